#!/bin/bash
# lane pairs: parity, then C2 / 512-infostate A/B (pairs on / off), then the multi-rank tests
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_c1.py tests/test_gpu_fixtures.py > gpurun_out/r4_pair_parity.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/env_sweep.py --workload c2 --contexts 2 "P=" "NP=DK_PAIR=0" > gpurun_out/r4_pair_c2.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/env_sweep.py --infostates 512 --contexts 2 --reps 4 "P=" "NP=DK_PAIR=0" > gpurun_out/r4_pair_small.log 2>&1 || exit 3
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_multi_rank.py > gpurun_out/r4_multirank.log 2>&1 || exit 4
