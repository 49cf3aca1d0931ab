#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py > gpurun_out/r4_touch_parity.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/env_sweep.py --infostates 18432 --contexts 2 --reps 3 "T=" "NT=LIB=libdoko_amd_nt.so" > gpurun_out/r4_touch_c3.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/env_sweep.py --workload c2 --contexts 2 "T=" "NT=LIB=libdoko_amd_nt.so" > gpurun_out/r4_touch_c2.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/env_sweep.py --infostates 512 --contexts 2 --reps 4 "T=" "NT=LIB=libdoko_amd_nt.so" > gpurun_out/r4_touch_small.log 2>&1 || exit 4
