#!/bin/bash
# Round-2 experiment 2: lane-interleaved pool layout (chunk 8 default) -- parity, then A/B against chunk 0 / 16
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bench_config.py tests/test_gpu_parity.py tests/test_gpu_fixtures.py > gpurun_out/t_e2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/t_e2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/env_sweep.py "c0=LIB=libdoko_amd_c0.so" "c8=LIB=libdoko_amd_c8.so" "c16=LIB=libdoko_amd_c16.so" --contexts 3 > gpurun_out/env_chunk.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -13 gpurun_out/env_chunk.log
exit $rc
