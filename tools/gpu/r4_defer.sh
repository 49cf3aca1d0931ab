#!/bin/bash
mkdir -p gpurun_out
L=master_doko_reinforcement_learning_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_fixtures.py tests/test_gpu_c1.py tests/test_gpu_inflight.py > gpurun_out/r4_defer_parity.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/env_sweep.py --infostates 18432 --contexts 4 --reps 3 "D=" "N=LIB=libdoko_amd_nd.so" > gpurun_out/r4_defer_c3.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/env_sweep.py --infostates 512 --contexts 2 --reps 4 "D=" "N=LIB=libdoko_amd_nd.so" > gpurun_out/r4_defer_small.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/env_sweep.py --workload c2 --contexts 2 "D=" "N=LIB=libdoko_amd_nd.so" > gpurun_out/r4_defer_c2.log 2>&1 || exit 6
DK_LIB=$PWD/$L/libdoko_amd_prof.so timeout -k 10 300 python -u tools/phase_prof.py --infostates 18432 > gpurun_out/r4_phase_c3.json 2> gpurun_out/r4_phase_c3.err || exit 4
timeout -k 10 300 python -u bench.py --workload impi --net-precision f32 --steps 2 --warmup 1 > gpurun_out/r4_impi_f32b.json 2> gpurun_out/r4_impi_f32b.err || exit 5
