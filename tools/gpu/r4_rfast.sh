#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_fixtures.py > gpurun_out/r4_rfast_parity.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/env_sweep.py --infostates 18432 --contexts 4 --reps 3 "F=" "S=LIB=libdoko_amd_rs.so" > gpurun_out/r4_rfast_c3.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/env_sweep.py --infostates 512 --contexts 2 --reps 4 "F=" "S=LIB=libdoko_amd_rs.so" > gpurun_out/r4_rfast_small.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/env_sweep.py --workload c2 --contexts 2 "F=" "S=LIB=libdoko_amd_rs.so" > gpurun_out/r4_rfast_c2.log 2>&1 || exit 4
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_gpu_network.py > gpurun_out/r4_net_tests.log 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --workload c5 --net-precision f32 --steps 2 --warmup 1 > gpurun_out/r4b/c5_f32b.json 2> gpurun_out/r4b/c5_f32b.err || exit 6
L=master_doko_reinforcement_learning_amd
for k in 1 2; do
  DK_LIB=$PWD/$L/libdoko_amd_ag.so timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4_mlp_ag.log 2>&1 || exit 7
  timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4_mlp_poly.log 2>&1 || exit 8
  DK_LIB=$PWD/$L/libdoko_amd_w4.so timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4_mlp_w4.log 2>&1 || exit 9
done
