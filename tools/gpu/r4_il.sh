#!/bin/bash
mkdir -p gpurun_out/r4k
L=master_doko_reinforcement_learning_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_network.py > gpurun_out/r4k/net_tests.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4k/mlp_il.log 2>&1 || exit 2
  DK_LIB=$PWD/$L/libdoko_amd_il0.so timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4k/mlp_il0.log 2>&1 || exit 3
done
DK_LIB=$PWD/$L/libdoko_amd_nprof.so timeout -k 10 120 python -u tools/mlp_prof.py > gpurun_out/r4k/mlp_prof_il.log 2>&1 || exit 4
