#!/bin/bash
mkdir -p gpurun_out/r4o
L=master_doko_reinforcement_learning_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_network.py > gpurun_out/r4o/net_tests.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4o/mlp_g6.log 2>&1 || exit 2
  DK_LIB=$PWD/$L/libdoko_amd_g7.so timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4o/mlp_g7.log 2>&1 || exit 3
done
