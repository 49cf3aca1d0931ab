#!/bin/bash
mkdir -p gpurun_out/r4l
L=master_doko_reinforcement_learning_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_network.py > gpurun_out/r4l/net_tests.log 2>&1 || exit 1
DK_LIB=$PWD/$L/libdoko_amd_bi.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_network.py -k "mlp or fused_network" > gpurun_out/r4l/net_tests_bi.log 2>&1 || exit 2
for k in 1 2; do
  timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4l/mlp_half.log 2>&1 || exit 3
  DK_LIB=$PWD/$L/libdoko_amd_g0.so timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4l/mlp_g0.log 2>&1 || exit 4
  DK_LIB=$PWD/$L/libdoko_amd_bi.so timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4l/mlp_bi.log 2>&1 || exit 5
done
