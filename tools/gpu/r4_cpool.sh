#!/bin/bash
mkdir -p gpurun_out/r4f
L=master_doko_reinforcement_learning_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_network.py > gpurun_out/r4f/net_tests.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 120 python -u tools/class_pool_bench.py >> gpurun_out/r4f/cpool_new.log 2>&1 || exit 2
  DK_LIB=$PWD/$L/libdoko_amd_cpold.so timeout -k 10 120 python -u tools/class_pool_bench.py >> gpurun_out/r4f/cpool_old.log 2>&1 || exit 3
done
