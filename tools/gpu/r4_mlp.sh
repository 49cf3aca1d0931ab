#!/bin/bash
mkdir -p gpurun_out/r4c
L=master_doko_reinforcement_learning_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_network.py > gpurun_out/r4c/net_tests.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4c/mlp_wide.log 2>&1 || exit 2
  DK_LIB=$PWD/$L/libdoko_amd_ns.so timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4c/mlp_narrow.log 2>&1 || exit 3
done
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/r4c/c5.json 2> gpurun_out/r4c/c5.err || exit 4
