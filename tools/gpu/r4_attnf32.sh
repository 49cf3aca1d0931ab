#!/bin/bash
mkdir -p gpurun_out/r4e
L=master_doko_reinforcement_learning_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_network.py > gpurun_out/r4e/net_tests.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 120 python -u tools/attn_f32_bench.py >> gpurun_out/r4e/attn_mfma.log 2>&1 || exit 2
  DK_LIB=$PWD/$L/libdoko_amd_a3.so timeout -k 10 120 python -u tools/attn_f32_bench.py >> gpurun_out/r4e/attn_w3.log 2>&1 || exit 3
done
timeout -k 10 300 python -u bench.py --workload c5 --net-precision f32 --steps 2 --warmup 1 > gpurun_out/r4e/c5_f32.json 2> gpurun_out/r4e/c5_f32.err || exit 4
