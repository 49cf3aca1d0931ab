#!/bin/bash
mkdir -p gpurun_out/r4h
L=master_doko_reinforcement_learning_amd
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_network.py > gpurun_out/r4h/net_tests.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 200 python -u tools/attn_bench.py >> gpurun_out/r4h/attn_new.log 2>&1 || exit 2
  DK_LIB=$PWD/$L/libdoko_amd_pold.so timeout -k 10 200 python -u tools/attn_bench.py >> gpurun_out/r4h/attn_old.log 2>&1 || exit 3
done
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/r4h/c5.json 2> gpurun_out/r4h/c5.err || exit 4
