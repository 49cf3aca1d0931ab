#!/bin/bash
mkdir -p gpurun_out/r4m
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests/test_gpu_network.py > gpurun_out/r4m/net_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c5 --net-precision f32 --steps 2 --warmup 1 > gpurun_out/r4m/c5_f32.json 2> gpurun_out/r4m/c5_f32.err || exit 2
timeout -k 10 300 python -u bench.py --workload impi --net-precision f32 --steps 2 --warmup 1 > gpurun_out/r4m/impi_f32.json 2> gpurun_out/r4m/impi_f32.err || exit 3
