#!/bin/bash
# round-4 bench legs: c1, prod (production search shape), c5/impi at f32, c2
mkdir -p gpurun_out/r4b
timeout -k 10 300 python -u bench.py --workload c1 --steps 1 --warmup 1 > gpurun_out/r4b/c1.json 2> gpurun_out/r4b/c1.err || exit 1
timeout -k 10 300 python -u bench.py --workload c2 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r4b/c2.json 2> gpurun_out/r4b/c2.err || exit 2
timeout -k 10 300 python -u bench.py --workload c5 --net-precision f32 --steps 2 --warmup 1 > gpurun_out/r4b/c5_f32.json 2> gpurun_out/r4b/c5_f32.err || exit 3
timeout -k 10 300 python -u bench.py --workload impi --net-precision f32 --steps 2 --warmup 1 > gpurun_out/r4b/impi_f32.json 2> gpurun_out/r4b/impi_f32.err || exit 4
timeout -k 10 420 python -u bench.py --workload prod > gpurun_out/r4b/prod.json 2> gpurun_out/r4b/prod.err || exit 5
