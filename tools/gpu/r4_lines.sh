#!/bin/bash
# every workload's bench line on one box (round-4 final numbers)
mkdir -p gpurun_out/r4final
run() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r4final/$n.json 2> gpurun_out/r4final/$n.err; }
run c3 --steps 5 --warmup 1 || exit 1
run c2 --workload c2 --steps 5 --warmup 1 || exit 2
run c2d --workload c2d --steps 3 --warmup 1 || exit 3
run c5 --workload c5 --steps 3 --warmup 1 || exit 4
run c5_f32 --workload c5 --net-precision f32 --steps 2 --warmup 1 || exit 5
run impi --workload impi --steps 3 --warmup 1 || exit 6
run impi_f32 --workload impi --net-precision f32 --steps 2 --warmup 1 || exit 7
run impid --workload impid --steps 3 --warmup 1 || exit 8
run c1 --workload c1 --steps 3 --warmup 1 || exit 9
