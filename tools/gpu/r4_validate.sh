#!/bin/bash
# final validation of the round's library: GPU suite, smoke, default bench line
mkdir -p gpurun_out/r4v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4v/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v/smoke.log 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > gpurun_out/r4v/bench_default.json 2> gpurun_out/r4v/bench_default.err || exit 3
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/r4v/c5.json 2> gpurun_out/r4v/c5.err || exit 4
