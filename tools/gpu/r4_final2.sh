#!/bin/bash
mkdir -p gpurun_out/r4f2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4f2/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f2/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/r4f2/c5.json 2> gpurun_out/r4f2/c5.err || exit 3
timeout -k 10 300 python -u bench.py --workload impi --steps 3 --warmup 1 > gpurun_out/r4f2/impi.json 2> gpurun_out/r4f2/impi.err || exit 4
timeout -k 10 400 python -u bench.py > gpurun_out/r4f2/c3.json 2> gpurun_out/r4f2/c3.err || exit 5
