#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/impitr
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/impitr/t -o t -- python3 bench.py --workload impi --steps 1 --warmup 1 > gpurun_out/impitr/impi.json 2> gpurun_out/impitr/impi.err || exit 1
f=$(find gpurun_out/impitr/t -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/impitr/impi_kernel_stats.csv
find gpurun_out/impitr/t -name "*kernel_trace.csv" -delete
