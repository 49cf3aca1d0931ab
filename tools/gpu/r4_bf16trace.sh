#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bf16tr
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bf16tr/t -o t -- python3 bench.py --workload c5 --steps 1 --warmup 1 > gpurun_out/bf16tr/c5.json 2> gpurun_out/bf16tr/c5.err || exit 1
f=$(find gpurun_out/bf16tr/t -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/bf16tr/c5_bf16_kernel_stats.csv
find gpurun_out/bf16tr/t -name "*kernel_trace.csv" -delete
