#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/f32tr
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f32tr/t -o t -- python3 bench.py --workload c5 --net-precision f32 --steps 1 --warmup 1 > gpurun_out/f32tr/c5.json 2> gpurun_out/f32tr/c5.err || exit 1
f=$(find gpurun_out/f32tr/t -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/f32tr/c5_f32_kernel_stats.csv
find gpurun_out/f32tr/t -name "*kernel_trace.csv" -delete
