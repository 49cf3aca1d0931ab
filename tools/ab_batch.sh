#!/bin/bash
# C3 rate by batch size (infostates of 64 roots each), interleaved reps.
set -u
for r in $(seq ${REPS:-2}); do
  for inf in ${INFS:-6144 9216 12288}; do
    out=$(timeout -k 10 300 python bench.py --workload ${WORKLOAD:-c3} --infostates $inf --steps 2 --warmup 1 --no-cpu-baseline) || exit $?
    echo "inf=$inf $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3f G/s kernel %.2f ms step %.1f ms" % (d["value"]/1e9, d["search_kernel_ms"], d["ms_per_step"]))')"
  done
done
