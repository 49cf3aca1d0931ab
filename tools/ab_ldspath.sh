#!/bin/bash
# C3 at the bench default batch: LDS path entries per lane (interleaved reps; box clocks
# drift, so compare medians).  "auto" = the per-launch choice (launch_search_t);
# DK_VERBOSE prints the residency each launch gets.
set -u
REPS=${REPS:-5}
for lp in auto 16 15 14; do
  if [ "$lp" = auto ]; then env_lp=""; else env_lp="DK_LDS_PATH=$lp"; fi
  env $env_lp DK_VERBOSE=1 timeout -k 10 300 python bench.py --workload ${WORKLOAD:-c3} --steps 1 --warmup 0 --no-cpu-baseline 2>&1 >/dev/null | grep "search n=" | sort | uniq -c || exit $?
done
for r in $(seq $REPS); do
  for lp in ${LPS:-16 15 14}; do
    if [ "$lp" = auto ]; then env_lp=""; else env_lp="DK_LDS_PATH=$lp"; fi
    out=$(env $env_lp timeout -k 10 300 python bench.py --workload ${WORKLOAD:-c3} --steps 3 --warmup 1 --no-cpu-baseline) || exit $?
    echo "lds_path=$lp $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3f G/s kernel %.2f ms" % (d["value"]/1e9, d["search_kernel_ms"]))')"
  done
done
