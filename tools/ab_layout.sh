#!/bin/bash
# A/B of the two hot-record layouts (DK_HOT_RECORD=16 / 32) against the per-launch
# default, alternating runs in one box session.  WORKLOAD=c3|c2|c2d, STEPS=n.
set -u
for r in 1 2; do
  for lay in default 16 32; do
    if [ $lay = default ]; then unset DK_HOT_RECORD; else export DK_HOT_RECORD=$lay; fi
    out=$(timeout -k 10 200 python bench.py --workload ${WORKLOAD:-c3} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline) || exit $?
    echo "${WORKLOAD:-c3} layout=$lay $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.2f ms/step kernel %.2f ms" % (d["ms_per_step"], d["search_kernel_ms"]))')"
  done
done
unset DK_HOT_RECORD
