#!/bin/bash
# A/B: root groups in queue order by cards left (default) vs index order (DK_GROUP_ORDER=0).
set -u
for w in c3 c2d; do
  for r in 1 2 3; do
    for o in 1 0; do
      out=$(DK_GROUP_ORDER=$o timeout -k 10 200 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline) || exit $?
      echo "$w order=$o $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3f G/s kernel %.2f ms" % (d["value"]/1e9, d["search_kernel_ms"]))')"
    done
  done
done
