#!/bin/bash
# C3: LDS path entries per lane (DK_LDS_PATH; 14 lets 12 workgroups fit a CU's LDS) and batch size.
set -u
for r in 1 2 3; do
  for cfg in "16 6144" "14 6144" "16 5632"; do
    set -- $cfg
    out=$(DK_LDS_PATH=$1 timeout -k 10 200 python bench.py --infostates $2 --steps 2 --warmup 1 --no-cpu-baseline) || exit $?
    echo "lds_path=$1 inf=$2 $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3f G/s kernel %.2f ms" % (d["value"]/1e9, d["search_kernel_ms"]))')"
  done
done
