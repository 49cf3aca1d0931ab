#!/bin/bash
# C3: LDS path entries per lane (DK_LDS_PATH) vs resident workgroups per CU.
set -u
for r in 1 2; do
  for lp in 16 14 12; do
    out=$(DK_LDS_PATH=$lp timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline) || exit $?
    echo "lds_path=$lp $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3f G/s kernel %.2f ms" % (d["value"]/1e9, d["search_kernel_ms"]))')"
  done
done
