#!/bin/bash
# A/B: default build (2 waves/SIMD) vs libdoko_amd_ab.so built with -DDK_SEARCH_MIN_WAVES=3
# (3 waves/SIMD; node pools sized for 12 single-wave workgroups per CU) on C3.
set -u
P=master_doko_reinforcement_learning_amd
for r in 1 2; do
  for cfg in "libdoko_amd.so 0" "libdoko_amd_ab.so 196608"; do
    set -- $cfg
    for inf in 4096 6144; do
      if [ $2 = 0 ]; then unset DK_POOL_ROOTS; else export DK_POOL_ROOTS=$2; fi
      out=$(DK_LIB=$P/$1 timeout -k 10 200 python bench.py --infostates $inf --steps 2 --warmup 1 --no-cpu-baseline) || exit $?
      echo "$1 inf=$inf $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3f G/s kernel %.2f ms" % (d["value"]/1e9, d["search_kernel_ms"]))')"
    done
  done
done
unset DK_POOL_ROOTS
