#!/bin/bash
# A/B timing of two builds of the library in one box session (alternating runs).
# A = libdoko_amd.so (current tree), B = libdoko_amd_ab.so (a reference build).
set -u
P=master_doko_reinforcement_learning_amd
for r in 1 2 3; do
  for lib in libdoko_amd.so libdoko_amd_ab.so; do
    out=$(DK_LIB=$P/$lib timeout -k 10 200 python bench.py --workload ${WORKLOAD:-c3} --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline) || exit $?
    echo "$lib $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3f G/s, %.2f ms/step kernel %.2f ms" % (d["value"]/1e9, d["ms_per_step"], d["search_kernel_ms"]))')"
  done
done
