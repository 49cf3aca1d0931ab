#!/bin/bash
# A/B of library builds on C3 (ABBA-interleaved reps; compare medians).  LIBS="a.so b.so", INF="18432 24576"
set -u
P=master_doko_reinforcement_learning_amd
REPS=${REPS:-3}
for lib in ${LIBS}; do
  DK_LIB=$P/$lib DK_VERBOSE=1 timeout -k 10 300 python bench.py --workload ${WORKLOAD:-c3} --infostates ${INF%% *} --steps 1 --warmup 0 --no-cpu-baseline --small-infostates 0 2>&1 >/dev/null | grep "search n=" | sort | uniq -c || exit $?
done
order="${LIBS}"
for r in $(seq $REPS); do
  for lib in $order; do
    for inf in ${INF}; do
      out=$(DK_LIB=$P/$lib timeout -k 10 300 python bench.py --workload ${WORKLOAD:-c3} --infostates $inf --steps ${STEPS:-2} --warmup 1 --no-cpu-baseline --small-infostates 0 ${EXTRA:-}) || exit $?
      echo "$lib inf=$inf $(echo "$out" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3f G/s kernel %.2f ms" % (d["value"]/1e9, d["search_kernel_ms"]))')"
    done
  done
  order=$(echo $order | tr ' ' '\n' | tac | tr '\n' ' ')
done
