#!/bin/bash
# PMC passes over one bench step (separate passes: counter slot limits; never combined with tracing).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
ARGS=${BENCH_ARGS:-"--steps 1 --warmup 0 --no-cpu-baseline"}
i=0
for set in "$@"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/p$i -o p$i --pmc $set -- python3 bench.py $ARGS > gpurun_out/pmc/p$i.log 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/pmc/p$i.log; exit $rc; fi
done
