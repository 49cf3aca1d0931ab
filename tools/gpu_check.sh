#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
set -u
mkdir -p gpurun_out
STEPS=${STEPS:-3}
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  # 0 ok, 1 = test/assert failure (no fault): keep going; anything else: stop
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
run gpu_tests 600 python -m pytest tests -m gpu -x -q
run smoke 180 python -c "import __graft_entry__ as g; g.smoke()"
run bench 300 python bench.py --steps "$STEPS" --warmup 1

true
