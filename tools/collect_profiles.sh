#!/bin/bash
# The profiles committed under profiles/<TAG>/ (run on the GPU box, after building in-tree):
#   1. rocprofv3 --kernel-trace --stats over the default bench command (C3, both legs) and over
#      the c2 / c2d workloads: per-kernel summaries whose search-kernel averages must agree with
#      the HIP-event times the traced bench lines print;
#   2. the PMC passes of tools/pmc_passes.sh over one bench step of C3 (both legs), C2 and C2d,
#      and over tools/pmc_calib (the counter calibration);
#   3. tools/pmc_finalize.py summaries: profiles/<TAG>/pmc_*.json.
# usage: TAG=r03 bash tools/collect_profiles.sh [trace|pmc|all]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r03}
WHAT=${1:-all}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT profiles/$TAG
run_trace() {   # name, bench args...
  local n=$1; shift
  echo "== trace $n"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$n -o t -- python3 bench.py "$@" \
    > $OUT/trace_$n.json 2> $OUT/trace_$n.err || { tail -20 $OUT/trace_$n.err; return 1; }
}
if [ "$WHAT" = trace ] || [ "$WHAT" = all ]; then
  run_trace c3 --steps 3 --no-cpu-baseline && \
  run_trace c2 --workload c2 --steps 5 --no-cpu-baseline && \
  run_trace c2d --workload c2d --steps 3 --no-cpu-baseline || exit 1
fi
if [ "$WHAT" = pmc ] || [ "$WHAT" = all ]; then
  PASS_TIMEOUT=120 bash tools/pmc_passes.sh $OUT/pmc_calib tools/pmc_calib && \
  PASS_TIMEOUT=240 bash tools/pmc_passes.sh $OUT/pmc_c3 python3 bench.py --steps 1 --warmup 0 --small-steps 1 \
    --no-cpu-baseline --host-readback-check && \
  PASS_TIMEOUT=180 bash tools/pmc_passes.sh $OUT/pmc_c2 python3 bench.py --workload c2 --steps 1 --warmup 0 --no-cpu-baseline && \
  PASS_TIMEOUT=180 bash tools/pmc_passes.sh $OUT/pmc_c2d python3 bench.py --workload c2d --steps 1 --warmup 0 --no-cpu-baseline \
    || exit 1
fi
