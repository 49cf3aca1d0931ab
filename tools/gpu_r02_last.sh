#!/bin/bash
# Last round-2 GPU evidence at the final build: every -m gpu test, smoke, the default bench
# line, small batches in flight on separate streams (M = 1, 2, 4), then the C3 profiles
# (kernel trace + PMC passes) into gpurun_out/prof_r02 (tools/summarize_profiles.py r02).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
for m in 1 2 4; do
  timeout -k 10 200 python tools/inflight_bench.py $m 8 512 >> gpurun_out/inflight.log 2>&1
  rc=$?; echo "inflight $m rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
rm -rf gpurun_out/prof_r02
TAG=r02 STEPS=3 bash tools/collect_profiles.sh
