#!/bin/bash
# Round-2 closing run: every -m gpu test, smoke, the default C3 bench line, C2 / C2d lines
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
for w in c2 c2d; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/bench_$w.log 2>&1
  rc=$?; echo "bench $w rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
