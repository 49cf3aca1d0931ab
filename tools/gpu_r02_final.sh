#!/bin/bash
# Round-2 GPU evidence: every -m gpu test, smoke, the default bench line, then the C3 profiles
# (kernel trace + PMC passes) into gpurun_out/prof_r02 (tools/summarize_profiles.py r02).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_all.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' gpurun_out/bench_default.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"]/1e9, d["search_kernel_ms"], d["roofline"]["frac"], d["small_batch"]["value"]/1e6, d["cpu_baseline"]["value"]/1e6)'; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof_r02
TAG=r02 STEPS=3 bash tools/collect_profiles.sh
