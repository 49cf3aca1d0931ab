#!/bin/bash
# Round-2 full GPU check: every -m gpu test, the default bench line, and the C3 kernel trace.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -6 gpurun_out/t_all.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 2500 gpurun_out/bench_default.log
[ $rc -ne 0 ] && exit $rc
[ "${TRACE:-1}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r02/trace -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r02_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -c 1500 gpurun_out/prof_r02_trace.log
exit $rc
