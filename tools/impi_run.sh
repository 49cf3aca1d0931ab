#!/bin/bash
# IMPI workload on the GPU box: parity tests, bench line, kernel-trace profile.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/impi
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_impi.py -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload impi --steps ${STEPS:-3} --warmup 1 > $OUT/bench.log 2>&1
rc=$?; grep '^{' $OUT/bench.log; [ $rc -ne 0 ] && { tail -20 $OUT/bench.log; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --workload impi --steps 2 --warmup 1 > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
