#!/bin/bash
# Parity tests of the default build, then an in-process A/B of two library builds on C3:
#   LIBS="libdoko_amd_prev.so libdoko_amd.so" CTX=3 bash tools/gpu_ab.sh
set -u
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_fixtures.py > gpurun_out/t_ab.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/t_ab.log; [ $rc -ne 0 ] && exit $rc
fi
set -- ${LIBS}
timeout -k 10 600 python -u tools/env_sweep.py "A=LIB=$1" "B=LIB=$2" --contexts ${CTX:-3} ${SWEEP_ARGS:-} > gpurun_out/ab.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -${TAILN:-9} gpurun_out/ab.log
exit $rc
