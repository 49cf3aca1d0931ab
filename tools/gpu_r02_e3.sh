#!/bin/bash
# Round-2 experiment 3: 8-B packed hot records -- parity, then A/B against the 16-B records
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_fixtures.py > gpurun_out/t_e3.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/t_e3.log; [ $rc -ne 0 ] && exit $rc
DK_VERBOSE=1 timeout -k 10 600 python -u tools/env_sweep.py "h16=DK_HOT_RECORD=16" "h8=DK_HOT_RECORD=8" --contexts 3 > gpurun_out/env_h8.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v "search n=" gpurun_out/env_h8.log | tail -9; grep "search n=" gpurun_out/env_h8.log | sort | uniq -c
exit $rc
