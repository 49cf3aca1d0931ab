#!/bin/bash
# round-4 GPU batch 3b: parity after the single-wave layout change, PC sampling probe
mkdir -p gpurun_out/pcs
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bench_config.py > gpurun_out/r4_parity.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval 1048576 -d gpurun_out/pcs/c3 -o c3 --output-format csv -- python3 tools/env_sweep.py --infostates 6144 --contexts 1 --reps 2 "D=" > gpurun_out/pcs/c3.log 2>&1
echo "rc=$?" >> gpurun_out/pcs/c3.log
ls -laR gpurun_out/pcs | head -40 >> gpurun_out/pcs/c3.log
