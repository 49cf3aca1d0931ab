#!/bin/bash
# round-4 GPU batch 1: new parity tests, C2 record/width sweep, f32 GEMM probe
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c1.py tests/test_gpu_inflight.py tests/test_gpu_parity.py -k "c1 or inflight or production or rng or reused or error or ttt or capacity" > gpurun_out/r4_t1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/env_sweep.py --workload c2 --contexts 2 "D=" "R16H8=DK_ROOTS_PER_WAVE=16,DK_HOT_RECORD=8" "R16H16=DK_ROOTS_PER_WAVE=16,DK_HOT_RECORD=16" "R32H16=DK_ROOTS_PER_WAVE=32,DK_HOT_RECORD=16" > gpurun_out/r4_c2_sweep.log 2>&1 || exit 2
timeout -k 10 120 python -u tools/fp32_gemm_probe.py gpurun_out/r4_fp32_probe.json > gpurun_out/r4_fp32_probe.log 2>&1 || exit 3
