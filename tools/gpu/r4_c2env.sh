#!/bin/bash
mkdir -p gpurun_out/r4p
timeout -k 10 400 python -u tools/env_sweep.py --workload c2 --contexts 3 "D=" "LN1=DK_LN_LDS=1" "H32=DK_HOT_RECORD=32" > gpurun_out/r4p/c2_env.log 2>&1 || exit 1
