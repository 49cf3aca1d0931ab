#!/bin/bash
mkdir -p gpurun_out/r4n
timeout -k 10 600 python -u tools/env_sweep.py --infostates 18432 --contexts 3 --reps 2 "D=" "L12=DK_LDS_PATH=12" "L16=DK_LDS_PATH=16" "G0=DK_GROUP_ORDER=0" > gpurun_out/r4n/c3_env.log 2>&1 || exit 1
