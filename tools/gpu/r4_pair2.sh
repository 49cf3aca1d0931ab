#!/bin/bash
mkdir -p gpurun_out
P=master_doko_reinforcement_learning_amd/libdoko_amd_prof.so
DK_LIB=$P timeout -k 10 120 python -u tools/phase_prof.py --workload c2 > gpurun_out/r4_phase_c2_pair.json 2>/dev/null || exit 1
DK_LIB=$P timeout -k 10 120 python -u tools/phase_prof.py --workload c3 --infostates 512 > gpurun_out/r4_phase_c3small_pair.json 2>/dev/null || exit 2
timeout -k 10 300 python -u tools/env_sweep.py --workload c2 --contexts 2 "P=" "PLN=DK_LN_LDS=1" > gpurun_out/r4_lnlds_c2.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/env_sweep.py --infostates 512 --contexts 2 --reps 4 "P=" "PLN=DK_LN_LDS=1" > gpurun_out/r4_lnlds_small.log 2>&1 || exit 4
