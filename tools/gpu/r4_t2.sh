#!/bin/bash
# round-4 GPU batch 2: phase profiles of the single-wave launches; record-layout sweeps
mkdir -p gpurun_out
P=master_doko_reinforcement_learning_amd/libdoko_amd_prof.so
DK_LIB=$P timeout -k 10 120 python -u tools/phase_prof.py --workload c2 > gpurun_out/r4_phase_c2.json 2>gpurun_out/r4_phase.err || exit 1
DK_LIB=$P timeout -k 10 120 python -u tools/phase_prof.py --workload c3 --infostates 512 > gpurun_out/r4_phase_c3small.json 2>>gpurun_out/r4_phase.err || exit 2
DK_LIB=$P timeout -k 10 120 python -u tools/phase_prof.py --workload c3 --infostates 18432 > gpurun_out/r4_phase_c3.json 2>>gpurun_out/r4_phase.err || exit 3
timeout -k 10 300 python -u tools/env_sweep.py --workload c2 --contexts 2 "D=" "H16=DK_HOT_RECORD=16" "H8=DK_HOT_RECORD=8" > gpurun_out/r4_c2_sweep2.log 2>&1 || exit 4
timeout -k 10 300 python -u tools/env_sweep.py --infostates 512 --contexts 2 --reps 4 "D=" "H16=DK_HOT_RECORD=16" "H8=DK_HOT_RECORD=8" > gpurun_out/r4_small_sweep.log 2>&1 || exit 5
