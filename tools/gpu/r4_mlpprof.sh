#!/bin/bash
mkdir -p gpurun_out/r4j
L=master_doko_reinforcement_learning_amd
DK_LIB=$PWD/$L/libdoko_amd_nprof.so timeout -k 10 120 python -u tools/mlp_prof.py > gpurun_out/r4j/mlp_prof.log 2>&1 || exit 1
