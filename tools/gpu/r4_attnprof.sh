#!/bin/bash
mkdir -p gpurun_out/r4g
L=master_doko_reinforcement_learning_amd
DK_LIB=$PWD/$L/libdoko_amd_nprof.so timeout -k 10 120 python -u tools/attn_prof.py 160 8192 > gpurun_out/r4g/attn_prof.log 2>&1 || exit 1
DK_LIB=$PWD/$L/libdoko_amd_nprof.so timeout -k 10 120 python -u tools/attn_prof.py 256 2048 >> gpurun_out/r4g/attn_prof.log 2>&1 || exit 2
