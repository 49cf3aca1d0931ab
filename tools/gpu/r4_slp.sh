#!/bin/bash
mkdir -p gpurun_out/r4i
L=master_doko_reinforcement_learning_amd
for k in 1 2; do
  timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4i/mlp_slp.log 2>&1 || exit 1
  DK_LIB=$PWD/$L/libdoko_amd_noslp.so timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4i/mlp_noslp.log 2>&1 || exit 2
done
timeout -k 10 200 python -u tools/attn_bench.py 10 160:8192 >> gpurun_out/r4i/attn_slp.log 2>&1 || exit 3
DK_LIB=$PWD/$L/libdoko_amd_noslp.so timeout -k 10 200 python -u tools/attn_bench.py 10 160:8192 >> gpurun_out/r4i/attn_noslp.log 2>&1 || exit 4
timeout -k 10 500 python -u tools/env_sweep.py --infostates 18432 --contexts 2 --reps 3 "D=" "N=LIB=libdoko_amd_noslp.so" > gpurun_out/r4i/c3.log 2>&1 || exit 5
