#!/bin/bash
mkdir -p gpurun_out/r4d
L=master_doko_reinforcement_learning_amd
for k in 1 2; do
  for v in def p12 p22 p1222; do
    if [ $v = def ]; then lib=""; else lib=$PWD/$L/libdoko_amd_$v.so; fi
    DK_LIB=$lib timeout -k 10 120 python -u tools/mlp_bench.py >> gpurun_out/r4d/mlp_$v.log 2>&1 || exit 1
  done
done
