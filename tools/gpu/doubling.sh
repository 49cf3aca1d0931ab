#!/bin/bash
# Phase pricing of the C3 search kernel by doubling (round 6; profiles/r06/valu_by_phase.json):
# measurement builds that run one phase a second time with its result discarded
# (tools/build_variant.sh: roll2 -DDK_ROLL_DOUBLE, exp2 -DDK_EXP_DOUBLE, pick2 -DDK_PICK_DOUBLE=64,
# trick16 / trick64 -DDK_TRICK_DOUBLE=16 / 64).  Per variant: an in-process A/B against the product
# build (tools/ab_inproc.py: kernel time, identical visits) and one PMC pass (instruction counts).
#   bash tools/gpu/doubling.sh <out-dir> <variant> ...
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
P=$PWD/master_doko_reinforcement_learning_amd
SETS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
BENCH=(python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --small-infostates 0)
for v in base "$@"; do
  lib=$P/libdoko_amd.so; [ "$v" != base ] && lib=$P/libdoko_amd_$v.so
  echo "== pmc $v"
  DK_LIB=$lib PMC_SETS="$SETS" PASS_TIMEOUT=180 bash tools/pmc_passes.sh "$OUT/pmc_$v" "${BENCH[@]}" > "$OUT/pmc_$v.log" 2>&1 \
    || { tail -20 "$OUT/pmc_$v.log"; exit 1; }
  if [ "$v" != base ]; then
    echo "== ab $v"
    timeout -k 10 400 python3 -u tools/ab_inproc.py "$P/libdoko_amd.so" "$lib" 36864 3 > "$OUT/ab_$v.log" 2>&1 \
      || { tail -20 "$OUT/ab_$v.log"; exit 2; }
  fi
done
echo "== done"
