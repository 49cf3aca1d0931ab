#!/bin/bash
# Search-kernel configuration sweep (phase-timer build) + parity under the chosen config.
set -u
mkdir -p gpurun_out
export DK_LIB=master_doko_reinforcement_learning_amd/libdoko_amd_prof.so
for cfg in ${SWEEP:-1:64 1:32 1:16}; do
  lay=${cfg%%:*}; rpw=${cfg##*:}
  DK_LAYOUT=$lay DK_ROOTS_PER_WAVE=$rpw timeout -k 10 120 python tools/phase_prof.py ${PROF_ARGS:-} >> gpurun_out/sweep.jsonl 2>> gpurun_out/sweep.err
  rc=$?
  echo "layout=$lay rpw=$rpw rc=$rc"; tail -n 1 gpurun_out/sweep.jsonl
  if [ $rc -ne 0 ]; then exit $rc; fi
done
