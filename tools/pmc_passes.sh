#!/bin/bash
# rocprofv3 PMC passes over one command, one counter set per pass (gfx950 slot limits: 8 SQ,
# 4 TCC (FETCH_SIZE takes 3, WRITE_SIZE 2), 2 GRBM per pass); kernel trace only, never combined
# with runtime/system tracing.  Every pass runs under its own time limit; the script stops at
# the first failing pass.
# usage: tools/pmc_passes.sh <out_dir> <command...>     (out_dir relative to the repo root)
# then:  python tools/pmc_report.py <out_dir> <kernel-name substring> ...
set -u
OUT=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
PASSES=(
  "FETCH_SIZE"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
  "TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE"
  "SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
)
# PMC_SETS="A B;C D" replaces the default passes (one pass per ';'-separated set)
if [ -n "${PMC_SETS:-}" ]; then IFS=';' read -r -a PASSES <<< "$PMC_SETS"; fi
i=0
for set in "${PASSES[@]}"; do
  i=$((i+1))
  echo "== pass $i: $set"
  timeout -k 10 ${PASS_TIMEOUT:-240} rocprofv3 --kernel-trace --output-format csv -d "$OUT/p$i" -o p$i --pmc $set -- "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; exit $rc; fi
done
