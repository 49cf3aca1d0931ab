#!/bin/bash
# Round-2 experiment 1 (GPU box): phase profile, allocation sweep (contiguous pools), PMC passes
# (lane utilisation, instruction mix, TLB) over one C3 bench step.
set -u
mkdir -p gpurun_out
echo "== phase profile"
DK_LIB=master_doko_reinforcement_learning_amd/libdoko_amd_prof.so timeout -k 10 200 python tools/phase_prof.py > gpurun_out/phase_r02.json 2> gpurun_out/phase_r02.err
rc=$?; echo "rc=$rc"; cat gpurun_out/phase_r02.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/phase_r02.err; exit $rc; }
echo "== alloc sweep"
DK_VERBOSE=1 timeout -k 10 400 python -u tools/env_sweep.py "hip=DK_POOL_CONTIG=0" "contig=DK_POOL_CONTIG=1" --contexts 3 > gpurun_out/env_contig.log 2>&1
rc=$?; echo "rc=$rc"; grep -v "search n=" gpurun_out/env_contig.log | tail -12; grep "contiguous" gpurun_out/env_contig.log | head -3; [ $rc -ne 0 ] && exit $rc
export BENCH_ARGS="--steps 1 --warmup 0 --no-cpu-baseline --small-infostates 0"
bash tools/pmc.sh \
  "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
  "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE" \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
  "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TCC_HIT_sum TCC_MISS_sum"
rc=$?; echo "pmc rc=$rc"
python tools/pmc_sum.py search_kernel gpurun_out/pmc > gpurun_out/pmc_r02.json; cat gpurun_out/pmc_r02.json
exit $rc
