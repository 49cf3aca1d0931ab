#!/bin/bash
# Round-2 experiment 4: 8-B records -- phase profile and PMC passes (icache, VALU, memory)
set -u
mkdir -p gpurun_out
DK_LIB=master_doko_reinforcement_learning_amd/libdoko_amd_prof.so timeout -k 10 200 python tools/phase_prof.py > gpurun_out/phase_h8.json 2> gpurun_out/phase_h8.err
rc=$?; echo "phase rc=$rc"; cat gpurun_out/phase_h8.json; [ $rc -ne 0 ] && { tail -5 gpurun_out/phase_h8.err; exit $rc; }
rm -rf gpurun_out/pmc
export BENCH_ARGS="--steps 1 --warmup 0 --no-cpu-baseline --small-infostates 0"
bash tools/pmc.sh \
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" \
  "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
  "FETCH_SIZE" "WRITE_SIZE" \
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
rc=$?; echo "pmc rc=$rc"
python tools/pmc_sum.py search_kernel gpurun_out/pmc > gpurun_out/pmc_h8.json; cat gpurun_out/pmc_h8.json
exit $rc
