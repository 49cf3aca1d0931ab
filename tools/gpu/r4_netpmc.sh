#!/bin/bash
mkdir -p gpurun_out
PMC_SETS="SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE;SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" PASS_TIMEOUT=240 bash tools/pmc_passes.sh gpurun_out/pmc_c5net python3 bench.py --workload c5 --steps 1 --warmup 0 || exit 1
python3 tools/pmc_report.py gpurun_out/pmc_c5net qkv_attn_ln_kernel mlp_ln_kernel class_pool_ln_kernel embed_ln > gpurun_out/pmc_c5net/report.json || exit 2
rm -rf gpurun_out/pmc_c5net/p1 gpurun_out/pmc_c5net/p2
