# card facts computed in registers (-DDK_CARD_ALU) against the LDS table, on the latency-bound
# single-wave launches: C3's 512-infostate batch in one process (both positions), C2 by bench
set -e
mkdir -p gpurun_out
P=master_doko_reinforcement_learning_amd
timeout -k 10 100 python tools/ab_inproc.py libdoko_amd.so libdoko_amd_alu.so 512 10 > gpurun_out/ab_alu_small1.log 2>&1
timeout -k 10 100 python tools/ab_inproc.py libdoko_amd_alu.so libdoko_amd.so 512 10 > gpurun_out/ab_alu_small2.log 2>&1
for r in 1 2; do
  for lib in libdoko_amd.so libdoko_amd_alu.so; do
    DK_LIB=$P/$lib timeout -k 10 200 python bench.py --workload c2 --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/ab_alu_c2_${lib}_$r.json
  done
done
