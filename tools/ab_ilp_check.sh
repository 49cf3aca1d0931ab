# max-ilp scheduler variant against the default build: C3 in one process (both orders),
# C2d / C2 through bench.py in alternating processes
set -e
mkdir -p gpurun_out
P=master_doko_reinforcement_learning_amd
timeout -k 10 150 python tools/ab_inproc.py libdoko_amd_ilp.so libdoko_amd.so 12288 6 > gpurun_out/ab2_c3.log 2>&1
for w in c2d c2; do
  for r in 1 2; do
    for lib in libdoko_amd.so libdoko_amd_ilp.so; do
      DK_LIB=$P/$lib timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab2_${w}_${lib}_$r.json
    done
  done
done
