# rs-doko trick-aligned rollout (libdoko_amd_dko.so) against the current library: C2 and C2d
# through bench.py in alternating processes
set -e
mkdir -p gpurun_out
P=master_doko_reinforcement_learning_amd
for w in c2 c2d; do
  for r in 1 2; do
    for lib in libdoko_amd.so libdoko_amd_dko.so; do
      DK_LIB=$P/$lib timeout -k 10 200 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --dump-acc gpurun_out/acc_${w}_${lib}.npy > gpurun_out/ab_dko_${w}_${lib}_$r.json
    done
  done
done
python -c "
import numpy as np
a=np.load('gpurun_out/acc_c2d_libdoko_amd.so.npy'); b=np.load('gpurun_out/acc_c2d_libdoko_amd_dko.so.npy')
print('c2d fusion accumulators equal:', bool((a==b).all()))"
