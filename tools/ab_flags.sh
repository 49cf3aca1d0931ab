set -e
mkdir -p gpurun_out
for v in ilp prio clause; do
  timeout -k 10 150 python tools/ab_inproc.py libdoko_amd.so libdoko_amd_$v.so 12288 6 > gpurun_out/ab_$v.log 2>&1
  timeout -k 10 100 python tools/ab_inproc.py libdoko_amd.so libdoko_amd_$v.so 512 8 > gpurun_out/ab_small_$v.log 2>&1
done
