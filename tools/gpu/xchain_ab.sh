# Same-box A/B of the d = 256 x-only chain (DK_F32_XCHAIN=1) against the h-in / h-out chain (0), IMPI f32 bench.
set -e
OUT=gpurun_out/r6z; mkdir -p $OUT
for r in 1 2 3; do
  for x in 1 0; do
    DK_F32_XCHAIN=$x timeout -k 10 300 python -u bench.py --workload impi --net-precision f32 --steps 2 --warmup 1 > $OUT/x${x}_$r.json 2> $OUT/x${x}_$r.err
  done
done
