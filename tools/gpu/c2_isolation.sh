set -u
O=gpurun_out/r6r; mkdir -p $O
for r in 1024 8192 32768; do
  DK_ROOTS_PER_WAVE=32 timeout -k 10 300 python -u bench.py --workload c2 --roots $r --steps 10 --warmup 2 --no-cpu-baseline > $O/c2_rpw32_$r.json 2> $O/c2_rpw32_$r.err || exit 1
done
