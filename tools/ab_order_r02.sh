# group queue order after the trick-aligned rollouts: C3 with longest-first (DK_GROUP_ORDER=1)
# against its default index order, C2d with index order (DK_GROUP_ORDER=0) against its default
set -e
mkdir -p gpurun_out
for r in 1 2; do
  for o in def 1; do
    if [ $o = def ]; then env=""; else env="DK_GROUP_ORDER=1"; fi
    env $env timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --small-infostates 0 > gpurun_out/ord_c3_${o}_$r.json
  done
  for o in def 0; do
    if [ $o = def ]; then env=""; else env="DK_GROUP_ORDER=0"; fi
    env $env timeout -k 10 200 python bench.py --workload c2d --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ord_c2d_${o}_$r.json
  done
done
