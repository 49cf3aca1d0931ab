# A/B of two libdoko_amd builds on the f32 MLP kernel (tools/mlp_f32_bench.py), after the f32 MLP /
# network tests under build B.   usage: bash tools/gpu/ab_mlp16.sh <out> <A> <B> [rows] [d]
set -e
OUT=gpurun_out/$1; A=$2; B=$3; ROWS=${4:-1523712}; D=${5:-256}
mkdir -p $OUT
L=$PWD/master_doko_reinforcement_learning_amd
DK_LIB=$L/libdoko_amd_$B.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "mlp_ln_f32x3 or f32_network" > $OUT/tests_$B.log 2>&1
for r in 1 2 3; do
  for v in $A $B; do
    DK_LIB=$L/libdoko_amd_$v.so timeout -k 10 120 python -u tools/mlp_f32_bench.py $ROWS $D 20 > $OUT/${v}_$r.log 2>&1
  done
done
