# Alternate a python tool over several builds of libdoko_amd:  bash tools/gpu/ab_variants.sh <out> "<tool + args>" <rounds> <variant>...
set -e
OUT=gpurun_out/$1; TOOL=$2; R=$3; shift 3
mkdir -p $OUT
L=$PWD/master_doko_reinforcement_learning_amd
for r in $(seq 1 $R); do
  for v in "$@"; do
    DK_LIB=$L/libdoko_amd_$v.so timeout -k 10 180 python -u $TOOL > $OUT/${v}_$r.log 2>&1
  done
done
