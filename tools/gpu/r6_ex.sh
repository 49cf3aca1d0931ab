# The d = 256 x-only chain: GPU tests, the IMPI f32 bench, and the d = 256 MLP kernel (h in) against the previous build.
set -e
OUT=gpurun_out/r6w; mkdir -p $OUT
L=$PWD/master_doko_reinforcement_learning_amd
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "ex_halves or f32_network or mlp_ln_f32x3 or attn_ln_f32x3 or class" > $OUT/tests.log 2>&1
timeout -k 10 300 python -u bench.py --workload impi --net-precision f32 --steps 2 --warmup 1 > $OUT/impif32.json 2> $OUT/impif32.err
for r in 1 2; do
  for v in cur main; do
    lib=$L/libdoko_amd_$v.so; [ $v = main ] && lib=$L/libdoko_amd.so
    DK_LIB=$lib timeout -k 10 120 python -u tools/mlp_f32_bench.py 1523712 256 20 > $OUT/mlp256_${v}_$r.log 2>&1
  done
done
