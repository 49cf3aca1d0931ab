# Round-6 end-of-session check: the GPU suite, smoke, and the bench lines of C3 (default), C2,
# C5 (f32, interleaved parts) and IMPI (f32, interleaved parts), each step under its own limit.
#   bash tools/gpu/final_r6.sh [out-dir under gpurun_out]
set -e
OUT=gpurun_out/${1:-final_r6}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err
timeout -k 10 400 python -u bench.py --workload c5 --steps 3 --warmup 1 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
timeout -k 10 400 python -u bench.py --workload impi --steps 2 --warmup 1 > $OUT/bench_impi.json 2> $OUT/bench_impi.err
echo done
