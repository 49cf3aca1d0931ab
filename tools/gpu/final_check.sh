# End-of-session check: the GPU suite, smoke, the default bench, the network benches, and a
# kernel trace of the IMPI f32 step.   usage: bash tools/gpu/final_check.sh [out-dir under gpurun_out]
set -e
OUT=gpurun_out/${1:-final}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 > $OUT/bench_c5.json 2> $OUT/bench_c5.err
timeout -k 10 300 python -u bench.py --workload c5 --net-precision f32 --steps 2 --warmup 1 > $OUT/bench_c5f32.json 2> $OUT/bench_c5f32.err
timeout -k 10 300 python -u bench.py --workload impi --net-precision f32 --steps 2 --warmup 1 > $OUT/bench_impif32.json 2> $OUT/bench_impif32.err
timeout -k 10 300 python -u bench.py --workload impi --steps 2 --warmup 1 > $OUT/bench_impi.json 2> $OUT/bench_impi.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_impif32 -o t -- python3 bench.py --workload impi --net-precision f32 --steps 1 --warmup 1 > $OUT/trace_impif32.json 2> $OUT/trace_impif32.err
