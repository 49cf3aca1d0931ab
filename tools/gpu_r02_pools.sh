# GPU check of the measured-capacity node pools + fallback pass (round 2)
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/t_pools.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -8 gpurun_out/t_pools.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_pools.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_pools.log
exit $rc
