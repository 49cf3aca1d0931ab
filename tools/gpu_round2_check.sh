set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bench_config.py tests/test_gpu_multi_rank.py > gpurun_out/t_new.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/t_new.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/bench2.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench2.log
