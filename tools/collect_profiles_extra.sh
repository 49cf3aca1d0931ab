#!/bin/bash
# Kernel-trace summaries of the non-default workloads (run on the GPU box):
#   c2d (determinized rs-doko: rule-based sampler + search), c2 (rs-doko roots), c5 (AlphaZero self-play),
#   impi (IMPI autoregressive determinization with the IMPI network)
# Output: gpurun_out/prof_extra/<workload>/ (rocprofv3 --kernel-trace --stats) + the traced bench line.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_extra${TAG:+_$TAG}
mkdir -p $OUT
for w in ${WORKLOADS:-c2d c2 c5 impi}; do
  case $w in
    c5) args="--workload c5 --steps 1 --warmup 1 --games 8192" ;;
    impi) args="--workload impi --steps 2 --warmup 1" ;;
    *)  args="--workload $w --steps 2 --warmup 1 --no-cpu-baseline" ;;
  esac
  echo "== trace $w"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$w -o run -- \
      python3 bench.py $args > $OUT/$w.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/$w.log; exit $rc; }
done
exit 0
