#!/bin/bash
# Profiles committed under profiles/ (run on the GPU box):
#   1. rocprofv3 --kernel-trace --stats over the default bench workload
#   2. separate PMC passes (FETCH_SIZE, WRITE_SIZE, EA request counts) over one bench step
#      of the dominant launch only (--small-infostates 0: twice, a counter pass left rows of
#      the small-batch leg's visits overwritten with u64 words of 1000, never outside rocprofv3
#      --pmc)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/trace.log; exit $rc; }
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "== pmc $i: $set"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/pmc$i -o p --pmc $set -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --small-infostates 0 > $OUT/pmc$i.log 2>&1
  rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/pmc$i.log; exit $rc; }
done
exit 0
