#!/bin/bash
# One parameterised GPU-box runner (replaces the per-experiment r4_*.sh scripts).
#   bash tools/gpu/run.sh <out-dir> <step> [<step> ...]
# Every step runs under its own time limit, output goes to gpurun_out/<out-dir>/<name>.{log,json,err},
# and the first failing step ends the script (no GPU step runs after a failure or a timeout).
# Steps:
#   tests[:<pytest -k expr>]     the GPU suite (or a -k subset)
#   smoke                        __graft_entry__.smoke()
#   bench:<name>[:<bench args>]  python bench.py <args>  (args: commas for spaces)
#   phase:<name>[:<args>]        tools/phase_prof.py with the profiling build (libdoko_amd_prof.so)
#   ab:<name>:<variantA>,<variantB>[:<args>]  tools/ab_inproc.py over two built variants
#   py:<name>:<script>[:<args>]  python <script> <args>
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
args_of() { echo "${1//,/ }"; }
for step in "$@"; do
  IFS=: read -r kind name rest more <<< "$step"
  case "$kind" in
    tests)
      K=(); [ -n "$name" ] && K=(-k "$name")
      echo "== tests ${name:-all}"
      timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" \
        > "$OUT/gpu_tests${name:+_sub}.log" 2>&1 || { tail -30 "$OUT/gpu_tests${name:+_sub}.log"; exit 1; } ;;
    smoke)
      echo "== smoke"
      timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 2; } ;;
    bench)
      echo "== bench $name"
      timeout -k 10 900 python -u bench.py $(args_of "$rest") > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 3; } ;;
    phase)
      echo "== phase $name"
      DK_LIB=$PWD/master_doko_reinforcement_learning_amd/libdoko_amd_prof.so timeout -k 10 600 python -u tools/phase_prof.py \
        $(args_of "$rest") > "$OUT/phase_$name.json" 2> "$OUT/phase_$name.err" || { tail -20 "$OUT/phase_$name.err"; exit 4; } ;;
    ab)
      echo "== ab $name"
      timeout -k 10 900 python -u tools/ab_inproc.py $(args_of "$rest") $(args_of "$more") > "$OUT/ab_$name.log" 2>&1 \
        || { tail -20 "$OUT/ab_$name.log"; exit 5; } ;;
    py)
      echo "== py $name"
      timeout -k 10 900 python -u "$rest" $(args_of "$more") > "$OUT/$name.log" 2>&1 || { tail -20 "$OUT/$name.log"; exit 6; } ;;
    *) echo "unknown step $step"; exit 9 ;;
  esac
done
echo "== done"
