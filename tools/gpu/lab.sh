#!/bin/bash
# Run measurement-harness binaries (tools/lab/<name>, built in the container) one after another:
#   bash tools/gpu/lab.sh <out-dir> <name>[:<args with commas>] ...
# each under its own time limit; the first failure ends the script.
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for step in "$@"; do
  IFS=: read -r name rest <<< "$step"
  echo "== $name"
  timeout -k 10 120 tools/lab/$name ${rest//,/ } > "$OUT/lab_$name.json" 2> "$OUT/lab_$name.err" || { tail -5 "$OUT/lab_$name.err"; exit 1; }
  cat "$OUT/lab_$name.json"
done
