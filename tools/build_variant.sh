#!/bin/bash
# Build an experiment variant of libdoko_amd.so: tools/build_variant.sh <name> [-DFLAG=...]
# -> master_doko_reinforcement_learning_amd/libdoko_amd_<name>.so (A/B with tools/ab_inproc.py)
set -eu
P=master_doko_reinforcement_learning_amd
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared "$@" -o $P/libdoko_amd_$name.so $P/csrc/doko_amd.hip
