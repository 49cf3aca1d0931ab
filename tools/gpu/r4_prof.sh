#!/bin/bash
mkdir -p gpurun_out
P=$PWD/master_doko_reinforcement_learning_amd/libdoko_amd_prof.so
DK_LIB=$P timeout -k 10 300 python -u tools/phase_prof.py --infostates 18432 > gpurun_out/r4_phase_c3.json 2> gpurun_out/r4_phase_c3.err || exit 1
DK_LIB=$P timeout -k 10 200 python -u tools/phase_prof.py --workload c2 > gpurun_out/r4_phase_c2.json 2> gpurun_out/r4_phase_c2.err || exit 2
timeout -k 10 300 python -u bench.py --workload impi --net-precision f32 --steps 2 --warmup 1 > gpurun_out/r4_impi_f32b.json 2> gpurun_out/r4_impi_f32b.err || exit 3
