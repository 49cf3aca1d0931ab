# max-ilp scheduling on the trick-aligned build, both A/B positions, C3 and the small batch
set -e
mkdir -p gpurun_out
timeout -k 10 150 python tools/ab_inproc.py libdoko_amd.so libdoko_amd_ilp.so 12288 6 > gpurun_out/ab_ilp2_c3_1.log 2>&1
timeout -k 10 150 python tools/ab_inproc.py libdoko_amd_ilp.so libdoko_amd.so 12288 6 > gpurun_out/ab_ilp2_c3_2.log 2>&1
timeout -k 10 100 python tools/ab_inproc.py libdoko_amd.so libdoko_amd_ilp.so 512 10 > gpurun_out/ab_ilp2_small_1.log 2>&1
timeout -k 10 100 python tools/ab_inproc.py libdoko_amd_ilp.so libdoko_amd.so 512 10 > gpurun_out/ab_ilp2_small_2.log 2>&1
