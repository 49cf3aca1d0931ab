# trick-aligned rollout with hands relative to the player on turn (-DDK_ROLLOUT_REL) against
# the per-ply loop: C3 and the 512-infostate batch, one process each, both A/B positions
set -e
mkdir -p gpurun_out
timeout -k 10 150 python tools/ab_inproc.py libdoko_amd.so libdoko_amd_rel.so 12288 6 > gpurun_out/ab_rel_c3_1.log 2>&1
timeout -k 10 150 python tools/ab_inproc.py libdoko_amd_rel.so libdoko_amd.so 12288 6 > gpurun_out/ab_rel_c3_2.log 2>&1
timeout -k 10 100 python tools/ab_inproc.py libdoko_amd.so libdoko_amd_rel.so 512 10 > gpurun_out/ab_rel_small_1.log 2>&1
timeout -k 10 100 python tools/ab_inproc.py libdoko_amd_rel.so libdoko_amd.so 512 10 > gpurun_out/ab_rel_small_2.log 2>&1
