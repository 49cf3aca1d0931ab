#!/bin/bash
# The bench's N>1 path on a one-GPU box: 2 ranks share cuda:0 and talk over gloo
# (the 8-GPU run uses RCCL, one rank per GPU).  The fused decisions of the 2-rank
# run (256 infostates per rank = 512 global, 32 samples each per rank) must equal
# a 1-rank run over the same 512 infostates x 64 samples (MaxN is exact).
set -u
mkdir -p gpurun_out
DK_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu-baseline \
    --infostates 256 --dump-actions gpurun_out/actions_2rank.npy || exit $?
timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --infostates 512 \
    --dump-actions gpurun_out/actions_1rank.npy || exit $?
python -c "
import numpy as np
a, b = np.load('gpurun_out/actions_2rank.npy'), np.load('gpurun_out/actions_1rank.npy')
print('2-rank vs 1-rank fused actions identical:', bool((a == b).all()), a.shape)
assert (a == b).all()
"
