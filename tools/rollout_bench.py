"""Rollout micro-benchmark: random playouts (A7) from the bench's C3 roots through
dk_env_rollout_batch_async, one lane per root, `reps` launches.  Prints rollouts/s
and the mean plies per rollout.  Usage (GPU box): python tools/rollout_bench.py [reps]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(reps=50):
    import torch

    import bench
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    L = _native.lib()
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    eng, step, n_roots, bufs = bench.make_workload(args, dk, L, dev, sp, 0, 1, 0)
    step()   # determinize (and one search) so that bufs["roots"] holds the C3 roots
    roots = bufs["roots"]
    rng = torch.tensor(dk.splitmix_rng_states(np.arange(n_roots, dtype=np.uint64) + np.uint64(77)).view(np.int64),
                       device=dev)
    rew = torch.zeros((n_roots, 4), dtype=torch.float64, device=dev)
    assert L.dk_env_rollout_batch_async(eng.ctx, roots.data_ptr(), rng.data_ptr(), n_roots, rew.data_ptr(), sp) == 0
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        assert L.dk_env_rollout_batch_async(eng.ctx, roots.data_ptr(), rng.data_ptr(), n_roots, rew.data_ptr(), sp) == 0
    e1.record()
    torch.cuda.synchronize(dev)
    assert L.dk_sync(eng.ctx, sp) == 0
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps({"roots": n_roots, "ms_per_launch": ms, "rollouts_per_s": n_roots / (ms / 1e3)}))
    eng.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:2]))
