"""Throughput with M independent C3 decision batches in flight on one GPU
(M streams, M engines; each step is one full C3 batch: determinize -> search ->
fuse).  Not the bench.py contract (that keeps one batch at a time); this
measures how much SIMD issue capacity a single 32,768-root batch leaves idle.
Usage (GPU box): DK_LDS_PATH=24 python tools/inflight_bench.py M steps
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(m=2, steps=6, infostates=2048):
    import torch

    import bench
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    sys.argv = [sys.argv[0], "--infostates", str(infostates)]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    L = _native.lib()
    works = []
    for i in range(m):
        st = torch.cuda.Stream(dev)
        with torch.cuda.stream(st):
            eng, step, n_roots, bufs = bench.make_workload(args, dk, L, dev, st.cuda_stream, 0, 1, 0)
        works.append((st, eng, step))
    for st, eng, step in works:            # warm-up
        with torch.cuda.stream(st):
            step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(steps):
        st, eng, step = works[s % m]
        with torch.cuda.stream(st):
            step()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    for st, eng, step in works:
        assert L.dk_sync(eng.ctx, st.cuda_stream) == 0
    print(json.dumps({"inflight": m, "steps": steps, "ms_per_step": el / steps * 1e3,
                      "rollouts_per_s": steps * n_roots * args.iterations / el,
                      "lds_path": os.environ.get("DK_LDS_PATH", "default")}))
    for st, eng, step in works:
        eng.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:4]))
