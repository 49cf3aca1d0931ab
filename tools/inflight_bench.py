"""Throughput with K independent C3 decision batches in flight on one GPU.

Modes:
  engine  one engine, DefaultImpiPolicy.execute_async on K streams (the product path:
          concurrent search slots over disjoint pool lanes)
  engines K engines, one per stream (round 2's caller-managed variant)
Each step issues K whole decisions (determinize -> search -> fuse -> select) and waits for
them; per-stream start/end events show whether the searches overlapped on the GPU.
Usage (GPU box): python tools/inflight_bench.py [engine|engines] K [steps] [infostates]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(mode="engine", k=2, steps=4, infostates=512):
    import torch

    import bench
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    k, steps, infostates = int(k), int(steps), int(infostates)
    sys.argv = [sys.argv[0], "--infostates", str(infostates)]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    L = _native.lib()
    S, iters = args.samples, args.iterations
    n = infostates * S
    main_st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(main_st)
    eng0, _, _, bufs = bench.make_workload(args, dk, L, dev, main_st.cuda_stream, 0, 1, 0)
    info = bufs["info"]
    if mode == "engines":
        engines = [eng0] + [dk.Engine(device=0, max_roots=n, max_iterations=iters) for _ in range(k - 1)]
    else:   # one engine whose pools hold the K batches' lanes at once
        eng0.close()
        engines = [dk.Engine(device=0, max_roots=k * n, max_iterations=iters)]
    pols = [dk.DefaultImpiPolicy(e, args.c, iters, S, dk.FUSE_MAXN) for e in engines]
    streams = [torch.cuda.Stream(dev) for _ in range(k)]
    seeds = []
    for b in range(k):
        base = np.uint64(0xE1000000 + (b << 24))
        sd = np.concatenate([np.arange(2 * n, dtype=np.uint64) + base])
        seeds.append(torch.tensor(sd.view(np.int64), device=dev))
    torch.cuda.synchronize(dev)

    def one_step(record=None):
        for b in range(k):
            st = streams[b]
            st.wait_stream(main_st)
            with torch.cuda.stream(st):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                pols[b % len(pols)].execute_async(info, seeds[b], game=dk.GAME_FULL_DOKO)
                e1.record()
                if record is not None:
                    record.append((b, e0, e1))
        for b in range(k):
            assert L.dk_sync(engines[b % len(engines)].ctx, streams[b].cuda_stream) == 0
        torch.cuda.synchronize(dev)

    one_step()
    rec = []
    t0 = time.perf_counter()
    for _ in range(steps):
        one_step(rec)
    el = time.perf_counter() - t0
    ref = rec[0][1]
    spans = [(b, ref.elapsed_time(e0), ref.elapsed_time(e1)) for b, e0, e1 in rec[:k]]
    print(json.dumps({"mode": mode, "inflight": k, "steps": steps, "infostates": infostates,
                      "ms_per_step": el / steps * 1e3, "rollouts_per_s": k * n * iters * steps / el,
                      "first_step_spans_ms": [[b, round(a, 2), round(z, 2)] for b, a, z in spans]}))
    for e in engines:
        e.close()


if __name__ == "__main__":
    main(*sys.argv[1:5])
