"""Search-kernel time against the node-state stride between lane regions (one process,
C3 roots).  Every stride gets a fresh context (DK_STATE_STRIDE, records per lane region),
the C3 search runs `reps` times (the first warms up); the stride list is run forward and
backward `rounds` times so that clock drift and the placement of individual contexts'
pools average out.  Results must not change with the stride (checked).

usage: python tools/state_stride_sweep.py s1,s2,... [infostates] [reps] [rounds]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main(strides, infostates=18432, reps=3, rounds=2):
    import torch
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    from cap_sweep import c3_roots
    L = _native.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    I, S, iters = infostates, 64, 1000
    n = I * S
    roots, d_srch = c3_roots(dk, L, dev, sp, I, S)
    v = torch.zeros((n, 39), dtype=torch.int32, device=dev)
    q = torch.zeros((n, 39), dtype=torch.float64, device=dev)
    bst = torch.zeros(n, dtype=torch.uint8, device=dev)
    times = {s: [] for s in strides}
    ref = None
    order = []
    for _ in range(rounds):
        order += strides + strides[::-1]
    for st in order:
        os.environ["DK_STATE_STRIDE"] = str(st)
        e = dk.Engine(device=0, max_roots=n, max_iterations=iters, slot_capacity=4096)
        got = []
        for r in range(reps):
            assert L.dk_search_batch_async(e.ctx, 0, roots.data_ptr(), d_srch.data_ptr(), n, iters, 2.5,
                                           v.data_ptr(), q.data_ptr(), bst.data_ptr(), sp) == 0
            assert L.dk_sync(e.ctx, sp) == 0
            if r > 0:
                got.append(e.last_search_ms())
        e.close()
        times[st] += got
        if ref is None:
            ref = v.clone()
        assert torch.equal(ref, v), "stride changed the results"
        print("stride %5d (%6d B)  %s ms" % (st, st * 64, " ".join("%.1f" % t for t in got)), flush=True)
    os.environ.pop("DK_STATE_STRIDE", None)
    for st in strides:
        print("stride %5d (%6d B) median %.1f ms mean %.1f ms" % (st, st * 64, float(np.median(times[st])),
                                                                  float(np.mean(times[st]))))


if __name__ == "__main__":
    args = sys.argv[1:]
    main([int(x) for x in args[0].split(",")], *(int(x) for x in args[1:]))
