"""Diagnostic: bench's two legs in one engine (the C3 batch, then the 512-infostate batch on
the same engine and stream), repeated, with every root's visit sum checked and the small
batch's outputs compared across repetitions.  Prints the roots whose sums are wrong.
Usage (GPU box): python tools/diag_small.py [big_infostates] [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(big=18432, reps=2):
    import copy

    import torch

    import bench
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    sys.argv = [sys.argv[0], "--infostates", str(big)]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    L = _native.lib()
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    sp = st.cuda_stream
    eng = None
    if big:
        eng, step, n, buf = bench.make_workload(args, dk, L, dev, sp, 0, 1, 0)
        step()
        torch.cuda.synchronize(dev)
        v = buf["visits"].cpu().numpy().sum(axis=1)
        print("big: roots %d bad %d" % (n, int((v != args.iterations).sum())), flush=True)
        del buf
    sa = copy.copy(args)
    sa.infostates = 512
    _, sstep, sn, sbuf = bench.make_workload(sa, dk, L, dev, sp, 0, 1, 0, eng=eng)
    ref = None
    for r in range(reps):
        sstep()
        torch.cuda.synchronize(dev)
        vis = sbuf["visits"].cpu().numpy()
        val = sbuf["values"].cpu().numpy()
        s = vis.sum(axis=1)
        bad = np.nonzero(s != sa.iterations)[0]
        print("small rep %d: bad %d %s" % (r, len(bad), [(int(i), int(s[i])) for i in bad[:12]]), flush=True)
        if ref is None:
            ref = (vis.copy(), val.copy())
        else:
            dv = np.nonzero((vis != ref[0]).any(axis=1))[0]
            print("  differs from rep 0 in %d roots %s" % (len(dv), dv[:12].tolist()), flush=True)
    hw, cap, ovf = (eng or dk.Engine).pool_high_water(sp) if eng is not None else (None, None, None)
    print("pool high water", hw, cap, ovf)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
