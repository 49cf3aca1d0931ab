"""Small-batch launch mapping experiment: the C3 small decision batch (512 infostates x 64
samples = 32,768 roots, one wave per SIMD, so the launch lasts as long as its slowest wave)
searched with the roots in three orders -- as built (each 32-root wave holds half of one
infostate's samples), interleaved (each wave holds 32 infostates of the same depth k), and a
random permutation.  Outputs are scattered back and must equal the as-built order's
bit for bit.  Prints the search-kernel HIP-event times.
Usage (GPU box): python tools/small_perm.py [infostates] [reps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(infostates=512, reps=3):
    import torch

    import bench
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    sys.argv = [sys.argv[0], "--infostates", str(infostates)]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    L = _native.lib()
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    sp = st.cuda_stream
    eng, step, n, buf = bench.make_workload(args, dk, L, dev, sp, 0, 1, 0)
    step()
    torch.cuda.synchronize(dev)
    roots, seeds_all = buf["roots"].clone(), None
    S = args.samples
    I = infostates
    j = np.arange(I)[:, None].repeat(S, 1)
    s = np.arange(S)[None, :].repeat(I, 0)
    k = j % 4
    seeds = (np.uint64(0xC3300000) + j.astype(np.uint64) * np.uint64(S) + s.astype(np.uint64)).reshape(-1)
    orders = {
        "built": np.arange(n),
        "interleave_k": np.lexsort((j.reshape(-1), s.reshape(-1), k.reshape(-1))),
        "random": np.random.default_rng(5).permutation(n),
    }
    ref = None
    res = {}
    for name, o in orders.items():
        ot = torch.tensor(o, device=dev)
        r = roots[ot].contiguous()
        d_seeds = torch.tensor(seeds[o].view(np.int64), device=dev)
        visits = torch.zeros((n, 39), dtype=torch.int32, device=dev)
        values = torch.zeros((n, 39), dtype=torch.float64, device=dev)
        best = torch.zeros(n, dtype=torch.uint8, device=dev)
        ms = []
        for _ in range(reps + 1):
            rc = L.dk_search_batch_async(eng.ctx, dk.GAME_FULL_DOKO, r.data_ptr(), d_seeds.data_ptr(), n,
                                         args.iterations, args.c, visits.data_ptr(), values.data_ptr(),
                                         best.data_ptr(), sp)
            assert rc == 0, rc
            ms.append(eng.last_search_ms())
        inv = torch.empty_like(ot)
        inv[ot] = torch.arange(n, device=dev)
        v = visits[inv].cpu().numpy()
        val = values[inv].cpu().numpy().view(np.uint64)
        if ref is None:
            ref = (v, val)
        else:
            assert (v == ref[0]).all() and (val == ref[1]).all(), name
        res[name] = ms[1:]
        print("%-14s %s ms" % (name, " ".join("%.1f" % x for x in ms[1:])), flush=True)
    print("outputs identical across orders")


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
