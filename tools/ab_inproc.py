"""In-process A/B of two builds of libdoko_amd.so on the C3 search kernel.

Box clocks drift with load (the second of two back-to-back bench processes runs several %
slower), so two builds are compared inside ONE process: both libraries are loaded (ctypes,
separate handles), each gets its own context, and their search launches alternate
A B B A ... over the same determinized roots.  Prints the per-launch HIP-event times and the
mean / median ratio.  Both builds must produce identical visits (checked).

usage: python tools/ab_inproc.py A.so B.so [infostates] [reps]
       python tools/ab_inproc.py A.so B.so c2 [reps]     (C2: 32,768 rs-doko roots after 4x Healthy, as bench.py)
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(path):
    from master_doko_reinforcement_learning_amd import _native
    saved = _native._lib
    _native._lib = None
    os.environ["DK_LIB"] = path
    L = _native.lib()
    _native._lib = saved
    return L


def main(a, b, infostates=12288, reps=6):
    import torch
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    P = os.path.join(ROOT, "master_doko_reinforcement_learning_amd")
    libs = [load(os.path.join(P, a)), load(os.path.join(P, b))]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    c2 = infostates == "c2"
    I, S, iters = (512 if c2 else int(infostates)), 64, 1000
    n = I * S
    ctxs = []
    for L in libs:
        cfg = _native.dk_config(0, n, iters, 4096)      # measured slot high-water ~2.4K
        ctx = L.dk_create(ctypes.byref(cfg))
        assert ctx
        ctxs.append(ctx)
    L0, c0 = libs[0], ctxs[0]
    seeds = torch.tensor((np.arange(I, dtype=np.uint64) + np.uint64(0xC3000000)).view(np.int64), device=dev)
    info = torch.zeros((I, 128), dtype=torch.uint8, device=dev)
    assert L0.dk_new_game_batch_async(c0, 0, seeds.data_ptr(), I, info.data_ptr(), sp) == 0
    h = torch.full((I,), 1 << 24, dtype=torch.int64, device=dev)
    for _ in range(4):
        assert L0.dk_env_step_batch_async(c0, info.data_ptr(), h.data_ptr(), I, sp) == 0
    plies = torch.tensor(np.array([[0, 8, 20, 32][j % 4] for j in range(I)], dtype=np.uint32).view(np.int32), device=dev)
    rng = torch.tensor(dk.splitmix_rng_states(np.arange(I, dtype=np.uint64) + np.uint64(0xC3100000)).view(np.int64), device=dev)
    assert L0.dk_env_random_plies_batch_async(c0, info.data_ptr(), rng.data_ptr(), plies.data_ptr(), I, sp) == 0
    j = np.arange(I, dtype=np.uint64)[:, None]
    s = np.arange(S, dtype=np.uint64)[None, :]
    d_samp = torch.tensor((np.uint64(0xC3200000) + j * np.uint64(S) + s).reshape(-1).view(np.int64), device=dev)
    d_srch = torch.tensor((np.uint64(0xC3300000) + j * np.uint64(S) + s).reshape(-1).view(np.int64), device=dev)
    roots = torch.zeros((n, 128), dtype=torch.uint8, device=dev)
    game = dk.GAME_FULL_DOKO
    if c2:
        # bench.py's C2 roots and search seeds (rs-doko deals SmallRng::seed_from_u64(0xD0C00000 + i), 4x Healthy)
        game = dk.GAME_DOKO
        gidx = np.arange(n, dtype=np.uint64)
        d_rs = torch.tensor((gidx + np.uint64(0xD0C00000)).view(np.int64), device=dev)
        assert L0.dk_new_game_batch_async(c0, dk.GAME_DOKO, d_rs.data_ptr(), n, roots.data_ptr(), sp) == 0
        h = torch.full((n,), 1 << 24, dtype=torch.int64, device=dev)
        for _ in range(4):
            assert L0.dk_env_step_batch_async(c0, roots.data_ptr(), h.data_ptr(), n, sp) == 0
        d_srch = torch.tensor((gidx * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)).view(np.int64), device=dev)
    else:
        assert L0.dk_determinize_batch_async(c0, info.data_ptr(), I, S, d_samp.data_ptr(), roots.data_ptr(), sp) == 0
    outs = []
    for _ in libs:
        outs.append((torch.zeros((n, 39), dtype=torch.int32, device=dev), torch.zeros((n, 39), dtype=torch.float64, device=dev),
                     torch.zeros(n, dtype=torch.uint8, device=dev)))
    times = [[], []]
    order = [0, 1]
    for r in range(reps + 1):
        for k in order:
            v, q, bst = outs[k]
            assert libs[k].dk_search_batch_async(ctxs[k], game, roots.data_ptr(), d_srch.data_ptr(), n, iters, 2.5,
                                                 v.data_ptr(), q.data_ptr(), bst.data_ptr(), sp) == 0
            assert libs[k].dk_sync(ctxs[k], sp) == 0
            ms = ctypes.c_float()
            libs[k].dk_last_search_ms(ctxs[k], ctypes.byref(ms))
            if r > 0:                       # the first round warms both up
                times[k].append(ms.value)
            print("%s %.2f ms" % ((a, b)[k], ms.value), flush=True)
        order = order[::-1]
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), "builds disagree"
    ta, tb = np.array(times[0]), np.array(times[1])
    print("A %s mean %.2f median %.2f | B %s mean %.2f median %.2f | B/A time %.4f (median %.4f)"
          % (a, ta.mean(), np.median(ta), b, tb.mean(), np.median(tb), tb.mean() / ta.mean(), np.median(tb) / np.median(ta)))
    for L, c in zip(libs, ctxs):
        L.dk_destroy(c)


if __name__ == "__main__":
    args = sys.argv[1:]
    main(args[0], args[1], *((x if x == "c2" else int(x)) for x in args[2:]))
