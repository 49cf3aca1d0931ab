"""Search-kernel time against the main pools' slot capacity (one process, C3 roots).

For every capacity a context is created, the C3 search runs `reps` times (first one
warms up), and the context is destroyed; the capacity list is then run again in reverse
order so that clock drift cancels.  Prints ms per launch and the pool high water.

usage: python tools/cap_sweep.py cap1,cap2,... [infostates] [reps]
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(caps, infostates=18432, reps=3):
    import torch
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
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
    times = {cap: [] for cap in caps}
    ref = None
    for cap in caps + caps[::-1]:
        e = dk.Engine(device=0, max_roots=n, max_iterations=iters, slot_capacity=cap)
        for r in range(reps):
            assert L.dk_search_batch_async(e.ctx, 0, roots.data_ptr(), d_srch.data_ptr(), n, iters, 2.5,
                                           v.data_ptr(), q.data_ptr(), bst.data_ptr(), sp) == 0
            assert L.dk_sync(e.ctx, sp) == 0
            ms = e.last_search_ms()
            if r > 0:
                times[cap].append(ms)
        hw = e.pool_high_water(sp)
        e.close()
        if ref is None:
            ref = v.clone()
        assert torch.equal(ref, v), "capacity changed the results"
        print("cap %6d  %s ms  high water %s  pool %.1f GB" % (cap, " ".join("%.1f" % t for t in times[cap][-(reps - 1):]),
                                                              hw, e_bytes(cap, n, iters)), flush=True)
    for cap in caps:
        print("cap %6d median %.1f ms" % (cap, float(np.median(times[cap]))))


def c3_roots(dk, L, dev, sp, I, S=64):
    """The bench's C3 roots (determinized on the device) and search seeds."""
    import torch
    n = I * S
    gen = dk.Engine(device=0, max_roots=n, max_iterations=1, slot_capacity=64)
    c0 = gen.ctx
    seeds = torch.tensor((np.arange(I, dtype=np.uint64) + np.uint64(0xC3000000)).view(np.int64), device=dev)
    info = torch.zeros((I, 128), dtype=torch.uint8, device=dev)
    assert L.dk_new_game_batch_async(c0, 0, seeds.data_ptr(), I, info.data_ptr(), sp) == 0
    h = torch.full((I,), 1 << 24, dtype=torch.int64, device=dev)
    for _ in range(4):
        assert L.dk_env_step_batch_async(c0, info.data_ptr(), h.data_ptr(), I, sp) == 0
    plies = torch.tensor(np.array([[0, 8, 20, 32][j % 4] for j in range(I)], dtype=np.uint32).view(np.int32), device=dev)
    rng = torch.tensor(dk.splitmix_rng_states(np.arange(I, dtype=np.uint64) + np.uint64(0xC3100000)).view(np.int64), device=dev)
    assert L.dk_env_random_plies_batch_async(c0, info.data_ptr(), rng.data_ptr(), plies.data_ptr(), I, sp) == 0
    j = np.arange(I, dtype=np.uint64)[:, None]
    s = np.arange(S, dtype=np.uint64)[None, :]
    d_samp = torch.tensor((np.uint64(0xC3200000) + j * np.uint64(S) + s).reshape(-1).view(np.int64), device=dev)
    d_srch = torch.tensor((np.uint64(0xC3300000) + j * np.uint64(S) + s).reshape(-1).view(np.int64), device=dev)
    roots = torch.zeros((n, 128), dtype=torch.uint8, device=dev)
    assert L.dk_determinize_batch_async(c0, info.data_ptr(), I, S, d_samp.data_ptr(), roots.data_ptr(), sp) == 0
    assert L.dk_sync(c0, sp) == 0
    gen.close()
    return roots, d_srch


def e_bytes(cap, n, iters):
    return min(n, 256 * 12 * 64) * cap * 48 / 1e9


if __name__ == "__main__":
    args = sys.argv[1:]
    main([int(x) for x in args[0].split(",")], *(int(x) for x in args[1:]))
