"""Several searches in flight on ONE engine (dk_search_batch_async on several streams).

Each launch takes its own search slot (queue counters, retry list, root orders, error
flag, events) and a range of pool lanes; a launch waits on the GPU for earlier launches
whose lanes it reuses.  These tests check that concurrency changes no result:
  * K independent decision batches through DefaultImpiPolicy.execute_many -- batched into
    one pass, or issued on K streams -- equal the same batches decided one at a time, and
    sampled roots equal oracle searches;
  * a full-pool batch and small batches issued on different streams at once (lanes that
    overlap, so the GPU-side waits must order them) equal their separate results;
  * more launches in flight than there are slots (slot reuse across streams).

Reference semantics: compare_impi.rs:212-371 (DefaultImpiPolicy::execute per decision),
mcts.rs:172-249; the evaluator runs many games at once (compare_impi/run.rs:775).
"""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu

ITERS = 300


def _info(j):
    st = ol.FdoState.new_game(0xF1000000 + j)
    for _ in range(4):
        st.play(24)
    st.random_plies(ol.rng_seed(0xF1100000 + j), [0, 8, 20, 32][j % 4], True)
    return st


def _batches(torch, dev, k, n_info, S):
    infos = [_info(j) for j in range(n_info)]
    packed = torch.tensor(np.frombuffer(b"".join(s.pack() for s in infos), dtype=np.uint8).reshape(-1, 128).copy(),
                          device=dev)
    out = []
    for b in range(k):
        sd = np.arange(2 * n_info * S, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1000 * b + 7)
        out.append((packed, torch.tensor(sd.view(np.int64), device=dev)))
    return infos, out


def test_execute_many_equals_sequential():
    import torch

    import master_doko_reinforcement_learning_amd as dk
    dev = torch.device("cuda", 0)
    S, n_info, k = 16, 96, 3
    eng = dk.Engine(device=0, max_roots=k * n_info * S, max_iterations=ITERS)
    try:
        pol = dk.DefaultImpiPolicy(eng, 2.5, ITERS, S, dk.FUSE_MAXN)
        infos, batches = _batches(torch, dev, k, n_info, S)
        many = pol.execute_many(batches, game=dk.GAME_FULL_DOKO)               # one batched pass
        many_st = pol.execute_many(batches, game=dk.GAME_FULL_DOKO, streams=k)   # concurrent streams
        one = []
        for b in batches:
            a, v = pol.execute_async(*b, game=dk.GAME_FULL_DOKO)
            torch.cuda.synchronize(dev)
            one.append((a.cpu().numpy(), v.cpu().numpy()))
        for res in (many, many_st):
            for (a, v), (a1, v1) in zip(res, one):
                assert np.array_equal(a.cpu().numpy(), a1)
                assert np.array_equal(v.cpu().numpy(), v1)
    finally:
        eng.close()
    # oracle: sampled roots of every batch (CAP sample, then the search on its seed)
    rng = np.random.default_rng(3)
    n = n_info * S
    for b, (a, v) in enumerate(one):
        sd = batches[b][1].cpu().numpy().view(np.uint64)
        for r in rng.choice(n, size=6, replace=False):
            j = r // S
            smp = infos[j].card_matching(ol.rng_seed(int(sd[r])))
            _, ov, _, _ = smp.search(ol.rng_seed(int(sd[n + r])), ITERS, 2.5)
            assert list(v[r]) == ov, (b, r)
        j = int(rng.integers(n_info))
        rows = [list(v[j * S + s]) for s in range(S)]
        exp, _ = ol.fuse_maxn(rows, infos[j].allowed())
        assert int(a[j]) == exp


def test_full_pool_and_small_batches_concurrently():
    """A batch that fills the pools on one stream while small batches run on two others: the
    lane ranges overlap, so the later launches must wait on the GPU; and eleven launches in
    flight cycle the eight slots."""
    import torch

    import master_doko_reinforcement_learning_amd as dk
    dev = torch.device("cuda", 0)
    S = 16
    eng = dk.Engine(device=0, max_roots=262144, max_iterations=ITERS)
    try:
        pol = dk.DefaultImpiPolicy(eng, 2.5, ITERS, S, dk.FUSE_MAXN)
        _, big = _batches(torch, dev, 1, 12288, S)         # 196,608 roots: every pool lane
        _, small = _batches(torch, dev, 10, 64, S)         # 1,024 roots each
        ref_big = pol.execute_many(big, game=dk.GAME_FULL_DOKO)[0][1].cpu().numpy()
        ref_small = [v.cpu().numpy() for _, v in pol.execute_many(small, game=dk.GAME_FULL_DOKO, streams=1)]
        streams = [torch.cuda.Stream(dev) for _ in range(3)]
        res = []
        with torch.cuda.stream(streams[0]):
            res.append(pol.execute_async(*big[0], game=dk.GAME_FULL_DOKO))
        for i, b in enumerate(small):
            with torch.cuda.stream(streams[1 + i % 2]):
                res.append(pol.execute_async(*b, game=dk.GAME_FULL_DOKO))
        L = dk._native.lib()
        for s in streams:
            assert L.dk_sync(eng.ctx, s.cuda_stream) == 0
        torch.cuda.synchronize(dev)
        assert np.array_equal(res[0][1].cpu().numpy(), ref_big)
        for (_, v), r in zip(res[1:], ref_small):
            assert np.array_equal(v.cpu().numpy(), r)
    finally:
        eng.close()


def test_error_of_reused_slot_reaches_dk_sync():
    """A malformed root on stream A (DK_E_STATE), then nine more launches on stream B before
    anyone syncs: the ninth reuses A's slot.  dk_sync(B) is clean and dk_sync(A) still
    reports A's error (it is folded into A's pending errors when the slot is reused)."""
    import torch

    import master_doko_reinforcement_learning_amd as dk
    dev = torch.device("cuda", 0)
    L = dk._native.lib()
    eng = dk.Engine(device=0, max_roots=1024, max_iterations=ITERS)
    try:
        s = ol.DoState.new_game(0xBAD)
        for _ in range(4):
            s.play(24)
        good = np.frombuffer(s.pack(), dtype=np.uint8).copy()
        bad = good.copy()
        bad[7] |= 0x01                                   # hand 0, bit 56: DK_E_STATE
        a, b = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        n = 64
        keep = []

        def launch(stream, root):
            roots = torch.tensor(np.tile(root, (n, 1)), device=dev)
            seeds = torch.arange(n, dtype=torch.int64, device=dev)
            vis = torch.empty((n, 39), dtype=torch.int32, device=dev)
            val = torch.empty((n, 39), dtype=torch.float64, device=dev)
            best = torch.empty(n, dtype=torch.uint8, device=dev)
            keep.append((roots, seeds, vis, val, best))
            return L.dk_search_batch_async(eng.ctx, dk.GAME_DOKO, roots.data_ptr(), seeds.data_ptr(), n, 50, 2.5,
                                           vis.data_ptr(), val.data_ptr(), best.data_ptr(), stream.cuda_stream)

        torch.cuda.synchronize(dev)
        assert launch(a, bad) == 0
        for _ in range(9):
            assert launch(b, good) == 0
        assert L.dk_sync(eng.ctx, b.cuda_stream) == 0
        assert L.dk_sync(eng.ctx, a.cuda_stream) == -3      # DK_E_STATE
        assert L.dk_sync(eng.ctx, a.cuda_stream) == 0       # reported once
        torch.cuda.synchronize(dev)
        for _, _, vis, _, _ in keep[1:]:
            assert bool((vis.sum(dim=1) == 50).all())
    finally:
        eng.close()


def test_reused_slot_lane_regions():
    """The lane-overlap pattern of a reused slot: X fills 60 % of the pool lanes on stream A,
    seven small launches take the other slots, X's slot is reused on stream A for the last
    lanes, and a launch on stream B wraps round to lanes X may still be using.  Its wait must
    come from the lane regions X covered, not from the slot's latest lane range.  Every
    result equals the same batch decided alone."""
    import torch

    import master_doko_reinforcement_learning_amd as dk
    dev = torch.device("cuda", 0)
    S = 16
    eng = dk.Engine(device=0, max_roots=65536, max_iterations=ITERS)
    try:
        pol = dk.DefaultImpiPolicy(eng, 2.5, ITERS, S, dk.FUSE_MAXN)
        sizes = [2456] + [205] * 7 + [205, 1229]           # infostates x 16 samples per launch
        batches = [_batches(torch, dev, 1, k, S)[1][0] for k in sizes]
        ref = [v.cpu().numpy() for _, v in pol.execute_many(batches, game=dk.GAME_FULL_DOKO, streams=1)]
        a, b = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        order = [a] + [b] * 7 + [a, b]
        res = []
        torch.cuda.synchronize(dev)
        for st, bt in zip(order, batches):
            with torch.cuda.stream(st):
                res.append(pol.execute_async(*bt, game=dk.GAME_FULL_DOKO))
        L = dk._native.lib()
        for st in (a, b):
            assert L.dk_sync(eng.ctx, st.cuda_stream) == 0
        torch.cuda.synchronize(dev)
        for (_, v), r in zip(res, ref):
            assert np.array_equal(v.cpu().numpy(), r)
    finally:
        eng.close()
