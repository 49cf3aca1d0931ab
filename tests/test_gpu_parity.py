"""GPU parity: the HIP path (through the C-ABI) against the ORACLE on identical inputs.

Integer / byte / index results are compared bit-exactly; the UCT values
(f64 win_score/visits) are compared bitwise too, because the kernel uses the
same IEEE f64 operations in the same order and glibc `log` values for ln(N).
"""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu

CMP = 117  # dk_fdo_state bytes with semantics (the rest is reserved/padding + tag at 127)


@pytest.fixture(scope="module")
def eng():
    import master_doko_reinforcement_learning_amd as dk
    e = dk.Engine(device=0, max_roots=4096, max_iterations=1000)
    yield e
    e.close()


def fdo_states(n_games, seed, with_announcements=True):
    """Random full-doko positions from oracle trajectories (all phases)."""
    rng = np.random.default_rng(seed)
    out = []
    for g in range(n_games):
        s = ol.FdoState.new_game(int(seed * 1000 + g))
        mode = g % 4
        while True:
            out.append(s.clone())
            info = s.info()
            if info["phase"] == 3:
                break
            legal = s.allowed()
            acts = [a for a in range(39) if legal >> a & 1]
            if info["phase"] == 0:
                a = 24
                if mode == 1 and (legal >> 25) & 1:
                    a = 25
                elif mode == 2 and rng.integers(3) == 0:
                    a = int(rng.choice([a for a in acts if a >= 26]))
            elif info["phase"] == 1:
                anns = [a for a in acts if 33 <= a <= 37]
                a = int(rng.choice(anns)) if (with_announcements and anns and rng.integers(3) == 0) else 38
            else:
                a = int(rng.choice(acts))
            s.play(a)
    return out


def pack_all(states):
    return np.frombuffer(b"".join(s.pack() for s in states), dtype=np.uint8).reshape(-1, 128).copy()


def test_new_game_fdo_and_doko(eng):
    seeds = np.arange(200, dtype=np.uint64) * 7919 + 3
    got = eng.new_games(0, seeds)
    exp = pack_all([ol.FdoState.new_game(int(x)) for x in seeds])
    assert np.array_equal(got[:, :CMP], exp[:, :CMP]) and np.all(got[:, 127] == 0)
    got = eng.new_games(1, seeds)
    exp = pack_all([ol.DoState.new_game(int(x)) for x in seeds])
    assert np.array_equal(got[:, :108], exp[:, :108]) and np.all(got[:, 127] == 1)


def test_env_allowed_and_step_fdo(eng):
    import master_doko_reinforcement_learning_amd as dk
    env = dk.McEnv(eng)
    states = fdo_states(24, 1)
    live = [s for s in states if s.info()["phase"] != 3]
    packed = pack_all(live)
    for first in (True, False):
        got = env.allowed_actions(packed, first)
        exp = np.array([s.env_allowed(first) for s in live], dtype=np.uint64)
        assert np.array_equal(got, exp)
    # step every state with a legal action and compare the resulting wire state
    rng = np.random.default_rng(5)
    acts = []
    nxt = []
    for s in live:
        legal = s.allowed()
        a = int(rng.choice([x for x in range(39) if legal >> x & 1]))
        acts.append(np.uint64(1) << np.uint64(a))
        t = s.clone()
        t.play(a)
        nxt.append(t)
    got = env.by_action(packed, np.array(acts, dtype=np.uint64))
    exp = pack_all(nxt)
    assert np.array_equal(got[:, :CMP], exp[:, :CMP])
    # illegal action -> DK_E_STATE
    bad = np.array([np.uint64(1) << np.uint64(38)], dtype=np.uint64)
    card_phase = [i for i, s in enumerate(live) if s.info()["phase"] == 2][0]
    with pytest.raises(dk.DokoError):
        env.by_action(packed[card_phase:card_phase + 1], bad)


def test_rewards_fdo(eng):
    import master_doko_reinforcement_learning_amd as dk
    env = dk.McEnv(eng)
    states = fdo_states(16, 2)
    packed = pack_all(states)
    has, r = env.rewards_or_none(packed)
    for i, s in enumerate(states):
        info = s.info()
        assert has[i] == bool(info["has_stats"])
        if has[i]:
            assert list(r[i]) == [float(x) for x in info["player_points"]]


def test_rollout_parity_fdo(eng):
    import master_doko_reinforcement_learning_amd as dk
    env = dk.McEnv(eng)
    states = fdo_states(40, 3)
    packed = pack_all(states)
    seeds = np.arange(len(states), dtype=np.uint64) * 31 + 11
    rs = dk.splitmix_rng_states(seeds)
    got_r, got_g = env.random_rollout(packed, rs)
    for i, s in enumerate(states):
        g = ol.arr(ol.ctypes.c_uint64, 4, [int(x) for x in rs[i]])
        exp = s.rollout(g)
        assert list(got_r[i]) == exp, i
        assert [int(x) for x in got_g[i]] == list(g), i


def test_rollout_parity_doko(eng):
    import master_doko_reinforcement_learning_amd as dk
    env = dk.McEnv(eng)
    states = []
    for g in range(300):
        s = ol.DoState.new_game(9000 + g)
        rng = ol.rng_seed(77 + g)
        s.random_plies(rng, g % 53)
        states.append(s)
    packed = pack_all(states)
    rs = dk.splitmix_rng_states(np.arange(len(states), dtype=np.uint64) + 5)
    got_r, got_g = env.random_rollout(packed, rs)
    for i, s in enumerate(states):
        g = ol.arr(ol.ctypes.c_uint64, 4, [int(x) for x in rs[i]])
        assert list(got_r[i]) == s.rollout(g)
        assert [int(x) for x in got_g[i]] == list(g)


def test_random_plies_match_oracle(eng):
    """C3 infostate generation: seeded deal, 4x Healthy, k plies of
    random_action_for_current_player_no_announcement."""
    import master_doko_reinforcement_learning_amd as dk
    env = dk.McEnv(eng)
    seeds = np.arange(64, dtype=np.uint64) + 100
    base = eng.new_games(0, seeds)
    base = env.by_action(base, np.full(64, np.uint64(1) << np.uint64(24)))
    for _ in range(3):
        base = env.by_action(base, np.full(64, np.uint64(1) << np.uint64(24)))
    plies = np.array([[0, 8, 20, 32][i % 4] for i in range(64)], dtype=np.uint32)
    rs = dk.splitmix_rng_states(seeds + np.uint64(5000))
    got, got_g = env.random_plies(base, rs, plies)
    for i in range(64):
        s = ol.FdoState.new_game(int(seeds[i]))
        for _ in range(4):
            s.play(24)
        g = ol.arr(ol.ctypes.c_uint64, 4, [int(x) for x in rs[i]])
        s.random_plies(g, int(plies[i]), True)
        assert got[i, :CMP].tobytes() == s.pack()[:CMP]
        assert [int(x) for x in got_g[i]] == list(g)


def _oracle_search(states, seeds, iters, c, kind):
    out = []
    for s, sd in zip(states, seeds):
        rng = ol.rng_seed(int(sd))
        if kind == "ttt":
            best, v, val = ol.ttt_search(s, rng, iters, c)
        else:
            best, v, val, _ = s.search(rng, iters, c)
        out.append((best, v, val))
    return out


@pytest.mark.parametrize("iters", [200, 1000])
def test_search_parity_fdo(eng, iters):
    import master_doko_reinforcement_learning_amd as dk
    pool = [s for s in fdo_states(30, 11) if s.info()["phase"] != 3]
    rng = np.random.default_rng(iters)
    pick = [pool[i] for i in rng.choice(len(pool), size=48 if iters == 200 else 16, replace=False)]
    seeds = rng.integers(0, 2**63, size=len(pick), dtype=np.uint64)
    visits, values, best = dk.CachedMCTS(eng, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(pick), 2.5, iters, seeds)
    for i, (b, v, val) in enumerate(_oracle_search(pick, seeds, iters, 2.5, "fdo")):
        assert list(visits[i]) == v, i
        assert values[i].tobytes() == np.array(val, dtype=np.float64).tobytes(), i
        assert int(best[i]) == (b if b >= 0 else 255), i


@pytest.mark.parametrize("env", [{"DK_LDS_PATH": "2"}, {"DK_ROOTS_PER_WAVE": "7"}, {"DK_ROOTS_PER_WAVE": "16"},
                                 {"DK_ROOTS_PER_WAVE": "32", "DK_LN_LDS": "1"},
                                 {"DK_POOL_ROOTS": "1", "DK_ROOTS_PER_WAVE": "4"},
                                 {"DK_POOL_ROOTS": "16", "DK_ROOTS_PER_WAVE": "5"},
                                 {"DK_HOT_RECORD": "16"}, {"DK_HOT_RECORD": "32"},
                                 {"DK_HOT_RECORD": "16", "DK_LDS_PATH": "2"},
                                 {"DK_HOT_RECORD": "16", "DK_POOL_ROOTS": "1", "DK_ROOTS_PER_WAVE": "4"},
                                 {"DK_HOT_RECORD": "8"}, {"DK_HOT_RECORD": "8", "DK_LDS_PATH": "2"},
                                 {"DK_HOT_RECORD": "8", "DK_POOL_ROOTS": "1", "DK_ROOTS_PER_WAVE": "4"},
                                 {"DK_HOT_RECORD": "8", "DK_ROOTS_PER_WAVE": "7"},
                                 {"DK_GROUP_ORDER": "1", "DK_POOL_ROOTS": "16", "DK_ROOTS_PER_WAVE": "5"},
                                 {"DK_PAIR": "0"}, {"DK_PAIR": "1", "DK_LDS_PATH": "2"},
                                 {"DK_PAIR": "1", "DK_POOL_ROOTS": "1", "DK_ROOTS_PER_WAVE": "4"},
                                 {"DK_PAIR": "1", "DK_ROOTS_PER_WAVE": "7", "DK_LN_LDS": "1"}])
def test_search_parity_fdo_launch_variants(env, monkeypatch):
    """Path overflow into global memory (2 LDS entries), partial / narrow waves, the LDS
    ln table, and batches larger than the node pools: with DK_POOL_ROOTS=1 one wave
    streams all six 4-root groups through a single pool region (stale trees of the
    previous group stay in it), with 16 four waves share five groups.  DK_HOT_RECORD
    forces a hot-record layout (8, 16 or 32 B; small batches pick 16-B records searched by lane
    pairs by themselves, DK_PAIR=0 / 1 switches the pairs off / on); DK_GROUP_ORDER=1 queues the
    root groups longest-first (group_order_kernel)."""
    import master_doko_reinforcement_learning_amd as dk
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    e = dk.Engine(device=0, max_roots=64, max_iterations=400)
    try:
        pool = [s for s in fdo_states(12, 23) if s.info()["phase"] != 3]
        rng = np.random.default_rng(5)
        pick = [pool[i] for i in rng.choice(len(pool), size=24, replace=False)]
        seeds = rng.integers(0, 2**63, size=len(pick), dtype=np.uint64)
        visits, values, best = dk.CachedMCTS(e, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(pick), 2.5, 400, seeds)
        for i, (b, v, val) in enumerate(_oracle_search(pick, seeds, 400, 2.5, "fdo")):
            assert list(visits[i]) == v, i
            assert values[i].tobytes() == np.array(val, dtype=np.float64).tobytes(), i
            assert int(best[i]) == (b if b >= 0 else 255), i
    finally:
        e.close()


@pytest.mark.parametrize("cap,env", [(120, {}), (600, {}), (600, {"DK_HOT_RECORD": "16"}),
                                     (120, {"DK_HOT_RECORD": "8"}), (600, {"DK_HOT_RECORD": "8"}),
                                     (300, {"DK_POOL_ROOTS": "1", "DK_ROOTS_PER_WAVE": "4"}),
                                     (500, {"DK_POOL_ROOTS": "16", "DK_ROOTS_PER_WAVE": "5", "DK_GROUP_ORDER": "1"})])
def test_search_capacity_fallback(cap, env, monkeypatch):
    """Main pools smaller than a search needs: roots that run out of child slots are
    searched again by the fallback launch (proven-capacity pool) and the results are the
    oracle's.  120 (256 after rounding) slots overflow most roots (400 iterations take
    ~2.4 slots each), 600 (768) a part of them; with DK_POOL_ROOTS=1 the fallback pool has one 4-root region, so one wave
    streams all retried roots through it.  dk_pool_high_water counts the overflowed roots
    and reports the demand of the largest search, which then exceeds the capacity."""
    import master_doko_reinforcement_learning_amd as dk
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    e = dk.Engine(device=0, max_roots=64, max_iterations=400, slot_capacity=cap)
    try:
        pool = [s for s in fdo_states(12, 29) if s.info()["phase"] != 3]
        rng = np.random.default_rng(cap)
        pick = [pool[i] for i in rng.choice(len(pool), size=24, replace=False)]
        seeds = rng.integers(0, 2**63, size=len(pick), dtype=np.uint64)
        visits, values, best = dk.CachedMCTS(e, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(pick), 2.5, 400, seeds)
        hw, got_cap, overflowed = e.pool_high_water()
        assert got_cap == (cap + 255) // 256 * 256          # region stride rounded to 256 slots
        assert overflowed > 0 and hw > cap      # an overflowed root needed more than the main pools hold
        for i, (b, v, val) in enumerate(_oracle_search(pick, seeds, 400, 2.5, "fdo")):
            assert list(visits[i]) == v, i
            assert values[i].tobytes() == np.array(val, dtype=np.float64).tobytes(), i
            assert int(best[i]) == (b if b >= 0 else 255), i
    finally:
        e.close()


@pytest.mark.parametrize("hot32", [True, False])
def test_search_wide_pools(hot32, monkeypatch, capfd):
    """A context sized for 200,000 iterations (compare_impi's setting).  With the 32-B records
    (DK_HOT_RECORD=32) its fallback pool's per-wave region (64 lanes x 2.4 M slots x 32 B) passes
    4 GiB, so every launch takes the 64-bit-offset records (NodeHot32W, launch line wide=1); with
    the default 16-B records (round 5) the region stays below 4 GiB and the 32-bit offsets hold
    (wide=0).  With a 256-slot main pool the roots overflow into the fallback pool; results
    equal the oracle's either way."""
    import master_doko_reinforcement_learning_amd as dk
    monkeypatch.setenv("DK_VERBOSE", "1")
    if hot32:
        monkeypatch.setenv("DK_HOT_RECORD", "32")
    e = dk.Engine(device=0, max_roots=64, max_iterations=200000, slot_capacity=256)
    try:
        pool = [s for s in fdo_states(8, 31) if s.info()["phase"] != 3]
        rng = np.random.default_rng(200000)
        pick = [pool[i] for i in rng.choice(len(pool), size=16, replace=False)]
        seeds = rng.integers(0, 2**63, size=len(pick), dtype=np.uint64)
        visits, values, best = dk.CachedMCTS(e, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(pick), 2.5, 1500, seeds)
        assert e.pool_high_water()[2] > 0          # roots overflowed into the (wide) fallback pool
    finally:
        e.close()
    err = capfd.readouterr().err
    if hot32:
        assert "wide=1" in err and "hot=32B" in err, err[-800:]
    else:
        assert "wide=0" in err and "hot=16B" in err, err[-800:]
    for i, (b, v, val) in enumerate(_oracle_search(pick, seeds, 1500, 2.5, "fdo")):
        assert list(visits[i]) == v, i
        assert values[i].tobytes() == np.array(val, dtype=np.float64).tobytes(), i
        assert int(best[i]) == (b if b >= 0 else 255), i


def test_search_malformed_doko_root(eng):
    """An rs-doko root whose hand has bits above the 48 card bits cannot be held by the 64-B
    node record: the search refuses it with DK_E_STATE (as for rs-full-doko roots) instead of
    silently truncating the hand."""
    import master_doko_reinforcement_learning_amd as dk
    s = ol.DoState.new_game(0xBAD)
    for _ in range(4):
        s.play(24)
    ok = np.frombuffer(s.pack(), dtype=np.uint8).copy()
    bad = ok.copy()
    bad[7] |= 0x01                                  # hand 0, bit 56
    m = dk.CachedMCTS(eng, dk.GAME_DOKO)
    v, _, _ = m.monte_carlo_tree_search(ok[None, :], 2.5, 50, np.array([5], dtype=np.uint64))
    assert int(v[0].sum()) == 50
    with pytest.raises(dk.DokoError, match="malformed"):
        m.monte_carlo_tree_search(bad[None, :], 2.5, 50, np.array([5], dtype=np.uint64))


def test_search_capacity_fallback_doko(monkeypatch):
    """The same fallback for rs-doko roots (longest-first queue order by default)."""
    import master_doko_reinforcement_learning_amd as dk
    monkeypatch.setenv("DK_POOL_ROOTS", "16")
    monkeypatch.setenv("DK_ROOTS_PER_WAVE", "5")
    e = dk.Engine(device=0, max_roots=64, max_iterations=500, slot_capacity=500)
    try:
        states = []
        for g in range(32):
            s = ol.DoState.new_game(0xD0C10000 + g)
            for _ in range(4):
                s.play(24)
            s.random_plies(ol.rng_seed(g), g % 30)
            states.append(s)
        seeds = np.arange(32, dtype=np.uint64) * 7 + 3
        visits, values, best = dk.CachedMCTS(e, dk.GAME_DOKO).monte_carlo_tree_search(pack_all(states), 2.5, 500, seeds)
        assert e.pool_high_water()[2] > 0
    finally:
        e.close()
    for i, (b, v, val) in enumerate(_oracle_search(states, seeds, 500, 2.5, "do")):
        assert list(visits[i]) == v
        assert values[i].tobytes() == np.array(val, dtype=np.float64).tobytes()
        assert int(best[i]) == b


@pytest.mark.parametrize("layout", [None, "16", "8", "ordered"])
def test_search_parity_doko(eng, layout, monkeypatch):
    """rs-doko search parity; "16" / "8" force those hot records, "ordered" streams 7 groups of 5
    roots through 3 pool regions so the rs-doko default longest-first queue order applies."""
    import master_doko_reinforcement_learning_amd as dk
    if layout in ("16", "8"):
        monkeypatch.setenv("DK_HOT_RECORD", layout)
    if layout == "ordered":
        monkeypatch.setenv("DK_POOL_ROOTS", "16")
        monkeypatch.setenv("DK_ROOTS_PER_WAVE", "5")
    if layout:
        eng = dk.Engine(device=0, max_roots=64, max_iterations=500)
    states = []
    for g in range(32):
        s = ol.DoState.new_game(0xD0C00000 + g)
        for _ in range(4):
            s.play(24)
        s.random_plies(ol.rng_seed(g), g % 30)
        states.append(s)
    seeds = np.arange(32, dtype=np.uint64) * 13 + 1
    visits, values, best = dk.CachedMCTS(eng, dk.GAME_DOKO).monte_carlo_tree_search(pack_all(states), 2.5, 500, seeds)
    if layout:
        eng.close()
    for i, (b, v, val) in enumerate(_oracle_search(states, seeds, 500, 2.5, "do")):
        assert list(visits[i]) == v
        assert values[i].tobytes() == np.array(val, dtype=np.float64).tobytes()
        assert int(best[i]) == b


def test_search_parity_ttt(eng):
    """Config 1 plumbing: tic-tac-toe from the empty board, c = 2.0, seed 999."""
    import master_doko_reinforcement_learning_amd as dk
    boards = [[0] * 9, [1, 0, 0, 2, 1, 0, 0, 0, 0], [1, 2, 1, 0, 2, 0, 0, 0, 0]]
    packed = np.frombuffer(b"".join(ol.ttt_pack(b) for b in boards), dtype=np.uint8).reshape(-1, 128).copy()
    seeds = np.array([999, 1, 2], dtype=np.uint64)
    visits, values, best = dk.CachedMCTS(eng, dk.GAME_TTT).monte_carlo_tree_search(packed, 2.0, 1000, seeds)
    for i, (b, v, val) in enumerate(_oracle_search(boards, seeds, 1000, 2.0, "ttt")):
        assert list(visits[i]) == v
        assert values[i].tobytes() == np.array(val, dtype=np.float64).tobytes()
        assert int(best[i]) == b


def test_determinize_parity(eng):
    import master_doko_reinforcement_learning_amd as dk
    pool = [s for s in fdo_states(20, 21) if s.info()["phase"] != 3]
    info = pool[::3]
    samples = 8
    seeds = np.arange(len(info) * samples, dtype=np.uint64) * 101 + 7
    got = dk.card_matching_full(eng, pack_all(info), samples, seeds)
    for i, s in enumerate(info):
        for k in range(samples):
            smp = s.card_matching(ol.rng_seed(int(seeds[i * samples + k])))
            row = got[i * samples + k]
            assert row[:32].tobytes() == smp.pack()[:32]          # hands
            assert row[92:98].tobytes() == smp.pack()[92:98]      # reservations round
            assert s.consistent_sample(smp)


def test_fusion_parity(eng):
    import master_doko_reinforcement_learning_amd as dk
    rng = np.random.default_rng(3)
    n_info, S = 40, 16
    visits = rng.integers(0, 50, size=(n_info, S, 39)).astype(np.uint32)
    visits[:, :, 30:] = 0
    visits[5] = 7  # all ties
    allowed = rng.integers(1, 2**39, size=n_info, dtype=np.uint64)
    got_m = dk.PolicyFusionMaxN().fuse(eng, visits, allowed)
    got_a = dk.PolicyFusionAverageStrategy().fuse(eng, visits, allowed)
    for i in range(n_info):
        em, _ = ol.fuse_maxn([list(r) for r in visits[i]], int(allowed[i]))
        ea, _ = ol.fuse_avg([list(r) for r in visits[i]])
        assert int(got_m[i]) == em
        assert int(got_a[i]) == ea


def test_fusion_sharded_accumulators(eng):
    """The multi-GPU split of bench.py on one device: each 'rank' accumulates its
    half of every infostate's samples, the accumulators are summed (what the RCCL
    all-reduce does), and the select equals the oracle's fusion over all samples."""
    import torch

    from master_doko_reinforcement_learning_amd import _native
    import master_doko_reinforcement_learning_amd as dk
    L = _native.lib()
    rng = np.random.default_rng(11)
    n_info, S, world = 24, 16, 2
    visits = rng.integers(0, 40, size=(n_info, S, 39)).astype(np.uint32)
    visits[:, :, 28:] = 0
    allowed = rng.integers(1, 2**39, size=n_info, dtype=np.uint64)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    with torch.cuda.stream(stream):
        sp = stream.cuda_stream
        d_allowed = torch.tensor(allowed.view(np.int64), device=dev)
        for mode in (dk.FUSE_MAXN, dk.FUSE_AVG):
            tot_u = torch.zeros((n_info, 39), dtype=torch.int32, device=dev)
            tot_f = torch.zeros((n_info, 39), dtype=torch.float32, device=dev)
            for r in range(world):
                part = np.ascontiguousarray(visits[:, r * S // world:(r + 1) * S // world])
                d_v = torch.tensor(part.view(np.int32), device=dev)
                acc_u = torch.zeros((n_info, 39), dtype=torch.int32, device=dev)
                acc_f = torch.zeros((n_info, 39), dtype=torch.float32, device=dev)
                assert L.dk_fuse_accumulate_async(eng.ctx, d_v.data_ptr(), n_info, S // world, d_allowed.data_ptr(),
                                                  mode, acc_u.data_ptr(), acc_f.data_ptr(), sp) == 0
                tot_u += acc_u
                tot_f += acc_f
            act = torch.zeros(n_info, dtype=torch.uint8, device=dev)
            assert L.dk_fuse_select_async(eng.ctx, n_info, mode, d_allowed.data_ptr(), tot_u.data_ptr(),
                                          tot_f.data_ptr(), act.data_ptr(), sp) == 0
            assert L.dk_sync(eng.ctx, sp) == 0
            got = act.cpu().numpy()
            for i in range(n_info):
                rows = [list(map(int, r)) for r in visits[i]]
                if mode == dk.FUSE_MAXN:
                    want, _ = ol.fuse_maxn(rows, int(allowed[i]))
                    assert int(got[i]) == want, i
                else:
                    want, probs = ol.fuse_avg(rows)
                    top = sorted(probs)[-2:]
                    if top[1] - top[0] > 1e-4:
                        assert int(got[i]) == want, i


def test_decide_end_to_end(eng):
    """DefaultImpiPolicy: CAP samples -> UCT -> MaxN fusion, against the oracle pipeline."""
    import master_doko_reinforcement_learning_amd as dk
    info = []
    for j in range(6):
        s = ol.FdoState.new_game(500 + j)
        for _ in range(4):
            s.play(24)
        s.random_plies(ol.rng_seed(900 + j), [0, 8, 20, 32][j % 4], True)
        info.append(s)
    S, iters = 8, 200
    seeds = np.arange(2 * len(info) * S, dtype=np.uint64) * 17 + 3
    pol = dk.DefaultImpiPolicy(eng, 2.5, iters, S, dk.FUSE_MAXN)
    actions, visits = pol.execute(pack_all(info), seeds, return_visits=True)
    n = len(info) * S
    for j, s in enumerate(info):
        rows = []
        for k in range(S):
            smp = s.card_matching(ol.rng_seed(int(seeds[j * S + k])))
            _, v, _, _ = smp.search(ol.rng_seed(int(seeds[n + j * S + k])), iters, 2.5)
            rows.append(v)
            assert list(visits[j * S + k]) == v
        exp, _ = ol.fuse_maxn(rows, s.allowed())
        assert int(actions[j]) == exp


def test_full_size_properties(eng, monkeypatch):
    """Bench-sized batch shape (4096 roots x 1000 iterations here): every root's
    visits sum to the iteration count, only root-legal actions are visited, a
    repeat run is bit-identical, and so is a run with the other hot-record layout."""
    import master_doko_reinforcement_learning_amd as dk
    n = 4096
    seeds = np.arange(n, dtype=np.uint64) + 1234
    roots = eng.new_games(0, seeds)
    env = dk.McEnv(eng)
    for _ in range(4):
        roots = env.by_action(roots, np.full(n, np.uint64(1) << np.uint64(24)))
    mcts = dk.CachedMCTS(eng, dk.GAME_FULL_DOKO)
    v1, val1, b1 = mcts.monte_carlo_tree_search(roots, 2.5, 1000, seeds)
    assert np.all(v1.sum(axis=1) == 1000)
    allowed = env.allowed_actions(roots, True)
    bits = (allowed[:, None] >> np.arange(39, dtype=np.uint64)[None, :]) & np.uint64(1)
    assert np.all((v1 > 0) <= (bits == 1))
    v2, val2, b2 = mcts.monte_carlo_tree_search(roots, 2.5, 1000, seeds)
    assert np.array_equal(v1, v2) and np.array_equal(val1.view(np.uint64), val2.view(np.uint64)) and np.array_equal(b1, b2)
    monkeypatch.setenv("DK_HOT_RECORD", "16")
    e16 = dk.Engine(device=0, max_roots=n, max_iterations=1000)
    try:
        v3, val3, b3 = dk.CachedMCTS(e16, dk.GAME_FULL_DOKO).monte_carlo_tree_search(roots, 2.5, 1000, seeds)
    finally:
        e16.close()
    assert np.array_equal(v1, v3) and np.array_equal(val1.view(np.uint64), val3.view(np.uint64)) and np.array_equal(b1, b3)
    # the default main-pool capacity (64 + 8 x iterations, 64 + 4 x when device memory is
    # short) holds every one of these searches
    hw, cap, overflowed = eng.pool_high_water()
    assert cap in (4096, 8192) and 0 < hw <= cap and overflowed == 0, (hw, cap, overflowed)
    # per-wave clocks of the last launch (dk_last_search_waves): one entry per wave of the grid
    # (4096 roots as 256 waves of 16: one wave per SIMD, launch_rpw), every wave busy for a
    # share of the span, and the span (100 MHz counter) within the launch's HIP-event time
    ms = eng.last_search_ms()
    w = eng.last_search_waves()
    assert w["waves"] == n // 16, w
    assert 0.0 < w["busy_frac"] <= 1.0 and 0.0 < w["first_end_ms"] <= w["median_end_ms"] <= w["span_ms"], w
    assert 0.5 * ms < w["span_ms"] <= ms * 1.02 + 0.05, (ms, w)


# ---------------------------------------------------------------- rs-doko rule-based sampler
def do_states(n_games, seed):
    """Random rs-doko positions from oracle trajectories (every third game a wedding when possible)."""
    rng = np.random.default_rng(seed)
    out = []
    for g in range(n_games):
        s = ol.DoState.new_game(int(seed * 1000 + g))
        while True:
            out.append(s.clone())
            info = s.info()
            if info["phase"] == 2:
                break
            legal = s.allowed()
            if info["phase"] == 0:
                a = 25 if (g % 3 == 1 and (legal >> 25) & 1) else 24
            else:
                a = int(rng.choice([a for a in range(24) if legal >> a & 1]))
            s.play(a)
    return out


def test_do_sample_assignment_parity(eng):
    """sample_assignment_full (rs-doko-assignment/src/assignment.rs:472-580) on the GPU
    == the oracle, all 128 bytes of every sample, at every phase of random games."""
    import master_doko_reinforcement_learning_amd as dk
    info = do_states(24, 5)[::2]
    samples = 8
    seeds = np.arange(len(info) * samples, dtype=np.uint64) * 977 + 11
    got = dk.sample_assignment_full(eng, pack_all(info), samples, seeds)
    for i, s in enumerate(info):
        for k in range(samples):
            smp = s.sample_assignment_full(ol.rng_seed(int(seeds[i * samples + k])))
            assert smp is not None
            assert got[i * samples + k].tobytes() == smp.pack()


def _card_counts(hands):
    """(n, 4) u64 hands -> (n, 4, 24) card multiplicities."""
    bits = (hands[..., None] >> np.arange(48, dtype=np.uint64)) & np.uint64(1)
    return (bits[..., :24] + bits[..., 24:]).astype(np.int32)


def test_do_sample_assignment_full_size_properties(eng):
    """4096 rs-doko infostates x 64 samples: hand sizes kept, the observer's cards
    kept, the hidden cards redistributed exactly, and every sampled hand
    consistent with the colours its player failed to follow."""
    import master_doko_reinforcement_learning_amd as dk
    n_info, S = 4096, 64
    seeds = np.arange(n_info, dtype=np.uint64) + 77
    info = eng.new_games(dk.GAME_DOKO, seeds)
    env = dk.McEnv(eng)
    for _ in range(4):
        info = env.by_action(info, np.full(n_info, np.uint64(1) << np.uint64(24)))
    plies = np.array([[0, 8, 20, 33][j % 4] for j in range(n_info)], dtype=np.uint32)
    info, _ = env.random_plies(info, dk.splitmix_rng_states(seeds * np.uint64(3)), plies)
    smp = dk.sample_assignment_full(eng, info, S, np.arange(n_info * S, dtype=np.uint64) * 3 + 5)
    h_in = np.repeat(info[:, :32].copy().view(np.uint64), S, axis=0)
    h_out = smp[:, :32].copy().view(np.uint64)
    assert np.array_equal(smp[:, 32:], np.repeat(info[:, 32:], S, axis=0))   # only the hands change
    c_in, c_out = _card_counts(h_in), _card_counts(h_out)
    assert np.array_equal(c_in.sum(axis=2), c_out.sum(axis=2))
    obs = info[:, 100].astype(np.int64)
    obs = np.where(obs == 255, 0, obs)
    obs = np.repeat(obs, S)
    rows = np.arange(n_info * S)
    assert np.array_equal(c_in[rows, obs], c_out[rows, obs])
    assert np.array_equal(c_in.sum(axis=1), c_out.sum(axis=1))
    # colour voids (normal-game colours): nobody holds a colour they failed to follow
    for j in range(0, n_info, 97):
        st = info[j]
        nc, start = int(st[98]), int(st[96])
        tw = int(st[88:92].copy().view(np.uint32)[0])
        trump = set(range(6)) | {7, 8, 9, 14, 15, 20, 21}
        color = lambda c: "T" if c in trump else "HCS"[c // 6 - 1]
        voids = [set() for _ in range(4)]
        for t in range(0, (nc + 3) // 4):
            lead = color(int(st[32 + 4 * t]))
            p0 = start if t == 0 else (tw >> (2 * (t - 1))) & 3
            for k in range(min(4, nc - 4 * t)):
                if color(int(st[32 + 4 * t + k])) != lead:
                    voids[(p0 + k) % 4].add(lead)
        for s_ in range(S):
            for p in range(4):
                held = {color(c) for c in range(24) if c_out[j * S + s_, p, c] > 0}
                assert not (held & voids[p]) or p == obs[j * S]


def test_decide_end_to_end_doko(eng):
    """DefaultImpiPolicy on rs-doko infostates: rule-based samples -> UCT -> MaxN fusion
    (the determinized C2 variant), against the oracle pipeline."""
    import master_doko_reinforcement_learning_amd as dk
    info = []
    for j in range(6):
        s = ol.DoState.new_game(0xD0C00000 + 40 + j)
        for _ in range(4):
            s.play(24)
        s.random_plies(ol.rng_seed(700 + j), [0, 8, 20, 33][j % 4])
        info.append(s)
    S, iters = 8, 200
    seeds = np.arange(2 * len(info) * S, dtype=np.uint64) * 19 + 5
    pol = dk.DefaultImpiPolicy(eng, 2.5, iters, S, dk.FUSE_MAXN)
    actions, visits = pol.execute(pack_all(info), seeds, return_visits=True)
    n = len(info) * S
    for j, s in enumerate(info):
        rows = []
        for k in range(S):
            smp = s.sample_assignment_full(ol.rng_seed(int(seeds[j * S + k])))
            _, v, _, _ = smp.search(ol.rng_seed(int(seeds[n + j * S + k])), iters, 2.5)
            rows.append(v)
            assert list(visits[j * S + k]) == v
        exp, _ = ol.fuse_maxn(rows, s.allowed())
        assert int(actions[j]) == exp


# ---------------------------------------------------------------- AlphaZero PUCT search
@pytest.mark.parametrize("drawn", [False, True, "beta"])
@pytest.mark.parametrize("temp_mode", [0, 1, 2])
def test_az_search_parity(eng, temp_mode, drawn):
    """AlphaZero mcts_search (rs-doko-alpha-zero async_mcts.rs:224-406) on the GPU ==
    the oracle restatement, with the synthetic hash network (oracle/az_eval.hpp) on both
    sides: root child visits, chosen action (greedy / uniform / T = 1) and the SmallRng end
    state for every game.  drawn: the root's Dirichlet([alpha; 39]) noise is drawn by each game
    from its own SmallRng, as the reference draws it (async_mcts.rs:111-113; rand_distr 0.5.1,
    parity unpinned: no reference vector), with alpha 0.8 / 1.0 / 0.5 (the three Gamma paths), or
    ("beta") 0.1 / 0.05 / 0.1, the crate's FromBeta construction (Cheng's BC on the device's
    restated glibc logf / expf); otherwise the caller's noise.  The drawn runs start from caller-held RNG states
    (dk_az_rng_async, the reference's &mut SmallRng) and read the end states back."""
    import torch
    import master_doko_reinforcement_learning_amd as dk
    pool = [s for s in fdo_states(24, 31) if s.info()["phase"] != 3]
    info = pool[::max(1, len(pool) // 64)][:64]
    n, iters, c, eps = len(info), 150, 2.5, 0.25
    epoch = 3 if temp_mode == 1 else 12
    rng = np.random.default_rng(temp_mode)
    noise = (rng.integers(0, 1000, size=(n, 39)) / 4000.0).astype(np.float32)
    seeds = rng.integers(0, 2**63, size=n, dtype=np.uint64)
    dev = torch.device("cuda", 0)

    def network(states):
        v, l = ol.az_hash_eval_np(states.cpu().numpy())
        return torch.from_numpy(v).to(dev), torch.from_numpy(l).to(dev)

    roots = torch.from_numpy(np.frombuffer(b"".join(s.pack_az() for s in info), dtype=np.uint8).reshape(-1, 160).copy()).to(dev)
    alpha = [0.1, 0.05, 0.1][temp_mode] if drawn == "beta" else [0.8, 1.0, 0.5][temp_mode]
    az = dk.AlphaZeroSearch(eng, c, eps, epoch, [None, float("inf"), 1.0][temp_mode], dirichlet_alpha=alpha)
    rs = None
    if drawn:
        start = np.array([list(ol.rng_seed(int(x) ^ 0x5EED)) for x in seeds], dtype=np.uint64)
        rs = torch.from_numpy(start.view(np.int64).copy()).to(dev)
    actions, visits = az.mcts_search(roots, network, None if drawn else torch.from_numpy(noise).to(dev), iters, seeds,
                                     rng_states=rs)
    actions, visits = actions.cpu().numpy(), visits.cpu().numpy()
    ends = rs.cpu().numpy().view(np.uint64) if drawn else None
    for g, s in enumerate(info):
        r = ol.rng_seed(int(seeds[g]) ^ 0x5EED) if drawn else ol.rng_seed(int(seeds[g]))
        a, v, _ = s.az_search(None if drawn else list(noise[g]), iters, c, eps, epoch, temp_mode, 1.0, r, alpha=alpha)
        assert list(visits[g]) == v
        assert int(actions[g]) == a
        if drawn:
            assert [int(x) for x in ends[g]] == list(r)


@pytest.mark.parametrize("first,stride,n", [(0, 127, (1 << 32) // 127 + 1), (0x3F000000, 1, 1 << 24),
                                             (0xC2D00000, 1, 1 << 21)])
def test_device_libm_f32(first, stride, n):
    """The device's glibc logf / expf (engine/libm_f32.h, the FromBeta noise's Beta draws) ==
    the host's glibc, bit for bit (NaN as NaN): every 127th f32 bit pattern over the whole range,
    all of [0.5, 2) (the Beta draws' u / (1 - u) around 1), and expf's underflow edge near -104."""
    import ctypes
    import torch
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    y = torch.empty(n, dtype=torch.float32, device="cuda")
    want = np.empty(n, dtype=np.float32)
    st = torch.cuda.current_stream().cuda_stream
    for fn in (0, 1):
        assert L.dk_f32_libm_async(fn, first, stride, n, y.data_ptr(), st) == 0
        ol.lib().or_libm_f32(fn, first, stride, n, want.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
        got = y.cpu().numpy()
        both_nan = np.isnan(got) & np.isnan(want)
        diff = (got.view(np.uint32) != want.view(np.uint32)) & ~both_nan
        assert not diff.any(), (fn, np.flatnonzero(diff)[:8], got[diff][:8], want[diff][:8])


def test_az_encode_and_step_parity(eng):
    """encode_state_pi on the GPU == the oracle's (311 tokens) at every position of random
    games with announcements, and dk_az_step (take_action with skip_single) keeps the
    records equal to the oracle's states and announcement lists."""
    import torch
    import master_doko_reinforcement_learning_amd as dk
    dev = torch.device("cuda", 0)
    states = [s for s in fdo_states(16, 41) if s.info()["phase"] != 3]
    recs = torch.from_numpy(np.frombuffer(b"".join(s.pack_az() for s in states), dtype=np.uint8).reshape(-1, 160).copy()).to(dev)
    tok = dk.az_encode(eng, recs).cpu().numpy()
    for i, s in enumerate(states):
        assert list(tok[i]) == s.encode_pi()
    # one skip-single step from every position: the first legal action
    acts = []
    nxt = []
    for s in states:
        legal = s.allowed()
        a = [b for b in range(39) if legal >> b & 1][0]
        acts.append(a)
        c = s.clone()
        c.az_take_action(a)
        nxt.append(c)
    dk.az_step(eng, recs, torch.tensor(acts, dtype=torch.uint8, device=dev))
    got = recs.cpu().numpy()
    for i, c in enumerate(nxt):
        want = np.frombuffer(c.pack_az(), dtype=np.uint8)
        assert got[i, :117].tobytes() == want[:117].tobytes()
        assert got[i, 128:153].tobytes() == want[128:153].tobytes()


def test_az_selfplay_with_network(eng):
    """C5 plumbing on the GPU: AlphaZeroSearch with the DokoAzNet evaluator (device encoder
    -> bf16 network) from fresh deals: every game's root children get exactly `iterations`
    visits, the chosen actions are legal, encoded tokens stay inside the embedding
    vocabularies, and dk_az_step plays the moves."""
    import torch
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd.az_network import VOCAB, AzEvaluator, DokoAzNet
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    G, iters = 32, 24
    st = torch.from_numpy(eng.new_games(dk.GAME_FULL_DOKO, np.arange(G, dtype=np.uint64) + 900)).to(dev)
    recs = dk.az_records(eng, st)
    ev = AzEvaluator(eng, DokoAzNet().to(dev))
    search = dk.AlphaZeroSearch(eng, 4.0, 0.3, 10, 0.5, dirichlet_alpha=0.8)
    noise = None   # drawn by every game from its own SmallRng (async_mcts.rs:111-113)
    for move in range(6):
        tok = dk.az_encode(eng, recs).cpu().numpy()
        for i, v in enumerate(VOCAB):
            part = tok[:, 62 * i:62 * (i + 1)] if i < 5 else tok[:, 310:]
            assert part.min() >= 0 and part.max() < v
        actions, visits = search.mcts_search(recs, ev, noise, iters, np.arange(G, dtype=np.uint64) + 7 * move)
        visits = visits.cpu().numpy()
        assert np.all(visits.sum(axis=1) == iters)
        legal = np.zeros(G, dtype=np.uint64)
        a = actions.cpu().numpy()
        for g in range(G):
            assert visits[g, a[g]] > 0
        dk.az_step(eng, recs, actions)


@pytest.mark.parametrize("iters,env,hot", [(1023, {"DK_HOT_RECORD": "8"}, "8B long=0"), (1024, {"DK_HOT_RECORD": "8"}, "16B"),
                                           (4095, {"DK_HOT_RECORD": "16"}, "16B long=0"),
                                           (4096, {"DK_HOT_RECORD": "16"}, "16B long=1"),
                                           (4096, {"DK_HOT_RECORD": "32"}, "32B long=0")])
def test_search_record_width_limits(iters, env, hot, monkeypatch, capfd):
    """The iteration limits of the packed hot records (search_core.h): 8-B records hold
    <= 1023 iterations (11-bit visits, 10-bit state indices), 16-B records compare means by
    24-bit cross products up to 4095 iterations and by 64-bit ones beyond (NodeHot16L, round 5);
    one iteration more takes the next layout even when a narrower one is forced, and the 32-B
    cached-mean records stay available (DK_HOT_RECORD=32).  Roots at the limit equal oracle
    searches bitwise."""
    import master_doko_reinforcement_learning_amd as dk
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("DK_VERBOSE", "1")
    e = dk.Engine(device=0, max_roots=16, max_iterations=iters)
    try:
        pool = [s for s in fdo_states(6, 41) if s.info()["phase"] != 3]
        rng = np.random.default_rng(iters)
        pick = [pool[i] for i in rng.choice(len(pool), size=6, replace=False)]
        seeds = rng.integers(0, 2**63, size=len(pick), dtype=np.uint64)
        visits, values, best = dk.CachedMCTS(e, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(pick), 2.5, iters, seeds)
        err = capfd.readouterr().err
        lines = [l for l in err.splitlines() if l.startswith("doko_amd: search")]
        h, _, lg = hot.partition(" ")
        assert lines and ("hot=%s" % h) in lines[0] and lg in lines[0], err[-1000:]
        for i, (b, v, val) in enumerate(_oracle_search(pick, seeds, iters, 2.5, "fdo")):
            assert sum(v) == iters and list(visits[i]) == v, i
            assert values[i].tobytes() == np.array(val, dtype=np.float64).tobytes(), i
            assert int(best[i]) == (b if b >= 0 else 255), i
    finally:
        e.close()


@pytest.mark.parametrize("iters,n,hot32", [(12000, 6, False), (50000, 2, False), (200000, 1, False), (200000, 1, True)])
def test_search_parity_production_shape(iters, n, hot32, monkeypatch):
    """Searches of the thesis's production length (run.rs:270-291 runs 200,000 iterations per
    sample; its grid goes to 2,000,000, run.rs:107-118): the long 16-B records (64-bit cross
    products, iterations > 4095) and deep LDS-path overflow; with DK_HOT_RECORD=32 the 32-B
    records with cached means, which at 200,000 iterations take 64-bit pool offsets (a wave's
    fallback region passes 4 GiB).  Visits, values (bitwise) and the best move equal the oracle's."""
    import master_doko_reinforcement_learning_amd as dk
    if hot32:
        monkeypatch.setenv("DK_HOT_RECORD", "32")
    pool = [s for s in fdo_states(8, 53) if s.info()["phase"] != 3 and s.info()["card_index"] < 24]
    rng = np.random.default_rng(iters)
    pick = [pool[i] for i in rng.choice(len(pool), size=n, replace=False)]
    seeds = rng.integers(0, 2**63, size=n, dtype=np.uint64)
    e = dk.Engine(device=0, max_roots=64, max_iterations=iters, slot_capacity=64 + 4 * iters)
    try:
        visits, values, best = dk.CachedMCTS(e, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(pick), 2.5, iters, seeds)
        _, _, overflowed = e.pool_high_water()
    finally:
        e.close()
    for i, (b, v, val) in enumerate(_oracle_search(pick, seeds, iters, 2.5, "fdo")):
        assert list(visits[i]) == v, i
        assert values[i].tobytes() == np.array(val, dtype=np.float64).tobytes(), i
        assert int(best[i]) == b, i
    assert overflowed == 0
