"""Searches that continue the caller's SmallRng (dk_search_batch_rng) and config 1 as the
reference runs it.

CachedMCTS::monte_carlo_tree_search takes `random: &mut SmallRng` (rs-doko-mcts/src/mcts/mcts.rs:
294-315); tic_tac_toe_player (rs-doko-mcts/src/example/tic_tac_toe_player.rs:8-52) threads ONE
seed_from_u64(999) stream through every search of 1000 games, c = 2.0, 1400 iterations, each move
max_by_key(visits).  The GPU must consume the stream exactly as the oracle does (every expansion's
random_single, every rollout, the final random_bool draw), so every later search -- and every
later game -- depends on the exact end state of every earlier one.

The reference's TicTacToeState leaves allowed_actions / by_action as todo!() (tic_tac_toe_impl.rs:
32-38); both sides use "empty cells as action bits 0-8" (oracle/ttt.hpp), as in round 1.
"""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import master_doko_reinforcement_learning_amd as dk
    e = dk.Engine(device=0, max_roots=4096, max_iterations=1400)
    yield e
    e.close()


def _oracle_player(games, iters, c=2.0):
    """tic_tac_toe_player on the oracle: one rng threaded through every search."""
    rng = ol.rng_seed(999)
    trace, res = [], [0, 0, 0]
    for g in range(games):
        b = [0] * 9
        while ol.lib().or_ttt_finish(ol.arr(ol.ctypes.c_int32, 9, b)) == 0:
            best, v, _ = ol.ttt_search(b, rng, iters, c)
            trace.append((g, list(b), v, best, [int(rng[k]) for k in range(4)]))
            x, o = b.count(1), b.count(2)
            b[best] = 1 if x == o else 2
        res[ol.lib().or_ttt_finish(ol.arr(ol.ctypes.c_int32, 9, b)) - 1] += 1
    return res, trace


@pytest.mark.parametrize("iters", [1400, 1000])
def test_tic_tac_toe_player_one_stream(eng, iters):
    """The first 12 games of tic_tac_toe_player: every move's board, visits, chosen move and
    the stream state after every search equal the oracle's."""
    import master_doko_reinforcement_learning_amd as dk
    games = 12
    exp_res, exp = _oracle_player(games, iters)
    trace = []
    res = dk.tic_tac_toe_player(eng, games, iterations=iters, uct_exploration_constant=2.0, trace=trace)
    assert len(trace) == len(exp)
    for (g, b, v, best, st), (eg, eb, ev, ebest, est) in zip(trace, exp):
        assert g == eg and list(b) == eb
        assert list(v[:9]) == ev[:9] and not v[9:].any()
        assert best == ebest
        assert [int(w) for w in st] == est
    assert res == exp_res


def test_search_rng_states_all_games(eng):
    """dk_search_batch_rng on rs-full-doko, rs-doko and tic-tac-toe roots with arbitrary
    (already advanced) stream states: results and end states equal the oracle's; a stream
    started with seed_from_u64 gives the seeded entry's results."""
    import master_doko_reinforcement_learning_amd as dk
    from test_gpu_parity import fdo_states, pack_all
    fdo = [s for s in fdo_states(6, 41) if s.info()["phase"] != 3][::9][:24]
    rng0 = np.random.default_rng(8)
    words = rng0.integers(0, 2**63, size=(len(fdo), 4), dtype=np.int64).astype(np.uint64)
    st = words.copy()
    v, val, best = dk.CachedMCTS(eng, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(fdo), 2.5, 400, st)
    for i, s in enumerate(fdo):
        r = ol.arr(ol.ctypes.c_uint64, 4, [int(w) for w in words[i]])
        b, ov, oval, _ = s.search(r, 400, 2.5)
        assert list(v[i]) == ov and val[i].tobytes() == np.array(oval, dtype=np.float64).tobytes()
        assert int(best[i]) == b
        assert [int(w) for w in st[i]] == [int(r[k]) for k in range(4)]
    # rs-doko
    dos = []
    for j in range(12):
        s = ol.DoState.new_game(700 + j)
        for _ in range(4):
            s.play(24)
        s.random_plies(ol.rng_seed(900 + j), 4 * (j % 8), )
        dos.append(s)
    st = words[:12].copy()
    v, _, best = dk.CachedMCTS(eng, dk.GAME_DOKO).monte_carlo_tree_search(pack_all(dos), 2.5, 300, st)
    for i, s in enumerate(dos):
        r = ol.arr(ol.ctypes.c_uint64, 4, [int(w) for w in words[i]])
        b, ov, _, _ = s.search(r, 300, 2.5)
        assert list(v[i]) == ov and int(best[i]) == b
        assert [int(w) for w in st[i]] == [int(r[k]) for k in range(4)]
    # seeded == continued from seed_from_u64
    seeds = np.arange(len(fdo), dtype=np.uint64) * 31 + 5
    v1, val1, b1 = dk.CachedMCTS(eng, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(fdo), 2.5, 200, seeds)
    gens = [dk.SmallRng.seed_from_u64(int(x)) for x in seeds]
    v2, val2, b2 = dk.CachedMCTS(eng, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(fdo), 2.5, 200, gens)
    assert np.array_equal(v1, v2) and val1.tobytes() == val2.tobytes() and np.array_equal(b1, b2)
    for i, g in enumerate(gens):
        r = ol.rng_seed(int(seeds[i]))
        fdo[i].search(r, 200, 2.5)
        assert [int(w) for w in g.state] == [int(r[k]) for k in range(4)]


def test_search_rng_capacity_fallback(monkeypatch):
    """A root that overflows the main pools is searched again by the fallback pass from the
    caller's stream state (not from the state the failed pass left): results and end states
    stay equal to the oracle's."""
    import master_doko_reinforcement_learning_amd as dk
    from test_gpu_parity import fdo_states, pack_all
    monkeypatch.setenv("DK_SLOT_CAPACITY", "256")
    e = dk.Engine(device=0, max_roots=256, max_iterations=600)
    try:
        roots = [s for s in fdo_states(4, 43) if s.info()["phase"] != 3][::5][:32]
        words = np.random.default_rng(2).integers(0, 2**63, size=(len(roots), 4), dtype=np.int64).astype(np.uint64)
        st = words.copy()
        v, _, _ = dk.CachedMCTS(e, dk.GAME_FULL_DOKO).monte_carlo_tree_search(pack_all(roots), 2.5, 600, st)
        _, _, ovf = e.pool_high_water()
        assert ovf > 0
        for i, s in enumerate(roots):
            r = ol.arr(ol.ctypes.c_uint64, 4, [int(w) for w in words[i]])
            _, ov, _, _ = s.search(r, 600, 2.5)
            assert list(v[i]) == ov
            assert [int(w) for w in st[i]] == [int(r[k]) for k in range(4)]
    finally:
        e.close()


def test_tic_tac_toe_games_lockstep(eng):
    """tic_tac_toe_games: independent games, each with its own stream, one launch per move over
    the unfinished games; every game equals the oracle's game on its own stream."""
    import master_doko_reinforcement_learning_amd as dk
    seeds = np.arange(64, dtype=np.uint64) + 999
    fin, moves, searches = dk.tic_tac_toe_games(eng, seeds, iterations=1000, uct_exploration_constant=2.0)
    assert searches == int(moves.sum())
    for g, sd in enumerate(seeds):
        rng = ol.rng_seed(int(sd))
        b, m = [0] * 9, 0
        while ol.lib().or_ttt_finish(ol.arr(ol.ctypes.c_int32, 9, b)) == 0:
            best, _, _ = ol.ttt_search(b, rng, 1000, 2.0)
            b[best] = 1 if b.count(1) == b.count(2) else 2
            m += 1
        assert int(fin[g]) == ol.lib().or_ttt_finish(ol.arr(ol.ctypes.c_int32, 9, b)) and int(moves[g]) == m
