"""The device against the committed ORACLE fixtures (tests/golden/oracle_*.json) directly:
1000 rollouts (points and the final RNG state), 100 CAP samples and 100 1000-simulation UCT
searches (visits, f64 values bitwise, best action) of C3 infostates."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _load(name):
    with open(os.path.join(HERE, "golden", name)) as fh:
        return json.load(fh)


@pytest.fixture(scope="module")
def eng():
    import master_doko_reinforcement_learning_amd as dk
    e = dk.Engine(device=0, max_roots=1024, max_iterations=1000)
    yield e
    e.close()


def _infostates(eng, n):
    """bench.py's C3 infostates 0..n-1, built on the GPU."""
    import master_doko_reinforcement_learning_amd as dk
    env = dk.McEnv(eng)
    s = eng.new_games(dk.GAME_FULL_DOKO, np.arange(n, dtype=np.uint64) + np.uint64(0xC3000000))
    for _ in range(4):
        s = env.by_action(s, np.full(n, np.uint64(1) << np.uint64(24)))
    plies = np.array([[0, 8, 20, 32][j % 4] for j in range(n)], dtype=np.uint32)
    s, _ = env.random_plies(s, dk.splitmix_rng_states(np.arange(n, dtype=np.uint64) + np.uint64(0xC3100000)), plies)
    return s


def test_rollouts_match_fixture(eng):
    import master_doko_reinforcement_learning_amd as dk
    want = _load("oracle_rollouts.json")
    info = _infostates(eng, 64)
    states = info[[w["info"] for w in want]]
    seeds = np.array([w["seed"] for w in want], dtype=np.uint64)
    pts, rng = dk.McEnv(eng).random_rollout(states, dk.splitmix_rng_states(seeds))
    for i, w in enumerate(want):
        assert [int(x) for x in pts[i]] == w["points"], i
        assert ["%016x" % int(x) for x in rng[i]] == w["rng_end"], i


def test_cap_samples_match_fixture(eng):
    import master_doko_reinforcement_learning_amd as dk
    want = _load("oracle_cap.json")
    info = _infostates(eng, 100)
    for i, w in enumerate(want):
        assert info[i, :117].tobytes() == bytes.fromhex(w["infostate"])[:117], i
    out = np.concatenate([dk.card_matching_full(eng, info[i:i + 1], 1, np.array([w["seed"]], dtype=np.uint64))
                          for i, w in enumerate(want)])
    for i, w in enumerate(want):
        assert out[i, :117].tobytes() == bytes.fromhex(w["sample"])[:117], i


def test_searches_match_fixture(eng):
    import master_doko_reinforcement_learning_amd as dk
    want = _load("oracle_searches.json")
    roots = np.stack([np.frombuffer(bytes.fromhex(w["root"]), dtype=np.uint8) for w in want])
    seeds = np.array([w["search_seed"] for w in want], dtype=np.uint64)
    visits, values, best = dk.CachedMCTS(eng, dk.GAME_FULL_DOKO).monte_carlo_tree_search(roots, 2.5, 1000, seeds)
    for i, w in enumerate(want):
        assert list(visits[i]) == w["visits"], i
        assert ["%016x" % int(x) for x in values[i].view(np.uint64)] == w["values"], i
        assert int(best[i]) == (w["best"] if w["best"] >= 0 else 255), i
