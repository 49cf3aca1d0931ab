"""CPU-only checks: oracle KATs, the host build of the engine headers against the
oracle (tests/native), host-side helpers, and that the C-ABI library exports
every symbol include/doko_amd.h declares.  No GPU compute here."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_lib as ol

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def native_bins():
    subprocess.run(["make", "-s", "-C", NATIVE], check=True)
    return NATIVE


def _run(binary, *args):
    out = subprocess.run([os.path.join(NATIVE, binary)] + [str(a) for a in args], capture_output=True, text=True,
                         timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("OK"), out.stdout
    return int(out.stdout.split()[1])


def test_engine_rules_vs_oracle(native_bins):
    """Legal masks, env masks, announcement offers, stepping on the wire format,
    rollouts (rewards + RNG stream position) and scoring of the gfx950 engine
    headers (host build) equal the oracle on random trajectories."""
    assert _run("fdo_engine_check", 300, 11) > 20000


def test_coin_flipper_runs_equal_item_by_item(native_bins):
    """rng.h choose_unsized (runs of tails per chunk, the CAP sampler's rule 4) == the item-by-item
    CoinFlipper reservoir: chosen index and generator state, 1.5 M random cases."""
    assert _run("coin_check", 1500000, 3) > 40000000


def test_engine_rules_vs_oracle_trick_replay(native_bins):
    """The same checks with every speculative fast-path trick of rollout_cards replayed through
    the exact per-ply draws (DK_TRICK_REPLAY_ALL): the replay path a rejected draw takes."""
    assert _run("fdo_engine_check_replay", 300, 11) > 20000


def test_do_engine_vs_oracle(native_bins):
    """do_engine.h (host build) = oracle rs-doko: legal masks, wire-format steps, and
    rollouts (fast card phase and stepwise; rewards + RNG stream position), weddings included."""
    assert _run("do_engine_check", 200, 7) > 30000


def test_do_engine_vs_oracle_trick_replay(native_bins):
    """do_engine.h with every speculative trick replayed through the exact per-ply draws."""
    assert _run("do_engine_check_replay", 200, 7) > 30000


def test_engine_search_vs_oracle(native_bins):
    """search_core.h (host build) = oracle UCT: visits, f64 values bitwise, best, RNG stream."""
    assert _run("search_check", 6, 400, 5) > 10
    assert _run("search_check", 20, 300, 17) > 30


def test_uct_pick_filter_exact(native_bins):
    """Filtered UCT pick (f32 estimate + exact f64 on candidates) == plain f64 UCT,
    with the f32 reciprocal / sqrt adversarially perturbed by up to 4 ulp."""
    assert _run("uct_pick_check", 1000000, 3) == 1000000
    assert _run("uct_pick_check8", 1000000, 4) == 1000000   # the same pick over 8-B records


def test_hot32_variant_exact(native_bins):
    """The 32-B hot-record build (DK_HOT16=0, cached exact means) stays exact as well."""
    assert _run("uct_pick_check32", 300000, 5) == 300000
    assert _run("search_check32", 6, 400, 5) > 10


def test_hot16l_variant_exact(native_bins):
    """The long 16-B records (NodeHot16L / NodeHot16PL: searches beyond 4,095 iterations, the
    production shape's 200,000) compare sibling means by 64-bit cross products: the filtered pick
    equals the plain f64 UCT for visit counts up to 2^22, and whole searches past the 24-bit
    limit equal the oracle's."""
    assert _run("uct_pick_check16l", 1000000, 6) == 1000000
    assert _run("search_check16l", 3, 5000, 21) > 2
    assert _run("search_check16l", 1, 12000, 31) >= 1


def test_hot8_variant_exact(native_bins):
    """The 8-B packed hot records (DK_HOT8: even-aligned child blocks, pair loads, the root
    in registers) give the oracle's searches exactly."""
    assert _run("search_check8", 8, 400, 9) > 10
    assert _run("search_check8", 4, 1000, 11, 2) > 4


def test_line_block_placement_exact(native_bins, monkeypatch):
    """Child blocks kept within 128-B lines (search_core.h block_base, DK_BLOCK_ALIGN=line): slot
    placement only, so the searches still equal the oracle's, for 8-B and 16-B records."""
    monkeypatch.setenv("DK_BALIGN_LINE", "1")
    assert _run("search_check8", 8, 400, 9) > 10
    assert _run("search_check8", 4, 1000, 11, 2) > 4
    assert _run("search_check", 6, 400, 5) > 10


def test_engine_cap_vs_oracle(native_bins):
    """cap_engine.h (host build) = oracle card_matching_full; samples always consistent."""
    assert _run("cap_check", 120, 3) > 5000


def test_engine_assignment_vs_oracle(native_bins):
    """assign_engine.h (host build) = oracle rs-doko sample_assignment_full
    (rs-doko-assignment/src/assignment.rs:472-580): hands, packed state, RNG stream
    position and panic cases at every decision point, weddings included."""
    assert _run("assign_check", 200, 3) > 40000


def test_dirichlet_vs_oracle(native_bins):
    """engine/rand_distr.h (the root noise the GPU draws, host build) = the oracle's rand_distr
    0.5.1 restatement: ziggurat tables, StandardNormal / Exp1 streams, Gamma on all three paths
    Beta<f32> on Cheng's BB and BC, and Dirichlet<f32, 39> on FromGamma and FromBeta (alpha 0.05,
    0.1), value for value with the RNG stream position (parity unpinned: no reference vector
    exists for these draws)."""
    assert _run("dirichlet_check", 20000, 3) == 3760000


def test_libm_f32_vs_glibc(native_bins):
    """engine/libm_f32.h -- glibc's logf / expf restated for the device (the FromBeta noise's
    Beta draws call them on arbitrary arguments; Rust's f32::ln / f32::exp are the platform libm)
    -- equals the host's glibc on all 2^32 f32 inputs, bit for bit."""
    assert _run("libm_check", 1, max(1, min(16, os.cpu_count() or 1))) == 1 << 32


def test_az_core_vs_oracle(native_bins):
    """az_core.h (host build, driven batch-wise like the GPU) = oracle AlphaZero
    mcts_search: root priors, visits, chosen action and RNG position, three temperature modes,
    with caller-supplied noise and with the Dirichlet noise the search draws itself."""
    assert _run("az_check", 120, 300, 5) == 960


def test_fusion_kats():
    """rs-doko-py-bridge/src/compare_impi/policy_fusion.rs:130-311."""
    with open(os.path.join(GOLD, "fusion_kats.json")) as fh:
        d = json.load(fh)
    assert len(d["cases"]) == 4
    for c in d["cases"]:
        allowed = sum(1 << a for a in c["allowed"])
        if c["mode"] == "maxn":
            got, _ = ol.fuse_maxn(c["visits"], allowed)
        else:
            got, _ = ol.fuse_avg(c["visits"])
        assert got == c["expect"], c["name"]


def test_splitmix_rng_states_match_oracle():
    import master_doko_reinforcement_learning_amd.api as api
    seeds = np.array([0, 1, 42, 2**63 + 5, 0xD0C00000], dtype=np.uint64)
    got = api.splitmix_rng_states(seeds)
    for i, s in enumerate(seeds):
        assert [int(x) for x in got[i]] == list(ol.rng_seed(int(s)))


def test_library_exports_every_header_symbol():
    from master_doko_reinforcement_learning_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        _native.build()
    with open(os.path.join(ROOT, "include", "doko_amd.h")) as fh:
        header = fh.read()
    body = re.sub(r"/\*.*?\*/", "", header, flags=re.S)  # declarations only, not comments
    declared = sorted(set(re.findall(r"\b(dk_\w+)\s*\(", body)))
    out = subprocess.run(["nm", "-D", "--defined-only", _native.LIB_PATH], capture_output=True, text=True, check=True)
    exported = set(line.split()[-1] for line in out.stdout.splitlines() if line.strip())
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    assert set(_native.EXPORTED) <= exported


def test_library_loads_without_gpu_compute():
    from master_doko_reinforcement_learning_amd import _native
    L = _native.lib()
    assert L.dk_abi_version() == 1
    assert L.dk_status_string(-2) == b"capacity exceeded"


def test_packed_state_layout():
    """The oracle's wire-format writer and the header agree on the 128-byte layout."""
    s = ol.FdoState.new_game(7)
    b = s.pack()
    assert len(b) == 128 and b[127] == 0
    hands = s.hands()
    assert [int.from_bytes(b[8 * i:8 * i + 8], "little") for i in range(4)] == hands
    assert all(x == 0xFF for x in b[32:80])
    info = s.info()
    assert b[100] == info["current_player"] and b[99] == 0


def test_oracle_samples_consistent():
    """Property of the reference's card_matching test (card_matching.rs:548-643)."""
    for g in range(20):
        s = ol.FdoState.new_game(300 + g)
        for _ in range(4):
            s.play(24)
        rng = ol.rng_seed(g)
        s.random_plies(rng, 4 * (g % 10), True)
        if s.info()["phase"] == 3:
            continue
        for k in range(5):
            smp = s.card_matching(ol.rng_seed(1000 * g + k))
            assert s.consistent_sample(smp)


def test_ar_engine_vs_oracle(native_bins):
    """ar_engine.h (host build, driven in lockstep rounds like the GPU) = oracle
    forward_pred_process_with_mask with the hash network: status, reason, sample, network
    calls and RNG stream position per lane, at temperatures 1, 0.35 and 4."""
    out = subprocess.run([os.path.join(NATIVE, "ar_check"), "200", "3", "9"], capture_output=True, text=True, check=True).stdout
    assert out.startswith("OK"), out
    lanes, ok, bad, panic = map(int, out.split()[1:5])
    assert lanes == 1800 and ok > 1000 and bad > 20


def test_bench_refuses_world_size_mismatch():
    """bench.py --gpus N inside a launcher that started a different number of ranks
    fails before any GPU call (it would otherwise report an N-GPU metric for fewer)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run(["python", os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                         text=True, timeout=60)
    assert out.returncode != 0
    assert "--gpus 2 but WORLD_SIZE=1" in out.stderr
