"""Parity of the configuration bench.py actually measures.

The bench's launch differs from the small parity tests' launches: with >= 2 groups
per resident wave the search kernel takes the 8-B hot records, the LDS path length
the occupancy calculator picks (14 entries at 64 roots per wave), a persistent grid
whose waves each stream several 64-root groups through one reused pool region, and
for rs-doko the longest-first group queue (group_order_kernel).  These tests build the
bench's own workloads with bench.make_workload at the bench's launch shape, run one
step, and compare roots spread over the whole queue -- the first groups, the groups at
the resident-grid boundary (a wave's second group, in a region that still holds the
previous group's trees) and the groups dequeued last -- with oracle searches on the same
seeds: visits, f64 values (bitwise), best move, and the fused action of whole
infostates.  Roots whose selection paths overflow the LDS path into the global
overflow stack are counted with the oracle's path-entry counter and must be present.

Reference: rs-doko-mcts/src/mcts/mcts.rs:172-249 (the loop), node.rs:202-277 (UCT),
compare_impi.rs:212-371 + policy_fusion.rs:23-74 (sample fan-out and MaxN fusion).
"""
import re
import sys

import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu

ITERS = 1000
LDS_ENTRIES_C3 = 14


def _bench_workload(argv, monkeypatch):
    import torch

    import bench
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    monkeypatch.setenv("DK_VERBOSE", "1")
    args = bench.parse()
    L = _native.lib()
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    eng, step, n_roots, bufs = bench.make_workload(args, dk, L, dev, sp, 0, 1, 0)
    step()
    assert L.dk_sync(eng.ctx, sp) == 0
    out = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in bufs.items()}
    eng.close()
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    return args, n_roots, out


def _launch_line(capfd):
    err = capfd.readouterr().err
    lines = [l for l in err.splitlines() if l.startswith("doko_amd: search")]
    assert lines, err[-2000:]
    m = dict(re.findall(r"(\w+(?:/\w+)?)=(\S+)", lines[-1]))
    return m


def _check_root(got_v, got_val, got_b, best, v, val, tag):
    assert list(got_v) == v, tag
    assert got_val.tobytes() == np.array(val, dtype=np.float64).tobytes(), tag
    assert int(got_b) == (best if best >= 0 else 255), tag


def _fdo_info(j):
    st = ol.FdoState.new_game(0xC3000000 + j)
    for _ in range(4):
        st.play(24)
    st.random_plies(ol.rng_seed(0xC3100000 + j), [0, 8, 20, 32][j % 4], True)
    return st


def _do_info(j):
    st = ol.DoState.new_game(0xC3000000 + j)
    for _ in range(4):
        st.play(24)
    st.random_plies(ol.rng_seed(0xC3100000 + j), [0, 8, 20, 32][j % 4])
    return st


def _picks(I, resident_groups, rng, n_random=8):
    """Infostates (= 64-root groups) spread over the queue."""
    edge = [0, 1, resident_groups - 1, resident_groups, resident_groups + 1, 2 * resident_groups, I - 2, I - 1]
    rand = rng.choice(I, size=n_random, replace=False).tolist()
    return sorted(set(j for j in edge + rand if 0 <= j < I))


def test_c3_bench_launch_parity(monkeypatch, capfd):
    """C3 at 6144 infostates x 64 CAP samples (393,216 roots: two groups per resident wave)."""
    import master_doko_reinforcement_learning_amd as dk
    I, S = 6144, 64
    args, n_roots, out = _bench_workload(["--infostates", str(I), "--iterations", str(ITERS)], monkeypatch)
    ln = _launch_line(capfd)
    assert ln["hot"] == "8B", ln
    grid, rpw = int(ln["grid"]), int(ln["rpw"])
    assert rpw == 64 and n_roots == I * S
    assert n_roots // rpw >= 2 * grid, ln           # waves stream >= 2 groups through their pool region
    lds_path = int(ln["lds_path"])
    assert lds_path <= 16
    rng = np.random.default_rng(2024)
    infos = _picks(I, grid, rng)
    checked = overflow = 0
    for j in infos:
        st = _fdo_info(j)
        for s in sorted(set([0, S - 1] + rng.choice(S, size=4, replace=False).tolist())):
            r = j * S + s
            smp = st.card_matching(ol.rng_seed(0xC3200000 + j * S + s))
            pk = smp.pack()
            assert out["roots"][r, :32].tobytes() == pk[:32] and out["roots"][r, 92:98].tobytes() == pk[92:98], r
            best, v, val, ctr = smp.search(ol.rng_seed(0xC3300000 + j * S + s), ITERS, args.c)
            _check_root(out["visits"][r], out["values"][r], out["best"][r], best, v, val, (j, s))
            checked += 1
            overflow += ctr[6] >= lds_path
    assert checked >= 64
    assert overflow >= 8, overflow      # roots whose deepest path spilled past the LDS entries
    # whole infostates: every sample searched by the oracle, MaxN fused == the device's action
    for j in (0, grid, I - 1):
        st = _fdo_info(j)
        rows = []
        for s in range(S):
            smp = st.card_matching(ol.rng_seed(0xC3200000 + j * S + s))
            _, v, _, _ = smp.search(ol.rng_seed(0xC3300000 + j * S + s), ITERS, args.c)
            assert list(out["visits"][j * S + s]) == v, (j, s)
            rows.append(v)
        exp, _ = ol.fuse_maxn(rows, st.allowed())
        assert int(out["actions"][j]) == exp, j


def test_c2d_bench_launch_parity(monkeypatch, capfd):
    """Determinized rs-doko (c2d) at 6144 infostates x 64 rule-based samples: 8-B records,
    longest-first group queue, pool reuse."""
    I, S = 6144, 64
    args, n_roots, out = _bench_workload(["--workload", "c2d", "--infostates", str(I), "--iterations", str(ITERS)],
                                         monkeypatch)
    ln = _launch_line(capfd)
    assert ln["hot"] == "8B", ln
    grid = int(ln["grid"])
    assert n_roots // int(ln["rpw"]) >= 2 * grid
    rng = np.random.default_rng(77)
    checked = 0
    for j in _picks(I, grid, rng):
        st = _do_info(j)
        for s in sorted(set([0, S - 1] + rng.choice(S, size=4, replace=False).tolist())):
            r = j * S + s
            smp = st.sample_assignment_full(ol.rng_seed(0xC3200000 + j * S + s))
            assert out["roots"][r].tobytes() == smp.pack(), r
            best, v, val, _ = smp.search(ol.rng_seed(0xC3300000 + j * S + s), ITERS, args.c)
            _check_root(out["visits"][r], out["values"][r], out["best"][r], best, v, val, (j, s))
            checked += 1
    assert checked >= 64


def test_c2_bench_parity_1000(monkeypatch, capfd):
    """C2 (rs-doko, 32,768 deals after 4x Healthy) at the config's 1000 iterations: the
    32-root waves and 32-B records the launch picks for this batch."""
    args, n_roots, out = _bench_workload(["--workload", "c2", "--iterations", str(ITERS)], monkeypatch)
    ln = _launch_line(capfd)
    assert n_roots == 32768
    rng = np.random.default_rng(5)
    picks = sorted(set([0, 1, 31, 32, 16383, 16384, 32766, 32767] + rng.choice(n_roots, size=60, replace=False).tolist()))
    for i in picks:
        st = ol.DoState.new_game(0xD0C00000 + i)
        for _ in range(4):
            st.play(24)
        assert out["roots"][i].tobytes() == st.pack(), i
        seed = (i * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF
        best, v, val, _ = st.search(ol.rng_seed(seed), ITERS, args.c)
        _check_root(out["visits"][i], out["values"][i], out["best"][i], best, v, val, (i, ln))


def test_c3_small_batch_parity(monkeypatch, capfd):
    """C3's small-batch leg (bench.py --small-infostates: 512 infostates x 64 CAP samples =
    32,768 roots): one group per wave, 32-root waves and the 32-B hot records the launch
    picks when the grid gives a SIMD fewer than two waves.  Every root's visits sum to the
    iterations, and roots spread over the batch match oracle searches bitwise."""
    I, S = 512, 64
    args, n_roots, out = _bench_workload(["--infostates", str(I), "--iterations", str(ITERS)], monkeypatch)
    ln = _launch_line(capfd)
    assert n_roots == I * S
    assert ln["hot"] == "32B" and int(ln["rpw"]) == 32, ln
    sums = out["visits"].astype(np.int64).sum(axis=1)
    bad = np.nonzero(sums != ITERS)[0]
    assert bad.size == 0, (bad[:16].tolist(), sums[bad[:16]].tolist())
    rng = np.random.default_rng(512)
    checked = 0
    for j in sorted(set([0, 1, 255, 256, I - 2, I - 1] + rng.choice(I, size=6, replace=False).tolist())):
        st = _fdo_info(j)
        for s in sorted(set([0, 31, 32, S - 1] + rng.choice(S, size=2, replace=False).tolist())):
            r = j * S + s
            smp = st.card_matching(ol.rng_seed(0xC3200000 + j * S + s))
            best, v, val, _ = smp.search(ol.rng_seed(0xC3300000 + j * S + s), ITERS, args.c)
            _check_root(out["visits"][r], out["values"][r], out["best"][r], best, v, val, (j, s))
            checked += 1
    assert checked >= 48
