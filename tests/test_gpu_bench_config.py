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


def _bench_workload(argv, monkeypatch, eng=None, keep=False, steps=1):
    """bench.make_workload with bench's argv; `steps` steps of the hot path; the device
    invariants of bench.check_visits; host copies of the buffers.  keep=True returns the
    engine (open) for a following leg, as bench.main runs its small leg on the same engine."""
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
    eng, step, n_roots, bufs = bench.make_workload(args, dk, L, dev, sp, 0, 1, 0, eng=eng)
    for _ in range(steps):
        step()
    assert L.dk_sync(eng.ctx, sp) == 0
    bench.check_visits(bufs, args.iterations, " ".join(argv))     # on the device: sums and best
    out = {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else v) for k, v in bufs.items()}
    del bufs, step
    if not keep:
        eng.close()
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    return (args, n_roots, out, eng) if keep else (args, n_roots, out)


def _host_invariants(out, iters):
    """The device invariants again on the host copy: row sums and best = an argmax."""
    v = out["visits"].astype(np.int64)
    sums = v.sum(axis=1)
    bad = np.nonzero(sums != iters)[0]
    assert bad.size == 0, (bad[:16].tolist(), sums[bad[:16]].tolist())
    b = out["best"].astype(np.int64)
    assert (b < 39).all()
    assert (v[np.arange(len(b)), b] == v.max(axis=1)).all()


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


def _c3_check_picks(out, args, I, S, picks, rng, lds_path=None, per_info=4):
    checked = overflow = 0
    for j in picks:
        st = _fdo_info(j)
        for s in sorted(set([0, S - 1] + rng.choice(S, size=per_info, replace=False).tolist())):
            r = j * S + s
            smp = st.card_matching(ol.rng_seed(0xC3200000 + j * args.samples + s))
            pk = smp.pack()
            assert out["roots"][r, :32].tobytes() == pk[:32] and out["roots"][r, 92:98].tobytes() == pk[92:98], r
            best, v, val, ctr = smp.search(ol.rng_seed(0xC3300000 + j * args.samples + s), ITERS, args.c)
            _check_root(out["visits"][r], out["values"][r], out["best"][r], best, v, val, (j, s))
            checked += 1
            if lds_path is not None:
                overflow += ctr[6] >= lds_path
    return checked, overflow


def test_c3_bench_two_legs(monkeypatch, capfd):
    """bench.main's exact sequence on one engine: the timed C3 batch at bench's default
    size (36,864 infostates x 64 CAP samples = 2,359,296 roots, twelve groups per resident
    wave), then the small-batch leg (512 infostates: 32-root waves, 16-B records) on the
    same engine with its own buffers.  Every root of both legs passes the device
    invariants (visit sum, best = an argmax) and the host re-check; roots spread over each
    queue equal oracle searches bitwise; whole infostates fuse to the oracle's action."""
    I, S = 36864, 64
    args, n_roots, out, eng = _bench_workload([], monkeypatch, keep=True)
    assert args.infostates == I and n_roots == I * S
    ln = _launch_line(capfd)
    assert ln["hot"] == "8B", ln
    grid, rpw = int(ln["grid"]), int(ln["rpw"])
    assert rpw == 64 and int(ln["resident/CU"]) * 256 >= grid
    assert n_roots // rpw >= 12 * grid, ln          # twelve groups per resident wave, as timed
    lds_path = int(ln["lds_path"])
    assert lds_path <= 16
    _host_invariants(out, ITERS)
    rng = np.random.default_rng(2024)
    checked, overflow = _c3_check_picks(out, args, I, S, _picks(I, grid, rng), rng, lds_path)
    assert checked >= 64
    assert overflow >= 4, overflow      # roots whose deepest path spilled past the LDS entries
    for j in (0, grid, I - 1):          # whole infostates: MaxN over every sample == the device's action
        st = _fdo_info(j)
        rows = []
        for s in range(S):
            smp = st.card_matching(ol.rng_seed(0xC3200000 + j * S + s))
            _, v, _, _ = smp.search(ol.rng_seed(0xC3300000 + j * S + s), ITERS, args.c)
            assert list(out["visits"][j * S + s]) == v, (j, s)
            rows.append(v)
        exp, _ = ol.fuse_maxn(rows, st.allowed())
        assert int(out["actions"][j]) == exp, j
    del out
    # second leg, same engine (bench.py --small-infostates 512, warm-up + timed steps)
    try:
        I2 = 512
        args2, n2, out2 = _bench_workload(["--infostates", str(I2)], monkeypatch, eng=eng, steps=2)
    finally:
        eng.close()
    ln2 = _launch_line(capfd)
    assert n2 == I2 * S
    assert ln2["hot"] == "16B" and int(ln2["rpw"]) == 32, ln2      # single wave per SIMD: 16-B records
    _host_invariants(out2, ITERS)
    rng = np.random.default_rng(512)
    checked, _ = _c3_check_picks(out2, args2, I2, S, sorted(set([0, 1, 255, 256, I2 - 2, I2 - 1] +
                                                                rng.choice(I2, size=6, replace=False).tolist())), rng)
    assert checked >= 48


def test_bench_cli_two_legs():
    """`bench.py` itself, both legs (bench's check_visits raises on any device violation),
    with the round-2 pageable host readbacks re-checked: no host copy may differ either."""
    import json
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--steps", "1", "--warmup", "0", "--small-steps",
                        "1", "--no-cpu-baseline", "--host-readback-check"], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["host_copy_bad_roots"] == {"batch": 0, "small": 0}, line["host_copy_bad_roots"]
    assert line["small_batch"]["roots_per_gpu"] == 32768
    assert line["roofline"]["achieved"] > 0 and line["node_pools"]["overflowed_roots"] >= 0


def test_root_window_sample_split(monkeypatch, capfd):
    """One rank's share of the C4 sample split at N = 8 (8 samples per infostate, so a
    64-root group holds 8 infostates of all four depth classes), searched in launch order
    and through depth-sorted windows (DK_ROOT_WINDOW): every root's visits, values and best
    are identical, and match oracle searches."""
    I, S = 16384, 8                     # 131,072 roots: two groups per SIMD, 8-B records
    monkeypatch.setenv("DK_ROOT_WINDOW", "0")
    args, n_roots, a = _bench_workload(["--infostates", str(I), "--samples", str(S)], monkeypatch)
    assert _launch_line(capfd)["root_window"] == "0"
    monkeypatch.delenv("DK_ROOT_WINDOW")   # the default window
    _, _, b = _bench_workload(["--infostates", str(I), "--samples", str(S)], monkeypatch)
    ln = _launch_line(capfd)
    assert ln["root_window"] == "1024" and ln["hot"] == "8B", ln
    for k in ("visits", "best", "actions"):
        assert np.array_equal(a[k], b[k]), k
    assert a["values"].tobytes() == b["values"].tobytes()
    rng = np.random.default_rng(8)
    checked, _ = _c3_check_picks(b, args, I, S, sorted(set([0, 1, 7, 8, I - 1] + rng.choice(I, 6, replace=False).tolist())),
                                 rng, per_info=2)
    assert checked >= 30


def test_c2d_bench_launch_parity(monkeypatch, capfd):
    """Determinized rs-doko (c2d) at bench's default 12,288 infostates x 64 rule-based samples: 8-B records,
    longest-first group queue, pool reuse."""
    I, S = 12288, 64
    args, n_roots, out = _bench_workload(["--workload", "c2d"], monkeypatch)
    assert args.infostates == I and n_roots == I * S
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
    32-root waves and 16-B records the launch picks for this batch."""
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


