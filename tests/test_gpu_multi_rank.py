"""The bench's N>1 path with the real HIP kernels (config C4 rehearsed on one GPU).

`bench.py --gpus 2` starts two ranks itself (torch.distributed.run, before touching
the GPU); with DK_DIST_BACKEND=gloo both ranks share cuda:0.  Two partitions:
  * infostates (default): each rank determinizes, searches and fuses its half of the
    infostates with all their samples, and the fused actions are all-gathered (gloo
    here, RCCL on an 8-GPU node): decisions AND accumulators equal the 1-rank run
    over the same global workload bit for bit, for both fusions;
  * samples: each rank searches its half of every infostate's samples, runs
    dk_fuse_accumulate_async on them, the accumulators are all-reduced and every rank
    runs dk_fuse_select_async.
Reference: the sample fan-out of DefaultImpiPolicy
(rs-doko-py-bridge/src/compare_impi/compare_impi.rs:217-291) and the fusions
(policy_fusion.rs:23-123).

With the sample split, MaxN fuses integer rank sums, so the 2-rank decision must
equal the 1-rank run over the same global workload bit for bit.  Average-strategy fusion sums f32
probabilities: the two ranks' partial sums added by the all-reduce are a different
f32 summation order than one rank's sequential sum (the reference's own order is
JoinSet completion order, compare_impi.rs:276-288), so the accumulators agree within
f32 rounding (rtol 1e-6 on sums of <= 64 terms <= 1) and the action agrees wherever
the top two sums are further apart than that.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

INFO_PER_RANK, ITERS = 48, 200


def _bench(tmp_path, gpus, infostates, fusion, tag, partition="samples", backend="gloo", extra=()):
    env = dict(os.environ)
    env["DK_DIST_BACKEND"] = backend
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    act = str(tmp_path / ("act_%s.npy" % tag))
    acc = str(tmp_path / ("acc_%s.npy" % tag))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--steps", "1", "--warmup", "0",
           "--no-cpu-baseline", "--small-infostates", "0", "--infostates", str(infostates),
           "--iterations", str(ITERS), "--fusion", fusion, "--dump-actions", act, "--dump-acc", acc,
           "--partition", partition] + list(extra)
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110 + 20 * gpus)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line), np.load(act), np.load(acc)


def test_bench_two_ranks_maxn_exact(tmp_path):
    r2, a2, acc2 = _bench(tmp_path, 2, INFO_PER_RANK, "maxn", "2")
    assert r2["n_gpus"] == 2 and r2["ranks"] == 2
    assert r2["config"]["roots_per_gpu"] == 2 * INFO_PER_RANK * 32
    r1, a1, acc1 = _bench(tmp_path, 1, 2 * INFO_PER_RANK, "maxn", "1")
    assert r1["n_gpus"] == 1
    assert a2.shape == (2 * INFO_PER_RANK,)
    assert np.array_equal(acc2, acc1)
    assert np.array_equal(a2, a1)


@pytest.mark.parametrize("fusion", ["maxn", "avg"])
def test_bench_two_ranks_infostate_partition_exact(tmp_path, fusion):
    r2, a2, acc2 = _bench(tmp_path, 2, INFO_PER_RANK, fusion, "i2" + fusion, "infostates")
    assert r2["n_gpus"] == 2 and r2["ranks"] == 2
    assert r2["config"]["roots_per_gpu"] == INFO_PER_RANK * 64          # the N = 1 shape per rank
    r1, a1, acc1 = _bench(tmp_path, 1, 2 * INFO_PER_RANK, fusion, "i1" + fusion, "infostates")
    assert a2.shape == (2 * INFO_PER_RANK,)
    assert np.array_equal(acc2, acc1)
    assert np.array_equal(a2, a1)


def test_bench_two_ranks_avg_tolerance(tmp_path):
    _, a2, acc2 = _bench(tmp_path, 2, INFO_PER_RANK, "avg", "2a")
    _, a1, acc1 = _bench(tmp_path, 1, 2 * INFO_PER_RANK, "avg", "1a")
    np.testing.assert_allclose(acc2, acc1, rtol=1e-6, atol=1e-6)
    for i in range(a1.shape[0]):
        if a1[i] != a2[i]:
            top = np.sort(acc1[i])[-2:]
            assert top[1] - top[0] <= 1e-5, (i, a1[i], a2[i], top)


@pytest.mark.parametrize("partition", ["infostates", "samples"])
def test_bench_rccl_one_rank(tmp_path, partition):
    """The N > 1 code path over RCCL on the MI355X (`--dist-one-rank`: a one-rank nccl process
    group, so the all-gather of the actions / all-reduce of the accumulators, the barriers and
    the max-over-ranks timing all run through RCCL on the device): decisions and accumulators
    equal the plain one-GPU run bit for bit."""
    r, a, acc = _bench(tmp_path, 1, 2 * INFO_PER_RANK, "maxn", "r" + partition, partition, backend="nccl",
                       extra=("--dist-one-rank",))
    assert r["dist_backend"] == "nccl" and r["ranks"] == 1, r
    r0, a0, acc0 = _bench(tmp_path, 1, 2 * INFO_PER_RANK, "maxn", "p" + partition, partition, backend="nccl")
    assert r0["dist_backend"] is None
    assert np.array_equal(acc, acc0) and np.array_equal(a, a0)


@pytest.mark.parametrize("ranks", [4, 8])
@pytest.mark.parametrize("partition", ["infostates", "samples"])
def test_bench_many_ranks(tmp_path, partition, ranks):
    """Four and eight ranks on one GPU (gloo): the all-gather of the actions (infostates) and
    the all-reduce of the accumulators (samples, the shape config 4 names: "RCCL visit
    all-reduce") at the width of a 4- and an 8-GPU run (C4's full width: 8 samples per
    infostate and rank with the sample split).  MaxN decisions and accumulators equal the
    1-rank run over the same global workload bit for bit, and the line attributes each rank's
    step: search-kernel and collective milliseconds per rank (compare_impi.rs:217-291)."""
    per = INFO_PER_RANK // 2          # --infostates: per rank (infostates) / global = ranks x per (samples)
    rN, aN, accN = _bench(tmp_path, ranks, per, "maxn", "q%d%s" % (ranks, partition), partition)
    assert rN["n_gpus"] == ranks and rN["ranks"] == ranks
    assert len(rN["search_kernel_ms_per_rank"]) == ranks and len(rN["collective_ms_per_rank"]) == ranks
    assert all(ms > 0 for ms in rN["search_kernel_ms_per_rank"]) and rN["collective_ms"] >= 0
    assert rN["collective"].startswith("all_gather" if partition == "infostates" else "all_reduce")
    total = ranks * per
    assert rN["config"]["roots_per_gpu"] == per * 64        # infostates: per x 64; samples: ranks per x 64/ranks
    r1, a1, acc1 = _bench(tmp_path, 1, total, "maxn", "q1%d%s" % (ranks, partition), partition)
    assert aN.shape == (total,)
    assert np.array_equal(accN, acc1) and np.array_equal(aN, a1)


def _bench_c5(tmp_path, gpus, tag, offset=0, extra=()):
    env = dict(os.environ)
    env["DK_DIST_BACKEND"] = "gloo"
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    rec = str(tmp_path / ("rec_%s" % tag))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "c5", "--gpus", str(gpus), "--steps", "2",
           "--warmup", "1", "--no-cpu-baseline", "--games", "96", "--az-iterations", "24",
           "--replica-offset", str(offset), "--dump-records", rec] + list(extra)
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=150 + 30 * gpus)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line), rec


def test_bench_c5_replicas_two_ranks(tmp_path):
    """Config 5 on N GPUs runs N independent self-play replicas (games do not interact; only the
    barriers and the max-over-ranks time are collective).  Two ranks on one GPU (gloo): each rank's
    games after three moves (every dk_az_state record: state, announcements) equal a 1-rank run of
    the same replica (--replica-offset), bit for bit, at the reference's f32 network precision."""
    r2, rec2 = _bench_c5(tmp_path, 2, "two")
    assert r2["n_gpus"] == 2 and r2["config"]["parallelism"] == "replicas x2"
    for rep in (0, 1):
        r1, rec1 = _bench_c5(tmp_path, 1, "one%d" % rep, offset=rep)
        assert r1["n_gpus"] == 1
        a, b = np.load("%s_r%d.npy" % (rec2, rep)), np.load("%s_r%d.npy" % (rec1, rep))
        assert a.shape == b.shape and np.array_equal(a, b), rep
    assert not np.array_equal(np.load("%s_r0.npy" % rec2), np.load("%s_r1.npy" % rec2))   # distinct replicas


def test_bench_c5_streams_equal_one_batch(tmp_path):
    """--c5-streams 8 (the default): the games split into eight searches on their own engines and
    streams, their iterations interleaved; every game's record after three moves equals the
    one-batch run (--c5-streams 1)."""
    r1, rec1 = _bench_c5(tmp_path, 1, "s1", extra=("--c5-streams", "1"))
    r2, rec2 = _bench_c5(tmp_path, 1, "s2", extra=("--c5-streams", "8"))
    assert r2["c5_streams"] == 8 and r1["c5_streams"] == 1
    a, b = np.load("%s_r0.npy" % rec1), np.load("%s_r0.npy" % rec2)
    assert a.shape == b.shape and np.array_equal(a, b)
