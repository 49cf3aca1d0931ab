"""Multi-rank decision path on CPU (gloo, world_size 2), both bench.py partitions:
  * samples: the samples of every infostate are split over the ranks, each rank fuses
    its share into summable accumulators (the arithmetic of fuse_accumulate_kernel:
    1-based stable ranks, 0 for disallowed actions; probability sums for Avg), one
    all-reduce(sum) combines them and every rank selects;
  * infostates (the default): each rank fuses its own infostates over all their samples
    and the fused actions are all-gathered.
The result must equal the oracle's fusion over all samples (policy_fusion.rs:23-123)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as ol

N_INFO, SAMPLES, ITERS = 6, 8, 60


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _workload():
    """Per infostate: legal mask and [SAMPLES][39] visits from oracle searches on CAP samples."""
    allowed, visits = [], []
    for j in range(N_INFO):
        st = ol.FdoState.new_game(0xC3000000 + j)
        for _ in range(4):
            st.play(24)
        st.random_plies(ol.rng_seed(0xC3100000 + j), [0, 8, 20, 32][j % 4], True)
        allowed.append(st.allowed())
        rows = []
        for s in range(SAMPLES):
            smp = st.card_matching(ol.rng_seed(0xC3200000 + j * SAMPLES + s))
            _, v, _, _ = smp.search(ol.rng_seed(0xC3300000 + j * SAMPLES + s), ITERS, 2.5)
            rows.append(v)
        visits.append(rows)
    return np.array(allowed, dtype=np.uint64), np.array(visits, dtype=np.uint32)


def _accumulate(visits, allowed, mode):
    """fuse_accumulate_kernel restated (test-side) for one rank's samples."""
    n_info, s_r, _ = visits.shape
    acc_u = np.zeros((n_info, 39), dtype=np.int64)
    acc_f = np.zeros((n_info, 39), dtype=np.float32)
    for i in range(n_info):
        al = [(int(allowed[i]) >> a) & 1 for a in range(39)]
        for s in range(s_r):
            row = visits[i, s]
            if mode == "maxn":
                for a in range(39):
                    if al[a]:
                        acc_u[i, a] += 1 + sum(1 for b in range(39) if al[b] and (row[b] > row[a] or (row[b] == row[a] and b < a)))
            else:
                tot = float(row.sum())
                for a in range(39):
                    acc_f[i, a] += np.float32(row[a] / tot if tot > 0 else 0.0)
    return acc_u, acc_f


def _select(acc_u, acc_f, allowed, mode):
    out = []
    for i in range(acc_u.shape[0]):
        if mode == "maxn":
            keys = [int(acc_u[i, a]) if (int(allowed[i]) >> a) & 1 else 2**32 - 1 for a in range(39)]
            out.append(int(np.argmin(keys)))                                  # first minimum
        else:
            best = 0
            for a in range(1, 39):
                if not acc_f[i, best] > acc_f[i, a]:
                    best = a                                                  # last maximum
            out.append(best)
    return out


def _worker(rank, world, port, allowed, visits, mode, q, partition="samples"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    if partition == "infostates":
        # bench.py --partition infostates: rank r owns infostates [r*I_r, (r+1)*I_r) with all samples,
        # fuses them locally and the actions are all-gathered (uint8, as on the device)
        i_r = N_INFO // world
        sl = slice(rank * i_r, (rank + 1) * i_r)
        acc_u, acc_f = _accumulate(visits[sl], allowed[sl], mode)
        mine = torch.tensor(_select(acc_u, acc_f, allowed[sl], mode), dtype=torch.uint8)
        parts = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        fparts = [torch.zeros((i_r, 39), dtype=torch.float32) for _ in range(world)]
        dist.all_gather(fparts, torch.from_numpy(acc_f))
        q.put((rank, torch.cat(parts).tolist(), torch.cat(fparts).numpy()))
        dist.destroy_process_group()
        return
    s_r = SAMPLES // world
    mine = visits[:, rank * s_r:(rank + 1) * s_r]          # bench.py: samples [rank*S_r, (rank+1)*S_r)
    acc_u, acc_f = _accumulate(mine, allowed, mode)
    tu = torch.from_numpy(acc_u)
    tf = torch.from_numpy(acc_f)
    dist.all_reduce(tu)
    dist.all_reduce(tf)
    q.put((rank, _select(tu.numpy(), tf.numpy(), allowed, mode), tf.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("partition", ["samples", "infostates"])
@pytest.mark.parametrize("mode", ["maxn", "avg"])
def test_two_rank_fusion_equals_single_process(mode, partition):
    allowed, visits = _workload()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, allowed, visits, mode, q, partition)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert res[0][1] == res[1][1], "ranks disagree"
    for i in range(N_INFO):
        rows = [list(map(int, r)) for r in visits[i]]
        if mode == "maxn":
            want, _ = ol.fuse_maxn(rows, int(allowed[i]))
            assert res[0][1][i] == want, i
        else:
            want, probs = ol.fuse_avg(rows)
            np.testing.assert_allclose(res[0][2][i], np.array(probs, dtype=np.float32), rtol=0, atol=1e-5)
            top = sorted(probs)[-2:]
            if top[1] - top[0] > 1e-4:    # summation order may flip only near-ties (reference order is nondeterministic)
                assert res[0][1][i] == want, i
