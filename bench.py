"""Benchmark: determinized rollouts/sec (48-card full game, 1000 sims/root).

One step = one determinized decision batch of BASELINE.json config 3 on every
GPU, entirely on the device:
    CAP determinization (card_matching_full)  -> 36864 infostates x 64 samples = 2,359,296 roots
    UCT search, 1000 simulations per root (select/expand/random rollout/backup)
    policy fusion (MaxN) of the per-sample visit counts per infostate
With N GPUs (config 4) the global batch holds 36864*N infostates (weak scaling,
2,359,296 roots per GPU).  By default every rank owns 36864 of them with all 64
samples, so its work has exactly the N = 1 shape, and the fused actions are
gathered with one RCCL all-gather over xGMI; --partition samples instead splits
every infostate's samples over the ranks and sums the fusion accumulators with one
RCCL all-reduce before the action is selected.

Rank 0 prints one JSON line.  `value` = simulations of all ranks / max-over-ranks
wall time of the K timed steps.  Inputs (the infostates) are synthesised on the
GPU before the timed region.
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "determinized rollouts/sec (48-card full game, 1000 sims/root) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def simds(dev):
    """SIMDs of the device (4 per CU on gfx950)."""
    import torch
    return 4 * torch.cuda.get_device_properties(dev).multi_processor_count


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--workload", choices=["c3", "c2", "c2d", "c5", "impi", "impid", "c1", "prod"], default="c3",
                   help="c3: rs-full-doko + CAP (default, the metric's config); c2: rs-doko roots after 4x Healthy; "
                        "c2d: rs-doko infostates determinized by the rule-based sampler; "
                        "c5: AlphaZero self-play moves (PUCT + policy/value network); "
                        "impi: autoregressive (IMPI) determinization of the c3 infostates with the IMPI network; "
                        "impid: the AR-determinized decision (mcts_ar_maxn_policy: AR samples -> UCT -> MaxN); "
                        "c1: tic-tac-toe games (tic_tac_toe_player: one SmallRng stream through every search, and "
                        "independent games in lockstep); prod: the thesis's production search shape (S samples x "
                        "200,000 iterations, run.rs:270-291): decision latency and decisions in flight")
    p.add_argument("--c1-games", type=int, default=1000, help="c1: independent games in lockstep per step")
    p.add_argument("--c1-serial-games", type=int, default=5,
                   help="c1: games of the one-stream tic_tac_toe_player timed on the GPU and on the oracle")
    p.add_argument("--prod-iterations", type=int, default=200000, help="prod: iterations per sample (run.rs:270-291)")
    p.add_argument("--prod-samples", default="5,10,50", help="prod: samples per decision, one leg each")
    p.add_argument("--prod-inflight", type=int, default=16, help="prod: decisions in flight in the batched leg")
    p.add_argument("--prod-capacity", type=int, default=-1,
                   help="prod: decisions of max(samples) samples in flight at the pools' capacity in one pass "
                        "(-1: as many as fit in the free device memory; 0: skip)")
    p.add_argument("--prod-slots-per-iter", type=float, default=2.5,
                   help="prod capacity leg: node slots per iteration and root (measured demand 1.95 at 200,000; a "
                        "root that outgrows them is searched again in the fallback pool, results unchanged)")
    p.add_argument("--games", type=int, default=8192, help="concurrent self-play games per GPU (c5)")
    p.add_argument("--az-iterations", type=int, default=200, help="PUCT iterations per move (c5)")
    p.add_argument("--impi-streams", type=int, default=8,
                   help="impi: split the infostates into this many independent AR samplings (one engine and HIP "
                        "stream each) whose network rounds are issued interleaved (api.sample_interleaved)")
    p.add_argument("--c5-streams", type=int, default=8,
                   help="c5: split the games into this many independent searches (one engine and HIP stream each) "
                        "whose iterations are issued interleaved, so one part's kernels fill the others' tails "
                        "(8: +4 %% against 1 and 16, profiles/r06/c5_streams/)")
    p.add_argument("--ar-samples", type=int, default=4, help="AR samples per infostate (impi)")
    p.add_argument("--net-precision", choices=["bf16", "f32"], default="f32",
                   help="c5 / impi / impid network: f32 (default) = the reference's precision (f32 activations at "
                        "matmul precision 'medium', az_doko.py:539-541 / main.py:508) on the hand-written f32 kernels, "
                        "GEMM products from bf16 hi / lo pieces (bf16x3, ~16-bit products, as fine as hipBLASLt's "
                        "'medium' measured: profiles/r04/fp32_gemm_probe.json; no hipBLASLt kernel runs); bf16 = the "
                        "fused bf16 kernels, NARROWER than the reference (bf16 activations and weights, opt-in)")
    p.add_argument("--ar-temperature", type=float, default=0.4, help="AR sampling temperature (impi; all_policies.rs:30)")
    p.add_argument("--iterations", type=int, default=1000)
    p.add_argument("--infostates", type=int, default=None,
                   help="infostates per GPU (c3: default 36864 x 64 samples = 2,359,296 roots, twelve 64-root groups "
                        "per resident wave (3072 waves): the persistent grid's drain tail is 4.5 %% of the launch, "
                        "against 7.5 %% at six groups (per-wave clocks, DESIGN.md §4.1); c2d, impi, impid: default 12288)")
    p.add_argument("--samples", type=int, default=64, help="samples per infostate (c3, c2d)")
    p.add_argument("--partition", choices=["infostates", "samples"], default="infostates",
                   help="N > 1 (c3, c2d): 'infostates' = each rank owns 1/N of the infostates with all their samples "
                        "(every rank's work has the N = 1 shape; one RCCL all-gather of the fused actions); "
                        "'samples' = the samples of every infostate split over the ranks (one RCCL all-reduce of "
                        "the fusion accumulators)")
    p.add_argument("--roots", type=int, default=32768, help="roots per GPU (c2)")
    p.add_argument("--c", type=float, default=2.5)
    p.add_argument("--fusion", choices=["maxn", "avg"], default="maxn")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--cpu-roots-per-thread", type=int, default=96)
    p.add_argument("--dump-actions", default="", help="rank 0 writes the fused actions (.npy) of the last step")
    p.add_argument("--replica-offset", type=int, default=0,
                   help="c5: replica index = rank + offset (seeds and network weights), so that a 1-rank run can "
                        "reproduce any rank of an N-rank run")
    p.add_argument("--dump-records", default="",
                   help="c5: every rank writes its games' dk_az_state records after the last step to <path>_r<replica>.npy")
    p.add_argument("--dump-acc", default="", help="rank 0 writes the all-reduced fusion accumulators (.npy) of the last step")
    p.add_argument("--small-infostates", type=int, default=512,
                   help="c3: also time the survey's small decision batch (512 infostates x 64 = 32,768 roots); 0 = skip")
    p.add_argument("--small-steps", type=int, default=5)
    p.add_argument("--inflight", default="2,4,8",
                   help="c3 small batch: also time K independent decision batches in flight on one engine "
                        "(DefaultImpiPolicy.execute_many), for each K in this list; empty = skip")
    p.add_argument("--dist-one-rank", action="store_true",
                   help="c3 / c2d at --gpus 1: initialise the process group anyway (RCCL, one rank) so that the "
                        "multi-GPU collectives (all-gather of the actions, all-reduce of the accumulators, barriers, "
                        "max-over-ranks timing) run on the device; results equal the plain N = 1 run")
    p.add_argument("--host-readback-check", action="store_true",
                   help="also copy every leg's visits to pageable host memory and check them there (the round-2 "
                        "sequence); a host-only violation is reported as host_copy_bad_roots, not raised")
    a = p.parse_args()
    if a.infostates is None:
        a.infostates = 36864 if a.workload == "c3" else 12288   # c2d: 2.18 G/s at 18432 against 2.24 at 12288
    return a


def make_workload(args, dk, L, dev, sp, rank, world, local_rank, dist=None, eng=None):
    """Build the synthetic inputs on the GPU (untimed) and return (engine, step,
    n_roots, buffers).  `step()` runs one pass of the hot path on stream `sp`."""
    import torch
    def ck(rc):
        if rc != 0:
            raise RuntimeError("doko_amd error %d: %s" % (rc, L.dk_status_string(rc).decode()))

    def ptr(t):
        return t.data_ptr()

    iters = args.iterations
    fuse_mode = dk.FUSE_MAXN if args.fusion == "maxn" else dk.FUSE_AVG

    determinized = args.workload in ("c3", "c2d")
    game = dk.GAME_FULL_DOKO if args.workload == "c3" else dk.GAME_DOKO
    by_info = args.partition == "infostates"
    if determinized:
        if not by_info and args.samples % world:
            raise SystemExit("samples must be divisible by the number of GPUs")
        # global infostates j = 0 .. infostates*world-1; this rank's: j0 .. j0+I-1 (all samples s0 .. s0+S_r-1)
        I = args.infostates if by_info else args.infostates * world
        S_r = args.samples if by_info else args.samples // world
        j0 = rank * I if by_info else 0
        s0 = 0 if by_info else rank * S_r
        n_roots = I * S_r
    else:
        I, S_r = 0, 0
        n_roots = args.roots
    if eng is None:
        eng = dk.Engine(device=local_rank, max_roots=n_roots, max_iterations=iters)

    # ------------------------------------------------------------ inputs (untimed, on the GPU)
    def healthy_round(states_t, n):
        a = torch.full((n,), 1 << 24, dtype=torch.int64, device=dev)
        for _ in range(4):
            ck(L.dk_env_step_batch_async(eng.ctx, ptr(states_t), ptr(a), n, sp))

    if determinized:
        gj = np.arange(j0, j0 + I, dtype=np.uint64)            # global infostate indices of this rank
        info_seeds = torch.tensor(gj + np.uint64(0xC3000000), device=dev)
        info = torch.zeros((I, 128), dtype=torch.uint8, device=dev)
        ck(L.dk_new_game_batch_async(eng.ctx, game, ptr(info_seeds), I, ptr(info), sp))
        healthy_round(info, I)
        plies = torch.tensor(np.array([[0, 8, 20, 32][j % 4] for j in range(j0, j0 + I)], dtype=np.uint32).view(np.int32),
                             device=dev)
        ply_rng = torch.tensor(dk.splitmix_rng_states(gj + np.uint64(0xC3100000)).view(np.int64), device=dev)
        ck(L.dk_env_random_plies_batch_async(eng.ctx, ptr(info), ptr(ply_rng), ptr(plies), I, sp))
        allowed = torch.zeros(I, dtype=torch.int64, device=dev)
        ck(L.dk_legal_actions_async(eng.ctx, ptr(info), I, ptr(allowed), sp))
        j = gj[:, None]
        s = np.arange(s0, s0 + S_r, dtype=np.uint64)[None, :]
        samp_seeds = (np.uint64(0xC3200000) + j * np.uint64(args.samples) + s).reshape(-1)
        srch_seeds = (np.uint64(0xC3300000) + j * np.uint64(args.samples) + s).reshape(-1)
        d_samp = torch.tensor(samp_seeds.view(np.int64), device=dev)
        d_srch = torch.tensor(srch_seeds.view(np.int64), device=dev)
        roots = torch.zeros((n_roots, 128), dtype=torch.uint8, device=dev)
        acc_u = torch.zeros((I, 39), dtype=torch.int32, device=dev)
        acc_f = torch.zeros((I, 39), dtype=torch.float32, device=dev)
        actions = torch.zeros(I, dtype=torch.uint8, device=dev)
        dist_on = dist is not None and dist.is_available() and dist.is_initialized()
        gather = by_info and dist_on
        actions_all = torch.zeros((world, I), dtype=torch.uint8, device=dev) if gather else actions
    else:
        gidx = np.arange(rank * n_roots, (rank + 1) * n_roots, dtype=np.uint64)
        d_rs = torch.tensor((gidx + np.uint64(0xD0C00000)).view(np.int64), device=dev)
        roots = torch.zeros((n_roots, 128), dtype=torch.uint8, device=dev)
        ck(L.dk_new_game_batch_async(eng.ctx, dk.GAME_DOKO, ptr(d_rs), n_roots, ptr(roots), sp))
        healthy_round(roots, n_roots)
        d_srch = torch.tensor((gidx * np.uint64(0x9E3779B97F4A7C15) + np.uint64(1)).view(np.int64), device=dev)
    visits = torch.zeros((n_roots, 39), dtype=torch.int32, device=dev)
    values = torch.zeros((n_roots, 39), dtype=torch.float64, device=dev)
    best = torch.zeros(n_roots, dtype=torch.uint8, device=dev)
    ck(L.dk_sync(eng.ctx, sp))
    # HIP events on the step's stream around the collectives (RCCL work is ordered between
    # them): per-rank collective time, so an N-GPU curve separates search from exchange
    coll_events = []

    def collective(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        coll_events.append((e0, e1))

    def step():
        if determinized:
            ck(L.dk_determinize_batch_async(eng.ctx, ptr(info), I, S_r, ptr(d_samp), ptr(roots), sp))
            ck(L.dk_search_batch_async(eng.ctx, game, ptr(roots), ptr(d_srch), n_roots, iters, args.c,
                                       ptr(visits), ptr(values), ptr(best), sp))
            ck(L.dk_fuse_accumulate_async(eng.ctx, ptr(visits), I, S_r, ptr(allowed), fuse_mode, ptr(acc_u), ptr(acc_f), sp))
            if dist_on and not by_info:
                collective(lambda: dist.all_reduce(acc_u if fuse_mode == dk.FUSE_MAXN else acc_f))  # RCCL over xGMI
            ck(L.dk_fuse_select_async(eng.ctx, I, fuse_mode, ptr(allowed), ptr(acc_u), ptr(acc_f), ptr(actions), sp))
            if gather:
                # RCCL over xGMI: every rank's decisions
                collective(lambda: dist.all_gather(list(actions_all.unbind(0)), actions))
        else:
            ck(L.dk_search_batch_async(eng.ctx, dk.GAME_DOKO, ptr(roots), ptr(d_srch), n_roots, iters, args.c,
                                       ptr(visits), ptr(values), ptr(best), sp))

    return eng, step, n_roots, {"visits": visits, "values": values, "best": best, "roots": roots, "I": I, "S_r": S_r,
                                "info": info if determinized else None, "game": game,
                                "actions": actions_all.reshape(-1) if determinized else None,
                                "coll_events": coll_events,
                                "acc": (acc_u if fuse_mode == dk.FUSE_MAXN else acc_f) if determinized else None}


def free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(args):
    """`--gpus N` outside a torchrun environment: start the N ranks (one process per GPU)
    as children under torch.distributed.run and return their exit status.  Called before
    this process touches the GPU (no HIP call, no torch.cuda query)."""
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def result_invariants(visits, best, iters):
    """Per-root invariants of a search result, evaluated ON THE DEVICE (torch ops on the
    current stream): the visits row sums to `iterations` (every simulation passes one root
    child, mcts.rs:172-249), and `best` is an action of maximal visits (max_by_key over the
    root children, mcts_policy.rs:95-111).  Returns a bool tensor, True = violated."""
    import torch
    s = visits.sum(dim=1, dtype=torch.int64)
    mx = visits.max(dim=1).values
    b = best.long()
    vb = torch.gather(visits, 1, b.clamp(max=38)[:, None])[:, 0]
    return (s != iters) | (b > 38) | (vb != mx)


def inflight_rates(args, dk, eng, sbufs, dev, world, dist, steps=3):
    """K independent small decision batches in flight on ONE engine (DefaultImpiPolicy.execute_many:
    batched into one device pass, results split per batch), the regime of an evaluator deciding
    many games at once (compare_impi/run.rs:775).  A step = K whole decisions
    (determinize -> search -> fuse -> select), complete; rate = K x roots x iterations / step time."""
    import torch
    info = sbufs["info"]
    I, S, iters = info.shape[0], sbufs["S_r"], args.iterations
    n = I * S
    fuse = dk.FUSE_MAXN if args.fusion == "maxn" else dk.FUSE_AVG
    policy = dk.DefaultImpiPolicy(eng, args.c, iters, S, fuse)
    out = {}
    for k in [int(x) for x in args.inflight.split(",") if x]:
        seeds = []
        for b in range(k):
            base = np.uint64(0xE1000000 + (b << 24))
            sd = np.concatenate([np.arange(n, dtype=np.uint64) + base, np.arange(n, dtype=np.uint64) + base + np.uint64(n)])
            seeds.append(torch.tensor(sd.view(np.int64), device=dev))
        batches = [(info, seeds[b]) for b in range(k)]
        policy.execute_many(batches, game=sbufs["game"])      # warm-up
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            res = policy.execute_many(batches, game=sbufs["game"])
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        for _, v in res:
            assert not bool((v.sum(dim=1) != iters).any().item()), "inflight: a root without exactly %d simulations" % iters
        out[str(k)] = {"batches_in_flight": k, "value": k * n * iters * steps * world / el, "unit": "rollouts/s",
                       "ms_per_step": el / steps * 1e3}
    return out


def check_visits(bufs, iters, leg):
    """Check every root of a leg with `result_invariants` on the device.  On a violation the
    device buffers are read back twice and compared, so the report says whether the DEVICE
    data is wrong or only a host copy of it (the round-2 failure under
    `rocprofv3 --pmc` was a stale pageable host copy, not a device write)."""
    bad = result_invariants(bufs["visits"], bufs["best"], iters)
    nbad = int(bad.sum().item())
    if nbad:
        idx = bad.nonzero()[:8, 0].cpu().numpy()
        v1, v2 = bufs["visits"].cpu().numpy(), bufs["visits"].cpu().numpy()
        best = bufs["best"].cpu().numpy()
        detail = [(int(i), int(v1[i].sum()), int(best[i]), v1[i].tolist()) for i in idx]
        raise AssertionError("%s: %d roots violate the result invariants on the device (visit sum %d, best = an "
                             "argmax); two host reads identical: %s; first: %s"
                             % (leg, nbad, iters, bool(np.array_equal(v1, v2)), detail))


def check_visits_host(v, iters, leg):
    """The same row-sum invariant on a host copy (reported separately from the device check)."""
    s = v.astype(np.int64).sum(axis=1)
    return np.nonzero(s != iters)[0]


def timed_steps(step, steps, warmup, eng, L, dev, world, dist, ck, sp, coll_events=None):
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize; returns
    (max-over-ranks wall seconds, per-step search-kernel ms, per-step collective ms of
    this rank)."""
    import torch
    search_ms = []
    for _ in range(warmup):
        step()
    ck(L.dk_sync(eng.ctx, sp))
    if coll_events is not None:
        coll_events.clear()
    dist_on = dist.is_available() and dist.is_initialized()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
        search_ms.append(eng.last_search_ms())  # waits for this step's search kernel (HIP events on its stream)
    torch.cuda.synchronize(dev)
    ck(L.dk_sync(eng.ctx, sp))
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    coll_ms = sum(e0.elapsed_time(e1) for e0, e1 in coll_events) / steps if coll_events else 0.0
    return float(t.item()), search_ms, coll_ms


def per_rank(value, dev, world, dist):
    """Every rank's `value` (a float), gathered on all ranks."""
    import torch
    if world == 1 or not (dist.is_available() and dist.is_initialized()):
        return [value]
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [float(p.item()) for p in parts]


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d (launch one rank per GPU)" % (args.gpus, world))
    import torch
    import torch.distributed as dist

    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native

    # one GPU per rank; DK_DIST_BACKEND=gloo + more ranks than GPUs is the
    # rehearsal mode for the multi-GPU path on a one-GPU box (ranks share a device)
    backend = os.environ.get("DK_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > ndev:
        raise SystemExit("bench.py: --gpus %d needs %d GPUs, %d visible (DK_DIST_BACKEND=gloo shares devices)"
                         % (world, world, ndev))
    device = local_rank % max(1, ndev) if backend != "nccl" else local_rank
    torch.cuda.set_device(device)
    dist_on = world > 1 or (args.dist_one_rank and args.workload in ("c3", "c2d"))
    if dist_on:
        if world == 1:   # one-rank group outside torchrun (--dist-one-rank)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))   # RCCL over xGMI
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus
    dev = torch.device("cuda", device)
    local_rank = device
    L = _native.lib()
    # one explicit stream for torch's allocations/copies AND the library's launches
    # (handle 0 would mean the library's own non-blocking stream: no ordering with torch)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    assert sp != 0

    def ck(rc):
        if rc != 0:
            raise RuntimeError("doko_amd error %d: %s" % (rc, L.dk_status_string(rc).decode()))

    if args.workload == "c5":
        return run_c5(args, dk, L, dev, stream, rank, world, local_rank, dist)
    if args.workload == "c1":
        return run_c1(args, dk, L, dev, stream, rank, world, local_rank, dist)
    if args.workload == "prod":
        return run_prod(args, dk, L, dev, stream, rank, world, local_rank, dist)
    if args.workload in ("impi", "impid"):
        return run_impi(args, dk, L, dev, stream, rank, world, local_rank, dist)
    eng, step, n_roots, bufs = make_workload(args, dk, L, dev, sp, rank, world, local_rank, dist)
    determinized = args.workload in ("c3", "c2d")
    iters = args.iterations
    visits = bufs["visits"]
    I = bufs["I"]

    elapsed, search_ms, coll_ms = timed_steps(step, args.steps, args.warmup, eng, L, dev, world, dist, ck, sp,
                                              bufs["coll_events"])
    # per-wave clocks of the last timed search launch: how much of it the persistent grid's
    # drain tail costs (the waves that ran out of groups wait for the slowest one)
    waves = eng.last_search_waves()
    clocks = eng.last_search_clocks()
    if rank == 0 and args.dump_actions and bufs["actions"] is not None:
        np.save(args.dump_actions, bufs["actions"].cpu().numpy())
    if args.dump_acc and bufs["acc"] is not None:
        acc = bufs["acc"]
        if dist_on and args.partition == "infostates" and args.workload in ("c3", "c2d"):
            parts = [torch.zeros_like(acc) for _ in range(world)]
            dist.all_gather(parts, acc)
            acc = torch.cat(parts)
        if rank == 0:
            np.save(args.dump_acc, acc.cpu().numpy())
    check_visits(bufs, iters, "batch")
    host_bad = {}
    if args.host_readback_check:
        host_bad["batch"] = check_visits_host(visits.cpu().numpy(), iters, "batch").size
    sims_total = n_roots * iters * args.steps * world
    kernel_ms = float(np.mean(search_ms))
    # attribution of an N-GPU step: every rank's search kernel and collective time (HIP events)
    rank_kernel_ms = per_rank(kernel_ms, dev, world, dist)
    rank_coll_ms = per_rank(coll_ms, dev, world, dist)
    del bufs, visits

    # the survey's C3 decision batch (512 infostates x 64 samples = 32,768 roots): the regime a
    # DefaultImpiPolicy caller with one decision batch per game step sees (same engine, own buffers)
    small = None
    if args.workload == "c3" and args.small_infostates:
        import copy
        sa = copy.copy(args)
        sa.infostates = args.small_infostates
        _, sstep, s_roots, sbufs = make_workload(sa, dk, L, dev, sp, rank, world, local_rank, dist, eng=eng)
        s_el, s_ms, _ = timed_steps(sstep, args.small_steps, 1, eng, L, dev, world, dist, ck, sp)
        s_waves = eng.last_search_waves()
        check_visits(sbufs, iters, "small batch")
        if args.host_readback_check:
            host_bad["small"] = check_visits_host(sbufs["visits"].cpu().numpy(), iters, "small batch").size
        small = {"infostates_per_gpu": args.small_infostates, "roots_per_gpu": s_roots, "steps": args.small_steps,
                 "value": s_roots * iters * args.small_steps * world / s_el, "unit": "rollouts/s",
                 "ms_per_step": s_el / args.small_steps * 1e3, "search_kernel_ms": float(np.mean(s_ms)),
                 "search_waves_busy_frac": round(s_waves["busy_frac"], 4)}
        if args.inflight:
            small["inflight"] = inflight_rates(args, dk, eng, sbufs, dev, world, dist)
        del sbufs

    result = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, dk)
        b_sim = alg_bytes_per_sim(args.workload)
        achieved = n_roots * iters * b_sim / (kernel_ms / 1e3) / 1e9 if b_sim else None
        pmc_path = pmc_summary_path(args.workload)
        traffic = pmc_traffic(n_roots, iters, pmc_path)
        valu = pmc_valu(pmc_path)
        workload_desc = {
            "c3": "C3 rs-full-doko determinized UCT: %d infostates x %d CAP samples/GPU-share, %d roots x %d sims per GPU"
                  % (I, args.samples, n_roots, iters),
            "c2d": "C2 determinized: rs-doko, %d infostates x %d rule-based samples/GPU-share "
                   "(rs-doko-assignment), %d roots x %d sims per GPU" % (I, args.samples, n_roots, iters),
            "c2": "C2 rs-doko random-rollout UCT: %d roots x %d sims per GPU" % (n_roots, iters),
        }[args.workload]
        data = {"c3": "synthetic: seeded deals (SmallRng::seed_from_u64), 4x Healthy, k in {0,8,20,32} random plies; "
                      "determinized on the GPU by CAP",
                "c2d": "synthetic: seeded rs-doko deals, 4x Healthy, k in {0,8,20,32} random plies; determinized "
                       "on the GPU by the rs-doko-assignment sampler",
                "c2": "synthetic: seeded rs-doko deals (SmallRng::seed_from_u64(0xD0C00000+i)), 4x Healthy"}[args.workload]
        stream_peak = stream_copy_gbs(torch, dev)
        hw, cap, overflowed = eng.pool_high_water(sp)
        pools = {"bytes": eng.pool_bytes(), "slot_capacity": cap, "proven_slot_bound": 42 + 12 * iters,
                 "slot_high_water": hw, "overflowed_roots": overflowed}
        result = {
            "metric": METRIC,
            "value": sims_total / elapsed,
            "unit": "rollouts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64+f64",
            "data": data,
            "config": {
                "workload": workload_desc,
                "roots_per_gpu": n_roots,
                "iterations": iters,
                "uct_c": args.c,
                "fusion": args.fusion if determinized else None,
                "parallelism": ("dp%d (infostates split over GPUs, all samples of an infostate on one rank; RCCL "
                                "all-gather of the fused actions)" if args.partition == "infostates" else
                                "dp%d (samples split over GPUs, RCCL all-reduce of fusion accumulators)") % world,
            },
            "kernel_only_rollouts_per_s": n_roots * iters * world / (kernel_ms / 1e3),
            "search_kernel_ms": kernel_ms,
            "search_kernel_ms_per_rank": rank_kernel_ms,
            "collective_ms": max(rank_coll_ms),
            "collective_ms_per_rank": rank_coll_ms,
            "collective": (None if not (dist_on and determinized) else
                           "all_gather of the fused actions (%d B per rank)" % I if args.partition == "infostates" else
                           "all_reduce of the fusion accumulators (%d B)" % (I * 39 * 4)),
            "search_waves": {"waves": waves["waves"], "busy_frac": round(waves["busy_frac"], 4),
                             "first_end_ms": round(waves["first_end_ms"], 2),
                             "median_end_ms": round(waves["median_end_ms"], 2), "span_ms": round(waves["span_ms"], 2),
                             "sclk_mhz": round(clocks["sclk_mhz"], 1),
                             "sclk_range_mhz": [round(clocks["sclk_min_mhz"], 1), round(clocks["sclk_max_mhz"], 1)],
                             # the launch's SIMD-cycles per simulation: event time x shader clock x SIMDs / simulations
                             # (comparable across boxes whose clocks differ)
                             "cycles_per_simulation": round(kernel_ms * 1e-3 * clocks["sclk_mhz"] * 1e6 * simds(dev)
                                                            / (n_roots * iters), 1),
                             "note": "each wave of the persistent grid stamps the 100 MHz counter and the shader clock "
                                     "(s_memtime) at start and once the group queue is dry for it; 1 - busy_frac = "
                                     "drain tail + launch ramp; sclk_mhz = shader cycles / real time over the waves; "
                                     "cycles_per_simulation = search_kernel_ms x sclk x SIMDs / simulations"},
            "roofline": {
                # bound: what binds the launch, measured (round-4 review): latency of the per-lane tree
                # walks -- neither VALU nor DRAM is saturated (valu below).  achieved/peak/frac stay the
                # north-star's HBM figures (algorithmic bytes / event-timed kernel vs 8 TB/s, the
                # resource it is priced against); traffic: calibrated DRAM bytes per launch (PMC)
                "bound": "latency",
                "priced_against": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS if achieved else None,
                "hbm_target_0p40_met": (achieved / HBM_PEAK_GBS >= 0.40) if achieved else None,
                "traffic": traffic,
                "alg_bytes_per_sim": b_sim,
                "stream_copy_peak_measured_gbs": stream_peak,
                "valu": valu,
                "limiter": "latency of the per-lane tree walks: VALU %s busy (measured), DRAM %s of the measured "
                           "random-line read peak, %s of wave cycles waiting on memory" % (
                               "%.0f%%" % (100 * valu["busy"]) if valu else "n/a",
                               "%.0f%%" % (100 * valu["dram_frac_of_random_line_peak"])
                               if valu and valu.get("dram_frac_of_random_line_peak") else "n/a",
                               "%.0f%%" % (100 * valu["mem_wait_frac"]) if valu else "n/a"),
                "note": "achieved = the SURVEY 8(d) algorithmic bytes (oracle counters, profiles/alg_bytes_<w>.json) / "
                        "event-timed search kernel; traffic = calibrated DRAM bytes per launch (128 B per read "
                        "request of the 128-B kind, WRITE_SIZE for writes: profiles/r04/pmc_calib.json) from "
                        "profiles/pmc_search.json, scaled to this launch",
            },
            "node_pools": pools,
            "small_batch": small,
            "host_copy_bad_roots": host_bad or None,
            "ranks": world,
            "dist_backend": backend if dist_on else None,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result))
    if dist_on:
        dist.destroy_process_group()
    eng.close()
    return result


AZ_FLOP_PER_EVAL = None


def az_flop_per_eval(d=160, seq=62, blocks=6, classes=43):
    """Algorithmic FLOPs of one DokoAzNet evaluation (multiply-add = 2): per block the
    projections 2*S*d*d*(3+1+1+4+4) and attention 4*S*S*d; the class heads 4*C*S*d + 2*C*d*d + 2*C*d."""
    return blocks * (26 * seq * d * d + 4 * seq * seq * d) + 4 * classes * seq * d + 2 * classes * d * d + 2 * classes * d


def net_precision(args, torch):
    """(torch dtype, dtype label, matrix peak TFLOP/s, note) of the network precision."""
    if args.net_precision == "f32":
        # the reference's settings (az_doko.py:539-541, main.py:402/508)
        torch.set_float32_matmul_precision("medium")
        torch.backends.cuda.matmul.allow_tf32 = True
        return (torch.float32, "f32 network (reference precision: f32 activations, matmul precision 'medium')", 2500.0 / 3,
                "f32 activations; GEMM products from bf16 pieces (bf16x3: three MFMAs per k-step, ~16-bit "
                "products, as hipBLASLt's 'medium' f32 GEMMs measured, profiles/r04/fp32_gemm_probe.json): at d = 160 "
                "and d = 256 every block as two HIP kernels (qkv_attn_ln_f32x3_kernel, mlp_ln_f32x3_kernel / "
                "mlp16_ln_f32x3_kernel; at d = 256 each half normalises the residual stream itself, x-only chain) and "
                "the heads as two (class_pool_ln_f32x3_kernel, class_mlp_f32x3_kernel), no hipBLASLt: peak = bf16 "
                "dense / 3")
    return (torch.bfloat16, "bf16 network (narrower than the reference's f32; opt-in --net-precision bf16)", 2500.0,
            "bf16 dense peak")


def run_c5(args, dk, L, dev, stream, rank, world, local_rank, dist):
    """Config 5: AlphaZero self-play.  One step = one move decision of every concurrent
    game: root evaluation, `az_iterations` x (PUCT select on the GPU -> encode_state_pi on
    the GPU -> DokoAzNet in bf16 -> backup), the temperature pick, the move
    (take_action with skip_single), and fresh deals for finished games.  Run parameters
    of the reference (az_doko.py:579-614): 8192 concurrent games, 200 iterations,
    Dirichlet alpha 0.8 / epsilon 0.3, c_puct 4.0, temperature 0.5.  Games are
    independent, so N GPUs run N replicas (weak scaling, no collective)."""
    import torch
    from master_doko_reinforcement_learning_amd.az_network import AzEvaluator, DokoAzNet
    rep = rank + args.replica_offset           # the replica's seeds and weights (--replica-offset)
    torch.manual_seed(1234 + rep)
    G, iters = args.games, args.az_iterations
    eng = dk.Engine(device=local_rank, max_roots=64, max_iterations=max(1, iters))
    sp = stream.cuda_stream

    def ck(rc):
        if rc != 0:
            raise RuntimeError("doko_amd error %d: %s" % (rc, L.dk_status_string(rc).decode()))

    seeds = np.arange(G, dtype=np.uint64) + np.uint64(0xA2000000 + rep * G)
    st = torch.zeros((G, 128), dtype=torch.uint8, device=dev)
    ck(L.dk_new_game_batch_async(eng.ctx, dk.GAME_FULL_DOKO, torch.tensor(seeds.view(np.int64), device=dev).data_ptr(),
                                 G, st.data_ptr(), sp))
    records = dk.az_records(eng, st)
    net = DokoAzNet().to(dev)
    ev_time = [0.0]

    class TimedEval(AzEvaluator):
        def __call__(self, recs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = super().__call__(recs)
            e1.record()
            ev_time.append((e0, e1))
            return out

    ndt, nlabel, npeak, nnote = net_precision(args, torch)
    evaluator = TimedEval(eng, net, dtype=ndt)
    search = dk.AlphaZeroSearch(eng, 4.0, 0.3, 10, 0.5, dirichlet_alpha=0.8)
    next_seed = [int(seeds[-1]) + 1]
    moves = [0, 0]
    # one SmallRng per game slot, carried across its searches (the reference's `rng: &mut SmallRng`);
    # each search draws its root's Dirichlet([0.8; 39]) noise from it (async_mcts.rs:111-113)
    rng_states = torch.from_numpy(dk.splitmix_rng_states(np.asarray(seeds, dtype=np.uint64) ^ np.uint64(0xA2))
                                  .view(np.int64).copy()).to(dev)

    from master_doko_reinforcement_learning_amd.api import AZ_STATE_BYTES
    H = max(1, args.c5_streams)
    if G % H:
        raise SystemExit("--games must be divisible by --c5-streams")
    parts = None
    if H > 1:
        # H independent searches over G/H games each: own engine (search state), own stream, own
        # evaluator (token buffer); the network weights are shared.  Games are independent and the
        # network is row-wise, so every game's search is the one-batch search (checked by the tests).
        parts = [(dk.Engine(device=local_rank, max_roots=64, max_iterations=max(1, iters)), torch.cuda.Stream(dev))
                 for _ in range(H)]
        part_evals = [TimedEval(e, net, dtype=ndt) for e, _ in parts]

    def search_parts(srch):
        """api.AlphaZeroSearch._search for the H parts, their launches interleaved per iteration."""
        Gh = G // H
        main = torch.cuda.current_stream(dev)
        st = []
        for h, (e, s) in enumerate(parts):
            s.wait_stream(main)
            sl = slice(h * Gh, (h + 1) * Gh)
            with torch.cuda.stream(s):
                seeds_t = torch.tensor(np.ascontiguousarray(srch[sl]).view(np.int64), device=dev)
                ev = torch.empty((Gh, AZ_STATE_BYTES), dtype=torch.uint8, device=dev)
                need = torch.empty(Gh, dtype=torch.uint8, device=dev)
                rs = rng_states[sl]
                ck(L.dk_az_begin_async(e.ctx, records[sl].data_ptr(), seeds_t.data_ptr(), Gh, iters, search.epoch,
                                       ev.data_ptr(), s.cuda_stream))
                ck(L.dk_az_rng_async(e.ctx, rs.data_ptr(), 1, s.cuda_stream))
                v, lg = part_evals[h](ev)
                v, lg = v.float().contiguous(), lg.float().contiguous()
                ck(L.dk_az_root_async(e.ctx, v.data_ptr(), lg.data_ptr(), None, search.alpha, search.eps, s.cuda_stream))
            st.append((e, s, ev, need, rs, seeds_t))
        for _ in range(iters):
            for h, (e, s, ev, need, rs, _) in enumerate(st):
                with torch.cuda.stream(s):
                    ck(L.dk_az_select_async(e.ctx, search.c, ev.data_ptr(), need.data_ptr(), s.cuda_stream))
                    v, lg = part_evals[h](ev)
                    v, lg = v.float().contiguous(), lg.float().contiguous()
                    ck(L.dk_az_backup_async(e.ctx, v.data_ptr(), lg.data_ptr(), s.cuda_stream))
        actions = torch.empty(G, dtype=torch.uint8, device=dev)
        visits = torch.empty((G, dk.NUM_ACTIONS), dtype=torch.int32, device=dev)
        for h, (e, s, ev, need, rs, _) in enumerate(st):
            with torch.cuda.stream(s):
                ck(L.dk_az_finish_async(e.ctx, 2, float(search.temperature), visits[h * Gh:(h + 1) * Gh].data_ptr(),
                                        actions[h * Gh:(h + 1) * Gh].data_ptr(), s.cuda_stream))
                ck(L.dk_az_rng_async(e.ctx, rs.data_ptr(), 0, s.cuda_stream))
            main.wait_stream(s)
        for e, s, *_ in st:
            ck(L.dk_sync(e.ctx, s.cuda_stream))
        return actions

    def step():
        srch = np.arange(G, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(next_seed[0])
        if parts is None:
            actions, _ = search.mcts_search(records, evaluator, None, iters, srch, rng_states=rng_states)
        else:
            actions = search_parts(srch)
        dk.az_step(eng, records, actions)
        fin = (records[:, 99] == 3).nonzero().flatten()      # phase byte: Finished -> a fresh deal
        moves[0] += int((actions != 255).sum().item())
        if fin.numel():
            k = fin.numel()
            fs = torch.tensor((np.arange(k, dtype=np.uint64) + np.uint64(next_seed[0])).view(np.int64), device=dev)
            next_seed[0] += k
            fresh = torch.zeros((k, 128), dtype=torch.uint8, device=dev)
            ck(L.dk_new_game_batch_async(eng.ctx, dk.GAME_FULL_DOKO, fs.data_ptr(), k, fresh.data_ptr(), sp))
            records[fin] = dk.az_records(eng, fresh)
            moves[1] += k

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ev_time[:] = [0.0]
    moves[:] = [0, 0]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    net_ms = sum(e0.elapsed_time(e1) for e0, e1 in ev_time[1:])
    if parts is not None:
        # the parts' network calls overlap each other: their event times do not add up to the
        # network's share of the step, so the whole step is charged to the network (an upper bound)
        net_ms = elapsed * 1e3
        for e, _ in parts:
            e.close()
    if args.dump_records:
        np.save("%s_r%d.npy" % (args.dump_records, rep), records.cpu().numpy())
    evals = G * (iters + 1) * args.steps
    flop = az_flop_per_eval()
    result = None
    if rank == 0:
        cpu = cpu_baseline_net(args, "c5") if world == 1 and not args.no_cpu_baseline else None
        achieved = flop * evals / (net_ms / 1e3) / 1e12
        result = {
            "metric": "AlphaZero self-play PUCT simulations/sec (one policy/value network leaf evaluation each)",
            "value": G * iters * args.steps * world / elapsed,
            "unit": "simulations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": nlabel + ", f32 tree statistics",
            "data": "synthetic: seeded full-doko deals, random-initialised DokoAzNet (d 160, 6 blocks); root "
                    "Dirichlet noise drawn on the device from each game's SmallRng (rand_distr 0.5.1)",
            "config": {"workload": "C5 AlphaZero self-play: %d concurrent games x %d PUCT iterations per move per GPU"
                                   % (G, iters),
                       "c_puct": 4.0, "dirichlet": [0.8, 0.3], "temperature": 0.5,
                       "moves_per_step": G, "games_finished": moves[1], "parallelism": "replicas x%d" % world},
            "network_ms_per_step": net_ms / args.steps,
            "search_ms_per_step": elapsed / args.steps * 1e3 - net_ms / args.steps if parts is None else None,
            "c5_streams": H,
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": npeak, "unit": "TFLOP/s",
                         "frac": achieved / npeak, "traffic": None,
                         "note": "network GEMMs/attention: %.1f MFLOP per leaf evaluation (algorithmic), %s; achieved "
                                 "over the network's event-timed share of the step" % (flop / 1e6, nnote)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()
    eng.close()
    return result


def _finish_dist(world, dist, t_elapsed, dev):
    """Max-over-ranks wall time (the driver's contract) for the replica workloads."""
    import torch
    t = torch.tensor([t_elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def run_c1(args, dk, L, dev, stream, rank, world, local_rank, dist):
    """Config 1: tic-tac-toe with rs-doko-mcts plain UCT (c = 2.0).  Two legs:
      * serial: tic_tac_toe_player (tic_tac_toe_player.rs:8-52) -- ONE seed_from_u64(999) stream
        threaded through every search of every game (dk_search_batch_rng, one root per launch), so
        the games are strictly sequential; timed on the GPU and on the oracle (one CPU thread,
        the reference's configuration) over the same --c1-serial-games games;
      * lockstep (`value`): --c1-games independent games, game g on its own stream
        seed_from_u64(999 + g), one search launch per move over every unfinished game.
    A step = one lockstep pass (all games played to the end)."""
    import torch
    iters = args.iterations if args.iterations != 1000 else 1400          # tic_tac_toe_player.rs:18
    G = args.c1_games
    eng = dk.Engine(device=local_rank, max_roots=max(G, 64), max_iterations=iters)
    seeds = np.arange(G, dtype=np.uint64) + np.uint64(999 + rank * G)
    for _ in range(args.warmup):
        dk.tic_tac_toe_games(eng, seeds, iters, 2.0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    searches, fin = 0, None
    for _ in range(args.steps):
        fin, moves, n = dk.tic_tac_toe_games(eng, seeds, iters, 2.0)
        searches += n
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = _finish_dist(world, dist, time.perf_counter() - t0, dev)
    # serial leg: the reference's one-stream player
    gs = args.c1_serial_games
    dk.tic_tac_toe_player(eng, 1, iters, 2.0)                              # warm-up game
    trace = []
    t1 = time.perf_counter()
    res_serial = dk.tic_tac_toe_player(eng, gs, iters, 2.0, trace=trace)
    serial_s = time.perf_counter() - t1
    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import ctypes

            import oracle_lib as ol
            rng = ol.rng_seed(999)
            t2 = time.perf_counter()
            ms, same = 0, True
            for g in range(gs):
                b = [0] * 9
                while ol.lib().or_ttt_finish(ol.arr(ctypes.c_int32, 9, b)) == 0:
                    best, _, _ = ol.ttt_search(b, rng, iters, 2.0)
                    if ms < len(trace):
                        same &= trace[ms][3] == best and [int(w) for w in trace[ms][4]] == [int(rng[k]) for k in range(4)]
                    b[best] = 1 if b.count(1) == b.count(2) else 2
                    ms += 1
            cpu_s = time.perf_counter() - t2
            cpu = {"value": ms * iters / cpu_s, "unit": "rollouts/s", "cores": 1, "kind": "port",
                   "sample": "the same %d one-stream games (%d searches x %d sims), oracle C++ restatement on one "
                             "thread (the reference's configuration)" % (gs, ms, iters),
                   "ms_per_search": cpu_s / ms * 1e3, "moves_equal_gpu": bool(same and ms == len(trace))}
        fin = np.asarray(fin)
        result = {
            "metric": "tic-tac-toe UCT simulations/sec (rs-doko-mcts plain UCT, %d sims/move, c = 2.0)" % iters,
            "value": searches * iters * world / elapsed,
            "unit": "rollouts/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u64+f64",
            "data": "tic-tac-toe from the empty board; game g's stream SmallRng::seed_from_u64(999 + g)",
            "config": {"workload": "C1 tic-tac-toe: %d independent games in lockstep per GPU, one search launch per "
                                   "move over the unfinished games, %d sims per search" % (G, iters),
                       "searches_per_step": searches // args.steps,
                       "results_x_o_draw": [int((fin == 1).sum()), int((fin == 2).sum()), int((fin == 3).sum())],
                       "parallelism": "replicas x%d" % world},
            "serial_one_stream": {
                "games": gs, "searches": len(trace), "results_x_o_draw": res_serial,
                "ms_per_search": serial_s / max(1, len(trace)) * 1e3,
                "rollouts_per_s": len(trace) * iters / serial_s,
                "note": "tic_tac_toe_player as the reference runs it: each search continues the previous one's "
                        "stream, so one root per launch, two host round trips per move (search, step)"},
            "roofline": None,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()
    eng.close()
    return result


def run_prod(args, dk, L, dev, stream, rank, world, local_rank, dist):
    """The thesis's production search shape: DefaultImpiPolicy with S CAP samples of
    200,000 UCT iterations each (compare_impi/run.rs:270-291; S in {5, 10, 50}).  Per S:
      * latency: ONE decision (S roots, determinize -> search -> fuse -> select) on the GPU;
      * in flight: --prod-inflight decisions batched into one pass (execute_many), the regime of
        the evaluator's 2 x available_parallelism concurrent games (run.rs:775);
      * cpu: the oracle on S threads, one sample per thread (the reference runs the samples of a
        decision as tokio tasks on MCTSWorkers threads), on the same roots.
    Each root's 200,000 simulations are sequential (the reference's semantics), so a decision's
    latency is one lane's sequential speed: the GPU loses on latency and wins on throughput."""
    import torch
    iters = args.prod_iterations
    Ss = [int(x) for x in args.prod_samples.split(",") if x]
    K = args.prod_inflight
    max_roots = max(Ss) * K
    # pools: 32-B records (iterations > 4095); 4 slots per iteration cover the measured demand
    eng = dk.Engine(device=local_rank, max_roots=max_roots, max_iterations=iters, slot_capacity=64 + 4 * iters)
    sp = stream.cuda_stream

    def ck(rc):
        if rc != 0:
            raise RuntimeError("doko_amd error %d: %s" % (rc, L.dk_status_string(rc).decode()))

    # K infostates: C3-style seeded deals, 4x Healthy, k in {0,8,20,32} random plies
    info_seeds = torch.tensor((np.arange(K, dtype=np.uint64) + np.uint64(0xC3000000)).view(np.int64), device=dev)
    info = torch.zeros((K, 128), dtype=torch.uint8, device=dev)
    ck(L.dk_new_game_batch_async(eng.ctx, dk.GAME_FULL_DOKO, info_seeds.data_ptr(), K, info.data_ptr(), sp))
    a = torch.full((K,), 1 << 24, dtype=torch.int64, device=dev)
    for _ in range(4):
        ck(L.dk_env_step_batch_async(eng.ctx, info.data_ptr(), a.data_ptr(), K, sp))
    plies = torch.tensor(np.array([[0, 8, 20, 32][j % 4] for j in range(K)], dtype=np.uint32).view(np.int32), device=dev)
    ply_rng = torch.tensor(dk.splitmix_rng_states(np.arange(K, dtype=np.uint64) + np.uint64(0xC3100000)).view(np.int64),
                           device=dev)
    ck(L.dk_env_random_plies_batch_async(eng.ctx, info.data_ptr(), ply_rng.data_ptr(), plies.data_ptr(), K, sp))
    ck(L.dk_sync(eng.ctx, sp))
    legs, v1_rows = [], {}
    for S in Ss:
        pol = dk.DefaultImpiPolicy(eng, args.c, iters, S, dk.FUSE_MAXN)

        def seeds_for(j):
            return torch.tensor(seeds_for_prod(j, S).view(np.int64), device=dev)

        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        act1, v1 = pol.execute_many([(info[:1], seeds_for(0))], game=dk.GAME_FULL_DOKO)[0]
        torch.cuda.synchronize(dev)
        lat = time.perf_counter() - t0
        k1 = eng.last_search_ms()
        v1_rows[S] = v1.cpu().numpy()
        batches = [(info[j:j + 1], seeds_for(j)) for j in range(K)]
        t0 = time.perf_counter()
        res = pol.execute_many(batches, game=dk.GAME_FULL_DOKO)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        kK = eng.last_search_ms()
        assert np.array_equal(res[0][1].cpu().numpy(), v1.cpu().numpy()), "prod: batched decision 0 differs"
        for _, v in res:
            assert bool((v.sum(dim=1) == iters).all().item()), "prod: a root without exactly %d simulations" % iters
        leg = {"samples": S, "decision_latency_s": lat, "search_kernel_ms_one": k1,
               "inflight_decisions": K, "inflight_s": el, "search_kernel_ms_inflight": kK,
               "inflight_decisions_per_s": K / el, "inflight_rollouts_per_s": K * S * iters / el,
               "one_decision_rollouts_per_s": S * iters / lat}
        legs.append(leg)
    hw, cap, overflowed = eng.pool_high_water(sp)
    pool_small = eng.pool_bytes()
    inflight_visits0 = res[0][1].cpu().numpy()   # decision 0 of the last S's in-flight leg
    eng.close()
    capleg = None
    if args.prod_capacity != 0:
        capleg = prod_capacity_leg(args, dk, L, dev, sp, Ss[-1], iters, local_rank, inflight_visits0, seeds_for_prod)
    result = None
    if rank == 0:
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import ctypes

            import oracle_lib as ol
            st = ol.FdoState.new_game(0xC3000000)
            for _ in range(4):
                st.play(24)
            rng = ol.arr(ctypes.c_uint64, 4, [int(x) for x in dk.splitmix_rng_states(np.array([0xC3100000], dtype=np.uint64))[0]])
            st.random_plies(rng, 0, True)
            for leg in legs:
                S = leg["samples"]
                roots = [st.card_matching(ol.rng_seed(0xC3200000 + s)) for s in range(S)]
                handles = (ctypes.c_void_p * S)(*[r.h for r in roots])
                vis = (ctypes.c_uint32 * (39 * S))()
                sd = ol.arr(ctypes.c_uint64, S, [0xC3200000 + 2048 + s for s in range(S)])
                cores, quota = cpu_quota_cores()
                thr = min(S, int(np.ceil(quota)) if quota else cores)
                secs = ol.lib().or_fdo_search_many(None, handles, sd, S, iters, args.c, vis, thr)
                same = all(list(vis[39 * s:39 * s + 39]) == [int(x) for x in v1_rows[S][s]] for s in range(S)) \
                    if S in v1_rows else None
                leg["cpu"] = {"decision_latency_s": secs, "threads": thr, "kind": "port",
                              "rollouts_per_s": S * iters / secs, "visits_equal_gpu": same}
                leg["gpu_over_cpu_latency"] = leg["decision_latency_s"] / secs
            if capleg is not None:
                capleg["oracle_check"] = prod_oracle_check(args, dk, iters, Ss[-1], capleg.pop("_check_rows"))
        if capleg is not None:
            capleg.pop("_check_rows", None)
        top = capleg if capleg is not None else {"rollouts_per_s": legs[-1]["inflight_rollouts_per_s"],
                                                 "s": legs[-1]["inflight_s"]}
        result = {
            "metric": "determinized decision latency and throughput at the production search shape "
                      "(S CAP samples x %d UCT iterations, MaxN)" % iters,
            "value": top["rollouts_per_s"],
            "unit": "rollouts/s",
            "n_gpus": world, "steps": 1, "warmup": 0,
            "ms_per_step": top["s"] * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64+f64",
            "data": "synthetic: C3-style seeded deals (4x Healthy, k in {0,8,20,32} random plies), CAP samples",
            "config": {"workload": "prod: S in %s samples x %d iterations; one decision, %d decisions in flight "
                                   "(execute_many), and %s decisions of %d samples at the pools' capacity"
                                   % (Ss, iters, K, capleg["decisions"] if capleg else 0, Ss[-1]),
                       "parallelism": "replicas x%d" % world},
            "legs": legs,
            "capacity": capleg,
            "node_pools": {"bytes": pool_small, "slot_capacity": cap, "slot_high_water": hw,
                           "overflowed_roots": overflowed},
            "roofline": None,
            "note": "a root's simulations are sequential (bit-exact reference semantics), so one decision's "
                    "latency is one GPU lane's sequential speed; throughput comes from decisions in flight",
        }
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()
    return result


def seeds_for_prod(j, S):
    """Sampler and search seeds of prod decision j (S samples): [S sampler seeds | S search seeds]."""
    base = np.uint64(0xC3200000 + j * 4096)
    return np.concatenate([np.arange(S, dtype=np.uint64) + base, np.arange(S, dtype=np.uint64) + base + np.uint64(2048)])


def prod_infostates(dk, L, eng, dev, sp, K):
    """K C3-style infostates: seeded deals, 4x Healthy, k in {0, 8, 20, 32} random plies (round robin)."""
    import torch
    info_seeds = torch.tensor((np.arange(K, dtype=np.uint64) + np.uint64(0xC3000000)).view(np.int64), device=dev)
    info = torch.zeros((K, 128), dtype=torch.uint8, device=dev)
    assert L.dk_new_game_batch_async(eng.ctx, dk.GAME_FULL_DOKO, info_seeds.data_ptr(), K, info.data_ptr(), sp) == 0
    a = torch.full((K,), 1 << 24, dtype=torch.int64, device=dev)
    for _ in range(4):
        assert L.dk_env_step_batch_async(eng.ctx, info.data_ptr(), a.data_ptr(), K, sp) == 0
    plies = torch.tensor(np.array([[0, 8, 20, 32][j % 4] for j in range(K)], dtype=np.uint32).view(np.int32), device=dev)
    ply_rng = torch.tensor(dk.splitmix_rng_states(np.arange(K, dtype=np.uint64) + np.uint64(0xC3100000)).view(np.int64),
                           device=dev)
    assert L.dk_env_random_plies_batch_async(eng.ctx, info.data_ptr(), ply_rng.data_ptr(), plies.data_ptr(), K, sp) == 0
    assert L.dk_sync(eng.ctx, sp) == 0
    return info


def prod_capacity_leg(args, dk, L, dev, sp, S, iters, local_rank, visits0, seeds_for):
    """As many decisions of S samples x `iters` iterations in flight as the device memory holds, in
    one pass (DefaultImpiPolicy.execute_many): the evaluator's regime (2 x available_parallelism
    concurrent games, run.rs:775) at this GPU's capacity.  Per root: the slots (16-B hot + 16-B cold
    records, --prod-slots-per-iter x iterations), the 64-B node states and the path overflow."""
    import torch
    slots = int(64 + args.prod_slots_per_iter * iters + 255) // 256 * 256
    per_root = slots * 32 + (iters + 1) * 64 + 512 * 12
    torch.cuda.empty_cache()
    free_b, _ = torch.cuda.mem_get_info(dev)
    reserve = (12 << 30) + (6 << 30)          # the fallback pool (<= 16 GB of 32-B records; ~11.5 GB here) + headroom
    K = args.prod_capacity
    if K < 0:
        K = max(1, int((free_b - reserve) * 0.95 // (per_root * S)))
    eng = dk.Engine(device=local_rank, max_roots=K * S, max_iterations=iters, slot_capacity=slots)
    try:
        info = prod_infostates(dk, L, eng, dev, sp, K)
        pol = dk.DefaultImpiPolicy(eng, args.c, iters, S, dk.FUSE_MAXN)
        batches = [(info[j:j + 1], torch.tensor(seeds_for(j, S).view(np.int64), device=dev)) for j in range(K)]
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        res = pol.execute_many(batches, game=dk.GAME_FULL_DOKO)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        kms = eng.last_search_ms()
        vis = torch.cat([v for _, v in res]).cpu().numpy()
        assert np.all(vis.sum(axis=1) == iters), "prod capacity: a root without exactly %d simulations" % iters
        # decision 0 equals its in-flight-leg result (a different batch, engine and pool placement)
        assert np.array_equal(vis[:S], visits0), "prod capacity: decision 0 differs from the 16-decision leg"
        hw, cap, overflowed = eng.pool_high_water(sp)
        last = K - 1
        rows = {"decisions": [last], "samples": list(range(min(S, 8))),
                "visits": {last: vis[last * S:last * S + min(S, 8)].tolist()}}
        return {"samples": S, "decisions": K, "roots": K * S, "s": el, "search_kernel_ms": kms,
                "decisions_per_s": K / el, "rollouts_per_s": K * S * iters / el,
                "pool_bytes": eng.pool_bytes(), "pool_bytes_per_root": eng.pool_bytes() / (K * S),
                "slot_capacity": cap, "slot_high_water": hw, "overflowed_roots": overflowed,
                "actions_of_decision_0_equal_inflight_leg": True, "_check_rows": rows}
    finally:
        eng.close()


def prod_oracle_check(args, dk, iters, S, rows):
    """The oracle (CPU restatement) on roots of the capacity leg's last decision: visits equal."""
    import ctypes
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as ol
    out = []
    for j in rows["decisions"]:
        st = ol.FdoState.new_game(0xC3000000 + j)
        for _ in range(4):
            st.play(24)
        rng = ol.arr(ctypes.c_uint64, 4, [int(x) for x in dk.splitmix_rng_states(np.array([0xC3100000 + j], dtype=np.uint64))[0]])
        st.random_plies(rng, [0, 8, 20, 32][j % 4], True)
        sd = seeds_for_prod(j, S)
        ks = rows["samples"]
        roots = [st.card_matching(ol.rng_seed(int(sd[k]))) for k in ks]
        handles = (ctypes.c_void_p * len(ks))(*[r.h for r in roots])
        vis = (ctypes.c_uint32 * (39 * len(ks)))()
        seeds = ol.arr(ctypes.c_uint64, len(ks), [int(sd[S + k]) for k in ks])
        cores, quota = cpu_quota_cores()
        thr = min(len(ks), int(np.ceil(quota)) if quota else cores)
        secs = ol.lib().or_fdo_search_many(None, handles, seeds, len(ks), iters, args.c, vis, thr)
        same = all(list(vis[39 * i:39 * i + 39]) == [int(x) for x in rows["visits"][j][i]] for i in range(len(ks)))
        out.append({"decision": j, "roots": len(ks), "visits_equal_gpu": same, "oracle_s": secs})
        assert same, "prod capacity: oracle visits differ on decision %d" % j
    return out


def impi_flop_per_eval(d=256, seq=62, blocks=4, classes=33):
    """Algorithmic FLOPs of one DokoImpiNet evaluation (create_ar.py:12-18 configuration)."""
    return az_flop_per_eval(d=d, seq=seq, blocks=blocks, classes=classes)


def run_impi(args, dk, L, dev, stream, rank, world, local_rank, dist):
    """§8(f) row 4: the ARSampling SamplingFn (compare_impi.rs:84-105), i.e.
    forward_pred_process_with_mask (rs-doko-impi/src/forward.rs:392-661), for
    `ar_samples` draws of each of the C3 infostates (12288 per GPU, 4 x Healthy then
    k in {0, 8, 20, 32} random plies).  One step = every card and hidden reservation
    of every sample guessed by the IMPI network (DokoImpiNet, d 256, 4 blocks, bf16),
    one batched network call per round, temperature 0.4 (all_policies.rs:30), then the
    consistency check.  Infostates are independent: N GPUs run N replicas.
    impid: the whole mcts_ar_maxn_policy decision (all_policies.rs:78-101) per step: the AR
    samples, then UCT (`iterations`, c) on each sample, MaxN fusion over the consistent ones
    and the random fallback (ArImpiPolicy)."""
    import torch
    from master_doko_reinforcement_learning_amd.impi_network import DokoImpiNet
    torch.manual_seed(4321 + rank)
    I, S = args.infostates, args.ar_samples
    decide = args.workload == "impid"
    eng = dk.Engine(device=local_rank, max_roots=I * S if decide else 64, max_iterations=args.iterations if decide else 1)
    sp = stream.cuda_stream

    def ck(rc):
        if rc != 0:
            raise RuntimeError("doko_amd error %d: %s" % (rc, L.dk_status_string(rc).decode()))

    info_seeds = torch.tensor((np.arange(I, dtype=np.uint64) + np.uint64(0xC3000000 + rank * I)).view(np.int64), device=dev)
    info = torch.zeros((I, 128), dtype=torch.uint8, device=dev)
    ck(L.dk_new_game_batch_async(eng.ctx, dk.GAME_FULL_DOKO, info_seeds.data_ptr(), I, info.data_ptr(), sp))
    a = torch.full((I,), 1 << 24, dtype=torch.int64, device=dev)
    for _ in range(4):
        ck(L.dk_env_step_batch_async(eng.ctx, info.data_ptr(), a.data_ptr(), I, sp))
    plies = torch.tensor(np.array([[0, 8, 20, 32][j % 4] for j in range(I)], dtype=np.uint32).view(np.int32), device=dev)
    ply_rng = torch.tensor(dk.splitmix_rng_states(np.arange(I, dtype=np.uint64) + np.uint64(0xC3100000 + rank * I)).view(np.int64),
                           device=dev)
    ck(L.dk_env_random_plies_batch_async(eng.ctx, info.data_ptr(), ply_rng.data_ptr(), plies.data_ptr(), I, sp))
    records = dk.az_records(eng, info)
    ndt, nlabel, npeak, nnote = net_precision(args, torch)
    net = DokoImpiNet().to(dev).eval().to(ndt)
    ev = []

    def network(tokens):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = net(tokens)
        e1.record()
        ev.append((e0, e1))
        return out

    ar = dk.ARSampling(eng, network, args.ar_temperature)
    seeds = np.arange(I * S, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(0xA5000000 + rank)
    P = max(1, args.impi_streams) if not decide else 1   # (impid: the policy splits its sampling itself)
    if I % P:
        raise SystemExit("--infostates must be divisible by --impi-streams")
    parts = None
    if P > 1:
        # P independent samplings over I/P infostates each (own engine: the AR state; own stream);
        # every lane's sample equals the one-batch sampling (tests/test_gpu_impi.py)
        Ip = I // P
        parts = [(dk.ARSampling(dk.Engine(device=local_rank, max_roots=64, max_iterations=1), network, args.ar_temperature),
                  torch.cuda.Stream(dev), records[k * Ip:(k + 1) * Ip], S, seeds[k * Ip * S:(k + 1) * Ip * S])
                 for k in range(P)]
    policy = dk.ArImpiPolicy(eng, network, args.c, args.iterations, S, dk.FUSE_MAXN, args.ar_temperature,
                             sampler_streams=max(1, args.impi_streams)) if decide else None
    pol_seeds = np.arange(2 * I * S + I, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(0xA6000000 + rank)
    stats = {"rows": 0, "consistent": 0, "lanes": 0}

    def step():
        with torch.inference_mode():
            if decide:
                _, succ, _ = policy.execute(records, pol_seeds)
                stats["rows"] += policy.sampler.rows
                stats["consistent"] += int(succ.sum().item())
            elif parts is None:
                _, status, _ = ar.sample(records, S, seeds)
                stats["rows"] += ar.rows
                stats["consistent"] += int((status == 0).sum().item())
            else:
                outs = dk.sample_interleaved(parts)
                stats["rows"] += sum(p[0].rows for p in parts)
                stats["consistent"] += sum(int((o[1] == 0).sum().item()) for o in outs)
        stats["lanes"] += I * S

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ev.clear()
    stats.update(rows=0, consistent=0, lanes=0)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    net_ms = sum(e0.elapsed_time(e1) for e0, e1 in ev)
    if parts is not None:
        # the parts' network calls overlap: the whole step is charged to the network (an upper bound)
        net_ms = elapsed * 1e3
        for p in parts:
            p[0].engine.close()
    flop = impi_flop_per_eval()
    result = None
    if rank == 0:
        cpu = cpu_baseline_net(args, "impi") if world == 1 and not decide and not args.no_cpu_baseline else None
        achieved = flop * stats["rows"] / (net_ms / 1e3) / 1e12
        result = {
            "metric": ("AR-determinized decisions/sec (mcts_ar_maxn_policy: %d AR samples x %d UCT simulations each)"
                       % (S, args.iterations)) if decide else
                      "IMPI autoregressive determinizations/sec (forward_pred_process_with_mask, one network call per guessed card)",
            "value": (I if decide else I * S) * args.steps * world / elapsed,
            "unit": "decisions/s" if decide else "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": nlabel + ", f32 softmax / weighted draw" + (", u64+f64 search" if decide else ""),
            "data": "synthetic: the C3 infostates (seeded deals, 4x Healthy, k in {0,8,20,32} random plies), "
                    "random-initialised DokoImpiNet (d 256, 4 blocks, 4 heads)",
            "config": {"workload": ("IMPI AR decision: %d infostates x %d AR samples x %d sims per GPU" % (I, S, args.iterations))
                                   if decide else "IMPI AR determinization: %d infostates x %d samples per GPU" % (I, S),
                       "temperature": args.ar_temperature,
                       "network_rounds": (policy.sampler.rounds if decide else
                                          ar.rounds if parts is None else max(p[0].rounds for p in parts)),
                       "impi_streams": P,
                       "network_rows_per_step": stats["rows"] // args.steps,
                       "consistent_fraction": stats["consistent"] / max(1, stats["lanes"]),
                       "parallelism": "replicas x%d" % world},
            "network_ms_per_step": net_ms / args.steps,
            ("search_sampler_fusion_ms_per_step" if decide else "sampler_ms_per_step"):
                elapsed / args.steps * 1e3 - net_ms / args.steps,
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": npeak, "unit": "TFLOP/s",
                         "frac": achieved / npeak, "traffic": None,
                         "note": "IMPI network: %.1f MFLOP per guess (algorithmic), rows = guesses actually needed "
                                 "(infostates ordered by guess count, each round runs the prefix of lanes still "
                                 "guessing); achieved over the network's event-timed share of the step; %s"
                                 % (flop / 1e6, nnote)},
            "cpu_baseline": cpu,
        }
        print(json.dumps(result))
    if world > 1:
        dist.destroy_process_group()
    eng.close()
    return result


def cpu_baseline_net(args, kind, target_s=3.0, batch=256):
    """CPU baseline of the network workloads (c5: AlphaZero self-play; impi: AR determinization)
    on this box's host cores, the reference's two parts timed separately on a bounded sample:
      net  : the reference architecture (DokoAzNet d 160 / DokoImpiNet d 256, random weights) in
             torch-CPU f32 at matmul precision "medium" (az_doko.py:539-541, main.py:508), batches of
             `batch` evaluations of random valid tokens -> evaluations/s;
      tree : the ORACLE's search around the network with its synthetic hash network -- c5:
             mcts_search (async_mcts.rs:224-406: PUCT, c 4.0, Dirichlet 0.8 / 0.3, T 0.5) on fresh
             deals; impi: forward_pred_process_with_mask (forward.rs:392-661, T 0.4) on the C3
             infostates -- one worker thread per usable core -> simulations (or samples) per second
             and network evaluations per unit.
    value = units/s with one network evaluation per simulation (c5) / per guess (impi), network and
    tree work serialised: 1 / (evals_per_unit / net_rate + 1 / tree_rate)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes
    from concurrent.futures import ThreadPoolExecutor

    import torch

    import oracle_lib as ol
    cores, quota = cpu_quota_cores()
    threads = args.cpu_threads or (min(cores, int(np.ceil(quota))) if quota else cores)
    prev_threads = torch.get_num_threads()
    try:
        prev_prec = torch.get_float32_matmul_precision()
    except RuntimeError:   # (the GPU leg set allow_tf32 through the legacy API: leave "medium" set after)
        prev_prec = "medium"
    torch.set_num_threads(threads)
    torch.set_float32_matmul_precision("medium")
    try:
        if kind == "c5":
            from master_doko_reinforcement_learning_amd.az_network import VOCAB as voc, DokoAzNet as Net
        else:
            from master_doko_reinforcement_learning_amd.impi_network import VOCAB_IPI as voc, DokoImpiNet as Net
        torch.manual_seed(99)
        net = Net().eval()
        g = torch.Generator().manual_seed(7)
        tok = torch.cat([torch.randint(0, v, (batch, 62 if i < 5 else 1), generator=g) for i, v in enumerate(voc)], dim=1)
        with torch.inference_mode():
            net(tok[:16])                                                   # warm-up
            n_ev, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < target_s or n_ev == 0:
                net(tok)
                n_ev += batch
            net_secs = time.perf_counter() - t0
        net_rate = n_ev / net_secs
    finally:
        torch.set_num_threads(prev_threads)
        torch.set_float32_matmul_precision(prev_prec)

    def timed_pool(work, n):
        t0 = time.perf_counter()
        with ThreadPoolExecutor(threads) as ex:
            out = list(ex.map(work, range(n)))
        return out, time.perf_counter() - t0

    if kind == "c5":
        iters = args.az_iterations

        def work(k):      # one move decision of a fresh deal (ctypes releases the GIL)
            st = ol.FdoState.new_game(0xA2000000 + k)
            st.az_search(None, iters, 4.0, 0.3, 10, 2, 0.5, ol.rng_seed(0xA2 ^ k), alpha=0.8)
            return iters

        _, t1 = timed_pool(work, threads)
        n = max(threads, int(threads * target_s / max(t1, 1e-3)))
        done, secs = timed_pool(work, n)
        tree_rate = sum(done) / secs
        evals_per_unit = 1.0
        unit, sample = "simulations/s", "%d searches of %d PUCT iterations on fresh deals" % (n, iters)
    else:
        def infostate(j):
            st = ol.FdoState.new_game(0xC3000000 + j)
            for _ in range(4):
                st.play(24)
            rng = ol.rng_seed(0xC3100000 + j)
            st.random_plies(rng, [0, 8, 20, 32][j % 4], True)
            return st

        def work(k):
            _, _, _, guesses = infostate(k % 4096).ipi_sample(ol.rng_seed(0xA5000000 + k), args.ar_temperature)
            return guesses

        _, t1 = timed_pool(work, threads)
        n = max(threads, int(threads * target_s / max(t1, 1e-3)))
        done, secs = timed_pool(work, n)
        tree_rate = n / secs
        evals_per_unit = float(np.mean(done))
        unit, sample = "samples/s", "%d AR samples of the C3 infostates (%.1f guesses each)" % (n, evals_per_unit)
    value = 1.0 / (evals_per_unit / net_rate + 1.0 / tree_rate)
    return {"value": value, "unit": unit, "cores": threads, "kind": "port", "cpu_quota_cores": quota,
            "network_evals_per_s": net_rate, "tree_units_per_s": tree_rate, "network_evals_per_unit": evals_per_unit,
            "sample": "network: %d evaluations in batches of %d (torch-CPU f32, matmul precision 'medium', %d threads, "
                      "%.1f s); tree: the oracle restatement with its hash network, %s on %d threads (%.1f s); "
                      "combined serially per evaluation" % (n_ev, batch, threads, net_secs, sample, threads, secs)}


def cpu_quota_cores():
    """CPU cores this process may use: the affinity set, capped by a cgroup v2 cpu.max quota."""
    cores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()
        if q != "max":
            quota = float(q) / float(per)
    except Exception:
        pass
    return cores, quota


def cpu_baseline(args, dk, target_s=5.0):
    """The ORACLE (C++ restatement of the reference hot path) timed on this box's host
    cores on a bounded sample of the same workload: one worker thread per usable core,
    root-parallel with a shared work queue like MCTSWorkers (mcts_policy.rs:55-126,
    run.rs:508-520), sized to about `target_s` seconds of wall time; plus a 1-thread figure."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes

    import oracle_lib as ol
    cores, quota = cpu_quota_cores()
    # one worker per core this process may actually use: on a box whose cgroup quota is
    # smaller than the visible CPUs, more threads only time-slice the same quota
    threads = args.cpu_threads or (min(cores, int(np.ceil(quota))) if quota else cores)
    eff = min(threads, quota) if quota else threads
    iters = args.iterations
    do = args.workload in ("c2", "c2d")

    def make_roots(n):
        roots, seeds = [], []
        for k in range(n):
            if args.workload in ("c3", "c2d"):
                j, s = k % args.infostates, (k // args.infostates) % args.samples
                st = (ol.DoState if do else ol.FdoState).new_game(0xC3000000 + j)
                for _ in range(4):
                    st.play(24)
                rng = ol.arr(ctypes.c_uint64, 4, [int(x) for x in dk.splitmix_rng_states(np.array([0xC3100000 + j], dtype=np.uint64))[0]])
                if do:
                    st.random_plies(rng, [0, 8, 20, 32][j % 4])
                    smp = st.sample_assignment_full(ol.rng_seed(0xC3200000 + j * args.samples + s))
                else:
                    st.random_plies(rng, [0, 8, 20, 32][j % 4], True)
                    smp = st.card_matching(ol.rng_seed(0xC3200000 + j * args.samples + s))
                roots.append(smp)
                seeds.append(0xC3300000 + j * args.samples + s)
            else:
                st = ol.DoState.new_game(0xD0C00000 + k)
                for _ in range(4):
                    st.play(24)
                roots.append(st)
                seeds.append((k * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF)
        return roots, seeds

    def run(roots, seeds, nthreads):
        n = len(roots)
        handles = (ctypes.c_void_p * n)(*[r.h for r in roots])
        vis = (ctypes.c_uint32 * (39 * n))()
        sd = ol.arr(ctypes.c_uint64, n, seeds)
        if do:
            return ol.lib().or_do_search_many(handles, sd, n, iters, args.c, vis, nthreads)
        return ol.lib().or_fdo_search_many(None, handles, sd, n, iters, args.c, vis, nthreads)

    n1 = 64
    r1, s1 = make_roots(n1)
    secs1 = run(r1, s1, 1)
    rate1 = n1 * iters / secs1
    n = int(np.ceil(target_s * rate1 * eff / iters / threads)) * threads
    n = max(n, threads)
    roots, seeds = make_roots(min(n, 8192))          # distinct roots, tiled beyond 8192 (Python setup time)
    roots = [roots[k % len(roots)] for k in range(n)]
    seeds = [seeds[k % len(seeds)] for k in range(n)]
    secs = run(roots, seeds, threads)
    model, phys = "", None
    try:
        ls = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
        kv = {l.split(":", 1)[0].strip(): l.split(":", 1)[1].strip() for l in ls.splitlines() if ":" in l}
        model = kv.get("Model name", "")
        phys = int(kv["Core(s) per socket"]) * int(kv["Socket(s)"])
    except Exception:
        model = model or platform.processor()
    return {"value": n * iters / secs, "unit": "rollouts/s", "cores": threads, "kind": "port",
            "host_cpus": os.cpu_count(), "host_physical_cores": phys, "cpu_quota_cores": quota,
            # NOT measured: the 1-thread rate times the host's physical cores (linear scaling,
            # no SMT gain), for comparison with a whole-machine MCTSWorkers pool
            "value_all_physical_cores_extrapolated": rate1 * phys if phys else None,
            "sample": "%d roots x %d sims of the same workload (oracle C++ restatement, one worker per usable core, "
                      "shared root queue like MCTSWorkers), %.1f s wall on %d threads of %s (%d CPUs visible, "
                      "cgroup quota %s cores); 1-thread figure on %d roots"
                      % (n, iters, secs, threads, model, os.cpu_count() or 0,
                         "%.1f" % quota if quota else "none", n1),
            "value_1_thread": rate1}


def alg_bytes_per_sim(workload):
    """SURVEY.md 8(d) byte model per simulation, measured by tools/alg_bytes.py
    on the oracle (committed as profiles/alg_bytes_c3.json)."""
    path = os.path.join(ROOT, "profiles", "alg_bytes_%s.json" % workload)
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        return json.load(fh)["b_sim"]


def stream_copy_gbs(torch, dev, nbytes=1 << 31, reps=10):
    """Measured device-to-device copy rate (read + write bytes / time) on this box."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize(dev)
    gbs = 2.0 * nbytes * reps / (e0.elapsed_time(e1) / 1e3) / 1e9
    del a, b
    return gbs


def pmc_valu(path=None):
    """Measured issue figures of the search launch from the committed PMC summary
    (tools/pmc_finalize.py): VALU busy = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x shader
    cycles), the 4 cycles calibrated by tools/pmc_calib.hip (a saturated integer VALU pipe
    reads 0.93-0.99 at 1-8 waves per SIMD); share of wave cycles waiting on memory; DRAM
    rate against the measured random-line read peak."""
    path = path or os.path.join(ROOT, "profiles", "pmc_search.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
        x = d["derived"]
        return {"busy": x["valu_busy"], "mem_wait_frac": x["mem_wait_frac"],
                "wave_insts_per_sim": d["valu_insts_per_sim_per_wave64"],
                "dram_gbs_under_pmc": x.get("dram_gbs"),
                "dram_frac_of_random_line_peak": d.get("dram_frac_of_random_line_peak"),
                "random_line_read_peak_gbs": d.get("random_line_read_peak_gbs_measured"),
                "source": os.path.relpath(path, ROOT), "calibration": d.get("calibration")}
    except Exception:
        return None


def pmc_summary_path(workload):
    """The committed PMC summary of a workload's search launch (tools/pmc_finalize.py):
    profiles/pmc_search.json for C3, profiles/pmc_search_<workload>.json otherwise."""
    return os.path.join(ROOT, "profiles", "pmc_search.json" if workload == "c3" else "pmc_search_%s.json" % workload)


def pmc_traffic(n_roots, iters, path):
    """Calibrated DRAM bytes per search launch from the committed PMC summary, scaled to
    this launch size; None if absent."""
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        d = json.load(fh)
    try:
        per_sim = d["hbm_bytes_per_launch"] / (d["roots"] * d["iterations"])
        return per_sim * n_roots * iters
    except Exception:
        return None


if __name__ == "__main__":
    main()
