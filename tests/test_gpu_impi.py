"""GPU parity of the IMPI autoregressive determinization (ARSampling, engine/ar_engine.h)
against the ORACLE forward_pred_process_with_mask (oracle/impi.hpp), and the IMPI network's
fused bf16 forward against its fp32 module."""
import numpy as np
import pytest

import oracle_lib as ol

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import master_doko_reinforcement_learning_amd as dk
    e = dk.Engine(device=0, max_roots=4096, max_iterations=200)
    yield e
    e.close()


def ar_positions(n, seed):
    """Positions of random games over all legal actions (weddings, solos, announcements),
    cut at a random ply; the reservation phase included."""
    rng = np.random.default_rng(seed)
    out = []
    g = 0
    while len(out) < n:
        s = ol.FdoState.new_game(int(seed * 100000 + g))
        g += 1
        stop = int(rng.integers(0, 56))
        for ply in range(80):
            if s.info()["phase"] == 3:
                break
            if ply == stop:
                out.append(s.clone())
                break
            legal = s.allowed()
            s.play(int(rng.choice([a for a in range(39) if legal >> a & 1])))
    return out


def _records(states):
    return np.frombuffer(b"".join(s.pack_az() for s in states), dtype=np.uint8).reshape(-1, 160).copy()


@pytest.mark.parametrize("temperature", [1.0, 0.35, 4.0])
def test_ar_sampling_parity(eng, temperature):
    """forward_pred_process_with_mask (rs-doko-impi/src/forward.rs:392-661) on the GPU ==
    the oracle, with the synthetic hash network (oracle/impi.hpp hash_eval) on both sides:
    per sample the status, the NotConsistentReason and the sampled deal + reservations."""
    import torch
    import master_doko_reinforcement_learning_amd as dk
    info = ar_positions(48, 7 + int(temperature * 100))
    S = 4
    rng = np.random.default_rng(int(temperature * 1000))
    seeds = rng.integers(0, 2**63, size=len(info) * S, dtype=np.uint64)
    dev = torch.device("cuda", 0)

    def network(tokens):
        return torch.from_numpy(ol.ipi_hash_eval_np(tokens.cpu().numpy())).to(dev)

    ar = dk.ARSampling(eng, network, temperature)
    out, status, reason = ar.sample(torch.from_numpy(_records(info)).to(dev), S, seeds)
    out, status, reason = out.cpu().numpy(), status.cpu().numpy(), reason.cpu().numpy()
    seen = set()
    for i in range(len(info) * S):
        st, rs, packed, _ = info[i // S].ipi_sample(ol.rng_seed(int(seeds[i])), temperature)
        assert int(status[i]) == st, i
        seen.add(st)
        if st == 1:
            assert int(reason[i]) == rs, i
        if st == 0:
            assert out[i, :117].tobytes() == packed[:117], i
    assert 0 in seen


def test_ar_sampling_full_size_properties(eng):
    """4096 infostates x 4 samples with the bf16 IMPI network (d 256, 4 layers): every
    consistent sample keeps the observer's hand and every hand size, deals exactly the
    hidden cards, and a repeat run is bit-identical."""
    import torch
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd.impi_network import DokoImpiNet
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = DokoImpiNet().to(dev).eval().bfloat16()
    n, S = 4096, 4
    seeds = np.arange(n, dtype=np.uint64) + 77
    roots = eng.new_games(0, seeds)
    env = dk.McEnv(eng)
    for _ in range(4):
        roots = env.by_action(roots, np.full(n, np.uint64(1) << np.uint64(24)))
    rng_states = dk.splitmix_rng_states(seeds + np.uint64(5))
    roots, _ = env.random_plies(roots, rng_states, np.array([0, 8, 20, 32] * (n // 4), dtype=np.uint32))
    recs = dk.az_records(eng, torch.from_numpy(roots).to(dev))
    ar = dk.ARSampling(eng, lambda t: net(t), 1.0)
    lane_seeds = np.arange(n * S, dtype=np.uint64) * 3 + 1
    with torch.inference_mode():
        o1, s1, r1 = ar.sample(recs, S, lane_seeds)
        o2, s2, r2 = ar.sample(recs, S, lane_seeds)
    assert torch.equal(o1, o2) and torch.equal(s1, s2) and torch.equal(r1, r2)
    assert ar.rounds == 36
    o, st = o1.cpu().numpy(), s1.cpu().numpy()
    info = recs.cpu().numpy()[:, :128]
    assert (st <= 1).all() and (st == 0).mean() > 0.5
    hands_o = o[:, :32].view(np.uint64)
    hands_i = np.repeat(info[:, :32].copy().view(np.uint64), S, axis=0)
    cp = np.repeat(info[:, 100], S)
    ok = st == 0
    for p in range(4):
        assert (np.vectorize(lambda x: bin(int(x)).count("1"))(hands_o[ok, p]) ==
                np.vectorize(lambda x: bin(int(x)).count("1"))(hands_i[ok, p])).all()
    rows = np.nonzero(ok)[0]
    assert (hands_o[rows, cp[rows]] == hands_i[rows, cp[rows]]).all()

    def counts(h):
        lo = (h[:, None] >> np.arange(24, dtype=np.uint64)) & np.uint64(1)
        hi = (h[:, None] >> (np.arange(24, dtype=np.uint64) + np.uint64(24))) & np.uint64(1)
        return (lo + hi).astype(np.int32)
    tot_o = sum(counts(hands_o[rows, p]) for p in range(4))
    tot_i = sum(counts(hands_i[rows, p]) for p in range(4))
    assert (tot_o == tot_i).all()


def test_impi_network_fused_matches_fp32_module():
    """DokoImpiNet's fused bf16 forward against the same weights run as the fp32 module."""
    import torch
    from master_doko_reinforcement_learning_amd.impi_network import VOCAB_IPI, DokoImpiNet
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net32 = DokoImpiNet().to(dev).eval()
    net16 = DokoImpiNet().to(dev).eval()
    net16.load_state_dict(net32.state_dict())
    net16 = net16.bfloat16()
    tok = torch.cat([torch.randint(0, v, (256, 62 if i < 5 else 1), device=dev) for i, v in enumerate(VOCAB_IPI)], 1).int()
    with torch.inference_mode():
        p32 = net32(tok)
        p16 = net16(tok)
    scale = p32.abs().max().item()
    assert (p16.float() - p32).abs().max().item() < 0.05 * scale + 0.02
    assert (p16.float().argmax(1) == p32.argmax(1)).float().mean().item() > 0.9


@pytest.mark.parametrize("fusion", ["maxn", "avg"])
@pytest.mark.parametrize("streams", [1, 3])
def test_ar_decide_end_to_end(eng, fusion, streams):
    """mcts_ar_maxn/avg_policy (all_policies.rs:78-127 -> DefaultImpiPolicy::execute,
    compare_impi.rs:212-371): AR samples (hash network) -> UCT on each -> fusion over the
    consistent samples, against the oracle pipeline (visits of every consistent sample,
    the number of consistent samples and the fused action of every infostate)."""
    import torch
    import master_doko_reinforcement_learning_amd as dk
    dev = torch.device("cuda", 0)
    info = ar_positions(10, 41)
    S, iters = 6, 120
    n = len(info)
    seeds = np.arange(2 * n * S + n, dtype=np.uint64) * 7919 + 5

    def network(tokens):
        return torch.from_numpy(ol.ipi_hash_eval_np(tokens.cpu().numpy())).to(dev)

    mode = dk.FUSE_MAXN if fusion == "maxn" else dk.FUSE_AVG
    pol = dk.ArImpiPolicy(eng, network, 2.5, iters, S, mode, 0.4, sampler_streams=streams)
    actions, successes, visits = pol.execute(torch.from_numpy(_records(info)).to(dev), seeds)
    actions, successes, visits = actions.cpu().numpy(), successes.cpu().numpy(), visits.cpu().numpy()
    for j, s in enumerate(info):
        rows = []
        for k in range(S):
            st, _, smp = s.ipi_sample_state(ol.rng_seed(int(seeds[j * S + k])), 0.4)
            if st != 0:
                continue
            _, v, _, _ = smp.search(ol.rng_seed(int(seeds[n * S + j * S + k])), iters, 2.5)
            assert list(visits[j * S + k]) == v
            rows.append(v)
        assert int(successes[j]) == len(rows)
        if rows:
            exp = ol.fuse_maxn(rows, s.allowed())[0] if fusion == "maxn" else ol.fuse_avg(rows)[0]
        else:
            ann = sum(1 << a for a in range(33, 38))
            bit = ol.random_single(s.allowed() & ~ann, ol.rng_seed(int(seeds[2 * n * S + j])))
            exp = bit.bit_length() - 1
        assert int(actions[j]) == exp, j


def test_ar_fallback_random_action(eng):
    """No consistent sample (compare_impi.rs:355-370): FdoAllowedActions::random over the legal
    actions minus the five announcements; infostates with a consistent sample keep the action
    the fusion wrote."""
    import torch
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd import _native
    dev = torch.device("cuda", 0)
    info = ar_positions(40, 5)
    n, S = len(info), 3
    allowed = np.array([s.allowed() for s in info], dtype=np.uint64)
    status = np.ones((n, S), dtype=np.uint8)
    status[::3, 1] = 0                       # every third infostate has one consistent sample
    seeds = np.arange(n, dtype=np.uint64) * 31 + 9
    d_status = torch.from_numpy(status.reshape(-1)).to(dev)
    d_allowed = torch.from_numpy(allowed.view(np.int64)).to(dev)
    d_seeds = torch.from_numpy(seeds.view(np.int64)).to(dev)
    act = torch.full((n,), 200, dtype=torch.uint8, device=dev)
    succ = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        rc = _native.lib().dk_ar_fallback_async(eng.ctx, n, S, d_status.data_ptr(), d_allowed.data_ptr(), d_seeds.data_ptr(),
                                                act.data_ptr(), succ.data_ptr(), side.cuda_stream)
    side.synchronize()
    assert rc == 0 and st is not None
    act, succ = act.cpu().numpy(), succ.cpu().numpy()
    ann = sum(1 << a for a in range(33, 38))
    for j in range(n):
        assert succ[j] == (1 if j % 3 == 0 else 0)
        if j % 3 == 0:
            assert act[j] == 200
        else:
            bit = ol.random_single(int(allowed[j]) & ~ann, ol.rng_seed(int(seeds[j])))
            assert int(act[j]) == bit.bit_length() - 1


def test_ar_sampling_interleaved_parts_equal_one_batch(eng):
    """sample_interleaved (bench.py --impi-streams): the infostates split into four samplings, each
    on its own Engine and stream, their network rounds issued interleaved, give every lane the
    sample, status and reason of the one-batch ARSampling (f32 IMPI network, d 256)."""
    import torch
    import master_doko_reinforcement_learning_amd as dk
    from master_doko_reinforcement_learning_amd.impi_network import DokoImpiNet
    dev = torch.device("cuda", 0)
    torch.manual_seed(3)
    net = DokoImpiNet().to(dev).eval()
    n, S, P = 1024, 4, 4
    seeds = np.arange(n, dtype=np.uint64) + 991
    roots = eng.new_games(0, seeds)
    env = dk.McEnv(eng)
    for _ in range(4):
        roots = env.by_action(roots, np.full(n, np.uint64(1) << np.uint64(24)))
    rng_states = dk.splitmix_rng_states(seeds + np.uint64(9))
    roots, _ = env.random_plies(roots, rng_states, np.array([0, 8, 20, 32] * (n // 4), dtype=np.uint32))
    recs = dk.az_records(eng, torch.from_numpy(roots).to(dev))
    lane_seeds = np.arange(n * S, dtype=np.uint64) * 5 + 3
    network = lambda t: net(t)   # noqa: E731
    with torch.inference_mode():
        o1, s1, r1 = dk.ARSampling(eng, network, 0.4).sample(recs, S, lane_seeds)
        m = n // P
        engines = [dk.Engine(device=0, max_roots=64, max_iterations=1) for _ in range(P)]
        parts = [(dk.ARSampling(engines[k], network, 0.4), torch.cuda.Stream(dev), recs[k * m:(k + 1) * m], S,
                  lane_seeds[k * m * S:(k + 1) * m * S]) for k in range(P)]
        outs = dk.sample_interleaved(parts)
    assert torch.equal(torch.cat([o[0] for o in outs]), o1)
    assert torch.equal(torch.cat([o[1] for o in outs]), s1)
    assert torch.equal(torch.cat([o[2] for o in outs]), r1)
    for e in engines:
        e.close()
