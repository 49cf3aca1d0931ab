"""Host-side mirror of the reference's operator interfaces for the hot path.

Names follow the Rust types they replace:

* ``Engine``                      — a dk_ctx (device, node/state pools)
* ``McEnv``                       — McEnvState (rs-doko-mcts/src/env/env_state.rs:7-28), batched
* ``CachedMCTS``                  — CachedMCTS::monte_carlo_tree_search (mcts.rs:284-315), batched over roots
* ``SmallRng``                    — rand 0.9 SmallRng state, continued by a search like ``&mut SmallRng``
* ``card_matching_full``          — CAP determinization (rs-full-doko/src/matching/card_matching.rs:469-497)
* ``sample_assignment_full``      — rs-doko rule-based determinization (rs-doko-assignment/src/assignment.rs:472-580)
* ``PolicyFusionMaxN`` / ``PolicyFusionAverageStrategy`` — policy_fusion.rs:18-123
* ``DefaultImpiPolicy``           — sample -> search -> fuse (compare_impi.rs:212-371)
* ``ArImpiPolicy``                — AR-determinized decision (mcts_ar_maxn/avg_policy, all_policies.rs:78-127)
* ``ARSampling``                  — IMPI autoregressive determinization (forward_pred_process_with_mask,
                                    rs-doko-impi/src/forward.rs:392-661), batched, network between launches
* ``AlphaZeroSearch``             — AlphaZero PUCT mcts_search (rs-doko-alpha-zero/src/alpha_zero/mcts/async_mcts.rs:224-406),
                                    batched over games, network evaluated between launches

States are ``numpy.uint8`` arrays of shape (n, 128) in the dk_state wire format
of include/doko_amd.h.  Every call runs on the GPU; errors raise DokoError
(the Rust path panics in the same situations).
"""
import ctypes

import numpy as np

from . import _native

GAME_FULL_DOKO = 0
GAME_DOKO = 1
GAME_TTT = 2
FUSE_MAXN = 0
FUSE_AVG = 1
NUM_ACTIONS = 39
STATE_BYTES = 128
AZ_STATE_BYTES = 160   # dk_az_state: packed state + announcement occurrence list
AZ_TOKENS = 311        # encode_state_pi
IPI_TOKENS = 311       # encode_state_ipi
IPI_CLASSES = 33       # ImperfectInformationOutput::COUNT
# ForwardPredResult / NotConsistentReason (rs-full-doko/src/matching/is_consistent.rs:26-36)
AR_CONSISTENT, AR_NOT_CONSISTENT, AR_PANIC, AR_UNFINISHED = 0, 1, 2, 3
NOT_CONSISTENT_REASONS = ("HandSizeMismatch", "NotInRemainingCards", "RemainingCardsLeft", "AlreadyDiscardedColor",
                          "HasClubQueenButSomeoneElseAnnouncedWedding", "HasNoClubQueenButAnnouncedRe",
                          "HasClubQueenButAnnouncedKontra", "WrongReservation", "WrongReservationClubQ")


class DokoError(RuntimeError):
    pass


def _check(rc):
    if rc != 0:
        raise DokoError("doko_amd: %s (%d)" % (_native.lib().dk_status_string(rc).decode(), rc))


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def _states(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    if a.ndim != 2 or a.shape[1] != STATE_BYTES:
        raise ValueError("states must have shape (n, 128)")
    return a


def splitmix_rng_states(seeds):
    """SmallRng::seed_from_u64(seed) states (Xoshiro256++ words) for a seed array."""
    seeds = np.asarray(seeds, dtype=np.uint64)
    out = np.empty((seeds.shape[0], 4), dtype=np.uint64)
    with np.errstate(over="ignore"):
        st = seeds.copy()
        for i in range(4):
            st = st + np.uint64(0x9E3779B97F4A7C15)
            z = st.copy()
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out[:, i] = z ^ (z >> np.uint64(31))
    return out


def _run_on_stream(dev, fn, *args):
    """Run fn(*args, stream_handle) on torch's current stream of `dev` when it is a real
    stream; on the legacy default stream (handle 0, which would select the library's own
    unordered stream) run it on a side stream ordered after the caller's work, make the
    caller wait for it, and record the caller's stream on every returned tensor so the
    caching allocator does not hand their blocks to new side-stream work while
    caller-stream kernels that read them are still queued."""
    import torch
    caller = torch.cuda.current_stream(dev)
    if caller.cuda_stream != 0:
        return fn(*args, caller.cuda_stream)
    side = torch.cuda.Stream(dev)
    side.wait_stream(caller)
    with torch.cuda.stream(side):
        out = fn(*args, side.cuda_stream)
    caller.wait_stream(side)
    for t in out:
        if isinstance(t, torch.Tensor):
            t.record_stream(caller)
    return out


class Engine:
    """A device context: node pools for `max_roots` searches of up to
    `max_iterations` iterations (the reference's CachedMCTS arenas, one per root)."""

    def __init__(self, device=0, max_roots=4096, max_iterations=1000, slot_capacity=0):
        L = _native.lib()
        cfg = _native.dk_config(device, max_roots, max_iterations, slot_capacity)
        self._ctx = L.dk_create(ctypes.byref(cfg))
        if not self._ctx:
            raise DokoError("dk_create failed: no usable gfx950 device %d (or out of device memory)" % device)
        self.max_roots = max_roots
        self.max_iterations = max_iterations

    @property
    def ctx(self):
        return self._ctx

    def close(self):
        if getattr(self, "_ctx", None):
            _native.lib().dk_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def pool_bytes(self):
        return int(_native.lib().dk_pool_bytes(self._ctx))

    def pool_high_water(self, stream=None):
        """(most child slots one search used, main-pool slots per root, roots that
        overflowed the main pools and were searched again in the fallback pool), since creation."""
        h, cap, ovf = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        _check(_native.lib().dk_pool_high_water(self._ctx, stream, ctypes.byref(h), ctypes.byref(cap), ctypes.byref(ovf)))
        return int(h.value), int(cap.value), int(ovf.value)

    def last_search_ms(self):
        ms = ctypes.c_float()
        _check(_native.lib().dk_last_search_ms(self._ctx, ctypes.byref(ms)))
        return float(ms.value)

    def last_search_waves(self):
        """Per-wave clocks of the last search launch (dk_last_search_waves): span_ms, the mean
        fraction of the span a wave had work, first / median wave end (ms), waves."""
        out = (ctypes.c_double * 5)()
        _check(_native.lib().dk_last_search_waves(self._ctx, out))
        return {"span_ms": out[0], "busy_frac": out[1], "first_end_ms": out[2], "median_end_ms": out[3],
                "waves": int(out[4])}

    def last_search_clocks(self):
        """Shader clock of the last search launch (dk_last_search_clocks): mean / slowest / fastest
        wave clock in MHz and the mean shader cycles a wave was busy."""
        out = (ctypes.c_double * 4)()
        _check(_native.lib().dk_last_search_clocks(self._ctx, out))
        return {"sclk_mhz": out[0], "sclk_min_mhz": out[1], "sclk_max_mhz": out[2], "wave_busy_cycles": out[3]}

    # ---- game construction (FdoState::new_game / DoState::new_game)
    def new_games(self, game, seeds):
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        out = np.zeros((seeds.shape[0], STATE_BYTES), dtype=np.uint8)
        _check(_native.lib().dk_new_game_batch(self._ctx, game, _ptr(seeds), seeds.shape[0], _ptr(out)))
        return out


class McEnv:
    """Batched McEnvState (rs-doko-mcts/src/env/env_state.rs:7-28) on the GPU."""

    def __init__(self, engine):
        self.engine = engine

    def allowed_actions(self, states, first_expansion):
        s = _states(states)
        m = np.zeros(s.shape[0], dtype=np.uint64)
        _check(_native.lib().dk_env_allowed_batch(self.engine.ctx, _ptr(s), s.shape[0], 1 if first_expansion else 0, _ptr(m)))
        return m

    def by_action(self, states, action_bits):
        s = _states(states).copy()
        a = np.ascontiguousarray(action_bits, dtype=np.uint64)
        _check(_native.lib().dk_env_step_batch(self.engine.ctx, _ptr(s), _ptr(a), s.shape[0]))
        return s

    def rewards_or_none(self, states):
        s = _states(states)
        has = np.zeros(s.shape[0], dtype=np.int32)
        r = np.zeros((s.shape[0], 4), dtype=np.float64)
        _check(_native.lib().dk_env_rewards_batch(self.engine.ctx, _ptr(s), s.shape[0], _ptr(has), _ptr(r)))
        return has.astype(bool), r

    def random_rollout(self, states, rng_states):
        """Returns (rewards[n,4], advanced rng states[n,4])."""
        s = _states(states)
        g = np.ascontiguousarray(rng_states, dtype=np.uint64).copy()
        r = np.zeros((s.shape[0], 4), dtype=np.float64)
        _check(_native.lib().dk_env_rollout_batch(self.engine.ctx, _ptr(s), _ptr(g), s.shape[0], _ptr(r)))
        return r, g

    def random_plies(self, states, rng_states, plies):
        s = _states(states).copy()
        g = np.ascontiguousarray(rng_states, dtype=np.uint64).copy()
        k = np.ascontiguousarray(plies, dtype=np.uint32)
        _check(_native.lib().dk_env_random_plies_batch(self.engine.ctx, _ptr(s), _ptr(g), _ptr(k), s.shape[0]))
        return s, g


class SmallRng:
    """rand 0.9 ``SmallRng`` (Xoshiro256++) held on the host as its four state words.  Passed to
    ``CachedMCTS.monte_carlo_tree_search`` it is advanced in place, exactly as the reference's
    ``&mut SmallRng`` is (rs-doko-mcts/src/mcts/mcts.rs:294-315)."""

    def __init__(self, state):
        self.state = np.array(state, dtype=np.uint64).reshape(4)

    @classmethod
    def seed_from_u64(cls, seed):
        return cls(splitmix_rng_states([seed])[0])

    def __eq__(self, other):
        return isinstance(other, SmallRng) and bool(np.array_equal(self.state, other.state))

    def __repr__(self):
        return "SmallRng(%s)" % ", ".join("0x%016x" % int(w) for w in self.state)


class CachedMCTS:
    """CachedMCTS::monte_carlo_tree_search (mcts.rs:294-315) for a batch of roots, one
    independent search per root.  `random` is either
      * u64 seeds [n]: root i searches with SmallRng::seed_from_u64(seeds[i]), or
      * the caller's generators, continued in place: a SmallRng (one root), a list of them, or a
        uint64 array [n, 4] of Xoshiro256++ states (dk_search_batch_rng).
    Returns (visits [n, 39], values [n, 39], best [n]): the Move list by action index and
    max_by_key(visits) over it (the last maximum), DK_NONE without children."""

    def __init__(self, engine, game=GAME_FULL_DOKO):
        self.engine = engine
        self.game = game

    def monte_carlo_tree_search(self, roots, uct_exploration_constant, iterations, random):
        s = _states(roots)
        n = s.shape[0]
        visits = np.zeros((n, NUM_ACTIONS), dtype=np.uint32)
        values = np.zeros((n, NUM_ACTIONS), dtype=np.float64)
        best = np.zeros(n, dtype=np.uint8)
        L = _native.lib()
        c = float(uct_exploration_constant)
        gens = [random] if isinstance(random, SmallRng) else random
        if isinstance(gens, (list, tuple)) and gens and isinstance(gens[0], SmallRng):
            st = np.stack([g.state for g in gens]).astype(np.uint64)
            if st.shape[0] != n:
                raise ValueError("need one SmallRng per root")
            _check(L.dk_search_batch_rng(self.engine.ctx, self.game, _ptr(s), _ptr(st), n, iterations, c,
                                         _ptr(visits), _ptr(values), _ptr(best)))
            for g, w in zip(gens, st):
                g.state[:] = w
            return visits, values, best
        arr = np.asarray(random)
        if arr.ndim == 2:
            if arr.shape != (n, 4) or arr.dtype != np.uint64 or not arr.flags.c_contiguous:
                raise ValueError("rng states must be a C-contiguous uint64 array [n, 4]")
            _check(L.dk_search_batch_rng(self.engine.ctx, self.game, _ptr(s), _ptr(arr), n, iterations, c,
                                         _ptr(visits), _ptr(values), _ptr(best)))
            return visits, values, best
        seeds = np.ascontiguousarray(arr, dtype=np.uint64)
        if seeds.shape != (n,):
            raise ValueError("need one seed per root")
        _check(L.dk_search_batch(self.engine.ctx, self.game, _ptr(s), _ptr(seeds), n, iterations, c,
                                 _ptr(visits), _ptr(values), _ptr(best)))
        return visits, values, best


# ---- tic-tac-toe (config 1: rs-doko-mcts/src/example/tic_tac_toe*.rs) -------------------------
TTT_NOT_FINISHED, TTT_XWON, TTT_OWON, TTT_DRAW = 0, 1, 2, 3
_TTT_LINES = ((0, 1, 2), (3, 4, 5), (6, 7, 8), (0, 3, 6), (1, 4, 7), (2, 5, 8), (0, 4, 8), (2, 4, 6))


def ttt_state(board=None, last_action=None):
    """The dk_ttt_state wire record of a TicTacToeState (0 empty, 1 X, 2 O per cell); its
    finish state is calc_finish_state (tic_tac_toe.rs:29-80)."""
    b = [0] * 9 if board is None else [int(v) for v in board]
    rec = np.zeros(STATE_BYTES, dtype=np.uint8)
    rec[:9] = b
    fin = TTT_NOT_FINISHED
    for ln in _TTT_LINES:
        if all(b[k] == 1 for k in ln):
            fin = TTT_XWON
            break
        if all(b[k] == 2 for k in ln):
            fin = TTT_OWON
            break
    if fin == TTT_NOT_FINISHED and 0 not in b:
        fin = TTT_DRAW
    rec[9] = fin
    rec[10] = 0xFF if last_action is None else int(last_action)
    rec[STATE_BYTES - 1] = GAME_TTT
    return rec


def tic_tac_toe_player(engine, games, iterations=1400, uct_exploration_constant=2.0, random=None, trace=None):
    """tic_tac_toe_player (rs-doko-mcts/src/example/tic_tac_toe_player.rs:8-52): `games` games
    from the empty board, ONE SmallRng (default seed_from_u64(999)) threaded through every
    search of every game, each move max_by_key(visits) of
    monte_carlo_tree_search(state, c, iterations, rng).  Every search and every move runs on
    the GPU (one root per launch: the stream makes the games strictly sequential).  Returns
    [X won, O won, draws]; `trace` (a list) receives (game, board, visits[39], best, rng state
    after the search) per move."""
    rng = SmallRng.seed_from_u64(999) if random is None else random
    mcts = CachedMCTS(engine, GAME_TTT)
    env = McEnv(engine)
    results = [0, 0, 0]
    for g in range(games):
        st = ttt_state()[None, :]
        while st[0, 9] == TTT_NOT_FINISHED:
            visits, _, best = mcts.monte_carlo_tree_search(st, uct_exploration_constant, iterations, rng)
            if trace is not None:
                trace.append((g, st[0, :9].copy(), visits[0].copy(), int(best[0]), rng.state.copy()))
            st = env.by_action(st, np.array([1 << int(best[0])], dtype=np.uint64))
        results[int(st[0, 9]) - 1] += 1
    return results


def tic_tac_toe_games(engine, seeds, iterations=1400, uct_exploration_constant=2.0):
    """Independent tic-tac-toe games in lockstep, game g with its own
    SmallRng::seed_from_u64(seeds[g]) threaded through its searches: one search launch per
    move over every unfinished game (the GPU-shaped form of tic_tac_toe_player).  Returns
    (finish state per game, moves per game, total searches)."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
    n = seeds.shape[0]
    rng = splitmix_rng_states(seeds)
    states = np.stack([ttt_state()] * n)
    mcts = CachedMCTS(engine, GAME_TTT)
    env = McEnv(engine)
    moves = np.zeros(n, dtype=np.int32)
    searches = 0
    while True:
        live = np.nonzero(states[:, 9] == TTT_NOT_FINISHED)[0]
        if live.size == 0:
            break
        r = np.ascontiguousarray(rng[live])
        _, _, best = mcts.monte_carlo_tree_search(states[live], uct_exploration_constant, iterations, r)
        rng[live] = r
        states[live] = env.by_action(states[live], np.left_shift(np.uint64(1), best.astype(np.uint64)))
        moves[live] += 1
        searches += int(live.size)
    return states[:, 9].copy(), moves, searches


def card_matching_full(engine, infostates, samples, seeds):
    """CAPSampling::sample for each infostate, `samples` times: returns
    (n_info*samples, 128) determinized states."""
    s = _states(infostates)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
    out = np.zeros((s.shape[0] * samples, STATE_BYTES), dtype=np.uint8)
    _check(_native.lib().dk_determinize_batch(engine.ctx, _ptr(s), s.shape[0], samples, _ptr(seeds), _ptr(out)))
    return out


def sample_assignment_full(engine, infostates, samples, seeds):
    """rs-doko `sample_assignment_full(state, &state.observation_for_current_player(), rng)`
    for each rs-doko infostate, `samples` times (rng i*samples+s =
    SmallRng::seed_from_u64(seeds[i*samples+s])): returns (n_info*samples, 128)
    determinized states.  Raises DokoError where the reference panics."""
    return card_matching_full(engine, infostates, samples, seeds)


class _Fusion:
    mode = None

    def fuse(self, engine, visits, allowed):
        """visits: (n_info, samples, 39); allowed: (n_info,) FdoAllowedActions bits."""
        v = np.ascontiguousarray(visits, dtype=np.uint32)
        n_info, samples = v.shape[0], v.shape[1]
        a = np.ascontiguousarray(allowed, dtype=np.uint64)
        out = np.zeros(n_info, dtype=np.uint8)
        _check(_native.lib().dk_fuse(engine.ctx, _ptr(v), n_info, samples, _ptr(a), self.mode, _ptr(out)))
        return out


class PolicyFusionMaxN(_Fusion):
    mode = FUSE_MAXN


class PolicyFusionAverageStrategy(_Fusion):
    mode = FUSE_AVG


class DefaultImpiPolicy:
    """Determinized decision: `num_samples` samples -> UCT each -> fusion.
    rs-full-doko infostates are sampled by CAP (compare_impi.rs:64-81), rs-doko
    infostates by the rule-based sampler (assignment.rs:472-580); one call
    holds infostates of one game."""

    def __init__(self, engine, uct_exploration_constant=2.5, iterations=1000, num_samples=64, fusion=FUSE_MAXN):
        self.engine = engine
        self.c = float(uct_exploration_constant)
        self.iterations = iterations
        self.num_samples = num_samples
        self.fusion = fusion

    def execute(self, infostates, seeds, return_visits=False):
        """seeds: 2*n_info*num_samples u64 (sampling seeds, then search seeds)."""
        s = _states(infostates)
        n_info = s.shape[0]
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        if seeds.shape[0] != 2 * n_info * self.num_samples:
            raise ValueError("need 2*n_info*num_samples seeds")
        actions = np.zeros(n_info, dtype=np.uint8)
        visits = np.zeros((n_info * self.num_samples, NUM_ACTIONS), dtype=np.uint32) if return_visits else None
        _check(_native.lib().dk_decide_batch(self.engine.ctx, _ptr(s), n_info, self.num_samples, _ptr(seeds),
                                             self.iterations, self.c, self.fusion, _ptr(actions),
                                             _ptr(visits) if return_visits else None))
        return (actions, visits) if return_visits else actions

    def execute_async(self, infostates, seeds, game=None):
        """DefaultImpiPolicy::execute entirely on the device, asynchronously on torch's current
        stream: `infostates` uint8 [n_info, 128] and `seeds` int64 [2 * n_info * num_samples]
        (sampling seeds, then search seeds) are CUDA tensors; returns CUDA tensors (actions
        uint8 [n_info], visits int32 [n_info * num_samples, 39]).  `game` (GAME_FULL_DOKO /
        GAME_DOKO) avoids reading the game tag back from the device.  Calls issued on
        different streams run concurrently on one engine: each search launch takes its own
        slot and range of pool lanes (dk_search_batch_async), so independent decision
        batches smaller than the resident grid overlap on the GPU.  Device-side errors
        surface at dk_sync of the stream (execute_many does that)."""
        if game is None:
            game = int(infostates[0, STATE_BYTES - 1].item())
        return _run_on_stream(infostates.device, self._execute_async, infostates, seeds, game)

    def _execute_async(self, infostates, seeds, game, st):
        import torch
        L = _native.lib()
        ctx = self.engine.ctx
        dev = infostates.device
        n_info, S = infostates.shape[0], self.num_samples
        n = n_info * S
        if seeds.numel() != 2 * n:
            raise ValueError("need 2*n_info*num_samples seeds")
        roots = torch.empty((n, STATE_BYTES), dtype=torch.uint8, device=dev)
        visits = torch.empty((n, NUM_ACTIONS), dtype=torch.int32, device=dev)
        values = torch.empty((n, NUM_ACTIONS), dtype=torch.float64, device=dev)
        best = torch.empty(n, dtype=torch.uint8, device=dev)
        allowed = torch.empty(n_info, dtype=torch.int64, device=dev)
        acc_u = torch.empty((n_info, NUM_ACTIONS), dtype=torch.int32, device=dev)
        acc_f = torch.empty((n_info, NUM_ACTIONS), dtype=torch.float32, device=dev)
        actions = torch.empty(n_info, dtype=torch.uint8, device=dev)
        sp = seeds.data_ptr()
        _check(L.dk_determinize_batch_async(ctx, infostates.data_ptr(), n_info, S, sp, roots.data_ptr(), st))
        _check(L.dk_search_batch_async(ctx, game, roots.data_ptr(), sp + 8 * n, n, self.iterations, self.c,
                                       visits.data_ptr(), values.data_ptr(), best.data_ptr(), st))
        _check(L.dk_legal_actions_async(ctx, infostates.data_ptr(), n_info, allowed.data_ptr(), st))
        _check(L.dk_fuse_accumulate_async(ctx, visits.data_ptr(), n_info, S, allowed.data_ptr(), self.fusion,
                                          acc_u.data_ptr(), acc_f.data_ptr(), st))
        _check(L.dk_fuse_select_async(ctx, n_info, self.fusion, allowed.data_ptr(), acc_u.data_ptr(), acc_f.data_ptr(),
                                      actions.data_ptr(), st))
        return actions, visits

    def execute_many(self, batches, game=None, streams=0):
        """Independent decision batches [(infostates, seeds), ...] (CUDA tensors as in
        execute_async) that are in flight at the same time -- the reference's evaluator
        decides many games at once (compare_impi/run.rs:775).  By default they are batched
        into ONE device pass (infostates and seeds concatenated, results split back): the
        roots of different decisions are independent and the fusion is per infostate, so
        every result equals its batch decided alone, while the launch gets the occupancy of
        the combined batch.  streams=K instead issues each batch on one of K streams (the
        engine's concurrent search slots); whether those overlap depends on how HIP maps
        the streams onto hardware queues.  Returns [(actions, visits), ...], complete;
        raises DokoError on a device-side error."""
        import torch
        if not batches:
            return []
        dev = batches[0][0].device
        caller = torch.cuda.current_stream(dev)
        L = _native.lib()
        S = self.num_samples
        if streams:
            groups = [[b] for b in batches]
        else:
            # one pass: seeds of batch b are [sampling n_b][search n_b] -> [all sampling][all search]
            sizes = [int(inf.shape[0]) for inf, _ in batches]
            info = torch.cat([inf for inf, _ in batches])
            seeds = torch.cat([sd[:n_b * S] for (_, sd), n_b in zip(batches, sizes)] +
                              [sd[n_b * S:] for (_, sd), n_b in zip(batches, sizes)])
            groups = [[(info, seeds)]]
        k = max(1, min(streams or 1, len(groups)))
        if len(getattr(self, "_streams", [])) < k:
            self._streams = [torch.cuda.Stream(dev) for _ in range(k)]
        res = []
        for i, g in enumerate(groups):
            s = self._streams[i % k]
            s.wait_stream(caller)
            with torch.cuda.stream(s):
                res.append(self.execute_async(*g[0], game))
        for s in self._streams[:k]:
            _check(L.dk_sync(self.engine.ctx, s.cuda_stream))
            caller.wait_stream(s)
        for a, v in res:
            a.record_stream(caller)
            v.record_stream(caller)
        if streams:
            return res
        actions, visits = res[0]
        out, i0 = [], 0
        for n_b in sizes:
            out.append((actions[i0:i0 + n_b], visits[i0 * S:(i0 + n_b) * S]))
            i0 += n_b
        return out


class ArImpiPolicy:
    """mcts_ar_maxn_policy / mcts_ar_avg_policy (rs-doko-py-bridge/src/compare_impi/all_policies.rs:78-127):
    DefaultImpiPolicy::execute (compare_impi.rs:212-371) with the ARSampling sampler.  Per
    infostate `num_samples` AR draws (network between launches), UCT on every draw, fusion
    over the consistent ones only; an infostate without a consistent draw takes a random
    legal non-announcement action.  Everything stays on the GPU (torch tensors).

    The reference continues each sample's SmallRng from the sampler into the search; here
    sampling, search and fallback take separate explicit seeds (production seeds are
    from_os_rng, so only the seeding scheme differs, not the distribution)."""

    def __init__(self, engine, network, uct_exploration_constant=2.5, iterations=1000, num_samples=64,
                 fusion=FUSE_MAXN, temperature=0.4, sampler_streams=1):
        """sampler_streams > 1: the AR sampling runs as that many interleaved parts, each on its own
        Engine and stream (sample_interleaved); results are those of one sampling."""
        self.engine = engine
        self.c = float(uct_exploration_constant)
        self.iterations = iterations
        self.num_samples = num_samples
        self.fusion = fusion
        self.sampler = ARSampling(engine, network, temperature)
        self.sampler_streams = int(sampler_streams)
        self._parts = None   # [(ARSampling on its own Engine, torch stream)], made on first use

    def execute(self, infostates, seeds):
        """infostates: uint8 [n, 160] dk_az_state records (GPU); seeds: uint64, n*S sampling seeds,
        then n*S search seeds, then n fallback seeds.  Returns (actions uint8 [n], successes int32 [n],
        visits int32 [n*S, 39]) as GPU tensors."""
        return _run_on_stream(infostates.device, self._execute, infostates, seeds)

    def _execute(self, infostates, seeds, st):
        import torch
        L = _native.lib()
        ctx = self.engine.ctx
        n, S = infostates.shape[0], self.num_samples
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        if seeds.shape[0] != 2 * n * S + n:
            raise ValueError("need 2*n*num_samples + n seeds")
        dev = infostates.device
        if self.sampler_streams > 1 and n >= self.sampler_streams:
            P = self.sampler_streams
            if self._parts is None:
                self._parts = [(ARSampling(Engine(device=dev.index or 0, max_roots=64, max_iterations=1), self.sampler.network,
                                           self.sampler.temperature, self.sampler.log_chance), torch.cuda.Stream(dev))
                               for _ in range(P)]
            cut = [n * k // P for k in range(P + 1)]
            outs = sample_interleaved([(smp, stm, infostates[cut[k]:cut[k + 1]], S, seeds[cut[k] * S:cut[k + 1] * S])
                                       for k, (smp, stm) in enumerate(self._parts)])
            samples = torch.cat([o[0] for o in outs])
            status = torch.cat([o[1] for o in outs])
            self.sampler.rounds = max(smp.rounds for smp, _ in self._parts)
            self.sampler.rows = sum(smp.rows for smp, _ in self._parts)
        else:
            samples, status, _ = self.sampler.sample(infostates, S, seeds[:n * S])
        srch = torch.as_tensor(seeds[n * S:2 * n * S].view(np.int64), device=dev)
        fb = torch.as_tensor(seeds[2 * n * S:].view(np.int64), device=dev)
        visits = torch.empty((n * S, NUM_ACTIONS), dtype=torch.int32, device=dev)
        values = torch.empty((n * S, NUM_ACTIONS), dtype=torch.float64, device=dev)
        best = torch.empty(n * S, dtype=torch.uint8, device=dev)
        _check(L.dk_search_batch_async(ctx, GAME_FULL_DOKO, samples.data_ptr(), srch.data_ptr(), n * S, self.iterations,
                                       self.c, visits.data_ptr(), values.data_ptr(), best.data_ptr(), st))
        info = infostates[:, :STATE_BYTES].contiguous()
        allowed = torch.empty(n, dtype=torch.int64, device=dev)
        _check(L.dk_legal_actions_async(ctx, info.data_ptr(), n, allowed.data_ptr(), st))
        valid = (status == AR_CONSISTENT).to(torch.uint8)
        acc_u = torch.zeros((n, NUM_ACTIONS), dtype=torch.int32, device=dev)
        acc_f = torch.zeros((n, NUM_ACTIONS), dtype=torch.float32, device=dev)
        actions = torch.empty(n, dtype=torch.uint8, device=dev)
        _check(L.dk_fuse_accumulate_masked_async(ctx, visits.data_ptr(), n, S, valid.data_ptr(), allowed.data_ptr(),
                                                 self.fusion, acc_u.data_ptr(), acc_f.data_ptr(), st))
        _check(L.dk_fuse_select_async(ctx, n, self.fusion, allowed.data_ptr(), acc_u.data_ptr(), acc_f.data_ptr(),
                                      actions.data_ptr(), st))
        successes = torch.empty(n, dtype=torch.int32, device=dev)
        _check(L.dk_ar_fallback_async(ctx, n, S, status.data_ptr(), allowed.data_ptr(), fb.data_ptr(), actions.data_ptr(),
                                      successes.data_ptr(), st))
        _check(L.dk_sync(ctx, st))
        return actions, successes, visits


class AlphaZeroSearch:
    """`mcts_search` of rs-doko-alpha-zero (async_mcts.rs:224-406) over FdoAzEnvState,
    batched over games: every iteration runs one PUCT selection per game on the GPU,
    then `network` on all leaves at once (the reference's batch processor), then the
    backup.  Everything stays on the device (torch tensors on the current stream).

    network(records) -> (value, logits): records = uint8 [n, 160] dk_az_state on the
    GPU (az_encode turns them into the 311-token network input); value = float32
    [n, 4] from each state's current player's point of view; logits = float32 [n, 39].
    temperature: None (greedy), float('inf') (uniform) or a finite T (select_action,
    mcts.rs:185-248)."""

    def __init__(self, engine, puct_exploration_constant=1.0, dirichlet_epsilon=0.25, epoch=10, temperature=None,
                 dirichlet_alpha=0.8):
        self.engine = engine
        self.c = float(puct_exploration_constant)
        self.eps = float(dirichlet_epsilon)
        self.alpha = float(dirichlet_alpha)   # AlphaZeroTrainOptions::dirichlet_alpha (az_doko.py:592: 0.8)
        self.epoch = int(epoch)
        self.temperature = temperature

    def mcts_search(self, roots, network, noise, iterations, seeds, rng_states=None):
        """roots: uint8 [n, 160] dk_az_state records (GPU); seeds: uint64 [n] (SmallRng per game).
        noise: None (the reference's way: each game draws Dirichlet([dirichlet_alpha; 39]) from its own
        SmallRng at the root, async_mcts.rs:111-113) or float32 [n, 39] samples (GPU) used instead.
        rng_states: None, or int64 [n, 4] (GPU) SmallRng states (Xoshiro256++ words) that game g
        continues instead of seeds[g] and that receive the end states (the reference's
        `rng: &mut SmallRng`, async_mcts.rs:224-406).
        Returns (actions uint8 [n], visits int32 [n, 39])."""
        # the launches need a real stream handle shared with torch (handle 0 would
        # select the library's own stream, unordered with the network's kernels)
        return _run_on_stream(roots.device, self._search, roots, network, noise, iterations, seeds, rng_states)

    def _search(self, roots, network, noise, iterations, seeds, rng_states, st):
        import torch
        L = _native.lib()
        ctx = self.engine.ctx
        n = roots.shape[0]
        dev = roots.device
        seeds_t = torch.as_tensor(np.ascontiguousarray(seeds, dtype=np.uint64).view(np.int64), device=dev)
        roots = roots.contiguous()
        noise = None if noise is None else noise.contiguous().float()
        # every argument is checked before the first launch (a refused call leaves no batch half begun)
        if not roots.is_cuda or seeds_t.shape[0] != n:
            raise ValueError("roots: uint8 [n, %d] on the GPU and seeds [n] expected" % AZ_STATE_BYTES)
        if noise is not None and (noise.device != dev or tuple(noise.shape) != (n, NUM_ACTIONS)):
            raise ValueError("noise: float32 [n, %d] on the roots' device expected" % NUM_ACTIONS)
        if rng_states is not None and (rng_states.dtype != torch.int64 or tuple(rng_states.shape) != (n, 4)
                                       or not rng_states.is_contiguous() or rng_states.device != dev):
            raise ValueError("rng_states: contiguous int64 [n, 4] on the roots' device expected")
        ev = torch.empty((n, AZ_STATE_BYTES), dtype=torch.uint8, device=dev)
        need = torch.empty(n, dtype=torch.uint8, device=dev)
        _check(L.dk_az_begin_async(ctx, roots.data_ptr(), seeds_t.data_ptr(), n, iterations, self.epoch,
                                   ev.data_ptr(), st))
        if rng_states is not None:
            _check(L.dk_az_rng_async(ctx, rng_states.data_ptr(), 1, st))
        value, logits = network(ev)
        value, logits = value.float().contiguous(), logits.float().contiguous()
        _check(L.dk_az_root_async(ctx, value.data_ptr(), logits.data_ptr(), None if noise is None else noise.data_ptr(),
                                  self.alpha, self.eps, st))
        for _ in range(iterations):
            _check(L.dk_az_select_async(ctx, self.c, ev.data_ptr(), need.data_ptr(), st))
            value, logits = network(ev)
            value, logits = value.float().contiguous(), logits.float().contiguous()
            _check(L.dk_az_backup_async(ctx, value.data_ptr(), logits.data_ptr(), st))
        visits = torch.empty((n, NUM_ACTIONS), dtype=torch.int32, device=dev)
        actions = torch.empty(n, dtype=torch.uint8, device=dev)
        t = self.temperature
        mode, temp = (0, 1.0) if t is None else ((1, 1.0) if np.isinf(t) else (2, float(t)))
        _check(L.dk_az_finish_async(ctx, mode, temp, visits.data_ptr(), actions.data_ptr(), st))
        if rng_states is not None:
            _check(L.dk_az_rng_async(ctx, rng_states.data_ptr(), 0, st))
        _check(L.dk_sync(ctx, st))
        return actions, visits


class ARSampling:
    """The ARSampling SamplingFn (rs-doko-py-bridge/src/compare_impi/compare_impi.rs:84-105):
    forward_pred_process_with_mask (rs-doko-impi/src/forward.rs:392-661) for `samples`
    draws of every infostate at once.  Each network call of the reference (one card or
    one hidden reservation of one player) is one row of a batched network evaluation;
    all lanes advance in lockstep rounds between two kernels (engine/ar_engine.h).

    network(tokens) -> logits: tokens = int32 [n, 311] encode_state_ipi rows on the GPU,
    logits = float [n, 33] (ImperfectInformationOutput order: 9 reservations, 24 cards).
    log_chance: the probability of the reference's log-file draw (one u64 per sample)."""

    def __init__(self, engine, network, temperature=1.0, log_chance=1.0 / 30000.0):
        self.engine = engine
        self.network = network
        self.temperature = float(temperature)
        self.log_chance = float(log_chance)
        self.rounds = 0   # network rounds of the last sample() call
        self.rows = 0     # network rows evaluated in it (the sum of the guesses, early stops aside)

    def sample(self, infostates, samples, seeds):
        """infostates: uint8 [n_info, 160] dk_az_state records (GPU); seeds: uint64 [n_info * samples].
        Returns (states uint8 [n, 128], status uint8 [n], reason uint8 [n]) with n = n_info * samples,
        lane = info * samples + sample; status AR_CONSISTENT rows hold the sample, the others the
        infostate (AR_NOT_CONSISTENT: reason = index into NOT_CONSISTENT_REASONS)."""
        return _run_on_stream(infostates.device, self._sample, infostates, samples, seeds)

    def _sample(self, infostates, samples, seeds, st):
        rounds = self._sample_rounds(infostates, samples, seeds, st)
        while True:
            try:
                next(rounds)
            except StopIteration as done:
                return done.value

    def _sample_rounds(self, infostates, samples, seeds, st, sync=True):
        """_sample as a generator that yields after each network round's launches (sample_interleaved,
        which synchronises the parts itself: sync=False)."""
        import torch
        L = _native.lib()
        ctx = self.engine.ctx
        info = infostates.contiguous()
        dev = info.device
        n_info = info.shape[0]
        n = n_info * samples
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        if seeds.shape[0] != n:
            raise ValueError("need one seed per (infostate, sample)")
        # order the infostates by descending number of guesses: the rows of round r are
        # then the prefix of lanes whose infostate needs more than r guesses
        counts = torch.empty(n_info, dtype=torch.int32, device=dev)
        _check(L.dk_ar_guesses_async(ctx, info.data_ptr(), n_info, counts.data_ptr(), st))
        counts = counts.cpu().numpy()
        order = np.argsort(-counts, kind="stable")
        sorted_counts = counts[order]
        info_s = info[torch.as_tensor(order, device=dev)].contiguous()
        seeds_s = seeds.reshape(n_info, samples)[order].reshape(-1)
        seeds_t = torch.as_tensor(seeds_s.view(np.int64), device=dev)
        rounds = torch.zeros(1, dtype=torch.int32, device=dev)
        tokens = torch.zeros((n, IPI_TOKENS), dtype=torch.int32, device=dev)
        _check(L.dk_ar_begin_async(ctx, info_s.data_ptr(), n_info, samples, seeds_t.data_ptr(), self.log_chance,
                                   rounds.data_ptr(), st))
        self.rounds = int(sorted_counts[0]) if n_info else 0
        self.rows = 0
        for r in range(self.rounds):
            rows = samples * int(np.count_nonzero(sorted_counts > r))
            _check(L.dk_ar_prepare_async(ctx, tokens.data_ptr(), st))
            logits = self.network(tokens[:rows]).float().contiguous()
            _check(L.dk_ar_choose_async(ctx, logits.data_ptr(), self.temperature, st))
            self.rows += rows
            yield r
        _check(L.dk_ar_prepare_async(ctx, tokens.data_ptr(), st))
        out_s = torch.empty((n, STATE_BYTES), dtype=torch.uint8, device=dev)
        status_s = torch.empty(n, dtype=torch.uint8, device=dev)
        reason_s = torch.empty(n, dtype=torch.uint8, device=dev)
        _check(L.dk_ar_output_async(ctx, out_s.data_ptr(), status_s.data_ptr(), reason_s.data_ptr(), st))
        inv = torch.as_tensor(np.argsort(order), device=dev)
        out = out_s.view(n_info, samples, STATE_BYTES)[inv].reshape(n, STATE_BYTES)
        status = status_s.view(n_info, samples)[inv].reshape(n)
        reason = reason_s.view(n_info, samples)[inv].reshape(n)
        if sync:
            _check(L.dk_sync(ctx, st))
        return out, status, reason


def sample_interleaved(parts):
    """Several independent ARSampling.sample calls whose network rounds are issued interleaved:
    parts = [(sampler, stream, infostates, samples, seeds)], each sampler on its own Engine (the
    AR state lives in the engine) and its own torch stream, so one part's kernels fill the tails
    of the others'.  Every part's result equals its sampler.sample(...) alone (lanes are
    independent and the networks row-wise).  The caller's stream waits for every part.
    Returns [(states, status, reason)] in part order."""
    import torch
    if not parts:
        return []
    dev = parts[0][2].device
    caller = torch.cuda.current_stream(dev)
    gens, outs = [], [None] * len(parts)
    for sampler, stream, info, samples, seeds in parts:
        stream.wait_stream(caller)
        with torch.cuda.stream(stream):
            gens.append(sampler._sample_rounds(info, samples, seeds, stream.cuda_stream, sync=False))
    live = list(range(len(parts)))
    while live:
        for k in list(live):
            with torch.cuda.stream(parts[k][1]):
                try:
                    next(gens[k])
                except StopIteration as done:
                    outs[k] = done.value
                    live.remove(k)
    for k, (sampler, stream, *_r) in enumerate(parts):
        _check(_native.lib().dk_sync(sampler.engine.ctx, stream.cuda_stream))
        caller.wait_stream(stream)
        for t in outs[k]:
            t.record_stream(caller)
    return outs


def _stream(t):
    """The caller's torch stream handle.  Handle 0 (torch's default stream) would select the
    library's own stream, which is not ordered after the caller's queued work: wait for that
    work first (the callers then dk_sync before returning)."""
    import torch
    st = torch.cuda.current_stream(t.device)
    if st.cuda_stream == 0:
        st.synchronize()
    return st.cuda_stream


def az_records(engine, states):
    """dk_az_state records (uint8 [n, 160], GPU) of packed rs-full-doko states without
    announcements (new games): the AlphaZero game records."""
    import torch
    states = states.contiguous()
    out = torch.empty((states.shape[0], AZ_STATE_BYTES), dtype=torch.uint8, device=states.device)
    st = _stream(states)
    _check(_native.lib().dk_az_records_async(engine.ctx, states.data_ptr(), states.shape[0], out.data_ptr(), st))
    _check(_native.lib().dk_sync(engine.ctx, st))
    return out


def az_step(engine, records, actions):
    """take_action_by_action_index(a, skip_single=true) (full_doko.rs:121-157) in place on
    every record whose action (uint8, GPU) is not 255: one self-play move."""
    st = _stream(records)
    _check(_native.lib().dk_az_step_async(engine.ctx, records.data_ptr(), actions.contiguous().data_ptr(),
                                          records.shape[0], st))
    _check(_native.lib().dk_sync(engine.ctx, st))
    return records


def az_encode(engine, records, out=None):
    """encode_state_pi (rs-doko-networks/src/full_doko/var1/encode_pi.rs:27-214) of each
    record: int32 [n, 311] tokens on the GPU (asynchronous on the current stream)."""
    import torch
    n = records.shape[0]
    if out is None:
        out = torch.empty((n, AZ_TOKENS), dtype=torch.int32, device=records.device)
    st = _stream(records)
    _check(_native.lib().dk_az_encode_async(engine.ctx, records.data_ptr(), n, out.data_ptr(), st))
    if st == 0:
        _check(_native.lib().dk_sync(engine.ctx, None))
    return out


# ---- state wire format from the reference's fields (host only; include/doko_amd.h) ----
class FdoFields(ctypes.Structure):
    """dk_fdo_fields: FdoState (rs-full-doko/src/state/state.rs:24-75) field by field."""
    _fields_ = [("hands", ctypes.c_uint64 * 4), ("player_eyes", ctypes.c_uint32 * 4),
                ("player_num_tricks", ctypes.c_uint32 * 4), ("res_start", ctypes.c_int8), ("res_len", ctypes.c_int8),
                ("reservations", ctypes.c_int8 * 4), ("n_tricks", ctypes.c_int8), ("trick_start", ctypes.c_int8 * 12),
                ("trick_cards", (ctypes.c_int8 * 4) * 12), ("ann_n", ctypes.c_int8),
                ("ann_card_index", ctypes.c_int8 * 12), ("ann_player", ctypes.c_int8 * 12),
                ("ann_announcement", ctypes.c_uint8 * 12), ("re_lowest", ctypes.c_uint8),
                ("contra_lowest", ctypes.c_uint8), ("ann_turns_without", ctypes.c_int8), ("ann_start", ctypes.c_int8),
                ("ann_allowed", ctypes.c_uint8), ("card_index", ctypes.c_int8), ("current_player", ctypes.c_int8),
                ("phase", ctypes.c_int8), ("rr_kind", ctypes.c_int8), ("rr_player", ctypes.c_int8),
                ("rr_reservation", ctypes.c_int8), ("game_type", ctypes.c_int8), ("team_kind", ctypes.c_int8),
                ("wedding_player", ctypes.c_int8), ("solved_trick", ctypes.c_int8), ("re_players", ctypes.c_uint8)]


class DoFields(ctypes.Structure):
    """dk_do_fields: DoState (rs-doko/src/state/state.rs:28-76) field by field."""
    _fields_ = [("hands", ctypes.c_uint64 * 4), ("player_eyes", ctypes.c_uint32 * 4),
                ("player_num_tricks", ctypes.c_uint32 * 4), ("res_start", ctypes.c_int8),
                ("reservations", ctypes.c_int8 * 4), ("trick_start", ctypes.c_int8 * 12),
                ("trick_cards", (ctypes.c_int8 * 4) * 12), ("current_player", ctypes.c_int8), ("phase", ctypes.c_int8),
                ("trick_index", ctypes.c_int8), ("rr_kind", ctypes.c_int8), ("rr_player", ctypes.c_int8),
                ("team_kind", ctypes.c_int8), ("wedding_player", ctypes.c_int8), ("solved_trick", ctypes.c_int8),
                ("re_players", ctypes.c_uint8)]


def fdo_from_fields(fields):
    """dk_fdo_from_fields: the 128-B packed state (bytes) of an FdoFields; DokoError on inconsistent fields."""
    out = (ctypes.c_uint8 * STATE_BYTES)()
    _check(_native.lib().dk_fdo_from_fields(ctypes.byref(fields), out))
    return bytes(out)


def fdo_to_fields(packed):
    f = FdoFields()
    buf = (ctypes.c_uint8 * STATE_BYTES).from_buffer_copy(bytes(packed))
    _check(_native.lib().dk_fdo_to_fields(buf, ctypes.byref(f)))
    return f


def do_from_fields(fields):
    """dk_do_from_fields: the 128-B packed rs-doko state (bytes) of a DoFields."""
    out = (ctypes.c_uint8 * STATE_BYTES)()
    _check(_native.lib().dk_do_from_fields(ctypes.byref(fields), out))
    return bytes(out)


def do_to_fields(packed):
    f = DoFields()
    buf = (ctypes.c_uint8 * STATE_BYTES).from_buffer_copy(bytes(packed))
    _check(_native.lib().dk_do_to_fields(buf, ctypes.byref(f)))
    return f
