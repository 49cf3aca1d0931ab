"""ctypes wrapper of the ORACLE (oracle/liboracle_doko.so) — test infrastructure only.

Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by
the product package.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
# ORACLE_LIB: another build of the restatement (the sanitizer build, oracle/_asan/)
LIB_PATH = os.environ.get("ORACLE_LIB") or os.path.join(ORACLE_DIR, "liboracle_doko.so")

_lib = None

u64p = ctypes.POINTER(ctypes.c_uint64)
u32p = ctypes.POINTER(ctypes.c_uint32)
i32p = ctypes.POINTER(ctypes.c_int32)
f64p = ctypes.POINTER(ctypes.c_double)
f32p = ctypes.POINTER(ctypes.c_float)
u8p = ctypes.POINTER(ctypes.c_uint8)
vp = ctypes.c_void_p


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "or_rng_seed": (None, [ctypes.c_uint64, u64p]),
            "or_rng_next_u64": (ctypes.c_uint64, [u64p]),
            "or_rng_range_u32": (ctypes.c_uint32, [u64p, ctypes.c_uint32, ctypes.c_uint32]),
            "or_rng_choose_unsized": (ctypes.c_int, [u64p, ctypes.c_uint32]),
            "or_select_by_rank": (ctypes.c_uint64, [ctypes.c_uint64, ctypes.c_uint64]),
            "or_fdo_new_game": (vp, [ctypes.c_uint64]),
            "or_fdo_from_hands": (vp, [u64p, ctypes.c_int]),
            "or_fdo_clone": (vp, [vp]),
            "or_fdo_free": (None, [vp]),
            "or_fdo_play": (None, [vp, ctypes.c_int]),
            "or_fdo_allowed": (ctypes.c_uint64, [vp]),
            "or_fdo_env_allowed": (ctypes.c_uint64, [vp, ctypes.c_int]),
            "or_fdo_hands": (None, [vp, u64p]),
            "or_fdo_info": (None, [vp, i32p]),
            "or_fdo_pack": (None, [vp, u8p]),
            "or_fdo_fields": (None, [vp, vp]),
            "or_do_fields": (None, [vp, vp]),
            "or_fdo_random_plies": (ctypes.c_int, [vp, u64p, ctypes.c_int, ctypes.c_int]),
            "or_fdo_rollout": (None, [vp, u64p, f64p]),
            "or_fdo_rewards": (ctypes.c_int, [vp, f64p]),
            "or_fdo_search": (ctypes.c_int, [vp, u64p, ctypes.c_uint32, ctypes.c_double, u32p, f64p, u64p]),
            "or_fdo_card_matching": (vp, [vp, u64p]),
            "or_fdo_sample_consistent": (ctypes.c_int, [vp, vp]),
            "or_fdo_visible_reservations": (None, [vp, ctypes.c_int, i32p]),
            "or_fdo_calc_allowed_announcements": (ctypes.c_int, [ctypes.c_int] * 7),
            "or_fdo_card_to_color": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
            "or_fdo_is_greater": (ctypes.c_int, [ctypes.c_int] * 4),
            "or_fdo_search_many": (ctypes.c_double, [vp, ctypes.POINTER(vp), u64p, ctypes.c_uint32, ctypes.c_uint32,
                                                     ctypes.c_double, u32p, ctypes.c_int]),
            "or_do_new_game": (vp, [ctypes.c_uint64]),
            "or_do_from_hands": (vp, [u64p, ctypes.c_int]),
            "or_do_clone": (vp, [vp]),
            "or_do_free": (None, [vp]),
            "or_do_play": (None, [vp, ctypes.c_int]),
            "or_do_allowed": (ctypes.c_uint64, [vp]),
            "or_do_hands": (None, [vp, u64p]),
            "or_do_info": (None, [vp, i32p]),
            "or_do_pack": (None, [vp, u8p]),
            "or_do_random_plies": (ctypes.c_int, [vp, u64p, ctypes.c_int]),
            "or_do_rollout": (None, [vp, u64p, f64p]),
            "or_do_search": (ctypes.c_int, [vp, u64p, ctypes.c_uint32, ctypes.c_double, u32p, f64p, u64p]),
            "or_do_search_many": (ctypes.c_double, [ctypes.POINTER(vp), u64p, ctypes.c_uint32, ctypes.c_uint32,
                                                    ctypes.c_double, u32p, ctypes.c_int]),
            "or_do_remaining_cards": (ctypes.c_uint64, [i32p, ctypes.c_uint64]),
            "or_do_allowed_to_have": (None, [ctypes.c_int, i32p, ctypes.c_uint64, ctypes.c_int, i32p, i32p]),
            "or_do_sample_assignment": (ctypes.c_int, [ctypes.c_int, i32p, ctypes.c_uint64, i32p, ctypes.c_int,
                                                       u64p, u64p]),
            "or_do_sample_full": (vp, [vp, u64p]),
            "or_az_hash_eval": (None, [u8p, f32p, f32p]),
            "or_az_search": (ctypes.c_int, [vp, f32p, ctypes.c_float, ctypes.c_uint32, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_float, u64p, u32p, f32p]),
            "or_dirichlet": (ctypes.c_int, [ctypes.c_float, ctypes.c_int, ctypes.c_uint32, u64p, f32p]),
            "or_gamma": (None, [ctypes.c_float, ctypes.c_uint32, u64p, f32p]),
            "or_beta": (None, [ctypes.c_float, ctypes.c_float, ctypes.c_uint32, u64p, f32p]),
            "or_libm_f32": (None, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, f32p]),
            "or_normal_f64": (None, [ctypes.c_uint32, u64p, f64p]),
            "or_exp1_f64": (None, [ctypes.c_uint32, u64p, f64p]),
            "or_ziggurat_tables": (None, [f64p]),
            "or_az_take_action": (None, [vp, ctypes.c_int]),
            "or_encode_pi": (None, [vp, ctypes.POINTER(ctypes.c_int64)]),
            "or_fdo_pack_az": (None, [vp, u8p]),
            "or_encode_pi_fields": (None, [i32p, u64p, ctypes.POINTER(ctypes.c_int64)]),
            "or_encode_ipi_fields": (ctypes.c_int, [i32p, u64p, u64p, i32p, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
            "or_ipi_encode": (ctypes.c_int, [vp, u64p, i32p, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]),
            "or_ipi_next_card": (ctypes.c_uint64, [vp, u64p, i32p, ctypes.c_int]),
            "or_ipi_next_reservation": (ctypes.c_uint32, [vp, u64p, ctypes.c_int]),
            "or_ipi_consistent": (ctypes.c_int, [vp, u64p, i32p]),
            "or_ipi_hash_eval": (None, [ctypes.POINTER(ctypes.c_int64), f32p]),
            "or_ipi_sample_state": (vp, [vp, u64p, ctypes.c_float, ctypes.c_float, i32p, i32p]),
            "or_fdo_random_single": (ctypes.c_uint64, [ctypes.c_uint64, u64p]),
            "or_ipi_sample": (ctypes.c_int, [vp, u64p, ctypes.c_float, ctypes.c_float, i32p, u8p, i32p]),
            "or_ttt_finish": (ctypes.c_int, [i32p]),
            "or_ttt_rollout": (None, [i32p, u64p, f64p]),
            "or_ttt_search": (ctypes.c_int, [i32p, u64p, ctypes.c_uint32, ctypes.c_double, u32p, f64p]),
            "or_ttt_pack": (None, [i32p, ctypes.c_int, u8p]),
            "or_fuse_maxn": (ctypes.c_int, [u32p, ctypes.c_int, ctypes.c_uint64, u32p]),
            "or_fuse_avg": (ctypes.c_int, [u32p, ctypes.c_int, f32p]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def arr(ctype, n, init=None):
    a = (ctype * n)()
    if init is not None:
        for i, v in enumerate(init):
            a[i] = v
    return a


def rng_seed(seed):
    s = arr(ctypes.c_uint64, 4)
    lib().or_rng_seed(seed, s)
    return s


class FdoState:
    """Handle to an oracle FdoState (rs-full-doko/src/state/state.rs:24-75)."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def new_game(cls, seed):
        return cls(lib().or_fdo_new_game(seed))

    @classmethod
    def from_hands(cls, hands, start):
        return cls(lib().or_fdo_from_hands(arr(ctypes.c_uint64, 4, hands), start))

    def clone(self):
        return FdoState(lib().or_fdo_clone(self.h))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.or_fdo_free(self.h)
            self.h = None

    def play(self, a):
        lib().or_fdo_play(self.h, a)

    def allowed(self):
        return lib().or_fdo_allowed(self.h)

    def env_allowed(self, first):
        return lib().or_fdo_env_allowed(self.h, 1 if first else 0)

    def hands(self):
        o = arr(ctypes.c_uint64, 4)
        lib().or_fdo_hands(self.h, o)
        return list(o)

    def info(self):
        o = arr(ctypes.c_int32, 40)
        lib().or_fdo_info(self.h, o)
        o = list(o)
        return {"phase": o[0], "current_player": o[1], "game_type": o[2], "eyes": o[3:7], "re_lowest": o[7],
                "contra_lowest": o[8], "has_stats": o[9], "player_points": o[10:14], "re_eyes": o[14],
                "kontra_eyes": o[15], "re_points": o[16], "kontra_points": o[17], "is_solo": o[18],
                "n_tricks": o[19], "trick_winners": o[20:32], "re_players": o[32], "card_index": o[33],
                "team_kind": o[34], "ann_turns": o[35], "ann_allowed": o[36], "n_ann": o[37]}

    def pack(self):
        o = arr(ctypes.c_uint8, 128)
        lib().or_fdo_pack(self.h, o)
        return bytes(o)

    def random_plies(self, rng, k, no_announcement=True):
        return lib().or_fdo_random_plies(self.h, rng, k, 1 if no_announcement else 0)

    def rollout(self, rng):
        o = arr(ctypes.c_double, 4)
        lib().or_fdo_rollout(self.h, rng, o)
        return list(o)

    def search(self, rng, iters, c):
        v = arr(ctypes.c_uint32, 39)
        val = arr(ctypes.c_double, 39)
        ctr = arr(ctypes.c_uint64, 8)
        best = lib().or_fdo_search(self.h, rng, iters, c, v, val, ctr)
        return best, list(v), list(val), list(ctr)

    def card_matching(self, rng):
        return FdoState(lib().or_fdo_card_matching(self.h, rng))

    def az_search(self, noise, iters, c, eps, epoch, temp_mode, temp, rng, alpha=0.8):
        """AlphaZero mcts_search (async_mcts.rs:224-406) with the synthetic hash
        network of oracle/az_eval.hpp -> (action, visits[39], root priors[39]).
        noise None: the search draws Dirichlet([alpha; 39]) from rng (rand_distr05.hpp)."""
        v = arr(ctypes.c_uint32, 39)
        pr = arr(ctypes.c_float, 39, [-1.0] * 39)
        nz = None if noise is None else arr(ctypes.c_float, 39, noise)
        a = lib().or_az_search(self.h, nz, ctypes.c_float(alpha), iters, c, eps, epoch, temp_mode, temp, rng, v, pr)
        return a, list(v), list(pr)

    def pack_az(self):
        """dk_az_state record (160 B): packed state + announcement occurrence list."""
        o = arr(ctypes.c_uint8, 160)
        lib().or_fdo_pack_az(self.h, o)
        return bytes(o)

    def encode_pi(self):
        """encode_state_pi (rs-doko-networks/src/full_doko/var1/encode_pi.rs:27-214) -> 311 tokens."""
        o = arr(ctypes.c_int64, 311)
        lib().or_encode_pi(self.h, o)
        return list(o)

    def ipi_encode(self, hands, res, guess):
        """encode_state_ipi (rs-doko-networks/src/full_doko/var1/encode_ipi.rs:48-282) -> 311 tokens
        (None where the reference panics)."""
        o = arr(ctypes.c_int64, 311)
        ok = lib().or_ipi_encode(self.h, arr(ctypes.c_uint64, 4, hands), arr(ctypes.c_int32, 4, res), guess, o)
        return list(o) if ok else None

    def ipi_next_card(self, hands, res, p):
        """next_possible_card (rs-doko-impi/src/next_consistent.rs:25-139) -> FdoHand bits."""
        return lib().or_ipi_next_card(self.h, arr(ctypes.c_uint64, 4, hands), arr(ctypes.c_int32, 4, res), p)

    def ipi_next_reservation(self, hands, p):
        """next_possible_reservation (next_consistent.rs:141-193) -> bit set over FdoReservation."""
        return lib().or_ipi_next_reservation(self.h, arr(ctypes.c_uint64, 4, hands), p)

    def ipi_consistent(self, hands, res):
        """_is_consistent (rs-full-doko/src/matching/is_consistent.rs:38-305) -> reason or -1."""
        return lib().or_ipi_consistent(self.h, arr(ctypes.c_uint64, 4, hands), arr(ctypes.c_int32, 4, res))

    def ipi_sample(self, rng, temperature, log_chance=1.0 / 30000.0):
        """forward_pred_process_with_mask (rs-doko-impi/src/forward.rs:392-661) with the hash
        network -> (status, reason, packed sample or None, network evaluations)."""
        reason = arr(ctypes.c_int32, 1)
        g = arr(ctypes.c_int32, 1)
        o = arr(ctypes.c_uint8, 128)
        st = lib().or_ipi_sample(self.h, rng, temperature, log_chance, reason, o, g)
        return st, reason[0], (bytes(o) if st == 0 else None), g[0]

    def ipi_sample_state(self, rng, temperature, log_chance=1.0 / 30000.0):
        """forward_pred_process_with_mask with the hash network -> (status, reason, FdoState or None)."""
        st = arr(ctypes.c_int32, 1)
        rs = arr(ctypes.c_int32, 1)
        h = lib().or_ipi_sample_state(self.h, rng, temperature, log_chance, st, rs)
        return st[0], rs[0], (FdoState(h) if h else None)

    def az_take_action(self, a):
        """FdoAzEnvState::take_action_by_action_index(a, skip_single=true)."""
        lib().or_az_take_action(self.h, a)

    def consistent_sample(self, sample):
        return bool(lib().or_fdo_sample_consistent(self.h, sample.h))


class DoState:
    """Handle to an oracle DoState (rs-doko/src/state/state.rs:28-76)."""

    def __init__(self, handle):
        self.h = handle

    @classmethod
    def new_game(cls, seed):
        return cls(lib().or_do_new_game(seed))

    @classmethod
    def from_hands(cls, hands, start):
        return cls(lib().or_do_from_hands(arr(ctypes.c_uint64, 4, hands), start))

    def clone(self):
        return DoState(lib().or_do_clone(self.h))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.or_do_free(self.h)
            self.h = None

    def play(self, a):
        lib().or_do_play(self.h, a)

    def allowed(self):
        return lib().or_do_allowed(self.h)

    def hands(self):
        o = arr(ctypes.c_uint64, 4)
        lib().or_do_hands(self.h, o)
        return list(o)

    def info(self):
        o = arr(ctypes.c_int32, 32)
        lib().or_do_info(self.h, o)
        o = list(o)
        return {"phase": o[0], "current_player": o[1], "eyes": o[2:6], "has_stats": o[6], "player_points": o[7:11],
                "re_eyes": o[11], "kontra_eyes": o[12], "re_points": o[13], "kontra_points": o[14],
                "trick_index": o[15], "trick_winners": o[16:28], "re_players": o[28]}

    def pack(self):
        o = arr(ctypes.c_uint8, 128)
        lib().or_do_pack(self.h, o)
        return bytes(o)

    def random_plies(self, rng, k):
        return lib().or_do_random_plies(self.h, rng, k)

    def rollout(self, rng):
        o = arr(ctypes.c_double, 4)
        lib().or_do_rollout(self.h, rng, o)
        return list(o)

    def sample_assignment_full(self, rng):
        """rs-doko-assignment sample_assignment_full for the current player's
        observation (assignment.rs:472-505); None where the reference panics."""
        h = lib().or_do_sample_full(self.h, rng)
        return DoState(h) if h else None

    def search(self, rng, iters, c):
        v = arr(ctypes.c_uint32, 39)
        val = arr(ctypes.c_double, 39)
        ctr = arr(ctypes.c_uint64, 8)
        best = lib().or_do_search(self.h, rng, iters, c, v, val, ctr)
        return best, list(v), list(val), list(ctr)


def _tricks_arr(tricks):
    flat = []
    for t in tricks:
        if t is None:
            flat += [-1, -1, -1, -1, -1]
        else:
            cs = list(t["cards"]) + [-1] * (4 - len(t["cards"]))
            flat += [t["start"]] + cs
    return arr(ctypes.c_int32, 60, flat)


def do_remaining_cards(tricks, hand):
    """assignment.rs:13-39 (tricks: 12 x None | {"start", "cards"})."""
    return lib().or_do_remaining_cards(_tricks_arr(tricks), hand)


def do_allowed_to_have(marriage, tricks, hand, observer):
    """assignment.rs:79-287 -> four card lists in the reference's order."""
    out = arr(ctypes.c_int32, 4 * 48)
    lens = arr(ctypes.c_int32, 4)
    lib().or_do_allowed_to_have(marriage, _tricks_arr(tricks), hand, observer, out, lens)
    return [list(out[48 * i:48 * i + lens[i]]) for i in range(4)]


def do_sample_assignment(marriage, tricks, hand, lengths, observer, rng):
    """assignment.rs:507-580 -> four hands (u64), or None where the reference panics."""
    out = arr(ctypes.c_uint64, 4)
    ok = lib().or_do_sample_assignment(marriage, _tricks_arr(tricks), hand, arr(ctypes.c_int32, 4, lengths),
                                       observer, rng, out)
    return list(out) if ok else None


def ttt_pack(board, last_action=-1):
    o = arr(ctypes.c_uint8, 128)
    lib().or_ttt_pack(arr(ctypes.c_int32, 9, board), last_action, o)
    return bytes(o)


def ttt_search(board, rng, iters, c):
    v = arr(ctypes.c_uint32, 39)
    val = arr(ctypes.c_double, 39)
    best = lib().or_ttt_search(arr(ctypes.c_int32, 9, board), rng, iters, c, v, val)
    return best, list(v), list(val)


def fuse_maxn(visits_rows, allowed):
    S = len(visits_rows)
    flat = arr(ctypes.c_uint32, 39 * S, [x for row in visits_rows for x in row])
    ranks = arr(ctypes.c_uint32, 39)
    return lib().or_fuse_maxn(flat, S, allowed, ranks), list(ranks)


def fuse_avg(visits_rows):
    S = len(visits_rows)
    flat = arr(ctypes.c_uint32, 39 * S, [x for row in visits_rows for x in row])
    probs = arr(ctypes.c_float, 39)
    return lib().or_fuse_avg(flat, S, probs), list(probs)


def az_hash_eval_np(packed):
    """numpy twin of oracle/az_eval.hpp hash_eval: (n, 128) uint8 -> value (n, 4), logits (n, 39) float32."""
    import numpy as np
    b = np.asarray(packed, dtype=np.uint8)
    h = np.full(b.shape[0], 0xCBF29CE484222325, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for i in range(117):
            h ^= b[:, i].astype(np.uint64)
            h *= np.uint64(0x100000001B3)
        value = np.stack([((h >> np.uint64(8 * k)) & np.uint64(15)).astype(np.int64) - 8 for k in range(4)], axis=1)
        logits = []
        for a in range(39):
            z = h + np.uint64(a) + np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            logits.append((z & np.uint64(31)).astype(np.int64) - 16)
    return (value.astype(np.float32) * np.float32(0.125)), (np.stack(logits, axis=1).astype(np.float32) * np.float32(0.25))


def _state_fields(res_start, res, tricks, announcements, current_player, phase, re_players):
    f = [0] * 119
    f[0], f[1] = res_start, len(res)
    for i, r in enumerate(res):
        f[2 + i] = r
    f[6] = len(tricks)
    for t, tr in enumerate(tricks):
        cs = list(tr["cards"]) + [-1] * (4 - len(tr["cards"]))
        f[7 + 6 * t:13 + 6 * t] = [tr["start"], len(tr["cards"])] + cs
    f[79] = len(announcements)
    for k, a in enumerate(announcements):
        f[80 + 3 * k:83 + 3 * k] = [a["card_index"], a["player"], a["bit"]]
    f[116], f[117], f[118] = current_player, phase, re_players
    return arr(ctypes.c_int32, 119, f)


def encode_pi_fields(res_start, res, tricks, hands, announcements, current_player, phase, re_players):
    """encode_state_pi of a state given by the fields the encoder reads (the encode_pi.rs test layout)."""
    o = arr(ctypes.c_int64, 311)
    lib().or_encode_pi_fields(_state_fields(res_start, res, tricks, announcements, current_player, phase, re_players),
                              arr(ctypes.c_uint64, 4, hands), o)
    return list(o)


def encode_ipi_fields(res_start, res, tricks, hands, announcements, current_player, phase, re_players,
                      assumed_hands, assumed_res, guess):
    """encode_state_ipi of a state given by its fields (the encode_ipi.rs test layout)."""
    o = arr(ctypes.c_int64, 311)
    ok = lib().or_encode_ipi_fields(_state_fields(res_start, res, tricks, announcements, current_player, phase, re_players),
                                    arr(ctypes.c_uint64, 4, hands), arr(ctypes.c_uint64, 4, assumed_hands),
                                    arr(ctypes.c_int32, 4, assumed_res), guess, o)
    return list(o) if ok else None


def random_single(mask, rng):
    """Bitflag::random_single (rs-game-utils/src/bit_flag.rs:86-92) -> the chosen bit."""
    return lib().or_fdo_random_single(mask, rng)


def ipi_hash_eval_np(tokens):
    """The oracle's synthetic IMPI network (oracle/impi.hpp hash_eval) over [n, 311] tokens -> [n, 33] f32."""
    import numpy as np
    t = np.ascontiguousarray(tokens, dtype=np.int64).reshape(-1, 311)
    out = np.zeros((t.shape[0], 33), dtype=np.float32)
    for i in range(t.shape[0]):
        lib().or_ipi_hash_eval(t[i].ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                               out[i].ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return out
