"""The HIP engine pinned directly to the reference's rule KATs (rule_kats_*.json).

tests/test_rule_kats.py checks the oracle against these vectors; here the same
positions go through the device engine via the C-ABI (dk_*_from_fields to build the
position, dk_env_step_batch / dk_env_allowed_batch / dk_env_rewards_batch /
dk_is_consistent_batch on the GPU) and must give the reference's expected values:

  card order     every KAT line (card/card_in_trick_logic.rs:226-1023) whose trick colour is
                 the colour of the earlier card in that game type -- the situations a game can
                 reach -- as a real trick [earlier card, later card, two off-colour fillers]
                 played on the device: the later card takes the trick iff the KAT says greater
  trick winners  trick/trick_winning_player_logic.rs:48-108
  teams          team/team_logic.rs:155-385: the reservation round and the tricks of each KAT
                 played on the device
  allowed announcements  calc_announcement.rs:232-300: the round the device opens after a card
  announcement rounds    announcement.rs:219-573: reservation end, then the KAT's announcements
  scoring        stats/stats.rs:245-778 as finished states -> rewards = player_points
  is_consistent  matching/is_consistent.rs:318-888 (dk_is_consistent_batch)
  rs-doko        allowed_actions.rs:210-312, teams/team_logic.rs:145-333, stats/stats.rs:144-238
"""
import ctypes

import numpy as np
import pytest

import oracle_lib as ol
from test_rule_kats import DO, FDO, arr, fdo_hand, kat_lib, replay

pytestmark = pytest.mark.gpu

# FdoGameType -> the FdoReservation that announces it (reservation_winning_logic.rs:16-33)
SOLO_RES = {2: 2, 3: 3, 4: 4, 5: 5, 6: 8, 7: 6, 8: 7}
CTC = {(k["card"], k["game_type"]): k["color"] for k in FDO["card_to_color"]}   # reference card_to_color table


@pytest.fixture(scope="module")
def eng():
    import master_doko_reinforcement_learning_amd as dk
    e = dk.Engine(device=0, max_roots=64, max_iterations=10)
    yield e
    e.close()


def ANN_TO_ACTION(bit):
    """FdoAnnouncement bit -> FdoAction (action/action.rs:295-310)."""
    return {1: 33, 2: 34, 4: 35, 8: 36, 16: 37, 64: 38}[bit]


def packed(rows):
    return np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(-1, 128).copy()


def winners(states):
    return states[:, 88:92].copy().view(np.uint32)[:, 0]


def base_fields(game_type, start):
    """PlayCard position at the start of trick 0 of `game_type`, reservations done."""
    import master_doko_reinforcement_learning_amd as dk
    f = dk.FdoFields()
    f.res_start = start
    f.res_len = 4
    res = [0, 0, 0, 0]
    if game_type == 1:
        res[0] = 1
        f.rr_kind, f.rr_player, f.team_kind, f.wedding_player = 2, start, 1, start
    elif game_type >= 2:
        res[0] = SOLO_RES[game_type]
        f.rr_kind, f.rr_player, f.rr_reservation, f.team_kind, f.re_players = 1, start, SOLO_RES[game_type], 3, 1 << start
    else:
        f.rr_kind, f.team_kind, f.re_players = 0, 3, 0b0101
    for i in range(4):
        f.reservations[i] = res[i]
    f.n_tricks = 1
    for t in range(12):
        f.trick_start[t] = -1
        for k in range(4):
            f.trick_cards[t][k] = -1
    f.trick_start[0] = start
    f.card_index = 0
    f.current_player = start
    f.phase = 2
    f.game_type = game_type
    f.ann_turns_without = 4
    f.ann_start = start
    return f


def play_tricks(eng, specs):
    """specs: (game_type, start, [c0..c3]) -> the device's trick winner of each."""
    import master_doko_reinforcement_learning_amd as dk
    rows = []
    for gt, start, cards in specs:
        f = base_fields(gt, start)
        for i, c in enumerate(cards):
            p = (start + i) % 4
            f.hands[p] = 1 << c                     # one card each: every play is legal
        rows.append(dk.fdo_from_fields(f))
    s = packed(rows)
    env = dk.McEnv(eng)
    for k in range(4):
        bits = np.array([1 << specs[i][2][k] for i in range(len(specs))], dtype=np.uint64)
        s = env.by_action(s, bits)
    return winners(s) & 3


def test_card_order_on_device(eng):
    specs, expect = [], []
    seen = set()
    for k in FDO["card_order"]:
        for gt in k["game_types"]:
            for col in k["colors"]:
                for prev in k["cards"]:
                    if CTC[(prev, gt)] != col or (gt, prev, k["cur"]) in seen:
                        continue
                    seen.add((gt, prev, k["cur"]))
                    fill = [x for x in range(24) if CTC[(x, gt)] not in (0, col) and x not in (prev, k["cur"])][:2]
                    if len(fill) < 2:
                        fill = fill * 2
                    specs.append((gt, 0, [prev, k["cur"], fill[0], fill[1]]))
                    expect.append(1 if k["greater"] else 0)
    got = play_tricks(eng, specs)
    bad = [(specs[i], expect[i], int(got[i])) for i in range(len(specs)) if got[i] != expect[i]]
    assert not bad, bad[:10]
    assert len(specs) > 1500 and {s[0] for s in specs} == set(range(9))


def test_trick_winners_on_device(eng):
    ks = [k for k in FDO["tricks"] if k["check"] == "winner"]
    assert ks
    got = play_tricks(eng, [(k["game_type"], k["start"], k["cards"]) for k in ks])
    for k, w in zip(ks, got):
        assert int(w) == k["expect"][0], k


def _reservation_position(hands, start, played):
    import master_doko_reinforcement_learning_amd as dk
    f = dk.FdoFields()
    for p in range(4):
        f.hands[p] = hands[p]
    f.res_start = start
    f.res_len = len(played)
    for i in range(4):
        f.reservations[i] = played[i] if i < len(played) else -1
    for t in range(12):
        f.trick_start[t] = -1
        for k in range(4):
            f.trick_cards[t][k] = -1
    f.current_player = (start + len(played)) % 4
    f.phase = 0
    f.rr_kind = -1
    f.game_type = -1
    return f


def test_team_resolution_on_device(eng):
    """The reservation round and the KAT's tricks played on the device; the team state it
    keeps must be the one FdoTeamState::resolve returns."""
    import master_doko_reinforcement_learning_amd as dk
    L = kat_lib()
    env = dk.McEnv(eng)
    checked = 0
    for k in FDO["team"]:
        if not _playable(L, k["tricks"], k["hands"]):
            continue                  # tricks that no game reaches (starts not the winners, a third copy)
        checked += 1
        rr = k["reservation_result"]
        hands = [list(h) for h in k["hands"]]
        for t in k["tricks"]:
            for i, c in enumerate(t[1:]):
                if c >= 0:
                    hands[(t[0] + i) % 4].append(c)
        actions = [24, 24, 24, 24]                           # start BOTTOM: B L T R
        if rr["kind"] == 2:
            actions[rr["player"]] = 25
        elif rr["kind"] == 1:
            actions[rr["player"]] = 24 + [0, 1, 2, 3, 4, 5, 7, 8, 6][rr["reservation"]]
        s = packed([dk.fdo_from_fields(_reservation_position([fdo_hand(L, h) for h in hands], 0, []))])
        for a in actions:
            s = env.by_action(s, np.array([1 << a], dtype=np.uint64))
        for t in k["tricks"]:
            for i, c in enumerate(t[1:]):
                f = dk.fdo_to_fields(s[0].tobytes())
                while f.phase == 1:                            # forced passes of announcement rounds
                    s = env.by_action(s, np.array([1 << 38], dtype=np.uint64))
                    f = dk.fdo_to_fields(s[0].tobytes())
                assert f.current_player == (t[0] + i) % 4, (k["test"], t, i)
                s = env.by_action(s, np.array([1 << c], dtype=np.uint64))
        f = dk.fdo_to_fields(s[0].tobytes())
        e = k["expect"]
        assert f.team_kind == e["kind"], k["test"]
        if e["kind"] != 1:
            assert all(f.re_players >> p & 1 for p in e["re_contains"]) and bin(f.re_players).count("1") == e["re_len"], k["test"]
        if e["wedding_player"] is not None:
            assert f.wedding_player == e["wedding_player"], k["test"]
        if e["solved"] is not None:
            assert f.solved_trick == e["solved"], k["test"]
    assert checked >= 4


def _playable(L, tricks, hands):
    """A KAT trick sequence a game can reach: every trick starts with the previous winner
    (the oracle's normal-game trick order, pinned by the trick KATs) and no card kind occurs
    more than twice."""
    count = [0] * 24
    for h in hands:
        for c in h:
            count[c] += 1
    prev = None
    for t in tricks:
        if prev is not None and t[0] != prev:
            return False
        out = (ctypes.c_int32 * 6)()
        L.or_kat_trick(arr(ctypes.c_int32, t), 0, out)
        prev = out[4]
        for c in t[1:]:
            count[c] += 1
    return max(count) <= 2


def test_allowed_announcements_on_device(eng):
    """calc_allowed_announcements KATs: the previous player plays a card, the device opens the
    announcement round at the KAT's player (hand of n_cards), whose offer must be the KAT set
    (an empty set: the device passes the round without stopping at that player)."""
    import master_doko_reinforcement_learning_amd as dk
    env = dk.McEnv(eng)
    ks = [k for k in FDO["calc_allowed"] if k["fn"] == "calc_allowed_announcements"]
    assert len(ks) == 4
    for k in ks:
        p, t = k["player"], k["team"]
        q = (p + 3) % 4
        f = base_fields(0, q)
        f.team_kind, f.re_players, f.wedding_player, f.solved_trick = t["kind"], t["re"], t["wedding_player"], t["solved"]
        f.re_lowest, f.contra_lowest = k["re_lowest"], k["contra_lowest"]
        hand = 0
        for c in range(k["n_cards"]):
            hand |= 1 << c
        f.hands[p] = hand
        f.hands[q] = 1 << 23                                 # the card q plays (not in p's hand)
        s = env.by_action(packed([dk.fdo_from_fields(f)]), np.array([1 << 23], dtype=np.uint64))
        g = dk.fdo_to_fields(s[0].tobytes())
        if k["expect"]:
            assert (g.phase, g.current_player, g.ann_allowed) == (1, p, k["expect"]), k
        else:
            assert g.phase == 2 and g.current_player == p, k


def test_announcement_rounds_on_device(eng):
    """announcement.rs rounds: the round the device opens when the reservations end (card_index
    0, the KAT's hand sizes; the club queens give the KAT's Re team), then the KAT's
    announcements stepped on the device; phase / player / counters / lowest announcements /
    offer after every step as the KAT states them."""
    import master_doko_reinforcement_learning_amd as dk
    env = dk.McEnv(eng)
    for k in FDO["ann_rounds"]:
        start = k["ops"][0]["op"][0]
        re = k["team"]["re"]
        hands = [0, 0, 0, 0]
        pool = [c for c in range(24) if c != 15] * 2
        for p in range(4):
            n = k["hand_lens"][p]
            cards = ([15] if re >> p & 1 else []) + [pool.pop() for _ in range(n - (1 if re >> p & 1 else 0))]
            for c in cards:
                hands[p] |= (1 << c) if not (hands[p] >> c & 1) else (1 << (c + 24))
        s = packed([dk.fdo_from_fields(_reservation_position(hands, start, [0, 0, 0]))])
        s = env.by_action(s, np.array([1 << 24], dtype=np.uint64))
        for i, o in enumerate(k["ops"]):
            if i > 0 and o["op"][1] == 32:
                # a CounterReContra is not an FdoAction: AnnouncementReContra records ReContra
                # (action/action.rs:295-310), so the env path diverges from the FdoAnnouncements-level
                # test here; the offers up to this point (which included it) were compared
                break
            if i > 0:
                s = env.by_action(s, np.array([1 << ANN_TO_ACTION(o["op"][1])], dtype=np.uint64))
            g = dk.fdo_to_fields(s[0].tobytes())
            c = o["checks"]
            ctx = (k["test"], i, c)
            if "result" in c:
                kind, player = c["result"]
                assert g.phase == (1 if kind == 0 else 2) and g.current_player == player, ctx
            if "n" in c:
                assert g.ann_n == c["n"], ctx
            if "starting_player" in c:
                assert g.ann_start == c["starting_player"], ctx
            if "turns" in c:
                assert g.ann_turns_without == c["turns"], ctx
            if "re_lowest" in c:
                assert g.re_lowest == c["re_lowest"], ctx
            if "contra_lowest" in c:
                assert g.contra_lowest == c["contra_lowest"], ctx
            if "allowed" in c:
                assert g.ann_allowed == c["allowed"], ctx


def _finished_fdo(k):
    """The stats KAT as a finished state.  The stats API takes no game type; the recorded
    tricks are used under the first FdoGameType whose trick order makes each trick start with
    the previous winner.  A solo's score reads no trick (extra points count in non-solo games
    only), and the solo KATs list tricks no game can reach (a third copy of a card), so a solo
    KAT's eyes / tricks won / teams / announcements sit on the tricks of a finished seeded game."""
    import master_doko_reinforcement_learning_amd as dk

    def fields(tricks, gt):
        f = dk.FdoFields()
        for p in range(4):
            f.player_eyes[p], f.player_num_tricks[p] = k["eyes"][p], k["ntricks"][p]
        f.res_start = tricks[0][0]
        f.res_len = 4
        f.n_tricks = 12
        for t, tr in enumerate(tricks):
            f.trick_start[t] = tr[0]
            for i in range(4):
                f.trick_cards[t][i] = tr[1 + i]
        f.re_lowest, f.contra_lowest = k["re_lowest"], k["contra_lowest"]
        f.card_index, f.current_player, f.phase, f.rr_kind, f.game_type = 48, -1, 3, 0, gt
        f.team_kind, f.re_players = 3, k["re_players"]
        return f

    for gt in range(9):
        try:
            return dk.fdo_from_fields(fields(k["tricks"], gt)), gt
        except dk.DokoError:
            continue
    if not k["expect"]["is_solo"]:
        return None, None     # extra points read these tricks, and no game reaches them
    g = ol.FdoState.new_game(11)
    for _ in range(4):
        g.play(24)
    g.random_plies(ol.rng_seed(11), 200, True)
    real = dk.fdo_to_fields(g.pack())
    tricks = [[real.trick_start[t]] + [real.trick_cards[t][i] for i in range(4)] for t in range(12)]
    return dk.fdo_from_fields(fields(tricks, real.game_type)), -1


def test_stats_on_device(eng):
    import master_doko_reinforcement_learning_amd as dk
    rows, exp = [], []
    unreachable = []
    for k in FDO["stats"]:
        row, gt = _finished_fdo(k)
        if row is None:
            # e.g. test_end_of_game_stats_normalspiel_kontra_verloren: trick 8 starts with LEFT
            # although RIGHT took trick 7, and every player_num_tricks is 0 -- checked on the
            # oracle only (tests/test_rule_kats.py::test_end_of_game_stats)
            unreachable.append(k["test"])
            continue
        if not k["expect"]["is_solo"]:
            assert gt in (0, 1), k["test"]        # extra points need the normal-game trick winners
        rows.append(row)
        exp.append(k["expect"]["player_points"])
    has, r = dk.McEnv(eng).rewards_or_none(packed(rows))
    assert has.all()
    assert r.astype(int).tolist() == exp
    assert len(rows) >= 2 and len(unreachable) <= 2, unreachable


def test_is_consistent_on_device(eng):
    from master_doko_reinforcement_learning_amd import _native
    L = kat_lib()
    recs, hands, res, exp = [], [], [], []
    for k in FDO["is_consistent"]:
        s = replay(L, k["start"], k["actions"])
        recs.append(s.pack_az())
        hands += [fdo_hand(L, h) for h in k["hands"]]
        r = [0xFF] * 4
        for i, x in enumerate(k["reservations"]):
            if x >= 0:
                r[(k["reservations_from"] + i) % 4] = x
        res += r
        exp.append(k["expect"])
    n = len(recs)
    rec = np.frombuffer(b"".join(recs), dtype=np.uint8).copy()
    h = np.array(hands, dtype=np.uint64)
    rr = np.array(res, dtype=np.uint8)
    out = np.zeros(n, dtype=np.uint8)
    rc = _native.lib().dk_is_consistent_batch(eng.ctx, rec.ctypes.data, h.ctypes.data, rr.ctypes.data, n, out.ctypes.data)
    assert rc == 0
    assert [bool(x == 0xFF) for x in out] == exp, list(out)


# ---------------------------------------------------------------- rs-doko
def _do_fields(hands, start, phase, current):
    import master_doko_reinforcement_learning_amd as dk
    f = dk.DoFields()
    for p in range(4):
        f.hands[p] = hands[p]
    f.res_start = start
    for t in range(12):
        f.trick_start[t] = -1
        for k in range(4):
            f.trick_cards[t][k] = -1
    f.current_player, f.phase = current, phase
    f.rr_kind = -1
    return f


def test_do_allowed_on_device(eng):
    """rs-doko legal actions: reservation phase from the KAT hand; card phase with the KAT's
    trick colour led by the previous player (♦9 trump, ♥9, ♠9, ♣9)."""
    import master_doko_reinforcement_learning_amd as dk
    L = kat_lib()
    env = dk.McEnv(eng)
    lead = {0: 0, 1: 6, 2: 18, 3: 12}
    n = 0
    for k in DO["allowed"]:
        h = 0
        for c in k["hand"]:
            h = L.or_kat_do_hand_add(h, c)
        if k["phase"] == 0:
            f = _do_fields([h, 0, 0, 0], 0, 0, 0)
            s = packed([dk.do_from_fields(f)])
        elif k["phase"] == 1:
            f = _do_fields([0, 0, 0, 0], 0, 1, 0)
            for i in range(4):
                f.reservations[i] = 1
            f.rr_kind, f.team_kind, f.re_players = 0, 3, 0b0101
            f.trick_start[0] = 0
            if k["trick_color"] < 0:
                f.hands[0] = h
                s = packed([dk.do_from_fields(f)])
            else:
                f.hands[0] = 1 << lead[k["trick_color"]]
                f.hands[1] = h
                s = env.by_action(packed([dk.do_from_fields(f)]), np.array([1 << lead[k["trick_color"]]], dtype=np.uint64))
        else:
            continue                                  # Finished: no actions (checked by the oracle test)
        got = env.allowed_actions(s, False)[0]
        assert [a for a in range(39) if int(got) >> a & 1] == sorted(k["expect"]), k
        n += 1
    assert n == 6


def test_do_stats_on_device(eng):
    """rs-doko scoring reads eyes, tricks won and the Re team: the KAT values on a finished
    rs-doko game (a seeded deal played out by the oracle)."""
    import master_doko_reinforcement_learning_amd as dk
    base = ol.DoState.new_game(7)
    base.random_plies(ol.rng_seed(7), 60)
    assert base.info()["phase"] == 2
    rows, exp = [], []
    for k in DO["stats"]:
        f = dk.do_to_fields(base.pack())
        for p in range(4):
            f.player_eyes[p], f.player_num_tricks[p] = k["eyes"][p], k["ntricks"][p]
        f.re_players = k["re_players"]
        rows.append(dk.do_from_fields(f))
        exp.append(k["expect"]["player_points"])
    has, r = dk.McEnv(eng).rewards_or_none(packed(rows))
    assert has.all() and r.astype(int).tolist() == exp
