"""The oracle against the reference's own rule-level unit tests.

tests/golden/make_rule_kats.py extracted every assertion of those tests into
rule_kats_fdo.json / rule_kats_do.json (inputs + expected outputs); each group below
feeds them through the oracle's restatement of the same function
(oracle/kats_capi.cpp) and must reproduce every expected value:

  card order (648 is_smaller / is_greater lines, all 9 game types)  card/card_in_trick_logic.rs:226-1023
  card colour (24 cards x 9 game types), colour masks, eyes        card/card_to_color.rs, card_color_masks.rs, card_to_eyes.rs
  trick colour / eyes / winner / next player                       trick/trick.rs, trick_winning_player_logic.rs
  team resolution                                                  team/team_logic.rs:155-385
  reservation winner, game type                                    reservation/reservation_winning_logic.rs
  allowed announcements (3 functions)                              announcement/calc_announcement.rs:232-516
  announcement rounds                                              announcement/announcement.rs:219-573
  DKV scoring and its building blocks                              stats/**
  is_consistent                                                    matching/is_consistent.rs:318-888
  rs-doko allowed actions, teams, scoring                          rs-doko/src/{action,teams,stats}
"""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle_lib as ol

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
i32, u32, u64 = ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64
I32P, U32P, U64P = ctypes.POINTER(i32), ctypes.POINTER(u32), ctypes.POINTER(u64)


def _load(name):
    with open(os.path.join(GOLD, name)) as fh:
        return json.load(fh)


FDO = _load("rule_kats_fdo.json")
DO = _load("rule_kats_do.json")


@pytest.fixture(scope="module")
def L():
    return kat_lib()


def kat_lib():
    lib = ol.lib()
    c = ctypes.c_int
    sigs = {
        "or_kat_card_eyes": (u32, [c]), "or_kat_color_masks": (None, [c, U64P]),
        "or_kat_trick": (None, [I32P, c, I32P]),
        "or_kat_team_resolve": (None, [c, c, c, I32P, c, U64P, I32P]),
        "or_kat_reservation_winner": (None, [c, I32P, c, I32P]), "or_kat_game_type_of": (c, [c, c, c]),
        "or_kat_all_higher_than": (u32, [c]), "or_kat_calc_allowed": (u32, [c] * 8),
        "or_kat_internal_calc_allowed": (u32, [c, u32, c, c]), "or_kat_cards_last_announcement": (c, [u32, c]),
        "or_kat_announcement_round": (None, [I32P, c, c, c, c, c, I32P, c, I32P]),
        "or_kat_stats": (None, [U32P, U32P, c, c, c, I32P, c, I32P]),
        "or_kat_re_won": (c, [u32, u32, u32, c, c]), "or_kat_kontra_won": (c, [u32, u32, u32, c, c]),
        "or_kat_basic_winning": (None, [u32, u32, c, u32, u32, u32, u32, I32P]),
        "or_kat_basic_draw": (None, [u32, u32, u32, u32, I32P]),
        "or_kat_additional": (None, [c, c, I32P, c, I32P]),
        "or_kat_do_allowed": (u64, [c, c, u64]), "or_kat_do_team_resolve": (None, [c, I32P, U64P, I32P]),
        "or_kat_do_stats": (None, [c, U32P, U32P, I32P]),
        "or_kat_do_hand_add": (u64, [u64, c]), "or_kat_fdo_hand_add": (u64, [u64, c]),
        "or_fdo_is_greater": (c, [c] * 4), "or_fdo_card_to_color": (c, [c, c]),
        "or_ipi_consistent": (c, [ctypes.c_void_p, U64P, I32P]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def arr(ct, xs):
    return (ct * len(xs))(*xs)


def tricks_arr(tricks):
    flat = [x for t in tricks for x in t] or [0]
    return arr(i32, flat)


def fdo_hand(L, cards):
    h = 0
    for c in cards:
        h = L.or_kat_fdo_hand_add(h, c)
    return h


def annset(L, s):
    return s["bits"] if "bits" in s else L.or_kat_all_higher_than(s["all_higher_than"])


# ---------------------------------------------------------------- cards and tricks
def test_card_order_all_game_types(L):
    """648 reference lines, each over its colours x cards x game types (several thousand checks)."""
    n = 0
    seen_gt = set()
    for k in FDO["card_order"]:
        for gt in k["game_types"]:
            seen_gt.add(gt)
            for col in k["colors"]:
                for c2 in k["cards"]:
                    got = L.or_fdo_is_greater(k["cur"], c2, col, gt)
                    assert bool(got) == k["greater"], (k, gt, col, c2)
                    n += 1
    assert len(FDO["card_order"]) == 648 and seen_gt == set(range(9)) and n > 5000


def test_card_to_color_and_masks(L):
    assert len(FDO["card_to_color"]) == 216
    for k in FDO["card_to_color"]:
        assert L.or_fdo_card_to_color(k["card"], k["game_type"]) == k["color"], k
    # card_color_masks.rs:250-315: the five masks of a game type agree with card_to_color
    for gt in range(9):
        m = (u64 * 5)()
        L.or_kat_color_masks(gt, m)
        for card in range(24):
            col = L.or_fdo_card_to_color(card, gt)
            assert [bool(m[x] >> card & 1) for x in range(5)] == [x == col for x in range(5)], (gt, card)


def test_card_eyes(L):
    for k in FDO["card_eyes"]:
        assert L.or_kat_card_eyes(k["card"]) == k["eyes"], k


def test_tricks(L):
    checks = {"color": 0, "eyes": 3, "winner": 4, "current_player": 1, "completed": 2}
    assert len(FDO["tricks"]) >= 15
    for k in FDO["tricks"]:
        t = [k["start"]] + k["cards"] + [-1] * (4 - len(k["cards"]))
        out = (i32 * 6)()
        L.or_kat_trick(arr(i32, t), k.get("game_type", 0), out)
        if k["check"] == "winner":
            assert [out[4], out[5]] == k["expect"], k
        elif k["check"] == "completed":
            assert bool(out[2]) == k["expect"], k
        else:
            assert out[checks[k["check"]]] == k["expect"], k


# ---------------------------------------------------------------- teams and reservations
def test_team_resolution(L):
    assert len(FDO["team"]) == 6
    for k in FDO["team"]:
        rr = k["reservation_result"]
        hands = arr(u64, [fdo_hand(L, h) for h in k["hands"]])
        out = (i32 * 4)()
        L.or_kat_team_resolve(rr["kind"], rr["player"], rr["reservation"], tricks_arr(k["tricks"]), len(k["tricks"]),
                              hands, out)
        e = k["expect"]
        assert out[0] == e["kind"], k["test"]
        if e["kind"] != 1:
            assert all(out[3] >> p & 1 for p in e["re_contains"]), k["test"]
            assert bin(out[3]).count("1") == e["re_len"], k["test"]
        if e["wedding_player"] is not None:
            assert out[1] == e["wedding_player"], k["test"]
        if e["solved"] is not None:
            assert out[2] == e["solved"], k["test"]


def test_reservation_winner_and_game_type(L):
    for k in FDO["reservation"]:
        out = (i32 * 4)()
        if k["check"] == "winner":
            L.or_kat_reservation_winner(k["start"], arr(i32, k["reservations"]), len(k["reservations"]), out)
            e = k["expect"]
            assert out[0] == e["kind"], k
            if e["kind"] != 0:
                assert out[1] == e["player"], k
            if e["kind"] == 1:
                assert out[2] == e["reservation"], k
        else:
            r = k["result"]
            assert L.or_kat_game_type_of(r["kind"], r["player"], r["reservation"]) == k["expect"], k


# ---------------------------------------------------------------- announcements
def test_calc_allowed_announcements(L):
    assert len(FDO["calc_allowed"]) == 23
    for k in FDO["calc_allowed"]:
        if k["fn"] == "calc_allowed_announcements":
            t = k["team"]
            got = L.or_kat_calc_allowed(k["player"], k["n_cards"], t["kind"], t["wedding_player"], t["solved"], t["re"],
                                        k["re_lowest"], k["contra_lowest"])
        elif k["fn"] == "internal_calc_allowed_annoucements":
            got = L.or_kat_internal_calc_allowed(k["n_cards"], annset(L, k["prev"]), k["wedding_solved"],
                                                 k["enemy_cards"])
        else:
            got = L.or_kat_cards_last_announcement(annset(L, k["set"]), k["wedding_solved"])
        assert got == k["expect"], k


def test_announcement_rounds(L):
    assert len(FDO["ann_rounds"]) == 3
    for k in FDO["ann_rounds"]:
        ops = k["ops"]
        t = k["team"]
        flat = [x for o in ops for x in o["op"]]
        out = (i32 * (21 * len(ops)))()
        L.or_kat_announcement_round(arr(i32, k["hand_lens"]), t["kind"], t["wedding_player"], t["solved"], t["re"],
                                    k["card_index"], arr(i32, flat), len(ops), out)
        for i, o in enumerate(ops):
            got = list(out[21 * i:21 * i + 21])
            c = o["checks"]
            ctx = (k["test"], i, c, got)
            if "result" in c:
                assert got[0:2] == c["result"], ctx
            for key, idx in (("n", 2), ("starting_player", 3), ("turns", 4), ("re_lowest", 5), ("contra_lowest", 6),
                             ("allowed", 7)):
                if key in c:
                    assert got[idx] == c[key], ctx
            for key, occ in c.items():
                if key.startswith("occurrence_"):
                    code = got[9 + int(key.split("_")[1])]
                    assert code >= 0, ctx
                    if "card_index" in occ:
                        assert code >> 8 == occ["card_index"], ctx
                    if "player" in occ:
                        assert (code >> 4) & 15 == occ["player"], ctx
                    if "announcement" in occ:
                        assert 1 << (code & 15) == occ["announcement"], ctx


# ---------------------------------------------------------------- scoring
def test_end_of_game_stats(L):
    names = FDO["fields"]
    assert len(FDO["stats"]) == 4
    for k in FDO["stats"]:
        out = (i32 * 57)()
        L.or_kat_stats(arr(u32, k["eyes"]), arr(u32, k["ntricks"]), k["re_players"], k["re_lowest"], k["contra_lowest"],
                       tricks_arr(k["tricks"]), len(k["tricks"]), out)
        e = k["expect"]
        ctx = k["test"]
        assert out[0] == e["re_players"] and bool(out[1]) == e["is_solo"], ctx
        assert [out[2], out[3], out[4], out[5]] == [e["re_eyes"], e["kontra_eyes"], e["re_points"], e["kontra_points"]], ctx
        assert list(out[6:10]) == e["player_points"], ctx
        w = e["basic_winning_point_details"]
        assert bool(out[10]) == (w is not None), ctx
        if w is not None:
            assert list(out[11:34]) == [w[f] for f in names["basic_winning"]], ctx
        d = e["basic_draw_points_details"]
        assert bool(out[34]) == (d is not None), ctx
        if d is not None:
            assert list(out[35:49]) == [d[f] for f in names["basic_draw"]], ctx
        a = e["additional_points_details"]
        assert bool(out[49]) == (a is not None), ctx
        if a is not None:
            assert list(out[50:57]) == [int(a[f]) for f in names["additional"]], ctx


def test_win_conditions(L):
    assert len(FDO["re_won"]) == 18 and len(FDO["kontra_won"]) == 12
    for fn, f in (("re_won", L.or_kat_re_won), ("kontra_won", L.or_kat_kontra_won)):
        for k in FDO[fn]:
            got = f(k["eyes"], annset(L, k["re_prev"]), annset(L, k["kontra_prev"]), int(k["re_all"]), int(k["kontra_all"]))
            assert bool(got) == k["expect"], (fn, k)


def test_basic_points(L):
    assert len(FDO["basic_winning"]) == 16 and len(FDO["basic_draw"]) == 3
    for k in FDO["basic_winning"]:
        out = (i32 * 25)()
        L.or_kat_basic_winning(k["winner_eyes"], k["loser_eyes"], int(k["winner_all"]), annset(L, k["re_prev"]),
                               annset(L, k["kontra_prev"]), k["re_eyes"], k["kontra_eyes"], out)
        assert list(out) == k["expect"], k
    for k in FDO["basic_draw"]:
        out = (i32 * 16)()
        L.or_kat_basic_draw(annset(L, k["re_prev"]), annset(L, k["kontra_prev"]), k["re_eyes"], k["kontra_eyes"], out)
        assert list(out) == k["expect"], k


def test_additional_points(L):
    add = FDO["additional"]
    for k in add["calculate"]:
        out = (i32 * 9)()
        L.or_kat_additional(k["re_players"], k["winning_team"], tricks_arr(k["tricks"]), len(k["tricks"]), out)
        assert [out[0], out[1]] == [k["expect"]["re"], k["expect"]["kontra"]], k
        assert list(out[2:9]) == k["expect"]["details"], k
    # the building blocks, each checked through the same restatement
    for key, lo in (("doppelkopf", 3), ("fuchs", 5), ("karlchen", 7)):
        assert add[key], key
        for k in add[key]:
            out = (i32 * 9)()
            L.or_kat_additional(k["re_players"], -1, tricks_arr(k["tricks"]), len(k["tricks"]), out)
            assert [out[lo], out[lo + 1]] == k["expect"], (key, k)
    for k in add["fuchs_in_trick"]:
        out = (i32 * 9)()
        L.or_kat_additional(k["re_players"], -1, tricks_arr([k["trick"]]), 1, out)
        assert [out[5], out[6]] == k["expect"], k
    # internal_calculate: the point arithmetic over given counts (additional_points.rs:61-128)
    for k in add["internal"]:
        dre, dko, fre, fko, kre, kko = k["counts"]
        re_pts = -1 if k["winning_team"] == 1 else 0
        re_pts += dre - dko + fre - fko + kre - kko
        assert [re_pts, -re_pts] == k["expect"][:2], k
        assert k["expect"][2] == int(k["winning_team"] == 1), k


# ---------------------------------------------------------------- is_consistent
def replay(L, start, actions):
    """The test's action list on the oracle.  The tests were written before two announcement-
    rule changes (as with the full-game traces): every real decision is replayed
    verbatim; NoAnnouncement passes are dropped where the current rules open no announcement
    phase and inserted where they do."""
    s = ol.FdoState.from_hands([fdo_hand(L, h) for h in start["hands"]], start["start_player"])
    for a in actions:
        phase = s.info()["phase"]
        if a == 38 and phase != 1:
            continue
        while a != 38 and a <= 23 and s.info()["phase"] == 1:
            s.play(38)
        s.play(a)
    return s



def test_is_consistent(L):
    assert len(FDO["is_consistent"]) == 21
    for k in FDO["is_consistent"]:
        s = replay(L, k["start"], k["actions"])
        ah = arr(u64, [fdo_hand(L, h) for h in k["hands"]])
        res = [-1] * 4
        for i, r in enumerate(k["reservations"]):
            res[(k["reservations_from"] + i) % 4] = r
        reason = L.or_ipi_consistent(s.h, ah, arr(i32, res))
        assert (reason < 0) == k["expect"], (k["test"], k["actions"][-3:], reason)


# ---------------------------------------------------------------- rs-doko
def test_do_allowed_actions(L):
    assert len(DO["allowed"]) == 7
    for k in DO["allowed"]:
        h = 0
        for c in k["hand"]:
            h = L.or_kat_do_hand_add(h, c)
        got = L.or_kat_do_allowed(k["phase"], k["trick_color"], h)
        assert [a for a in range(39) if got >> a & 1] == sorted(k["expect"]), k


def test_do_team_resolution(L):
    assert len(DO["team"]) == 5
    for k in DO["team"]:
        tr = []
        for t in k["tricks"]:
            tr += t if t is not None else [-1, -1, -1, -1, -1]
        hands = []
        for h in k["hands"]:
            x = 0
            for c in h:
                x = L.or_kat_do_hand_add(x, c)
            hands.append(x)
        out = (i32 * 4)()
        L.or_kat_do_team_resolve(k["wedding_player"], arr(i32, tr), arr(u64, hands), out)
        e = k["expect"]
        assert out[0] == e["kind"], k["test"]
        if e["kind"] != 1:
            assert all(out[3] >> p & 1 for p in e["re_contains"]) and bin(out[3]).count("1") == e["re_len"], k["test"]
        if e["wedding_player"] is not None:
            assert out[1] == e["wedding_player"], k["test"]
        if e["solved"] is not None:
            assert out[2] == e["solved"], k["test"]


def test_do_stats(L):
    assert len(DO["stats"]) == 4
    for k in DO["stats"]:
        out = (i32 * 10)()
        L.or_kat_do_stats(k["re_players"], arr(u32, k["eyes"]), arr(u32, k["ntricks"]), out)
        e = k["expect"]
        got = {"winning_team": out[0], "is_solo": bool(out[1]), "re_eyes": out[2], "kontra_eyes": out[3],
               "re_points": out[4], "kontra_points": out[5], "player_points": list(out[6:10]),
               "player_eyes": k["eyes"]}
        for key, v in e.items():
            assert got[key] == v, (k["test"], key)
