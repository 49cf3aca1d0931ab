"""Extract the reference's rule-level known-answer tests into JSON fixtures.

Run HERE (the container that has /root/reference); the GPU box never reads the
reference.  It reads the reference's #[test] functions as text (rustexpr.py parses
their literal expressions; nothing is executed) and writes inputs + expected
outputs only:

tests/golden/rule_kats_fdo.json (rs-full-doko):
  card_order       card/card_in_trick_logic.rs:226-1023   is_smaller / is_greater over all game types
  card_to_color    card/card_to_color.rs:261-530
  card_eyes        card/card_to_eyes.rs:45-77
  tricks           trick/trick.rs:121-315, trick/trick_winning_player_logic.rs:48-108
  team             team/team_logic.rs:155-385
  reservation      reservation/reservation_winning_logic.rs:75-140
  calc_allowed     announcement/calc_announcement.rs:232-516 (three functions)
  ann_rounds       announcement/announcement.rs:219-573
  stats            stats/stats.rs:245-778
  re_won/kontra_won, basic_winning, basic_draw, additional, doppelkopf, fuchs, karlchen
                   stats/{win_conditions,basic_points,additional_points}/*.rs tests
  is_consistent    matching/is_consistent.rs:318-888
tests/golden/rule_kats_do.json (rs-doko):
  allowed          action/allowed_actions.rs:210-312
  team             teams/team_logic.rs:145-333
  stats            stats/stats.rs:144-238

Usage: python tests/golden/make_rule_kats.py
"""
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rustexpr import balanced, parse_expr, parse_tokens, statements, test_functions, tokenize  # noqa: E402

REF = "/root/reference"
FDO = os.path.join(REF, "rs-full-doko", "src")
DO = os.path.join(REF, "rs-doko", "src")
OUT = os.path.dirname(os.path.abspath(__file__))

SUITS = ["Diamond", "Heart", "Club", "Spade"]
RANKS = ["Nine", "Ten", "Jack", "Queen", "King", "Ace"]
CARD_NAMES = [s + r for s in SUITS for r in RANKS]      # FdoCard order (card/cards.rs:8-36)
SYM_SUIT = {"♦": "Diamond", "♥": "Heart", "♣": "Club", "♠": "Spade"}
SYM_RANK = {"9": "Nine", "10": "Ten", "J": "Jack", "Q": "Queen", "K": "King", "A": "Ace"}
PLAYERS = {"BOTTOM": 0, "LEFT": 1, "TOP": 2, "RIGHT": 3}
GAME_TYPES = ["Normal", "Wedding", "DiamondsSolo", "HeartsSolo", "SpadesSolo", "ClubsSolo", "TrumplessSolo",
              "QueensSolo", "JacksSolo"]
COLORS = ["Trump", "Diamond", "Heart", "Spade", "Club"]   # FdoColor (basic/color.rs)
COLOR_SYM = {"T": 0, "♦": 1, "♥": 2, "♠": 3, "♣": 4}
ANN = {"ReContra": 1, "No90": 2, "No60": 4, "No30": 8, "Black": 16, "CounterReContra": 32, "NoAnnouncement": 64}
RESERVATIONS = ["Healthy", "Wedding", "DiamondsSolo", "HeartsSolo", "SpadesSolo", "ClubsSolo", "QueensSolo",
                "JacksSolo", "TrumplessSolo"]            # FdoReservation (reservation/reservation.rs:11-24)
ACTIONS = ["Card" + c for c in CARD_NAMES] + [
    "ReservationHealthy", "ReservationWedding", "ReservationDiamondsSolo", "ReservationHeartsSolo",
    "ReservationSpadesSolo", "ReservationClubsSolo", "ReservationTrumplessSolo", "ReservationQueensSolo",
    "ReservationJacksSolo", "AnnouncementReContra", "AnnouncementNo90", "AnnouncementNo60",
    "AnnouncementNo30", "AnnouncementBlack", "NoAnnouncement"]
DO_COLORS = {"Trump": 0, "Heart": 1, "Spade": 2, "Club": 3}   # DoColor (rs-doko/src/basic/color.rs)


def read(path):
    with open(path, encoding="utf-8") as fh:
        return fh.read()


def lineno(text, idx):
    return text.count("\n", 0, idx) + 1


# ---------------------------------------------------------------- value converters
def last(path):
    return path.split("::")[-1]


def card(e):
    if isinstance(e, str):                         # "♦9"
        return CARD_NAMES.index(SYM_SUIT[e[0]] + SYM_RANK[e[1:]])
    assert e[0] == "path", e
    return CARD_NAMES.index(last(e[1]))


def card_syms(s):
    return [card(x) for x in s.split()]


def cards(e):
    if e[0] == "list":
        return [card(x) for x in e[1]]
    raise ValueError(e)


def player(e):
    assert e[0] == "path", e
    return PLAYERS[last(e[1]).replace("PLAYER_", "")]


def pset(e):
    if e[0] == "call" and last(e[1]) == "from_vec":
        m = 0
        for p in e[2][0][1]:
            m |= 1 << player(p)
        return m
    if e[0] == "call" and last(e[1]) in ("empty", "new"):
        return 0
    if e[0] == "call" and last(e[1]) == "all":
        return 15
    if isinstance(e, int):                         # rs-doko player sets are plain integers
        return e
    raise ValueError(e)


def ann(e):
    """Option<FdoAnnouncement> / FdoAnnouncement -> bit (0 = None)."""
    if e == ("path", "None"):
        return 0
    if e[0] == "call" and e[1] == "Some":
        return ann(e[2][0])
    return ANN[last(e[1])]


def annset(e):
    """FdoAnnouncementSet expression -> {"bits": b} or {"all_higher_than": lowest bit}."""
    name = last(e[1])
    if name == "new":
        return {"bits": 0}
    if name == "from_vec":
        b = 0
        for a in e[2][0][1]:
            b |= ann(a)
        return {"bits": b}
    if name == "all_higher_than":
        return {"all_higher_than": ann(e[2][0])}
    raise ValueError(e)


def opt_int(e):
    if e == ("path", "None"):
        return -1
    if e[0] == "call" and e[1] == "Some":
        return e[2][0]
    return e


def game_type(e):
    return GAME_TYPES.index(last(e[1]))


def team_state(e):
    if e[0] == "path":
        assert last(e[1]) == "InReservations"
        return {"kind": 0, "wedding_player": 0, "solved": 0, "re": 0}
    kind = {"WeddingUnsolved": 1, "WeddingSolved": 2, "NoWedding": 3}[last(e[1])]
    f = e[2]
    return {"kind": kind, "wedding_player": player(f["wedding_player"]) if "wedding_player" in f else 0,
            "solved": f.get("solved_trick_index", 0), "re": pset(f["re_players"]) if "re_players" in f else 0}


def trick(e, env=None):
    while e[0] == "ref":
        e = e[1]
    if e[0] == "method" and e[2] == "clone":
        e = e[1]
    if e[0] == "path" and env is not None:
        e = env[e[1]]
    assert e[0] == "call" and last(e[1]) == "existing", e
    cs = cards(e[2][1])
    return [player(e[2][0])] + cs + [-1] * (4 - len(cs))


def trick_list(e, env=None):
    """&heapless::Vec::from_slice(&[..]).unwrap() -> [[start, c0..c3], ...]"""
    while e[0] in ("ref", "method"):
        e = e[1]
    if e[0] == "call":
        e = e[2][0]
    while e[0] == "ref":
        e = e[1]
    return [trick(t, env) for t in e[1]]


def hand(e):
    assert e[0] == "call" and last(e[1]) in ("from_vec", "hand_from_vec"), e
    return cards(e[2][0])


def zero_arr(e):
    assert e[0] == "call" and last(e[1]) == "from_full", e
    return e[2][0][1]


def reservation_result(e):
    if e[0] == "path":
        return {"kind": 0, "player": 0, "reservation": 0}
    name = last(e[1])
    if name == "Wedding":
        return {"kind": 2, "player": player(e[2][0]), "reservation": 0}
    if name == "Solo":
        return {"kind": 1, "player": player(e[2][0]), "reservation": RESERVATIONS.index(last(e[2][1][1]))}
    raise ValueError(e)


def stmt_text(tokens):
    return " ".join(t[1] for t in tokens)


def strip_let(tokens):
    """`let [mut] name [: ty] = expr` -> (name, expr tokens) or (None, tokens)"""
    if tokens and tokens[0][1] == "let":
        i = 1
        if tokens[i][1] == "mut":
            i += 1
        if tokens[i][1] == "(":                    # let (a, b, c) = ...
            j = i
            depth = 0
            while True:
                depth += tokens[j][1] == "("
                depth -= tokens[j][1] == ")"
                j += 1
                if depth == 0:
                    break
            names = [t[1] for t in tokens[i + 1:j - 1] if t[1] != ","]
            return names, tokens[j + 1:]
        name = tokens[i][1]
        j = i + 1
        if tokens[j][1] == ":":                    # skip a type annotation up to '='
            while tokens[j][1] != "=":
                j += 1
        return name, tokens[j + 1:]
    return None, tokens


def macro_args(tokens):
    """assert_eq!(a, b) / assert!(x) tokens -> parsed argument list"""
    e = parse_tokens(tokens)
    assert e[0] == "call" and e[1].endswith("!"), e
    return e[1], e[2]


# ---------------------------------------------------------------- rs-full-doko groups
def card_order():
    text = read(os.path.join(FDO, "card", "card_in_trick_logic.rs"))
    body = dict(test_functions(text))["test_is_greater_in_trick"]
    env = {}
    out = []
    for st in statements(body):
        name, toks = strip_let(st)
        if name:
            env[name] = [game_type(g) for g in parse_tokens(toks)[1]]
            continue
        e = parse_tokens(st)
        if e[0] != "call" or e[1] not in ("is_smaller", "is_greater"):
            continue
        cur, colors, cs, gts = e[2]
        gts = env[gts[1][1]] if gts[0] == "ref" else [game_type(g) for g in gts[1]]
        out.append({"cur": card(cur), "colors": [COLOR_SYM[c] for c in colors], "cards": card_syms(cs),
                    "game_types": gts, "greater": e[1] == "is_greater"})
    return out


def card_to_color():
    text = read(os.path.join(FDO, "card", "card_to_color.rs"))
    out = []
    for m in re.finditer(r"card_to_color\(FdoCard::(\w+), FdoGameType::(\w+)\) == FdoColor::(\w+)", text):
        out.append({"card": CARD_NAMES.index(m.group(1)), "game_type": GAME_TYPES.index(m.group(2)),
                     "color": COLORS.index(m.group(3))})
    return out


def card_eyes():
    text = read(os.path.join(FDO, "card", "card_to_eyes.rs"))
    return [{"card": CARD_NAMES.index(m.group(1)), "eyes": int(m.group(2))}
            for m in re.finditer(r"FdoCard::(\w+)\.eyes\(\), (\d+)\)", text)]


def tricks_group():
    """Every assertion on a trick built by FdoTrick::empty/existing (+ play_card)."""
    out = []
    for fname in (os.path.join(FDO, "trick", "trick.rs"), os.path.join(FDO, "trick", "trick_winning_player_logic.rs")):
        text = read(fname)
        for tname, body in test_functions(text):
            cur = None
            env = {}
            for st in statements(body):
                name, toks = strip_let(st)
                e = parse_tokens(toks)
                if name == "trick":
                    if e[0] == "call" and last(e[1]) == "empty":
                        cur = [player(e[2][0])]
                    elif e[0] == "call" and last(e[1]) == "existing":
                        cs = e[2][1]
                        cur = [player(e[2][0])] + cards(env[cs[1]] if cs[0] == "path" else cs)
                    continue
                if name:
                    env[name] = e
                    continue
                if name is None and e[0] == "method" and e[2] == "play_card":
                    cur = cur + [card(e[2 + 1][0])]
                    continue
                if e[0] != "call" or e[1] != "assert_eq!":
                    continue
                lhs, rhs = e[2][:2]
                if lhs[0] != "method" or lhs[1] != ("path", "trick"):
                    continue
                entry = {"test": tname, "start": cur[0], "cards": cur[1:]}
                meth = lhs[2]
                if meth == "color":
                    entry.update(check="color", game_type=game_type(lhs[3][0]),
                                 expect=-1 if rhs == ("path", "None") else COLORS.index(last(rhs[2][0][1])))
                elif meth == "eyes":
                    entry.update(check="eyes", expect=rhs)
                elif meth == "calc_winning_player_in_trick":
                    entry.update(check="winner", game_type=game_type(lhs[3][0]),
                                 expect=[player(rhs[1][0]), card(rhs[1][1])])
                elif meth == "current_player":
                    entry.update(check="current_player", expect=-1 if rhs == ("path", "None") else player(rhs[2][0]))
                elif meth == "is_completed":
                    entry.update(check="completed", expect=rhs)
                else:
                    continue
                out.append(entry)
    return out


def team_group():
    text = read(os.path.join(FDO, "team", "team_logic.rs"))
    out = []
    for tname, body in test_functions(text):
        if not tname.startswith("test_resolve"):
            continue
        env, expect = {}, None
        for st in statements(body):
            name, toks = strip_let(st)
            if name:
                env[name] = parse_tokens(toks)
                continue
            if st[0][1] == "match":
                # match team_state { FdoTeamState::K { fields } => { asserts } _ => panic }
                text_st = stmt_text(st)
                m = re.search(r"FdoTeamState::(\w+)", text_st)
                kind = {"WeddingUnsolved": 1, "WeddingSolved": 2, "NoWedding": 3}[m.group(1)]
                expect = {"kind": kind, "re_contains": [], "re_len": None, "wedding_player": None, "solved": None}
                for c in re.finditer(r"re_players \. contains \( FdoPlayer::(\w+) \)", text_st):
                    expect["re_contains"].append(PLAYERS[c.group(1)])
                m = re.search(r"re_players \. len \( \) , (\d+)", text_st)
                expect["re_len"] = int(m.group(1)) if m else None
                m = re.search(r"assert_eq ! \( wedding_player , FdoPlayer::(\w+) \)", text_st)
                expect["wedding_player"] = PLAYERS[m.group(1)] if m else None
                m = re.search(r"assert_eq ! \( solved_trick_index , (\d+) \)", text_st)
                expect["solved"] = int(m.group(1)) if m else None
        hands = [hand(h) for h in zero_arr(env["hands"])]
        out.append({"test": tname, "reservation_result": reservation_result(env["reservation_results"]),
                    "tricks": trick_list(env["tricks"]), "hands": hands, "expect": expect})
    return out


def reservation_group():
    text = read(os.path.join(FDO, "reservation", "reservation_winning_logic.rs"))
    out = []
    for tname, body in test_functions(text):
        env = {}
        for st in statements(body):
            name, toks = strip_let(st)
            if name:
                env[name] = parse_tokens(toks)
                continue
            e = parse_tokens(st)
            if e[0] != "call" or e[1] != "assert_eq!":
                continue
            lhs, rhs = e[2][:2]
            if lhs[0] == "call" and lhs[1] == "winning_player_in_reservation_round":
                rr = env["reservation_round"]
                out.append({"check": "winner", "start": player(rr[2][0]),
                            "reservations": [RESERVATIONS.index(last(r[1])) for r in rr[2][1][1]],
                            "expect": reservation_result(rhs)})
            elif lhs[0] == "method" and lhs[2] == "to_game_type":
                rr = lhs[1]
                out.append({"check": "game_type", "result": reservation_result(rr), "expect": game_type(rhs)})
    return out


def calc_allowed_group():
    text = read(os.path.join(FDO, "announcement", "calc_announcement.rs"))
    out = []
    for tname, body in test_functions(text):
        for st in statements(body):
            e = parse_tokens(st)
            if e[0] != "call" or e[1] != "assert_eq!":
                continue
            lhs, rhs = e[2][:2]
            fn = lhs[1]
            if fn == "calc_allowed_announcements":
                p, n, ts, rl, cl = lhs[2]
                out.append({"fn": fn, "player": player(p), "n_cards": n, "team": team_state(ts), "re_lowest": ann(rl),
                            "contra_lowest": ann(cl), "expect": annset(rhs)["bits"]})
            elif fn == "internal_calc_allowed_annoucements":
                n, prev, w, enemy = lhs[2]
                out.append({"fn": fn, "n_cards": n, "prev": annset(prev), "wedding_solved": opt_int(w),
                            "enemy_cards": opt_int(enemy), "expect": annset(rhs)["bits"]})
            elif fn == "calc_number_of_cards_announcement_possible_for_last_announcement":
                s, w = lhs[2]
                out.append({"fn": fn, "set": annset(s), "wedding_solved": opt_int(w), "expect": opt_int(rhs)})
    return out


def ann_rounds_group():
    text = read(os.path.join(FDO, "announcement", "announcement.rs"))
    out = []
    for tname, body in test_functions(text):
        env = {}
        ops = []          # [{"op": [player, ann], "checks": {...}}]
        for st in statements(body):
            name, toks = strip_let(st)
            e = parse_tokens(toks)
            if name == "result":
                if e[2] == "start_round":
                    ci, p, _, _ = e[3]
                    env["card_index_used"] = ci
                    ops.append({"op": [player(p), 0], "checks": {}})
                else:
                    p, a, _, _, _ = e[3]
                    ops.append({"op": [player(p), ann(a)], "checks": {}})
                continue
            if name:
                env[name] = e
                continue
            if e[0] != "call" or e[1] != "assert_eq!":
                continue
            lhs, rhs = e[2][:2]
            chk = ops[-1]["checks"]
            key = stmt_text(tokenize(stmt_text(st)))
            if lhs == ("path", "result"):
                chk["result"] = [0 if last(rhs[1]) == "NextPlayerIs" else 1, player(rhs[2][0])]
            elif lhs[0] == "method" and lhs[2] == "len":
                chk["n"] = rhs
            elif lhs[0] == "field" and lhs[2] == "starting_player":
                chk["starting_player"] = player(rhs)
            elif lhs[0] == "field" and lhs[2] == "number_of_turns_without_announcement":
                chk["turns"] = rhs
            elif lhs[0] == "field" and lhs[2] == "re_lowest_announcement":
                chk["re_lowest"] = ann(rhs)
            elif lhs[0] == "field" and lhs[2] == "contra_lowest_announcement":
                chk["contra_lowest"] = ann(rhs)
            elif lhs[0] == "field" and lhs[2] == "current_player_allowed_announcements":
                chk["allowed"] = annset(rhs)["bits"]
            elif lhs[0] == "field" and lhs[1][0] == "call":
                pass
            elif lhs[0] == "field" and lhs[1][0] == "index" and lhs[2] in ("player", "card_index", "announcement"):
                # announcements.announcements[k].field
                occ = chk.setdefault("occurrence_%d" % lhs[1][2], {})
                occ[lhs[2]] = player(rhs) if lhs[2] == "player" else (ann(rhs) if lhs[2] == "announcement" else rhs)
            else:
                raise ValueError("unhandled announcement assertion: %s" % key)
        hl = zero_arr(env["current_player_number_of_cards_on_hand"])
        out.append({"test": tname, "hand_lens": hl, "team": team_state(env["team_state"]),
                    "card_index": env["card_index"], "ops": ops})
    return out


def stats_struct(e):
    """FdoEndOfGameStats { .. } -> dict of the fields the tests state"""
    f = e[2]
    out = {"re_players": pset(f["re_players"]), "is_solo": f["is_solo"], "player_eyes": zero_arr(f["player_eyes"]),
           "re_eyes": f["re_eyes"], "kontra_eyes": f["kontra_eyes"], "re_points": f["re_points"],
           "kontra_points": f["kontra_points"], "player_points": zero_arr(f["player_points"])}
    for key in ("basic_winning_point_details", "basic_draw_points_details", "additional_points_details"):
        v = f[key]
        if v == ("path", "None"):
            out[key] = None
        else:
            out[key] = {k: x for k, x in v[2][0][2].items()}
    return out


def stats_group():
    text = read(os.path.join(FDO, "stats", "stats.rs"))
    out = []
    for tname, body in test_functions(text):
        env = {}
        for st in statements(body):
            name, toks = strip_let(st)
            if name:
                env[name] = parse_tokens(toks)
        a = env["actual"]
        eyes, ntr, re_players, rl, cl, tricks = a[2]
        out.append({"test": tname, "eyes": zero_arr(eyes), "ntricks": zero_arr(ntr), "re_players": pset(re_players),
                    "re_lowest": ann(rl), "contra_lowest": ann(cl), "tricks": trick_list(tricks),
                    "expect": stats_struct(env["expected"])})
    return out


def simple_asserts(path, fn_names):
    """assert_eq!(fn(args..), expected) over the test functions of one file -> [(fn, args, expected)]"""
    text = read(path)
    out = []
    for tname, body in test_functions(text):
        env = {}
        for st in statements(body):
            name, toks = strip_let(st)
            if name and not isinstance(name, list):
                env[name] = parse_tokens(toks)
                continue
            if name:
                env[tuple(name)] = parse_tokens(toks)
                continue
            e = parse_tokens(st)
            if e[0] == "call" and e[1] == "assert_eq!" and e[2][0][0] == "call" and last(e[2][0][1]) in fn_names:
                out.append((tname, last(e[2][0][1]), e[2][0][2], e[2][1], env))
            elif e[0] == "call" and e[1] == "assert_eq!":
                out.append((tname, None, e[2][0], e[2][1], env))
    return out


def win_conditions():
    res = {}
    for fn in ("re_won", "kontra_won"):
        out = []
        for tname, f, args, rhs, _ in simple_asserts(os.path.join(FDO, "stats", "win_conditions", fn + ".rs"), {fn}):
            if f != fn:
                continue
            eyes, rp, kp, ra, ka = args
            out.append({"eyes": eyes, "re_prev": annset(rp), "kontra_prev": annset(kp), "re_all": ra, "kontra_all": ka,
                        "expect": rhs})
        res[fn] = out
    return res


WIN_FIELDS = ["winning_points", "winning_under_90", "winning_under_60", "winning_under_30", "winning_black",
              "re_announcement", "kontra_announcement", "re_under_90_announcement", "re_under_60_announcement",
              "re_under_30_announcement", "re_black_announcement", "kontra_under_90_announcement",
              "kontra_under_60_announcement", "kontra_under_30_announcement", "kontra_black_announcement",
              "re_reached_120_against_no_90", "re_reached_90_against_no_60", "re_reached_60_against_no_30",
              "re_reached_30_against_black", "kontra_reached_120_against_no_90", "kontra_reached_90_against_no_60",
              "kontra_reached_60_against_no_30", "kontra_reached_30_against_black"]
DRAW_FIELDS = ["winning_under_90_re", "winning_under_60_re", "winning_under_30_re", "winning_under_90_kontra",
               "winning_under_60_kontra", "winning_under_30_kontra", "re_reached_120_against_no_90",
               "re_reached_90_against_no_60", "re_reached_60_against_no_30", "re_reached_30_against_black",
               "kontra_reached_120_against_no_90", "kontra_reached_90_against_no_60",
               "kontra_reached_60_against_no_30", "kontra_reached_30_against_black"]
ADD_FIELDS = ["against_club_queens", "number_of_doppelkopf_re", "number_of_doppelkopf_kontra", "fuchs_gefangen_re",
              "fuchs_gefangen_kontra", "karlchen_last_trick_re", "karlchen_last_trick_kontra"]


def basic_points():
    win, draw = [], []
    for _, f, args, rhs, _ in simple_asserts(os.path.join(FDO, "stats", "basic_points", "basic_winning_points.rs"),
                                             {"calculate"}):
        if f != "calculate":
            continue
        we, le, wall, rp, kp, re_e, ko_e = args
        det = rhs[1][2][2]
        win.append({"winner_eyes": we, "loser_eyes": le, "winner_all": wall, "re_prev": annset(rp),
                    "kontra_prev": annset(kp), "re_eyes": re_e, "kontra_eyes": ko_e,
                    "expect": [rhs[1][0], rhs[1][1]] + [det[k] for k in WIN_FIELDS]})
    for _, f, args, rhs, _ in simple_asserts(os.path.join(FDO, "stats", "basic_points", "basic_draw_points.rs"),
                                             {"calculate"}):
        if f != "calculate":
            continue
        rp, kp, re_e, ko_e = args
        det = rhs[1][2][2]
        draw.append({"re_prev": annset(rp), "kontra_prev": annset(kp), "re_eyes": re_e, "kontra_eyes": ko_e,
                     "expect": [rhs[1][0], rhs[1][1]] + [det[k] for k in DRAW_FIELDS]})
    return win, draw


def winning_team(e):
    if e == ("path", "None"):
        return -1
    return {"Re": 0, "Kontra": 1}[last(e[2][0][1])]


def additional_group():
    """additional_points.rs test_calculate (+ internal_calculate), doppelkopf, fuchs, karlchen."""
    res = {"calculate": [], "internal": [], "doppelkopf": [], "fuchs": [], "fuchs_in_trick": [], "karlchen": []}
    base = os.path.join(FDO, "stats", "additional_points")
    # calculate: let (re, kontra, details) = calculate(...); asserts on the three
    text = read(os.path.join(base, "additional_points.rs"))
    for tname, body in test_functions(text):
        env, pend = {}, None
        for st in statements(body):
            name, toks = strip_let(st)
            e = parse_tokens(toks)
            if isinstance(name, list):
                pend = {"re_players": pset(e[2][0]), "winning_team": winning_team(e[2][1]),
                        "tricks": trick_list(e[2][2], env), "expect": {}}
                res["calculate"].append(pend)
                continue
            if name:
                env[name] = e
                continue
            if e[0] != "call" or e[1] != "assert_eq!":
                continue
            lhs, rhs = e[2][:2]
            if lhs == ("path", "re_points"):
                pend["expect"]["re"] = rhs
            elif lhs == ("path", "kontra_points"):
                pend["expect"]["kontra"] = rhs
            elif lhs == ("path", "details"):
                pend["expect"]["details"] = [int(rhs[2][k]) for k in ADD_FIELDS]
            elif lhs[0] == "call" and last(lhs[1]) == "internal_calculate":
                a = lhs[2]
                det = rhs[1][2][2]
                res["internal"].append({"re_players": pset(a[0]), "winning_team": winning_team(a[1]),
                                        "counts": [int(x) for x in a[2:]],
                                        "expect": [rhs[1][0], rhs[1][1]] + [int(det[k]) for k in ADD_FIELDS]})
    for key, fname, fn in (("doppelkopf", "doppelkopf.rs", "calc_number_of_doppelkopf"),
                           ("fuchs", "fuchs_gefangen.rs", "calc_fuchs_gefangen"),
                           ("karlchen", "last_trick_karlchen.rs", "calc_trick_karlchen")):
        text = read(os.path.join(base, fname))
        for tname, body in test_functions(text):
            env = {}
            for st in statements(body):
                name, toks = strip_let(st)
                e = parse_tokens(toks)
                if isinstance(name, list) and e[0] == "call" and last(e[1]) == fn:
                    env["__pending"] = {"re_players": pset(e[2][0]), "tricks": trick_list(e[2][1], env), "names": name}
                    continue
                if name:
                    env[name] = e
                    continue
                if e[0] != "call" or e[1] != "assert_eq!":
                    continue
                lhs, rhs = e[2][:2]
                if lhs[0] == "call" and last(lhs[1]) == fn:
                    res[key].append({"re_players": pset(lhs[2][0]), "tricks": trick_list(lhs[2][1], env),
                                     "expect": [rhs[1][0], rhs[1][1]]})
                elif lhs[0] == "call" and last(lhs[1]) == "calc_fuchs_gefangen_in_trick":
                    res["fuchs_in_trick"].append({"trick": trick(lhs[2][0], env), "re_players": pset(lhs[2][1]),
                                                  "expect": [rhs[1][0], rhs[1][1]]})
                elif lhs[0] == "tuple" or (lhs[0] == "path" and "__pending" in env):
                    pend = env["__pending"]
                    names = pend["names"]
                    if lhs[0] == "tuple":
                        res[key].append({"re_players": pend["re_players"], "tricks": pend["tricks"],
                                         "expect": [rhs[1][0], rhs[1][1]]})
                    else:
                        pend.setdefault("expect", [None, None])[names.index(lhs[1])] = rhs
                        if None not in pend["expect"]:
                            res[key].append({"re_players": pend["re_players"], "tricks": pend["tricks"],
                                             "expect": pend["expect"]})
                            env.pop("__pending")
    return res


def is_consistent_group():
    text = read(os.path.join(FDO, "matching", "is_consistent.rs"))
    out = []
    for tname, body in test_functions(text):
        env, actions, start = {}, [], None
        for st in statements(body):
            name, toks = strip_let(st)
            e = parse_tokens(toks)
            if name == "state":
                start = {"hands": [hand(h) for h in zero_arr(e[2][0])], "start_player": player(e[2][1])}
                continue
            if name:
                env[name] = e
                continue
            if e[0] == "method" and e[2] == "play_action":
                actions.append(ACTIONS.index(last(e[3][0][1])))
                continue
            if e[0] == "call" and e[1] == "assert_eq!" and e[2][0][0] == "call" and last(e[2][0][1]) == "is_consistent":
                hands = [hand(h) for h in zero_arr(env["hands"])]
                r = env["reservations"]
                r_start = player(r[2][0])
                rs = [-1 if x == ("path", "None") else RESERVATIONS.index(last(x[2][0][1])) for x in r[2][1][1]]
                out.append({"test": tname, "start": start, "actions": list(actions), "hands": hands,
                            "reservations_from": r_start, "reservations": rs, "expect": e[2][1]})
    return out


# ---------------------------------------------------------------- rs-doko groups
def do_card(e):
    return CARD_NAMES.index(last(e[1]))


def do_allowed():
    text = read(os.path.join(DO, "action", "allowed_actions.rs"))
    out = []
    for tname, body in test_functions(text):
        for st in statements(body):
            e = parse_tokens(st)
            if e[0] != "call" or e[1] != "assert_eq!":
                continue
            lhs, rhs = e[2][:2]
            ordered = False
            if lhs[0] == "method" and lhs[2] == "to_vec":
                lhs = lhs[1][2][0]
                ordered = True
            phase, color, h = lhs[2]
            ph = {"Reservation": 0, "PlayCard": 1, "Finished": 2}[last(phase[1])]
            col = -1 if color == ("path", "None") else DO_COLORS[last(color[2][0][1])]
            if rhs == 0:
                exp = []
            elif ordered:
                exp = [ACTIONS.index(last(a[1])) for a in rhs[1]]
            else:
                exp = [ACTIONS.index(last(a[1])) for a in rhs[2][0][1]]
            out.append({"phase": ph, "trick_color": col, "hand": [do_card(c) for c in h[2][0][1]],
                        "expect": sorted(exp) if not ordered else exp, "ordered": ordered})
    return out


def do_trick(e):
    if e == ("path", "None"):
        return None
    # Some(DoTrick::existing(PLAYER_X, vec![..])) or DoTrick { .. }
    inner = e[2][0] if e[0] == "call" and e[1] == "Some" else e
    if inner[0] == "call" and last(inner[1]) == "existing":
        cs = [do_card(c) for c in inner[2][1][1]]
        return [player(inner[2][0])] + cs + [-1] * (4 - len(cs))
    raise ValueError(inner)


def do_team():
    text = read(os.path.join(DO, "teams", "team_logic.rs"))
    out = []
    for tname, body in test_functions(text):
        if not tname.startswith("test_resolve"):
            continue
        env, expect = {}, None
        for st in statements(body):
            name, toks = strip_let(st)
            if name:
                env[name] = parse_tokens(toks)
                continue
            if st[0][1] == "match":
                text_st = stmt_text(st)
                m = re.search(r"DoTeamState::(\w+)", text_st)
                kind = {"WeddingUnsolved": 1, "WeddingSolved": 2, "NoWedding": 3}[m.group(1)]
                expect = {"kind": kind, "re_contains": [PLAYERS[c.group(1)] for c in
                                                        re.finditer(r"player_set_contains \( re_players , PLAYER_(\w+) \)", text_st)]}
                m = re.search(r"player_set_len \( re_players \) , (\d+)", text_st)
                expect["re_len"] = int(m.group(1)) if m else None
                m = re.search(r"assert_eq ! \( wedding_player , PLAYER_(\w+) \)", text_st)
                expect["wedding_player"] = PLAYERS[m.group(1)] if m else None
                m = re.search(r"assert_eq ! \( solved_trick_index , (\d+) \)", text_st)
                expect["solved"] = int(m.group(1)) if m else None
        rr = env["reservation_results"]
        wp = -1 if rr[0] == "path" else player(rr[2][0])
        tricks = [do_trick(t) for t in env["tricks"][1]]
        hands = [[do_card(c) for c in h[2][0][1]] for h in env["hands"][1]]
        out.append({"test": tname, "wedding_player": wp, "tricks": tricks, "hands": hands, "expect": expect})
    return out


def do_stats():
    text = read(os.path.join(DO, "stats", "stats.rs"))
    out = []
    for tname, body in test_functions(text):
        env, exp = {}, {}
        for st in statements(body):
            name, toks = strip_let(st)
            e = parse_tokens(toks)
            if name:
                env[name] = e
                continue
            if e[0] != "call" or e[1] != "assert_eq!":
                continue
            lhs, rhs = e[2][:2]
            if lhs[0] == "field" and lhs[1] == ("path", "end_of_game_stats"):
                key = lhs[2]
                if key == "winning_team":
                    rhs = {"Re": 0, "Kontra": 1}[last(rhs[1])]
                elif key == "re_players":
                    continue
                elif isinstance(rhs, tuple) and rhs[0] == "list":
                    rhs = rhs[1]
                exp[key] = rhs
        re = 0
        for p in env["re_players"][2][0][1]:
            re |= 1 << player(p)
        out.append({"test": tname, "re_players": re, "eyes": env["player_eyes"][1],
                    "ntricks": env["player_num_tricks"][1], "expect": exp})
    return out


def jsonable(x):
    if isinstance(x, tuple):
        return [x[0]] + [jsonable(v) for v in x[1:]]
    if isinstance(x, list):
        return [jsonable(v) for v in x]
    if isinstance(x, dict):
        return {k: jsonable(v) for k, v in x.items()}
    return x


def main():
    win, draw = basic_points()
    wc = win_conditions()
    fdo = {
        "source": "rs-full-doko unit tests (see the docstring of tests/golden/make_rule_kats.py for file:line)",
        "card_order": card_order(), "card_to_color": card_to_color(), "card_eyes": card_eyes(),
        "tricks": tricks_group(), "team": team_group(), "reservation": reservation_group(),
        "calc_allowed": calc_allowed_group(), "ann_rounds": ann_rounds_group(), "stats": stats_group(),
        "re_won": wc["re_won"], "kontra_won": wc["kontra_won"], "basic_winning": win, "basic_draw": draw,
        "additional": additional_group(), "is_consistent": is_consistent_group(),
        "fields": {"basic_winning": WIN_FIELDS, "basic_draw": DRAW_FIELDS, "additional": ADD_FIELDS},
    }
    do = {"source": "rs-doko unit tests", "allowed": do_allowed(), "team": do_team(), "stats": do_stats()}
    with open(os.path.join(OUT, "rule_kats_fdo.json"), "w") as fh:
        json.dump(jsonable(fdo), fh, separators=(",", ":"))
    with open(os.path.join(OUT, "rule_kats_do.json"), "w") as fh:
        json.dump(do, fh, separators=(",", ":"))
    for k, v in fdo.items():
        if isinstance(v, list):
            print("fdo", k, len(v))
        elif k == "additional":
            print("fdo additional", {a: len(b) for a, b in v.items()})
    for k, v in do.items():
        if isinstance(v, list):
            print("do", k, len(v))


if __name__ == "__main__":
    main()
