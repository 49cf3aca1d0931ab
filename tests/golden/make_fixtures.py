"""Extract golden vectors from the reference's own test code into JSON fixtures.

Run HERE (the container that has /root/reference); the GPU box never reads the
reference. The output files are data only (inputs + expected outputs):

* fdo_traces.json — the four full-game traces written as (commented) tests in
  rs-full-doko/src/state/state.rs:551-951, :955-1346, :1350-1552, :1558-1808:
  initial hands, start player, every action, and after every action the
  expected phase / current player / legal-action set / eyes / trick winners /
  lowest announcements, ending in the expected FdoEndOfGameStats.
* fdo_deal_seed42.json — the seeded deal of rs-full-doko/src/hand/hand.rs:558-585.
* do_display_game.json — the finished rs-doko game of
  rs-doko/src/display/display.rs:242-280 (tricks + expected eyes / re points).
* bitflag_select_rank.json — rs-game-utils/src/bit_flag.rs:186-192.
* ttt_kats.json — rs-doko-mcts/src/example/tic_tac_toe.rs tests (finish states).
* fusion_kats.json — rs-doko-py-bridge/src/compare_impi/policy_fusion.rs:130-311.
* do_assignment_kats.json — rs-doko-assignment/src/assignment.rs:593-1190 (rule-based sampler).
* encode_pi_kat.json — rs-doko-networks/src/full_doko/var1/encode_pi.rs:237-797 (AlphaZero network input).

Usage: python tests/golden/make_fixtures.py
"""
import json
import os
import re

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))

CARD_NAMES = [
    "DiamondNine", "DiamondTen", "DiamondJack", "DiamondQueen", "DiamondKing", "DiamondAce",
    "HeartNine", "HeartTen", "HeartJack", "HeartQueen", "HeartKing", "HeartAce",
    "ClubNine", "ClubTen", "ClubJack", "ClubQueen", "ClubKing", "ClubAce",
    "SpadeNine", "SpadeTen", "SpadeJack", "SpadeQueen", "SpadeKing", "SpadeAce",
]
ACTION_NAMES = ["Card" + c for c in CARD_NAMES] + [
    "ReservationHealthy", "ReservationWedding", "ReservationDiamondsSolo", "ReservationHeartsSolo",
    "ReservationSpadesSolo", "ReservationClubsSolo", "ReservationTrumplessSolo", "ReservationQueensSolo",
    "ReservationJacksSolo", "AnnouncementReContra", "AnnouncementNo90", "AnnouncementNo60",
    "AnnouncementNo30", "AnnouncementBlack", "NoAnnouncement",
]
PLAYERS = {"BOTTOM": 0, "LEFT": 1, "TOP": 2, "RIGHT": 3}
PHASES = {"Reservation": 0, "Announcement": 1, "PlayCard": 2, "Finished": 3}
GAME_TYPES = {"Normal": 0, "Wedding": 1, "DiamondsSolo": 2, "HeartsSolo": 3, "SpadesSolo": 4,
              "ClubsSolo": 5, "TrumplessSolo": 6, "QueensSolo": 7, "JacksSolo": 8}
ANN = {"ReContra": 1, "No90": 2, "No60": 4, "No30": 8, "Black": 16, "CounterReContra": 32}


def _uncomment(lines):
    out = []
    for ln in lines:
        s = ln.lstrip()
        if s.startswith("//"):
            s = s[2:]
        out.append(s)
    return out


def _bracket(text, start):
    """Return the substring of balanced {...} starting at text[start] == '{'."""
    depth = 0
    for i in range(start, len(text)):
        if text[i] == "{":
            depth += 1
        elif text[i] == "}":
            depth -= 1
            if depth == 0:
                return text[start:i + 1]
    raise ValueError("unbalanced")


def _parse_obs(obs):
    d = {}
    d["phase"] = PHASES[re.search(r"phase: FdoPhase::(\w+)", obs).group(1)]
    m = re.search(r"current_player: (None|Some\(FdoPlayer::(\w+)\))", obs)
    d["current_player"] = -1 if m.group(1) == "None" else PLAYERS[m.group(2)]
    m = re.search(r"allowed_actions_current_player: FdoAllowedActions::from_vec\(vec!\[([^\]]*)\]\)", obs)
    names = [x.strip() for x in m.group(1).split(",") if x.strip()]
    d["allowed"] = sorted(ACTION_NAMES.index(n) for n in names)
    m = re.search(r"game_type: (None|Some\(FdoGameType::(\w+)\))", obs)
    d["game_type"] = -1 if m.group(1) == "None" else GAME_TYPES[m.group(2)]
    m = re.search(r"player_eyes: \[(\d+), (\d+), (\d+), (\d+)\]", obs)
    d["player_eyes"] = [int(x) for x in m.groups()]
    d["trick_winners"] = [(-1 if w == "None" else PLAYERS[w2]) for w, w2 in
                          re.findall(r"winning_player: (None|Some\(FdoPlayer::(\w+)\))", obs.split("visible_reservations")[0])]
    m = re.search(r"re_lowest_announcement: (None|Some\((\w+)\))", obs)
    d["re_lowest"] = -1 if m.group(1) == "None" else ANN[m.group(2)]
    m = re.search(r"contra_lowest_announcement: (None|Some\((\w+)\))", obs)
    d["contra_lowest"] = -1 if m.group(1) == "None" else ANN[m.group(2)]
    m = re.search(r"observing_player_hand: FdoHand::from_vec\(vec!\[([^\]]*)\]\)", obs)
    d["observing_hand"] = sorted(CARD_NAMES.index(x.strip()) for x in m.group(1).split(",") if x.strip())
    m = re.search(r"phi_re_players: (None|Some\(FdoPlayerSet::from_vec\(vec!\[([^\]]*)\]\)\))", obs)
    if m.group(1) == "None":
        d["re_players"] = -1
    else:
        d["re_players"] = sum(1 << PLAYERS[p.strip().split("::")[1]] for p in m.group(2).split(",") if p.strip())
    fs = obs.find("finished_stats: Some(")
    if fs >= 0:
        st = _bracket(obs, obs.find("{", fs))
        f = {}
        for key in ("re_eyes", "kontra_eyes", "re_points", "kontra_points"):
            f[key] = int(re.search(key + r": (-?\d+)", st).group(1))
        f["is_solo"] = re.search(r"is_solo: (\w+)", st).group(1) == "true"
        f["player_points"] = [int(x) for x in re.search(r"player_points: \[(-?\d+), (-?\d+), (-?\d+), (-?\d+)\]", st).groups()]
        d["finished"] = f
    else:
        d["finished"] = None
    return d


def fdo_traces():
    path = os.path.join(REF, "rs-full-doko/src/state/state.rs")
    with open(path, encoding="utf-8") as fh:
        all_lines = fh.readlines()
    spans = [("full_normal_game", 551, 951), ("full2_clubs_solo", 955, 1346),
             ("test_full3_wedding", 1350, 1552), ("test_full4_silent_solo", 1558, 1808)]
    games = []
    for name, a, b in spans:
        text = "\n".join(_uncomment(all_lines[a - 1:b]))
        hands = [sorted(CARD_NAMES.index(c.strip()) for c in h.split(","))
                 for h in re.findall(r"FdoHand::from_vec\(vec!\[([^\]]*)\]\)", text.split(");")[0])][:4]
        start = PLAYERS[re.search(r"\],\s*FdoPlayer::(\w+),", text).group(1)]
        steps = []
        # The first assertion describes the initial state.
        pos = 0
        pending_action = None
        token = re.compile(r"state\.play_action\((\w+)\);|assert_eq!\(state\.observation_for_current_player\(\), FdoObservation ")
        while True:
            m = token.search(text, pos)
            if not m:
                break
            if m.group(1):
                pending_action = ACTION_NAMES.index(m.group(1))
                pos = m.end()
            else:
                obs = _bracket(text, text.find("{", m.end() - 1))
                steps.append({"action": pending_action, "expect": _parse_obs(obs)})
                pending_action = None
                pos = m.end() + len(obs)
        games.append({"name": name, "source": "rs-full-doko/src/state/state.rs:%d-%d" % (a, b),
                      "hands": hands, "start_player": start, "steps": steps})
    return games


def deal_seed42():
    path = os.path.join(REF, "rs-full-doko/src/hand/hand.rs")
    with open(path, encoding="utf-8") as fh:
        lines = fh.readlines()
    text = "".join(lines[557:585])
    vals = [int(x, 2) for x in re.findall(r"0b([01]+)", text)]
    return {"source": "rs-full-doko/src/hand/hand.rs:558-585", "seed": 42, "hands": vals[:4]}


def do_display_game():
    path = os.path.join(REF, "rs-doko/src/display/display.rs")
    with open(path, encoding="utf-8") as fh:
        lines = fh.readlines()
    text = "".join(lines[241:280])
    tricks = []
    for sp, cards in re.findall(r"DoTrick::existing\((PLAYER_\w+), vec!\[([^\]]*)\]\)", text):
        tricks.append({"start": PLAYERS[sp.split("_")[1]],
                       "cards": [CARD_NAMES.index(c.strip().split("::")[1]) for c in cards.split(",")]})
    eyes = [int(x) for x in re.search(r"player_eyes: \[(\d+), (\d+), (\d+), (\d+)\]", text).groups()]
    fin = re.search(r"re_eyes: (\d+), kontra_eyes: (\d+), re_points: (-?\d+), kontra_points: (-?\d+)", text)
    return {"source": "rs-doko/src/display/display.rs:242-280", "tricks": tricks, "player_eyes": eyes,
            "re_eyes": int(fin.group(1)), "kontra_eyes": int(fin.group(2)),
            "re_points": int(fin.group(3)), "kontra_points": int(fin.group(4)),
            "note": "player_points/phi_team_eyes in that fixture are hand-typed and inconsistent; "
                    "eyes, re/kontra eyes and points are the checked fields"}


def select_rank():
    path = os.path.join(REF, "rs-game-utils/src/bit_flag.rs")
    with open(path, encoding="utf-8") as fh:
        lines = fh.readlines()
    text = "".join(lines[185:193])
    cases = [{"v": int(v, 2), "r": int(r), "expect": int(e, 2)}
             for v, r, e in re.findall(r"select_by_rank\(0b([01]+), (\d+)\), 0b([01]+)\)", text)]
    return {"source": "rs-game-utils/src/bit_flag.rs:186-192", "cases": cases}


def ttt_kats():
    path = os.path.join(REF, "rs-doko-mcts/src/example/tic_tac_toe.rs")
    with open(path, encoding="utf-8") as fh:
        text = fh.read()
    tests = text[text.find("#[cfg(test)]"):]
    fin = {"Xwon": 1, "Owon": 2, "Draw": 3, "NotFinished": 0}
    cases = []
    for board, st in re.findall(r'str_to_state\("([ XO]{9})"\);\s*let finish_state = state\.finish_state\(\);\s*'
                                r'assert_eq!\(TicTacToeFinishState::(\w+), finish_state\)', tests):
        cases.append({"board": board, "finish": fin[st]})
    succ = []
    for body in re.findall(r'fn test_possible_states_\w+\(\) \{(.*?)\n    \}', tests, re.S):
        m = re.search(r'str_to_state\("([ XO]{9})"\)', body)
        parent = "         " if "TicTacToeState::new()" in body else m.group(1)
        children = re.findall(r'assert_eq!\(str_to_state\("([ XO]{9})"\), possible_states\[\d+\]\)', body)
        succ.append({"board": parent, "successors": children})
    return {"source": "rs-doko-mcts/src/example/tic_tac_toe.rs:236-317", "cases": cases, "successors": succ}


def fusion_kats():
    path = os.path.join(REF, "rs-doko-py-bridge/src/compare_impi/policy_fusion.rs")
    with open(path, encoding="utf-8") as fh:
        text = fh.read()
    tests = text[text.find("#[cfg(test)]"):]
    names = {"idx_ten": 1, "idx_nine": 0, "idx_jack": 2, "idx_queen": 3,
             "a1_idx": 1, "a2_idx": 0, "a3_idx": 2, "a4_idx": 3}

    def action(tok):
        tok = tok.strip()
        m = re.match(r"FdoAction::from_index\((\d+)\)", tok)
        if m:
            return int(m.group(1))
        return ACTION_NAMES.index(tok.split("::")[1])

    cases = []
    for name, body in re.findall(r"async fn (test_\w+)\(\) \{(.*?)\n    \}\n", tests, re.S):
        mode = "maxn" if "PolicyFusionMaxN" in body else "avg"
        rows = []
        for blk in re.findall(r"\{\s*let mut s = dummy;(.*?)\bs\s*\}", body, re.S):
            row = [0] * 39
            for k, v in re.findall(r"s\[(\w+)\]\s*=\s*(\d+)", blk):
                row[int(k) if k.isdigit() else names[k]] = int(v)
            rows.append(row)
        allowed_blk = body[body.find("from_vec("):]
        allowed = [action(t) for t in re.findall(r"FdoAction::(?:from_index\(\d+\)|\w+)", allowed_blk.split("))")[0])]
        exp = re.search(r"assert_eq!\(\s*result,\s*(FdoAction::(?:from_index\(\d+\)|\w+))", body).group(1)
        cases.append({"name": name, "mode": mode, "visits": rows, "allowed": sorted(set(allowed)),
                      "expect": action(exp)})
    return {"source": "rs-doko-py-bridge/src/compare_impi/policy_fusion.rs:130-311", "cases": cases}


def _strip_line_comments(text):
    return "\n".join(ln.split("//")[0] for ln in text.split("\n"))


def _paren(text, start):
    """Return the content of the balanced (...) whose '(' is at text[start]."""
    depth = 0
    for i in range(start, len(text)):
        if text[i] in "([":
            depth += 1
        elif text[i] in ")]":
            depth -= 1
            if depth == 0:
                return text[start + 1:i]
    raise ValueError("unbalanced")


def _split_top(args):
    out, depth, cur = [], 0, ""
    for ch in args:
        if ch in "([":
            depth += 1
        elif ch in ")]":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _player(tok):
    tok = tok.strip()
    if tok.isdigit():
        return int(tok)
    return PLAYERS[tok.split("_")[1]]


def _cards(tok):
    return [CARD_NAMES.index(c.strip().split("::")[-1]) for c in tok.split(",") if c.strip()]


def _vec_cards(tok):
    m = re.match(r"\s*vec!\[(.*)\]\s*$", tok, re.S)
    return _cards(m.group(1))


def _tricks(tok):
    body = tok.strip()[2:-1]  # &[ ... ]
    tricks = []
    for t in _split_top(body):
        if t == "None":
            tricks.append(None)
            continue
        m = re.match(r"Some\(DoTrick::existing\(\s*(\w+)\s*,\s*vec!\[(.*)\]\s*\)\)$", t, re.S)
        tricks.append({"start": _player(m.group(1)), "cards": _cards(m.group(2))})
    assert len(tricks) == 12
    return tricks


def _hand(tok):
    tok = tok.strip()
    if tok.isdigit():
        return int(tok)
    m = re.match(r"hand_from_vec\((.*)\)$", tok, re.S)
    h = 0
    for c in _vec_cards(m.group(1)):
        h |= (1 << (c + 24)) if (h >> c) & 1 else (1 << c)
    return h


def _marriage(tok):
    tok = tok.strip()
    return -1 if tok == "None" else _player(re.match(r"Some\((\w+)\)", tok).group(1))


def do_assignment_kats():
    """rs-doko-assignment/src/assignment.rs:593-1190: player_allowed_to_have
    lists, calc_remaining_cards, and the support sets of 1000 seeded samples."""
    path = os.path.join(REF, "rs-doko-assignment/src/assignment.rs")
    with open(path, encoding="utf-8") as fh:
        text = fh.read()
    tests = _strip_line_comments(text[text.find("#[cfg(test)]"):])
    calls = []
    for m in re.finditer(r"(?<!fn )\b(player_allowed_to_have|calc_remaining_cards|brute_force_assignments)\(", tests):
        calls.append((m.start(), m.group(1), m.end() - 1))
    allowed, remaining, support = [], [], []
    for k, (pos, name, par) in enumerate(calls):
        args = _split_top(_paren(tests, par))
        tail = tests[par:calls[k + 1][0] if k + 1 < len(calls) else len(tests)]
        if name == "player_allowed_to_have":
            exp = {}
            for i, v in re.findall(r"assert_eq!\(result\[(\d)\], vec!\[([^\]]*)\]\);", tail):
                exp[int(i)] = _cards(v)
            allowed.append({"marriage": _marriage(args[0]), "tricks": _tricks(args[1]), "hand": _hand(args[2]),
                            "observer": _player(args[3]), "expect": [exp[i] for i in range(4)]})
        elif name == "calc_remaining_cards":
            v = re.search(r"assert_eq!\(remaining_cards_as_vec, vec!\[([^\]]*)\]\)", tail, re.S).group(1)
            remaining.append({"tricks": _tricks(args[0]), "hand": _hand(args[1]), "expect": _cards(v)})
        elif name == "brute_force_assignments":
            n = re.search(r"assert_eq!\(result\.len\(\), (\d+)\)", tail)
            sets = [[_cards(h) for h in re.findall(r"vec!\[([^\]]*)\]", blk)]
                    for blk in re.findall(r"result\.contains\(&\[(.*?)\]\)\);", tail, re.S)]
            support.append({"marriage": _marriage(args[0]), "tricks": _tricks(args[1]), "hand": _hand(args[2]),
                            "lengths": [int(x) for x in re.findall(r"\d+", args[3])], "observer": _player(args[4]),
                            "seed": 42, "draws": 1000, "expect_len": int(n.group(1)) if n else None,
                            "expect_contains": sets})
    return {"source": "rs-doko-assignment/src/assignment.rs:593-1190",
            "note": "support cases draw 1000 samples from ONE SmallRng::seed_from_u64(42) stream; expect_len is the "
                    "number of distinct (sorted) assignments; a case without expect_len must only not panic",
            "allowed_to_have": allowed, "remaining": remaining, "support": support}


def _var2_tables():
    """Token tables of the encoder helpers, read from their match arms
    (rs-doko-networks/src/full_doko/var2/encode_reservation_or_card_or_none.rs)."""
    path = os.path.join(REF, "rs-doko-networks/src/full_doko/var2/encode_reservation_or_card_or_none.rs")
    with open(path, encoding="utf-8") as fh:
        text = fh.read()
    def arms(fn, enum):
        body = text[text.find("pub fn " + fn):]
        body = body[:body.find("\npub fn ", 10) if "\npub fn " in body[10:] else len(body)]
        return {k: int(v) for k, v in re.findall(enum + r"::(\w+) => \[(\d+)\]", body)}, \
               int(re.search(r"None => \[(\d+)\]", body).group(1)) if re.search(r"None => \[(\d+)\]", body) else None
    return {"card": arms("encode_reservation_or_card_or_none_card", "FdoCard"),
            "pi_ann": arms("encode_reservation_or_card_or_pi_announcement", "FdoAnnouncement"),
            "pi_res": arms("encode_reservation_or_card_or_pi_reservation", "FdoReservation"),
            "vis_res": arms("encode_reservation_or_card_or_reservation", "FdoVisibleReservation")}


FDO_RES = ["Healthy", "Wedding", "DiamondsSolo", "HeartsSolo", "SpadesSolo", "ClubsSolo", "QueensSolo", "JacksSolo",
           "TrumplessSolo"]
ANN_BITS = {"ReContra": 1, "No90": 2, "No60": 4, "No30": 8, "Black": 16, "CounterReContra": 32}


def _kat_state(t):
    """Fields of the FdoState literal of an encoder test (tricks, hands, announcements ...)."""
    card = lambda n: CARD_NAMES.index(n.split("::")[-1].strip())
    m = re.search(r"reservations: PlayerOrientedVec::from_full\(FdoPlayer::(\w+), vec!\[(.*?)\]\)", t, re.S)
    res_start = PLAYERS[m.group(1)]
    res = [FDO_RES.index(x.strip().split("::")[-1]) for x in m.group(2).split(",") if x.strip()]
    tricks = []
    for sp, cs in re.findall(r"FdoTrick \{\s*cards: PlayerOrientedVec::from_full\(FdoPlayer::(\w+), vec!\[(.*?)\]\)", t, re.S):
        tricks.append({"start": PLAYERS[sp], "cards": [card(x) for x in cs.split(",") if x.strip()]})
    hm = re.search(r"hands: PlayerZeroOrientedArr::from_full\(\[(.*?)\]\),\s*announcements", t, re.S).group(1)
    hands = _hands_of(hm)
    anns = [{"card_index": int(ci), "player": PLAYERS[p], "bit": ANN_BITS[a]}
            for ci, p, a in re.findall(r"FdoAnnouncementOccurrence \{\s*card_index: (\d+),\s*player: FdoPlayer::(\w+),\s*"
                                       r"announcement: (\w+),", t, re.S)]
    cur = PLAYERS[re.search(r"current_player: Some\(FdoPlayer::(\w+)\)", t).group(1)]
    phase = PHASES[re.search(r"current_phase: FdoPhase::(\w+)", t).group(1)]
    re_players = 0
    for p in re.findall(r"FdoPlayer::(\w+)", re.search(r"re_players: FdoPlayerSet::from_vec\(vec!\[(.*?)\]\)", t).group(1)):
        re_players |= 1 << PLAYERS[p]
    return {"res_start": res_start, "res": res, "tricks": tricks, "hands": hands, "announcements": anns,
            "current_player": cur, "phase": phase, "re_players": re_players}


def _hands_of(text):
    """FdoHand::from_vec literals -> FdoHand bits (add: first copy, then second copy)."""
    card = lambda n: CARD_NAMES.index(n.split("::")[-1].strip())
    hands = []
    for cs in re.findall(r"FdoHand::from_vec\(vec!\[(.*?)\]\)", text, re.S):
        h = 0
        for c in [card(x) for x in cs.split(",") if x.strip()]:
            h |= (1 << (c + 24)) if (h >> c) & 1 else (1 << c)
        hands.append(h)
    return hands


def _kat_tokens(t):
    """The expected tokens: the test's assert_eq_inc! helper calls, evaluated with the helpers' tables."""
    pl = lambda n: PLAYERS[n.split("::")[-1].strip()]
    tab = _var2_tables()

    def ev(fn, arg):
        arg = arg.strip()
        a0 = arg.split(",")[0].strip()
        if fn == "encode_reservation_or_card_or_reservation":
            return tab["vis_res"][0][re.search(r"FdoVisibleReservation::(\w+)", arg).group(1)]
        if fn == "encode_reservation_or_card_or_none_card":
            return tab["card"][0][re.search(r"FdoCard::(\w+)", arg).group(1)] if "Some" in arg else tab["card"][1]
        if fn == "encode_reservation_or_card_or_pi_announcement":
            return tab["pi_ann"][0][re.search(r"Some\((\w+)\)", arg).group(1)] if "Some" in arg else tab["pi_ann"][1]
        if fn == "encode_position_or_unknown_int":
            return int(a0) + 1
        if fn == "encode_position_or_unknown_hand":
            if a0 == "None":
                return 0
            return (pl(re.search(r"Some\(FdoPlayer::(\w+)\)", arg).group(1)) - pl(arg.split(",")[1])) % 4 + 1 + 52
        if fn == "encode_player_or_none":
            if a0 == "None":
                return 0
            return (pl(re.search(r"Some\(FdoPlayer::(\w+)\)", arg).group(1)) - pl(arg.split(",")[1])) % 4 + 1
        if fn == "encode_subposition_card":
            return 0 if a0 == "None" else {0: 11, 1: 12}[int(re.search(r"Some\((\d+)\)", arg).group(1))]
        if fn == "encode_subposition_pos":
            return 0 if a0 == "None" else int(re.search(r"Some\((\d+)\)", arg).group(1)) + 1
        if fn == "encode_announcement_team":
            return 0 if a0 == "None" else {"Re": 1, "Kontra": 2}[re.search(r"FdoTeam::(\w+)", arg).group(1)]
        if fn == "encode_phase":
            return PHASES[re.search(r"FdoPhase::(\w+)", arg).group(1)]
        raise ValueError(fn)

    calls = re.findall(r"assert_eq_inc!\(result\[i\.\.i\+1\], (\w+)\((.*?)\)\);", t)
    tokens = [ev(fn, arg) for fn, arg in calls]
    assert len(tokens) == 311
    return tokens


def encode_pi_kat():
    """rs-doko-networks/src/full_doko/var1/encode_pi.rs:237-797 (test_encode_state):
    the state's fields and the expected 311 tokens, the latter evaluated from the
    test's 311 helper-call assertions with the helpers' own token tables."""
    path = os.path.join(REF, "rs-doko-networks/src/full_doko/var1/encode_pi.rs")
    with open(path, encoding="utf-8") as fh:
        text = fh.read()
    t = text[text.find("fn test_encode_state"):]
    out = {"source": "rs-doko-networks/src/full_doko/var1/encode_pi.rs:237-797"}
    out.update(_kat_state(t))
    out["expect"] = _kat_tokens(t)
    return out


def encode_ipi_kat():
    """rs-doko-networks/src/full_doko/var1/encode_ipi.rs:307-888 (test_encode_state): the
    state, the assumed hands / reservations and the player to guess for, and the
    expected 311 tokens (evaluated from the test's helper-call assertions)."""
    path = os.path.join(REF, "rs-doko-networks/src/full_doko/var1/encode_ipi.rs")
    with open(path, encoding="utf-8") as fh:
        text = fh.read()
    t = text[text.find("fn test_encode_state"):]
    out = {"source": "rs-doko-networks/src/full_doko/var1/encode_ipi.rs:307-888"}
    out.update(_kat_state(t))
    call = t[t.find("let result = encode_state_ipi("):]
    call = call[:call.find(");")]
    out["assumed_hands"] = _hands_of(call)
    rm = re.search(r"PlayerZeroOrientedArr::from_full\(\s*\[(.*?)\]\s*\),\s*FdoPlayer::(\w+)",
                   call[call.rfind("PlayerZeroOrientedArr::from_full("):], re.S)
    out["assumed_res"] = [-1 if x.strip() == "None" else FDO_RES.index(re.search(r"FdoReservation::(\w+)", x).group(1))
                          for x in rm.group(1).split(",") if x.strip()]
    out["guess"] = PLAYERS[rm.group(2)]
    out["expect"] = _kat_tokens(t)
    return out


def main():
    with open(os.path.join(OUT, "fdo_traces.json"), "w") as fh:
        json.dump(fdo_traces(), fh, indent=0)
    with open(os.path.join(OUT, "fdo_deal_seed42.json"), "w") as fh:
        json.dump(deal_seed42(), fh, indent=1)
    with open(os.path.join(OUT, "do_display_game.json"), "w") as fh:
        json.dump(do_display_game(), fh, indent=1)
    with open(os.path.join(OUT, "bitflag_select_rank.json"), "w") as fh:
        json.dump(select_rank(), fh, indent=1)
    with open(os.path.join(OUT, "ttt_kats.json"), "w") as fh:
        json.dump(ttt_kats(), fh, indent=1)
    with open(os.path.join(OUT, "fusion_kats.json"), "w") as fh:
        json.dump(fusion_kats(), fh, indent=1)
    with open(os.path.join(OUT, "do_assignment_kats.json"), "w") as fh:
        json.dump(do_assignment_kats(), fh, indent=None)
    with open(os.path.join(OUT, "encode_pi_kat.json"), "w") as fh:
        json.dump(encode_pi_kat(), fh, indent=None)
    with open(os.path.join(OUT, "encode_ipi_kat.json"), "w") as fh:
        json.dump(encode_ipi_kat(), fh, indent=None)
    print("wrote fixtures to", OUT)


if __name__ == "__main__":
    main()
