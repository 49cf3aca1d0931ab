// ORACLE — test infrastructure only. Never linked into the product library.
// Restates rs-full-doko (/root/reference/rs-full-doko/src); each function cites
// the reference location it follows.
#include "full_doko.hpp"
#include <cstdio>
#include <cstdlib>

namespace oracle {
namespace fdo {

static void panic(const char* msg) { fprintf(stderr, "oracle panic: %s\n", msg); abort(); }

// hand/hand.rs:215-229
void Hand::add(int c) {
    if (bits >> c & 1) bits |= 1ULL << (c + SECOND);
    else bits |= 1ULL << c;
}
// hand/hand.rs:235-247 — the second copy (bit c+24) is removed first.
void Hand::remove(int c) {
    if (bits >> (c + SECOND) & 1) bits &= ~(1ULL << (c + SECOND));
    else if (bits >> c & 1) bits &= ~(1ULL << c);
    else panic("Karte nicht in Hand");
}
// hand/hand.rs:256-266
void Hand::remove_both(int c) {
    if (contains(c)) { remove(c); if (contains(c)) remove(c); }
    else panic("Karte nicht in Hand (remove_both)");
}
// hand/hand.rs:45-62
void Hand::remove_color(int color, int game_type) {
    uint64_t m[5]; color_masks(game_type, m);
    bits &= ~(m[color] | (m[color] << SECOND));
}
// hand/hand.rs:68-82 — iterates FdoCard::iter() (declaration order).
Hand Hand::plus_hand(const Hand& other) const {
    Hand h = *this;
    for (int c = 0; c < 24; ++c) {
        if (other.contains_both(c)) { h.add(c); h.add(c); }
        else if (other.contains(c)) h.add(c);
    }
    return h;
}

// card/card_to_color.rs:11-259.  Suit of kind k: 0 diamond, 1 heart, 2 club, 3 spade.
static int suit_color(int card) {
    switch (card / 6) { case 0: return Diamond; case 1: return Heart; case 2: return Club; default: return Spade; }
}
static bool is_jack(int c) { return c % 6 == 2; }
static bool is_queen(int c) { return c % 6 == 3; }
int card_to_color(int card, int game_type) {
    switch (game_type) {
        case Normal: case GWedding: case GDiamondsSolo:
            if (card / 6 == 0 || card == HeartTen || is_jack(card) || is_queen(card)) return Trump;
            return suit_color(card);
        case GHeartsSolo:
            if (card / 6 == 1 || is_jack(card) || is_queen(card)) return Trump;
            return suit_color(card);
        case GSpadesSolo:
            if (card / 6 == 3 || card == HeartTen || is_jack(card) || is_queen(card)) return Trump;
            return suit_color(card);
        case GClubsSolo:
            if (card / 6 == 2 || card == HeartTen || is_jack(card) || is_queen(card)) return Trump;
            return suit_color(card);
        case GTrumplessSolo: return suit_color(card);
        case GQueensSolo: return is_queen(card) ? Trump : suit_color(card);
        case GJacksSolo: return is_jack(card) ? Trump : suit_color(card);
    }
    panic("bad game type");
    return 0;
}
// card/card_to_eyes.rs:11-41
uint32_t card_eyes(int card) {
    static const uint32_t e[6] = {0, 10, 2, 3, 4, 11};
    return e[card % 6];
}
// card/card_color_masks.rs:7-249 (the masks equal the card_to_color partition).
void color_masks(int game_type, uint64_t out[5]) {
    for (int i = 0; i < 5; ++i) out[i] = 0;
    for (int c = 0; c < 24; ++c) out[card_to_color(c, game_type)] |= 1ULL << c;
}

// card/card_in_trick_logic.rs:17-86 (trump_to_rank)
static int trump_to_rank(int card) {
    switch (card) {
        case DiamondNine: return 0; case DiamondKing: return 1; case DiamondTen: return 2; case DiamondAce: return 3;
        case HeartNine: return 0; case HeartKing: return 1; case HeartAce: return 2;
        case SpadeNine: return 0; case SpadeKing: return 1; case SpadeTen: return 2; case SpadeAce: return 3;
        case ClubNine: return 0; case ClubKing: return 1; case ClubTen: return 2; case ClubAce: return 3;
        case DiamondJack: return 4; case HeartJack: return 5; case SpadeJack: return 6; case ClubJack: return 7;
        case DiamondQueen: return 8; case HeartQueen: return 9; case SpadeQueen: return 10; case ClubQueen: return 11;
        case HeartTen: return 12;
    }
    panic("bad card");
    return 0;
}
// card/card_in_trick_logic.rs:95-141
bool is_greater_in_trick(int cur, int prev, int trick_color, int game_type) {
    const int cc = card_to_color(cur, game_type), pc = card_to_color(prev, game_type);
    const bool ct = cc == Trump, pt = pc == Trump;
    if (ct && !pt) return true;
    if (!ct && pt) return false;
    if (ct && pt) return trump_to_rank(prev) < trump_to_rank(cur);
    const bool ctc = cc == trick_color, ptc = pc == trick_color;
    if (ctc && !ptc) return true;
    if (ctc && ptc) return card_eyes(cur) > card_eyes(prev);
    return false;
}
// trick/trick.rs:30-37
int trick_color(const Trick& t, int game_type) {
    if (t.len == 0) return -1;
    return card_to_color(t.cards[0], game_type);
}
// trick/trick.rs:86-107 + trick_winning_player_logic.rs:15-44
void trick_play_card(Trick& t, int card, int game_type) {
    if (t.len >= 4) panic("trick complete");
    t.cards[t.len++] = card;
    if (t.len == 4) {
        const int tc = trick_color(t, game_type);
        int wc = t.cards[0], wp = t.player_at(0);
        for (int i = 1; i < 4; ++i) {
            if (is_greater_in_trick(t.cards[i], wc, tc, game_type)) { wc = t.cards[i]; wp = t.player_at(i); }
        }
        t.winning_player = wp;
        t.winning_card = wc;
    }
}

// rs-game-utils/src/bit_flag.rs:104-171 — the bit with rank r counted from the MSB.
uint64_t select_by_rank(uint64_t v, uint64_t r) {
    for (int b = 63; b >= 0; --b) {
        if (v >> b & 1) { if (r == 0) return 1ULL << b; --r; }
    }
    panic("select_by_rank out of range");
    return 0;
}
// rs-game-utils/src/bit_flag.rs:86-92
uint64_t random_single(uint64_t mask, SmallRng& rng) {
    const uint32_t n = (uint32_t)__builtin_popcountll(mask);
    if (n == 0) panic("cannot sample empty range");
    const uint32_t index = rng.random_range_u32(0, n);
    return select_by_rank(mask, index);
}

// action/allowed_actions.rs:68-169
uint64_t calculate_allowed_actions(int phase, int tcolor, Hand hand, int game_type, uint32_t allowed_ann) {
    switch (phase) {
        case Reservation: {
            uint64_t a = abit(A_ReservationHealthy);
            if (hand.contains_both(ClubQueen)) a |= abit(A_ReservationWedding);
            a |= abit(A_ReservationJacksSolo) | abit(A_ReservationQueensSolo) | abit(A_ReservationDiamondsSolo) |
                 abit(A_ReservationHeartsSolo) | abit(A_ReservationSpadesSolo) | abit(A_ReservationClubsSolo) |
                 abit(A_ReservationTrumplessSolo);
            return a;
        }
        case PlayCard: {
            const uint64_t single = (hand.bits | (hand.bits >> 24)) & 0xFFFFFFULL;
            if (tcolor < 0) return single;
            uint64_t m[5]; color_masks(game_type, m);
            const uint64_t mask = m[tcolor];
            if (single & mask) return single & mask;
            return single;
        }
        case Finished: panic("Es sind keine Aktionen mehr moeglich"); return 0;
        case Announcement: {
            uint64_t a = 0;
            if ((allowed_ann & CounterReContra) || (allowed_ann & ReContra)) a |= abit(A_AnnouncementReContra);
            if (allowed_ann & No90) a |= abit(A_AnnouncementNo90);
            if (allowed_ann & No60) a |= abit(A_AnnouncementNo60);
            if (allowed_ann & No30) a |= abit(A_AnnouncementNo30);
            if (allowed_ann & Black) a |= abit(A_AnnouncementBlack);
            a |= abit(A_NoAnnouncement);
            return a;
        }
    }
    panic("bad phase");
    return 0;
}

// announcement/announcement_set.rs:25-61
uint32_t all_higher_than(int lowest) {
    switch (lowest) {
        case -1: return 0;
        case ReContra: return ReContra;
        case No90: return ReContra | No90;
        case No60: return ReContra | No90 | No60;
        case No30: return ReContra | No90 | No60 | No30;
        case Black: return ReContra | No90 | No60 | No30 | Black;
        case CounterReContra: return CounterReContra;
        default: return 0;
    }
}

// announcement/calc_announcement.rs:21-48
static int calc_cards_last_announcement(uint32_t prev, int w, bool* some) {
    *some = true;
    if (prev & Black) return 7 - w;
    if (prev & No30) return 8 - w;
    if (prev & No60) return 9 - w;
    if (prev & No90) return 10 - w;
    if (prev & ReContra) return 11 - w;
    *some = false;
    return 0;
}

// announcement/calc_announcement.rs:51-174
static uint32_t internal_calc_allowed(int n, uint32_t prev, int w, bool enemy_some, int enemy_cards) {
    const int a0 = 11 - w, a90 = 10 - w, a60 = 9 - w, a30 = 8 - w, ab = 7 - w;
    uint32_t rem = 0;
    const bool p = n >= a0;
    const bool p90 = p || (n >= a90 && (prev & ReContra));
    const bool p60 = p90 || (n >= a60 && (prev & No90));
    const bool p30 = p60 || (n >= a30 && (prev & No60));
    const bool pb = p30 || (n >= ab && (prev & No30));
    if (p) rem |= ReContra;
    if (p90) rem |= No90;
    if (p60) rem |= No60;
    if (p30) rem |= No30;
    if (pb) rem |= Black;
    rem &= ~(prev & (ReContra | No90 | No60 | No30 | Black));
    if (rem & ReContra) rem &= ~(No90 | No60 | No30 | Black);
    if (rem & No90) rem &= ~(No60 | No30 | Black);
    if (rem & No60) rem &= ~(No30 | Black);
    if (rem & No30) rem &= ~Black;
    const bool regular = rem != 0;
    if (enemy_some && !regular) {
        const bool by_cards = n >= enemy_cards - 1;
        const bool counter_done = prev & CounterReContra;
        const bool regular_done = prev & ReContra;
        if (by_cards && !counter_done && !(counter_done || regular_done)) rem |= CounterReContra;
    }
    return rem;
}

// announcement/calc_announcement.rs:177-229
uint32_t calc_allowed_announcements(int player, int n_cards, const TeamState& ts, int re_lowest, int contra_lowest) {
    int w = 0;
    uint8_t re = 0;
    switch (ts.kind) {
        case InReservations: panic("should not happen"); break;
        case WeddingUnsolved: return 0;
        case WeddingSolved: w = ts.solved_trick_index; re = ts.re_players; break;
        case NoWedding: re = ts.re_players; break;
    }
    const bool is_re = re >> player & 1;
    const int own = is_re ? re_lowest : contra_lowest;
    const int enemy = is_re ? contra_lowest : re_lowest;
    bool some;
    const int enemy_cards = calc_cards_last_announcement(all_higher_than(enemy), w, &some);
    return internal_calc_allowed(n_cards, all_higher_than(own), w, some, enemy_cards);
}

// announcement/announcement.rs:182-215
static void internal_play_announcement(Announcements& a, int player, uint32_t ann, int card_index, const TeamState& ts) {
    if (ann == NoAnnouncement) { a.turns_without += 1; return; }
    a.turns_without = 0;
    if (a.n < 12) a.list[a.n++] = AnnOccurrence{card_index, player, ann};  // heapless push result ignored
    if (!ts.has_re()) panic("team unknown at announcement");
    if (ts.re_players >> player & 1) a.re_lowest = (int)ann;
    else a.contra_lowest = (int)ann;
}

enum { NextPlayerIs = 0, RoundIsOver = 1 };
// announcement/announcement.rs:137-180
static int internal_progress(Announcements& a, int player, int card_index, const int hand_lens[4], const TeamState& ts, int* next) {
    int cp = player;
    for (;;) {
        if (a.turns_without == 4) { a.allowed = 0; *next = a.starting_player; return RoundIsOver; }
        const uint32_t allowed = calc_allowed_announcements(cp, hand_lens[cp], ts, a.re_lowest, a.contra_lowest);
        if (allowed == 0) internal_play_announcement(a, cp, NoAnnouncement, card_index, ts);
        else { a.allowed = allowed; *next = cp; return NextPlayerIs; }
        cp = (cp + 1) % 4;
    }
}

static void hand_lens(const State& s, int out[4]) { for (int i = 0; i < 4; ++i) out[i] = s.hands[i].len(); }

// state/state.rs:184-206
static void progress_next_card_or_announcement(State& s) {
    int hl[4]; hand_lens(s, hl);
    s.announcements.turns_without = 0;                 // start_round (announcement.rs:83-101)
    s.announcements.starting_player = s.current_player;
    int next;
    const int r = internal_progress(s.announcements, s.current_player, s.card_index, hl, s.team_state, &next);
    s.phase = r == NextPlayerIs ? Announcement : PlayCard;
    s.current_player = next;
}

// team/team_logic.rs:37-122
TeamState team_resolve(const ReservationResult& rr, const Trick* tricks, int n_tricks, const Hand* hands) {
    TeamState t;
    switch (rr.kind) {
        case NoReservation: {
            t.kind = NoWedding;
            for (int p = 0; p < 4; ++p) if (hands[p].contains(ClubQueen)) t.re_players |= 1 << p;
            return t;
        }
        case RWedding: {
            int partner = -1, solved = -1, completed = 0;
            for (int i = 0; i < 3; ++i) {
                if (i >= n_tricks) break;
                if (!tricks[i].is_completed()) break;
                completed += 1;
                const int winner = tricks[i].winning_player;
                if (winner != rr.player) { partner = winner; solved = i; break; }
            }
            t.wedding_player = rr.player;
            if (partner >= 0) {
                t.kind = WeddingSolved; t.solved_trick_index = solved;
                t.re_players = (uint8_t)((1 << rr.player) | (1 << partner));
                return t;
            }
            if (completed == 3) {
                t.kind = WeddingSolved; t.solved_trick_index = 2; t.re_players = (uint8_t)(1 << rr.player);
                return t;
            }
            t.kind = WeddingUnsolved;
            return t;
        }
        case Solo: {
            t.kind = NoWedding; t.re_players = (uint8_t)(1 << rr.player);
            return t;
        }
    }
    return t;
}

// reservation/reservation_winning_logic.rs:37-73
ReservationResult winning_player_in_reservation_round(const State& s) {
    ReservationResult rr;
    int wedding = -1;
    for (int i = 0; i < s.res_len; ++i) {
        const int player = (s.res_start + i) % 4;
        const int r = s.res[i];
        if (r == Wedding) wedding = player;
        else if (r == Healthy) {}
        else { rr.kind = Solo; rr.player = player; rr.reservation = r; return rr; }
    }
    if (wedding < 0) { rr.kind = NoReservation; return rr; }
    rr.kind = RWedding; rr.player = wedding;
    return rr;
}
// reservation_winning_logic.rs:16-33
int reservation_to_game_type(const ReservationResult& rr) {
    switch (rr.kind) {
        case NoReservation: return Normal;
        case RWedding: return GWedding;
        case Solo:
            switch (rr.reservation) {
                case DiamondsSolo: return GDiamondsSolo; case HeartsSolo: return GHeartsSolo;
                case SpadesSolo: return GSpadesSolo; case ClubsSolo: return GClubsSolo;
                case QueensSolo: return GQueensSolo; case JacksSolo: return GJacksSolo;
                case TrumplessSolo: return GTrumplessSolo;
            }
    }
    panic("not a valid solo");
    return 0;
}

static uint32_t trick_eyes(const Trick& t) { uint32_t e = 0; for (int i = 0; i < t.len; ++i) e += card_eyes(t.cards[i]); return e; }

// stats/win_conditions/re_won.rs:5-117 and kontra_won.rs:4-114
struct AnnFlags { bool ann, u90, u60, u30, black, none, only_ann, only_u90, only_u60, only_u30, only_black; };
static AnnFlags ann_flags(uint32_t prev) {
    AnnFlags f;
    f.ann = (prev & ReContra) || (prev & CounterReContra);
    f.u90 = prev & No90; f.u60 = prev & No60; f.u30 = prev & No30; f.black = prev & Black;
    f.none = __builtin_popcount(prev) == 0;
    f.only_ann = f.ann && !f.u90; f.only_u90 = f.u90 && !f.u60; f.only_u60 = f.u60 && !f.u30;
    f.only_u30 = f.u30 && !f.black; f.only_black = f.black;
    return f;
}
bool re_won(uint32_t re_eyes, uint32_t re_prev, uint32_t ko_prev, bool re_all, bool ko_all) {
    const AnnFlags r = ann_flags(re_prev), k = ann_flags(ko_prev);
    if (re_eyes >= 121 && r.none && k.none) return true;
    if (re_eyes >= 121 && r.only_ann && !k.ann) return true;
    if (re_eyes >= 121 && r.only_ann && k.only_ann) return true;
    if (re_eyes >= 120 && !r.ann && k.only_ann) return true;
    if (re_eyes >= 151 && r.only_u90) return true;
    if (re_eyes >= 181 && r.only_u60) return true;
    if (re_eyes >= 211 && r.only_u30) return true;
    if (re_all && r.only_black) return true;
    if (re_eyes >= 90 && k.only_u90 && !r.u90) return true;
    if (re_eyes >= 60 && k.only_u60 && !r.u90) return true;
    if (re_eyes >= 30 && k.only_u30 && !r.u90) return true;
    if (!ko_all && k.only_black && !r.u90) return true;
    return false;
}
bool kontra_won(uint32_t ko_eyes, uint32_t re_prev, uint32_t ko_prev, bool re_all, bool ko_all) {
    const AnnFlags r = ann_flags(re_prev), k = ann_flags(ko_prev);
    if (ko_eyes >= 120 && r.none && k.none) return true;
    if (ko_eyes >= 120 && r.only_ann && !k.ann) return true;
    if (ko_eyes >= 120 && r.only_ann && k.only_ann) return true;
    if (ko_eyes >= 121 && !r.ann && k.only_ann) return true;
    if (ko_eyes >= 151 && k.only_u90) return true;
    if (ko_eyes >= 181 && k.only_u60) return true;
    if (ko_eyes >= 211 && k.only_u30) return true;
    if (ko_all && k.only_black) return true;
    if (ko_eyes >= 90 && r.only_u90 && !k.u90) return true;
    if (ko_eyes >= 60 && r.only_u60 && !k.u90) return true;
    if (ko_eyes >= 30 && r.only_u30 && !k.u90) return true;
    if (!re_all && r.only_black && !k.u90) return true;
    return false;
}

// stats/basic_points/basic_winning_points.rs:48-285
// details[23] in the field order of FdoBasicWinningPointsDetails (basic_winning_points.rs:8-46)
void basic_winning_points(uint32_t loser_eyes, bool winner_all, uint32_t re_prev, uint32_t ko_prev,
                          uint32_t re_eyes, uint32_t ko_eyes, int* win, int* lose, int* details) {
    const AnnFlags r = ann_flags(re_prev), k = ann_flags(ko_prev);
    int d[23] = {0};
    d[0] = 1;                                        // (a) won
    d[1] = loser_eyes < 90; d[2] = loser_eyes < 60; d[3] = loser_eyes < 30; d[4] = winner_all;
    d[5] = r.ann ? 2 : 0;                            // (b)
    d[6] = k.ann ? 2 : 0;
    d[7] = r.u90; d[8] = r.u60; d[9] = r.u30; d[10] = r.black;       // (c)
    d[11] = k.u90; d[12] = k.u60; d[13] = k.u30; d[14] = k.black;    // (d)
    d[15] = re_eyes >= 120 && k.u90; d[16] = re_eyes >= 90 && k.u60; // (e)
    d[17] = re_eyes >= 60 && k.u30; d[18] = re_eyes >= 30 && k.black;
    d[19] = ko_eyes >= 120 && r.u90; d[20] = ko_eyes >= 90 && r.u60; // (f)
    d[21] = ko_eyes >= 60 && r.u30; d[22] = ko_eyes >= 30 && r.black;
    int w = 0;
    for (int i = 0; i < 23; ++i) w += d[i];
    if (details) for (int i = 0; i < 23; ++i) details[i] = d[i];
    *win = w; *lose = -w;
}
// stats/basic_points/basic_draw_points.rs:27-175
// details[14] in the field order of FdoBasicDrawPointsDetails (basic_draw_points.rs:8-25):
// winning_under_{90,60,30}_re, winning_under_{90,60,30}_kontra, re_reached_*, kontra_reached_*
void basic_draw_points(uint32_t re_prev, uint32_t ko_prev, uint32_t re_eyes, uint32_t ko_eyes, int* re, int* ko,
                       int* details) {
    const AnnFlags r = ann_flags(re_prev), k = ann_flags(ko_prev);
    int d[14] = {0};
    d[0] = ko_eyes < 90; d[1] = ko_eyes < 60; d[2] = ko_eyes < 30;      // Re's gains
    d[3] = re_eyes < 90; d[4] = re_eyes < 60; d[5] = re_eyes < 30;      // Kontra's gains
    d[6] = re_eyes >= 120 && k.u90; d[7] = re_eyes >= 90 && k.u60; d[8] = re_eyes >= 60 && k.u30; d[9] = re_eyes >= 30 && k.black;
    d[10] = ko_eyes >= 120 && r.u90; d[11] = ko_eyes >= 90 && r.u60; d[12] = ko_eyes >= 60 && r.u30; d[13] = ko_eyes >= 30 && r.black;
    const int rp = d[0] + d[1] + d[2] + d[6] + d[7] + d[8] + d[9];
    const int kp = d[3] + d[4] + d[5] + d[10] + d[11] + d[12] + d[13];
    if (details) for (int i = 0; i < 14; ++i) details[i] = d[i];
    *re = rp - kp; *ko = kp - rp;
}

// stats/additional_points/*.rs
AdditionalDetails additional_points(uint8_t re_players, int winning_team /*0 re,1 ko,-1 none*/,
                                           const Trick* tricks, int n_tricks, int* re_add, int* ko_add) {
    AdditionalDetails d{};
    for (int i = 0; i < n_tricks; ++i) {                       // doppelkopf.rs:8-28
        if (trick_eyes(tricks[i]) >= 40) {
            if (re_players >> tricks[i].winning_player & 1) d.doko_re++; else d.doko_kontra++;
        }
    }
    for (int i = 0; i < n_tricks; ++i) {                       // fuchs_gefangen.rs:9-61
        const Trick& t = tricks[i];
        const bool win_re = re_players >> t.winning_player & 1;
        for (int j = 0; j < t.len; ++j) {
            const int p = t.player_at(j);
            const bool p_re = re_players >> p & 1;
            if (t.cards[j] == DiamondAce && p_re != win_re) { if (win_re) d.fuchs_re++; else d.fuchs_kontra++; }
        }
    }
    const Trick& last = tricks[11];                            // last_trick_karlchen.rs:6-29
    if (last.winning_card == ClubJack) {
        if (re_players >> last.winning_player & 1) d.karlchen_re = true; else d.karlchen_kontra = true;
    }
    int ra = 0, ka = 0;                                        // additional_points.rs:61-128
    if (winning_team == 1) { ka += 1; ra -= 1; d.against_club_queens = true; }
    ra += d.doko_re; ka -= d.doko_re; ra -= d.doko_kontra; ka += d.doko_kontra;
    ra += d.fuchs_re; ka -= d.fuchs_re; ra -= d.fuchs_kontra; ka += d.fuchs_kontra;
    if (d.karlchen_re) { ra += 1; ka -= 1; }
    if (d.karlchen_kontra) { ra -= 1; ka += 1; }
    *re_add = ra; *ko_add = ka;
    return d;
}

// stats/stats.rs:46-243
EndOfGameStats calculate_stats(const uint32_t eyes[4], const uint32_t ntricks[4], uint8_t re_players,
                               int re_lowest, int contra_lowest, const Trick* tricks, int n_tricks) {
    EndOfGameStats s{};
    uint32_t re_tricks = 0, ko_tricks = 0, re_eyes = 0, ko_eyes = 0;
    for (int p = 0; p < 4; ++p) {
        if (re_players >> p & 1) { re_eyes += eyes[p]; re_tricks += ntricks[p]; }
        else { ko_eyes += eyes[p]; ko_tricks += ntricks[p]; }
    }
    const bool re_all = re_tricks == 12, ko_all = ko_tricks == 12;
    const uint32_t re_prev = all_higher_than(re_lowest), ko_prev = all_higher_than(contra_lowest);
    const bool rw = re_won(re_eyes, re_prev, ko_prev, re_all, ko_all);
    const bool kw = kontra_won(ko_eyes, re_prev, ko_prev, re_all, ko_all);
    const bool is_solo = __builtin_popcount(re_players) == 1;
    const int winning_team = rw ? 0 : (kw ? 1 : -1);
    int re_pts, ko_pts;
    if (!rw && !kw) {
        int rb, kb; basic_draw_points(re_prev, ko_prev, re_eyes, ko_eyes, &rb, &kb, s.draw_details);
        int ra = 0, ka = 0;
        if (!is_solo) { s.additional = additional_points(re_players, winning_team, tricks, n_tricks, &ra, &ka); s.has_additional = true; }
        re_pts = rb + ra; ko_pts = kb + ka;
        s.has_draw_details = true;
    } else {
        const uint32_t loser_eyes = rw ? ko_eyes : re_eyes;
        const bool winner_all = rw ? re_all : (kw ? ko_all : false);
        int wp, lp; basic_winning_points(loser_eyes, winner_all, re_prev, ko_prev, re_eyes, ko_eyes, &wp, &lp, s.win_details);
        int ra = 0, ka = 0;
        if (!is_solo) { s.additional = additional_points(re_players, winning_team, tricks, n_tricks, &ra, &ka); s.has_additional = true; }
        re_pts = rw ? wp + ra : lp + ra;
        ko_pts = kw ? wp + ka : lp + ka;
        s.has_winning_details = true;
    }
    if (is_solo) re_pts *= 3;
    s.re_players = re_players; s.is_solo = is_solo;
    for (int p = 0; p < 4; ++p) { s.player_eyes[p] = eyes[p]; s.player_points[p] = (re_players >> p & 1) ? re_pts : ko_pts; }
    s.re_eyes = re_eyes; s.kontra_eyes = ko_eyes; s.re_points = re_pts; s.kontra_points = ko_pts;
    return s;
}

// state/state.rs:121-162
State new_game_from_hand_and_start_player(const Hand hands[4], int start_player) {
    State s;
    s.res_start = start_player;
    for (int p = 0; p < 4; ++p) s.hands[p] = hands[p];
    s.current_player = start_player;
    s.phase = Reservation;
    return s;
}
// state/state.rs:165-176 + hand.rs:172-186 + player.rs:43-47
State new_game(SmallRng& rng) {
    const int start = (int)rng.random_range_usize(0, 4);
    int cards[48];
    for (int i = 0; i < 24; ++i) { cards[2 * i] = i; cards[2 * i + 1] = i; }
    shuffle(cards, 48, rng);
    Hand hands[4];
    for (int p = 0; p < 4; ++p) for (int j = 0; j < 12; ++j) hands[p].add(cards[p * 12 + j]);
    return new_game_from_hand_and_start_player(hands, start);
}

// state/state.rs:360-372
int current_trick_color(const State& s) {
    if (s.n_tricks > 0 && s.n_tricks < 12) return trick_color(s.tricks[s.n_tricks - 1], s.game_type);
    return -1;
}

// state/state.rs:208-358
void play_action(State& s, int a) {
    if (s.phase == Finished) panic("play_action on finished game");
    const int cp = s.current_player;
    if (a <= 23) {
        // Card
        if (!s.has_reservation_result) panic("no reservation result");
        s.hands[cp].remove(a);
        Trick& t = s.tricks[s.n_tricks - 1];
        trick_play_card(t, a, s.game_type);
        s.card_index += 1;
        if (t.is_completed()) {
            const int w = t.winning_player;
            s.player_eyes[w] += trick_eyes(t);
            s.player_num_tricks[w] += 1;
            if (!s.team_state.is_final()) s.team_state = team_resolve(s.reservation_result, s.tricks, s.n_tricks, s.hands);
            if (s.n_tricks == 12) {
                s.phase = Finished;
                s.current_player = -1;
                if (!s.team_state.has_re()) panic("teams unknown at game end");
                s.stats = calculate_stats(s.player_eyes, s.player_num_tricks, s.team_state.re_players,
                                          s.announcements.re_lowest, s.announcements.contra_lowest, s.tricks, s.n_tricks);
                s.has_stats = true;
                return;
            }
            s.current_player = w;
            s.tricks[s.n_tricks] = Trick(); s.tricks[s.n_tricks].start = w; s.n_tricks += 1;
            progress_next_card_or_announcement(s);
            return;
        }
        s.current_player = (cp + 1) % 4;
        progress_next_card_or_announcement(s);
    } else if (a <= 32) {
        // Reservation; action order differs from the FdoReservation enum order.
        static const int map[9] = {Healthy, Wedding, DiamondsSolo, HeartsSolo, SpadesSolo, ClubsSolo, TrumplessSolo, QueensSolo, JacksSolo};
        if (s.res_len >= 4) panic("reservation round complete");
        s.res[s.res_len++] = map[a - 24];
        const int np = (cp + 1) % 4;
        s.current_player = np;
        if (s.res_len == 4) {
            const ReservationResult rr = winning_player_in_reservation_round(s);
            s.reservation_result = rr; s.has_reservation_result = true;
            s.game_type = reservation_to_game_type(rr);
            if (!s.team_state.is_final()) s.team_state = team_resolve(rr, s.tricks, s.n_tricks, s.hands);
            s.tricks[s.n_tricks] = Trick(); s.tricks[s.n_tricks].start = np; s.n_tricks += 1;
            progress_next_card_or_announcement(s);
        }
    } else {
        // Announcement (action_to_type maps AnnouncementReContra -> ReContra)
        static const uint32_t map[6] = {ReContra, No90, No60, No30, Black, NoAnnouncement};
        const uint32_t ann = map[a - 33];
        int hl[4]; hand_lens(s, hl);
        internal_play_announcement(s.announcements, cp, ann, s.card_index, s.team_state);
        int next;
        const int r = internal_progress(s.announcements, (cp + 1) % 4, s.card_index, hl, s.team_state, &next);
        if (r == NextPlayerIs) s.current_player = next;
        else { s.phase = PlayCard; s.current_player = next; }
    }
}

static uint64_t allowed_now(const State& s) {
    return calculate_allowed_actions(s.phase, current_trick_color(s), s.hands[s.current_player], s.game_type, s.announcements.allowed);
}
// state/state.rs:378-397
bool random_action_for_current_player(State& s, SmallRng& rng) {
    if (s.phase == Finished) return true;
    const uint64_t a = allowed_now(s);
    play_action(s, __builtin_ctzll(random_single(a, rng)));
    return false;
}
// state/state.rs:401-431
bool random_action_for_current_player_no_announcement(State& s, SmallRng& rng) {
    if (s.phase == Finished) return true;
    uint64_t a = allowed_now(s);
    a &= ~(abit(A_AnnouncementReContra) | abit(A_AnnouncementNo90) | abit(A_AnnouncementNo60) |
           abit(A_AnnouncementNo30) | abit(A_AnnouncementBlack));
    play_action(s, __builtin_ctzll(random_single(a, rng)));
    return false;
}
// state/state.rs:434-481 (allowed_actions_current_player of the observation)
uint64_t observation_allowed_actions(const State& s) {
    if (s.phase == Finished) return 0;
    const int obs = s.current_player < 0 ? 0 : s.current_player;
    return calculate_allowed_actions(s.phase, current_trick_color(s), s.hands[obs], s.game_type, s.announcements.allowed);
}

// reservation/visible_reservations_logic.rs:7-66 (zero-oriented output)
void visible_reservations(const State& s, int observing, int out[4]) {
    for (int p = 0; p < 4; ++p) out[p] = V_NoneYet;
    const bool completed = s.res_len == 4;
    bool higher = false;
    for (int i = 0; i < s.res_len; ++i) {
        const int p = (s.res_start + i) % 4;
        const int r = s.res[i];
        if (r == Healthy) out[p] = V_Healthy;
        else if (r == Wedding) out[p] = (completed || p == observing) ? V_Wedding : V_NotRevealed;
        else {
            if (completed && !higher) {
                static const int vmap[9] = {0, 0, V_DiamondsSolo, V_HeartsSolo, V_SpadesSolo, V_ClubsSolo, V_QueensSolo, V_JacksSolo, V_TrumplessSolo};
                out[p] = vmap[r];
                higher = true;
            } else out[p] = V_NotRevealed;
        }
    }
}

// ---- env adapter (rs-doko-mcts/src/env/envs/env_state_full_doko.rs) ----------
// :136-181
uint64_t Env::allowed_actions(bool first_expansion) const {
    uint64_t a = observation_allowed_actions(doko);
    if (!first_expansion) {
        for (int i = 0; i < doko.res_len; ++i) {
            const int r = doko.res[i];
            if (r != Healthy && r != Wedding) {
                a &= ~(abit(A_ReservationClubsSolo) | abit(A_ReservationSpadesSolo) | abit(A_ReservationDiamondsSolo) |
                       abit(A_ReservationHeartsSolo) | abit(A_ReservationTrumplessSolo) | abit(A_ReservationJacksSolo) |
                       abit(A_ReservationQueensSolo) | abit(A_ReservationWedding));
            }
        }
        a &= ~(abit(A_AnnouncementReContra) | abit(A_AnnouncementNo90) | abit(A_AnnouncementNo60) |
               abit(A_AnnouncementNo30) | abit(A_AnnouncementBlack));
    }
    return a;
}
// :183-189
Env Env::by_action(int action_idx) const {
    Env e; e.doko = doko; play_action(e.doko, action_idx); e.last_action = action_idx; return e;
}
// :42-55, :191-196
bool Env::rewards_or_none(double out[4]) const {
    if (!doko.has_stats) return false;
    for (int p = 0; p < 4; ++p) out[p] = (double)doko.stats.player_points[p];
    return true;
}
// :198-220
void Env::random_rollout(SmallRng& rng, double out[4]) const {
    State r = doko;
    for (;;) { if (random_action_for_current_player_no_announcement(r, rng)) break; }
    for (int p = 0; p < 4; ++p) out[p] = (double)r.stats.player_points[p];
}

}  // namespace fdo
}  // namespace oracle

// ---- public entry points for the reference's rule KATs (tests/test_rule_kats.py) ----
namespace oracle {
namespace fdo {
int announcements_start_round(Announcements& a, int card_index, int start, const int hand_lens[4], const TeamState& ts,
                              int* next) {
    a.turns_without = 0;                                   // start_round (announcement.rs:83-101)
    a.starting_player = start;
    return internal_progress(a, start, card_index, hand_lens, ts, next);
}
int announcements_play(Announcements& a, int player, uint32_t ann, int card_index, const int hand_lens[4],
                       const TeamState& ts, int* next) {
    internal_play_announcement(a, player, ann, card_index, ts);   // play_announcement (announcement.rs:103-124)
    return internal_progress(a, (player + 1) % 4, card_index, hand_lens, ts, next);
}
int calc_cards_last_announcement_pub(uint32_t set, int wedding_solved, bool* some) {
    return calc_cards_last_announcement(set, wedding_solved, some);
}
uint32_t internal_calc_allowed_pub(int n_cards, uint32_t prev, int wedding_solved, bool enemy_some, int enemy_cards) {
    return internal_calc_allowed(n_cards, prev, wedding_solved, enemy_some, enemy_cards);
}
}  // namespace fdo
}  // namespace oracle
