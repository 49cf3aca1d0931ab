// rs-full-doko rules as a register-resident bitboard state machine for gfx950.
//
// Reference behaviour (all under /root/reference/rs-full-doko/src):
//   legal mask ............ action/allowed_actions.rs:68-169
//   card order / winner ... card/card_in_trick_logic.rs:17-141, trick/trick_winning_player_logic.rs:15-44
//   colours / masks ....... card/card_to_color.rs:11-259, card/card_color_masks.rs:7-249
//   play_action ........... state/state.rs:184-358
//   announcements ......... announcement/announcement.rs:83-215, announcement/calc_announcement.rs:21-229
//   teams ................. team/team_logic.rs:37-122
//   reservations .......... reservation/reservation_winning_logic.rs:16-73
//   DKV scoring ........... stats/**
//   rollout ............... state.rs:401-431 + rs-doko-mcts env_state_full_doko.rs:198-220
//
// Design (not a translation): the whole game state is ~90 bytes of scalars
// (FdoWork) that live in VGPRs during a rollout — no trick history is kept;
// scoring uses per-player accumulators (eyes, tricks, >=40-eye tricks, fox
// events, Karlchen).  In the card phase of a rollout nobody announces, so each
// announcement round collapses to "advance the RNG once per player whose
// offer set is non-empty" (fdo_rollout, proven equal to the step-by-step path
// by tests/native and the GPU parity tests).
#pragma once
#include "../../../include/doko_amd.h"
#include "common.h"
#include "rng.h"

namespace dk {
namespace fdo {

enum : uint32_t { PH_RESERVATION = 0, PH_ANNOUNCEMENT = 1, PH_PLAYCARD = 2, PH_FINISHED = 3 };
enum : uint32_t { GT_NORMAL = 0, GT_WEDDING, GT_DIAMONDS, GT_HEARTS, GT_SPADES, GT_CLUBS, GT_TRUMPLESS, GT_QUEENS, GT_JACKS };
enum : uint32_t { C_TRUMP = 0, C_DIAMOND, C_HEART, C_SPADE, C_CLUB };
enum : uint32_t { TK_INRES = 0, TK_WED_UNSOLVED, TK_WED_SOLVED, TK_NOWEDDING };
enum : uint32_t { RR_NONE = 0, RR_SOLO = 1, RR_WEDDING = 2 };
enum : uint32_t { R_HEALTHY = 0, R_WEDDING, R_DIAMONDS, R_HEARTS, R_SPADES, R_CLUBS, R_QUEENS, R_JACKS, R_TRUMPLESS };
enum : uint32_t { AN_RE = 1, AN_90 = 2, AN_60 = 4, AN_30 = 8, AN_BLACK = 16, AN_COUNTER = 32 };
enum : int { A_HEALTHY = 24, A_WEDDING = 25, A_RE = 33, A_NOANN = 38 };
static constexpr uint64_t ANN_ACTIONS = 0x1FULL << 33;          // ReContra..Black
static constexpr uint64_t SOLO_WEDDING_ACTIONS = 0xFFULL << 25; // Wedding + 7 solos
static constexpr int CLUB_QUEEN = 15, CLUB_JACK = 14, DIAMOND_ACE = 5;

// ---- card tables ------------------------------------------------------------
// trump cards per game type (24-bit masks)
DK_HD uint32_t trump_mask(uint32_t gt) {
    const uint32_t JQ = 0x30C30Cu;      // all jacks and queens (kinds 2,3,8,9,14,15,20,21)
    const uint32_t H10 = 1u << 7;
    switch (gt) {
        case GT_NORMAL: case GT_WEDDING: case GT_DIAMONDS: return 0x3Fu | H10 | JQ;
        case GT_HEARTS: return (0x3Fu << 6) | JQ;
        case GT_SPADES: return (0x3Fu << 18) | H10 | JQ;
        case GT_CLUBS: return (0x3Fu << 12) | H10 | JQ;
        case GT_TRUMPLESS: return 0u;
        case GT_QUEENS: return 0x208208u;   // kinds 3, 9, 15, 21
        default: return 0x104104u;          // GT_JACKS: kinds 2, 8, 14, 20
    }
}
DK_HD uint32_t suit_color(int card) {
    const int s = card / 6;  // 0 diamond, 1 heart, 2 club, 3 spade
    return s == 0 ? C_DIAMOND : (s == 1 ? C_HEART : (s == 2 ? C_CLUB : C_SPADE));
}
DK_HD uint32_t card_color(int card, uint32_t gt) { return (trump_mask(gt) >> card & 1u) ? C_TRUMP : suit_color(card); }
DK_HD uint32_t color_mask(uint32_t color, uint32_t gt) {
    const uint32_t t = trump_mask(gt);
    switch (color) {
        case C_TRUMP: return t;
        case C_DIAMOND: return 0x00003Fu & ~t;
        case C_HEART: return 0x000FC0u & ~t;
        case C_CLUB: return 0x03F000u & ~t;
        default: return 0xFC0000u & ~t;
    }
}
DK_HD uint32_t card_eyes(int card) { return (uint32_t)((0x0B040302'0A00ULL >> (8 * (card % 6))) & 0xFF); }
// trump rank (card_in_trick_logic.rs:53-83), 4 bits per card kind
DK_HD uint32_t trump_rank(int card) {
    // kinds 0..15 in RANK_LO, 16..23 in RANK_HI
    const uint64_t RANK_LO = 0xB720'2195'C031'8420ULL;  // see tests: D9 0,D10 2,DJ 4,DQ 8,DK 1,DA 3,H9 0,H10 12,HJ 5,HQ 9,HK 1,HA 2,C9 0,C10 2,CJ 7,CQ 11
    const uint64_t RANK_HI = 0x0000'0000'31A6'2031ULL;  // CK 1,CA 3,S9 0,S10 2,SJ 6,SQ 10,SK 1,SA 3
    return card < 16 ? (uint32_t)((RANK_LO >> (4 * card)) & 15) : (uint32_t)((RANK_HI >> (4 * (card - 16))) & 15);
}
// Strength of a card in a trick: trumps above everything, then the trick
// colour by eyes (which order the colour cards), other colours never win.
DK_HD int trick_key(int card, uint32_t trick_color, uint32_t gt) {
    const uint32_t col = card_color(card, gt);
    if (col == C_TRUMP) return 32 + (int)trump_rank(card);
    return col == trick_color ? (int)card_eyes(card) : -1;
}

// ---- working state ----------------------------------------------------------
struct Work {
    uint64_t h[4];
    uint32_t trick_cards;   // current trick, 8 bits per card in play order
    uint32_t trick_winners; // 2 bits per completed trick
    uint32_t eyes;          // 8 bits per player
    uint32_t ntricks;       // 8 bits per player
    uint32_t doko;          // tricks of >= 40 eyes won, per player
    uint32_t res;           // reservation round entries, 8 bits each
    uint8_t fox_n, fox0, fox1, karl;  // fox events (played_by<<2|winner); karl = 1+winner if last trick won by the club jack
    uint8_t trick_len, trick_start, n_tricks, card_index;
    uint8_t phase, cur, game_type, rr_kind;
    uint8_t rr_player, rr_res, team_kind, wedding_player;
    uint8_t solved_trick, re_players, re_lowest, contra_lowest;
    uint8_t ann_turns, ann_start, ann_allowed, ann_count;
    uint8_t ann_players, res_start, res_len, pad0;
    uint32_t pad1;          // explicit tail padding (88 B): stored as 0, never carried through registers
};

DK_HD int hand_len(const Work& w, int p) { return popc64(sel4(w.h, p)); }

// ---- announcements ----------------------------------------------------------
DK_HD uint32_t all_higher_than(uint32_t lowest) {
    switch (lowest) {
        case AN_RE: return AN_RE;
        case AN_90: return AN_RE | AN_90;
        case AN_60: return AN_RE | AN_90 | AN_60;
        case AN_30: return AN_RE | AN_90 | AN_60 | AN_30;
        case AN_BLACK: return AN_RE | AN_90 | AN_60 | AN_30 | AN_BLACK;
        case AN_COUNTER: return AN_COUNTER;
        default: return 0;
    }
}
// calc_announcement.rs:51-229
DK_HD uint32_t allowed_announcements(const Work& w, int player, int n) {
    if (w.team_kind == TK_WED_UNSOLVED || w.team_kind == TK_INRES) return 0;
    const int ws = w.team_kind == TK_WED_SOLVED ? (int)w.solved_trick : 0;
    const bool is_re = (w.re_players >> player) & 1;
    const uint32_t prev = all_higher_than(is_re ? w.re_lowest : w.contra_lowest);
    const uint32_t enemy = all_higher_than(is_re ? w.contra_lowest : w.re_lowest);
    const bool p0 = n >= 11 - ws;
    const bool p90 = p0 || (n >= 10 - ws && (prev & AN_RE));
    const bool p60 = p90 || (n >= 9 - ws && (prev & AN_90));
    const bool p30 = p60 || (n >= 8 - ws && (prev & AN_60));
    const bool pb = p30 || (n >= 7 - ws && (prev & AN_30));
    uint32_t rem = (p0 ? AN_RE : 0u) | (p90 ? AN_90 : 0u) | (p60 ? AN_60 : 0u) | (p30 ? AN_30 : 0u) | (pb ? AN_BLACK : 0u);
    rem &= ~prev;
    rem &= (0u - rem) | ~0x1Fu;  // keep only the lowest set bit among the five levels ("one below the current")
    if (rem == 0) {
        int ec = -1;
        if (enemy & AN_BLACK) ec = 7 - ws;
        else if (enemy & AN_30) ec = 8 - ws;
        else if (enemy & AN_60) ec = 9 - ws;
        else if (enemy & AN_90) ec = 10 - ws;
        else if (enemy & AN_RE) ec = 11 - ws;
        if (ec >= 0 && n >= ec - 1 && !(prev & (AN_COUNTER | AN_RE))) rem |= AN_COUNTER;
    }
    return rem;
}

// ---- card-phase rollout fast path ------------------------------------------------
// The card phase of a rollout rewritten for a 64-wide SIMD: 32-bit words only,
// selects instead of branches, and the per-card announcement round reduced to
// arithmetic.  With nobody announcing, player p is offered an announcement
// after a card iff its hand size n_p >= theta_p (allowed_announcements is
// monotone in n; the thresholds change only when a wedding is resolved), so
// the forced NoAnnouncement draws of a round are popc over 4 byte compares.
//
//   theta (own levels)  = 11 - ws - |prev & {Re,90,60,30}|      unless Black is in prev
//   theta (counter)     = 11 - ws - |enemy levels|               if enemy announced and
//                                                                prev has neither Re nor Counter
// (calc_announcement.rs:51-229; derivation in DESIGN.md).  Equality with the
// step-by-step path is checked by tests/native/fdo_engine_check and the GPU tests.
DK_HD uint32_t ann_theta(uint32_t prev, uint32_t enemy, int ws) {
    uint32_t t = 99u;
    if (!(prev & AN_BLACK)) t = (uint32_t)(11 - ws - popc32(prev & 0xFu));
    if ((enemy & 0x1Fu) && !(prev & (AN_COUNTER | AN_RE))) {
        const uint32_t tc = (uint32_t)(11 - ws - popc32(enemy & 0x1Fu));
        t = tc < t ? tc : t;
    }
    return t;
}
// theta_p packed one byte per player (99 = never offered)
DK_HD uint32_t ann_thetas(uint32_t team_kind, uint32_t solved_trick, uint32_t re_players, uint32_t re_lowest,
                          uint32_t contra_lowest) {
    if (team_kind == TK_WED_UNSOLVED || team_kind == TK_INRES) return 0x63636363u;
    const int ws = team_kind == TK_WED_SOLVED ? (int)solved_trick : 0;
    const uint32_t pr = all_higher_than(re_lowest), pk = all_higher_than(contra_lowest);
    const uint32_t tre = ann_theta(pr, pk, ws), tko = ann_theta(pk, pr, ws);
    uint32_t out = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) out |= (((re_players >> p) & 1u) ? tre : tko) << (8 * p);
    return out;
}
DK_HD uint32_t sel4u(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t p) {
    const uint32_t lo = (p & 1u) ? a1 : a0, hi = (p & 1u) ? a3 : a2;
    return (p & 2u) ? hi : lo;
}
// trump rank nibbles (same table as trump_rank), 8 cards per word
DK_HD uint32_t rank_fast(uint32_t c) {
    const uint32_t wv = c < 8u ? 0xC0318420u : (c < 16u ? 0xB7202195u : 0x31A62031u);
    return (wv >> (4u * (c & 7u))) & 15u;
}
DK_HD uint32_t suit_of(uint32_t c) { return (c * 43u) >> 8; }   // c / 6 for c < 24
DK_HD uint32_t eyes_fast(uint32_t c) { return (0xB432A0u >> (4u * (c - 6u * suit_of(c)))) & 15u; }
// colour class mask of card c (trumps, or its suit minus trumps)
DK_HD uint32_t class_mask(uint32_t c, uint32_t tm) {
    return ((tm >> c) & 1u) ? tm : ((0x3Fu << (6u * suit_of(c))) & ~tm);
}
// key of card c in a trick led with colour class `lead` (trick_key)
DK_HD int key_fast(uint32_t c, uint32_t tm, uint32_t lead) {
    const int k_t = 32 + (int)rank_fast(c), k_c = (int)eyes_fast(c);
    return ((tm >> c) & 1u) ? k_t : (((lead >> c) & 1u) ? k_c : -1);
}

// Per-(game type, card) facts for the rollout, one 8-byte entry:
//   x = colour-class mask of the card (24 bits) | eyes << 24 | trump << 28
//   y = trick key when it can win: 32 + trump rank for trumps, eyes otherwise
// On the GPU the 9 x 24 table lives in LDS (built by card_table_init at kernel
// start); on the host it is computed on the fly.
struct CardInfo { uint32_t x, y; };
DK_HD CardInfo card_info_calc(uint32_t gt, uint32_t c) {
    const uint32_t tm = trump_mask(gt);
    const bool tr = (tm >> c) & 1u;
    CardInfo ci;
    ci.x = class_mask(c, tm) | (eyes_fast(c) << 24) | (tr ? 1u << 28 : 0u);
    ci.y = tr ? 32u + rank_fast(c) : eyes_fast(c);
    return ci;
}
// Position of the set bit of rank k (from the LSB) in a byte: bit_rank_calc(v, k).
DK_HD uint32_t bit_rank_calc(uint32_t v, uint32_t k) {
    for (uint32_t b = 0; b < 8u; ++b)
        if ((v >> b) & 1u) { if (k == 0) return b; --k; }
    return 0;
}
#if defined(__HIP_DEVICE_COMPILE__)
__shared__ uint2 dk_card_tab[9 * 24];
__shared__ uint8_t dk_bit_rank_tab[256 * 8];   // [byte][rank] -> bit position (2 KB)
__device__ inline void card_table_init() {
    for (uint32_t i = threadIdx.x; i < 9u * 24u; i += blockDim.x) {
        const CardInfo ci = card_info_calc(i / 24u, i % 24u);
        dk_card_tab[i] = make_uint2(ci.x, ci.y);
    }
    for (uint32_t i = threadIdx.x; i < 256u * 8u; i += blockDim.x) dk_bit_rank_tab[i] = (uint8_t)bit_rank_calc(i >> 3, i & 7u);
    __syncthreads();
}
__device__ inline uint32_t bit_rank(uint32_t v, uint32_t k) { return dk_bit_rank_tab[v * 8u + k]; }
__device__ inline CardInfo card_info(uint32_t gt, uint32_t c) {
    const uint2 v = dk_card_tab[gt * 24u + c];
    CardInfo ci;
    ci.x = v.x; ci.y = v.y;
    return ci;
}
#else
inline void card_table_init() {}
inline CardInfo card_info(uint32_t gt, uint32_t c) { return card_info_calc(gt, c); }
inline uint32_t bit_rank(uint32_t v, uint32_t k) { return bit_rank_calc(v, k); }
#endif
// Position of the set bit of rank k (from the LSB) in a 24-bit mask with more than k set
// bits: the byte holding it from two byte popcounts, the bit from the [byte][rank] table.
DK_HD uint32_t nth_set_bit24(uint32_t m, uint32_t k) {
    const uint32_t c0 = (uint32_t)popc32(m & 0xFFu), c1 = (uint32_t)popc32(m & 0xFF00u);
    const bool ge0 = k >= c0;
    const uint32_t k1 = k - c0;
    const bool ge1 = ge0 && k1 >= c1;
    const uint32_t sh = ge1 ? 16u : (ge0 ? 8u : 0u);
    const uint32_t kk = ge1 ? k1 - c1 : (ge0 ? k1 : k);
    return sh + bit_rank((m >> sh) & 0xFFu, kk);
}


// announcement.rs:182-215 (the announcing player's team decides which lowest moves)
DK_HD void internal_play_announcement(Work& w, int player, uint32_t ann) {
    if (ann == 0) { w.ann_turns += 1; return; }  // NoAnnouncement
    w.ann_turns = 0;
    if (w.ann_count < 12) { w.ann_count += 1; w.ann_players |= (uint8_t)(1u << player); }
    if ((w.re_players >> player) & 1) w.re_lowest = (uint8_t)ann; else w.contra_lowest = (uint8_t)ann;
}
// announcement.rs:137-180. Returns true if the round is over.  The players are
// asked in order from `player`; one without an offer passes automatically
// (number_of_turns_without_announcement += 1) and the round ends after four
// consecutive passes.  Offers are non-empty iff hand size >= theta (see
// ann_theta), so the first player to ask is found from the thresholds and only
// that player's offer set is computed.
DK_HD bool internal_progress(Work& w, int player) {
    const uint32_t theta = ann_thetas(w.team_kind, w.solved_trick, w.re_players, w.re_lowest, w.contra_lowest);
    const uint32_t t = w.ann_turns;
    uint32_t found = 4;   // index (from `player`) of the first offered player within the round
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
        const uint32_t p = ((uint32_t)player + i) & 3u;
        const bool offered = (uint32_t)hand_len(w, (int)p) >= ((theta >> (8u * p)) & 0xFFu);
        found = (found == 4u && i + t < 4u && offered) ? i : found;
    }
    if (found == 4u) {
        w.ann_turns = 4; w.ann_allowed = 0; w.cur = w.ann_start;
        return true;
    }
    const int p = (player + (int)found) & 3;
    w.ann_turns = (uint8_t)(t + found);
    w.ann_allowed = (uint8_t)allowed_announcements(w, p, hand_len(w, p));
    w.cur = (uint8_t)p;
    return false;
}
// state.rs:184-206
DK_HD void progress_next_card_or_announcement(Work& w) {
    w.ann_turns = 0;
    w.ann_start = w.cur;
    const bool over = internal_progress(w, w.cur);
    w.phase = over ? PH_PLAYCARD : PH_ANNOUNCEMENT;
}

// ---- legal actions ------------------------------------------------------------
DK_HD uint32_t current_trick_color(const Work& w) {
    // state.rs:360-372: no colour while the trick is empty, and none during the 12th trick
    if (w.trick_len == 0 || w.n_tricks >= 12 || w.n_tricks == 0) return 0xFF;
    return card_color((int)(w.trick_cards & 0xFF), w.game_type);
}
DK_HD uint64_t legal_actions(const Work& w) {
    switch (w.phase) {
        case PH_RESERVATION: {
            const uint64_t h = sel4(w.h, w.cur);
            uint64_t a = (0x1FFULL << 24) & ~(1ULL << A_WEDDING);
            if ((h >> CLUB_QUEEN & 1) && (h >> (CLUB_QUEEN + 24) & 1)) a |= 1ULL << A_WEDDING;
            return a;
        }
        case PH_PLAYCARD: {
            const uint64_t h = sel4(w.h, w.cur);
            const uint64_t single = (h | (h >> 24)) & 0xFFFFFFULL;
            const uint32_t tc = current_trick_color(w);
            if (tc == 0xFF) return single;
            const uint64_t follow = single & color_mask(tc, w.game_type);
            return follow ? follow : single;
        }
        case PH_ANNOUNCEMENT: {
            const uint32_t al = w.ann_allowed;
            uint64_t a = 1ULL << A_NOANN;
            if (al & (AN_COUNTER | AN_RE)) a |= 1ULL << 33;
            if (al & AN_90) a |= 1ULL << 34;
            if (al & AN_60) a |= 1ULL << 35;
            if (al & AN_30) a |= 1ULL << 36;
            if (al & AN_BLACK) a |= 1ULL << 37;
            return a;
        }
        default: return 0;
    }
}
// McFullDokoEnvState::allowed_actions (env_state_full_doko.rs:136-181)
DK_HD uint64_t env_allowed(const Work& w, bool first_expansion) {
    uint64_t a = legal_actions(w);
    if (!first_expansion) {
        bool any_solo = false;
        for (int i = 0; i < 4; ++i)
            if (i < w.res_len) { const uint32_t r = byte_get(w.res, i); any_solo |= r >= R_DIAMONDS; }
        if (any_solo) a &= ~SOLO_WEDDING_ACTIONS;
        a &= ~ANN_ACTIONS;
    }
    return a;
}

// ---- transitions ----------------------------------------------------------------
// reservation_winning_logic.rs:37-73 + :16-33, team_logic.rs:37-122 (reservation end)
DK_HD void finish_reservations(Work& w) {
    int wedding = -1;
    w.rr_kind = RR_NONE;
    for (int i = 0; i < 4; ++i) {
        const int p = (w.res_start + i) & 3;
        const uint32_t r = byte_get(w.res, i);
        if (w.rr_kind == RR_SOLO) continue;
        if (r == R_WEDDING) wedding = p;
        else if (r >= R_DIAMONDS) { w.rr_kind = RR_SOLO; w.rr_player = (uint8_t)p; w.rr_res = (uint8_t)r; }
    }
    if (w.rr_kind != RR_SOLO && wedding >= 0) { w.rr_kind = RR_WEDDING; w.rr_player = (uint8_t)wedding; }
    if (w.rr_kind == RR_SOLO) {
        // FdoReservation -> FdoGameType (nibble r of 0x687543200)
        w.game_type = (uint8_t)((0x687543200ULL >> (4 * w.rr_res)) & 15);
        w.team_kind = TK_NOWEDDING; w.re_players = (uint8_t)(1u << w.rr_player);
    } else if (w.rr_kind == RR_WEDDING) {
        w.game_type = GT_WEDDING;
        w.team_kind = TK_WED_UNSOLVED; w.wedding_player = w.rr_player; w.re_players = 0;
    } else {
        w.game_type = GT_NORMAL;
        uint8_t re = 0;
        for (int p = 0; p < 4; ++p) {
            const uint64_t h = sel4(w.h, p);
            if ((h >> CLUB_QUEEN & 1) || (h >> (CLUB_QUEEN + 24) & 1)) re |= (uint8_t)(1u << p);
        }
        w.team_kind = TK_NOWEDDING; w.re_players = re;
    }
}

// One completed trick: winner, eyes, scoring accumulators, wedding resolution.
// Returns the winner.
DK_HD int complete_trick(Work& w) {
    const uint32_t tm = trump_mask(w.game_type);
    const uint32_t lead = class_mask(w.trick_cards & 0xFFu, tm);
    int best_key = -2, best_i = 0;
    uint32_t e = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t c = (w.trick_cards >> (8 * i)) & 0xFFu;
        const int k = key_fast(c, tm, lead);
        const bool better = k > best_key;
        best_key = better ? k : best_key;
        best_i = better ? i : best_i;
        e += eyes_fast(c);
    }
    const int winner = (w.trick_start + best_i) & 3;
    const int win_card = (int)((w.trick_cards >> (8 * best_i)) & 0xFF);
    const int t = w.n_tricks - 1;
    w.trick_winners |= (uint32_t)winner << (2 * t);
    w.eyes = byte_add(w.eyes, winner, e);
    w.ntricks = byte_add(w.ntricks, winner, 1);
    if (e >= 40) w.doko = byte_add(w.doko, winner, 1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if ((int)((w.trick_cards >> (8 * i)) & 0xFF) == DIAMOND_ACE) {
            const uint8_t ev = (uint8_t)((((w.trick_start + i) & 3) << 2) | winner);
            if (w.fox_n == 0) w.fox0 = ev; else w.fox1 = ev;
            w.fox_n += 1;
        }
    }
    if (t == 11 && win_card == CLUB_JACK) w.karl = (uint8_t)(1 + winner);
    if (w.team_kind == TK_WED_UNSOLVED && t < 3) {
        if (winner != w.wedding_player) {
            w.team_kind = TK_WED_SOLVED; w.solved_trick = (uint8_t)t;
            w.re_players = (uint8_t)((1u << w.wedding_player) | (1u << winner));
        } else if (t == 2) {
            w.team_kind = TK_WED_SOLVED; w.solved_trick = 2; w.re_players = (uint8_t)(1u << w.wedding_player);
        }
    }
    return winner;
}

// Remove one copy of `card` from player p's hand (second copy first, hand.rs:235-247).
DK_HD void hand_remove(Work& w, int p, int card) {
    const uint64_t h = sel4(w.h, p);
    const uint64_t hi = 1ULL << (card + 24);
    set4(w.h, p, (h & hi) ? (h & ~hi) : (h & ~(1ULL << card)));
}

// Plays a card for w.cur. Returns true when the game finished.
DK_HD bool play_card_core(Work& w, int card) {
    const int cp = w.cur;
    hand_remove(w, cp, card);
    w.trick_cards |= (uint32_t)card << (8 * w.trick_len);
    w.trick_len += 1;
    w.card_index += 1;
    if (w.trick_len == 4) {
        const int winner = complete_trick(w);
        if (w.n_tricks == 12) { w.phase = PH_FINISHED; w.cur = 0xFF; return true; }
        w.cur = (uint8_t)winner;
        w.trick_cards = 0; w.trick_len = 0; w.trick_start = (uint8_t)winner; w.n_tricks += 1;
        return false;
    }
    w.cur = (uint8_t)((cp + 1) & 3);
    return false;
}

// FdoState::play_action (state.rs:208-358) for any phase.  The three action
// kinds share ONE announcement-round progression (internal_progress), so a wave
// whose lanes play different kinds of actions runs it once.
DK_HD void play_action(Work& w, int a) {
    int start = -1;   // player the announcement round continues from (-1: no round step)
    if (a <= 23) {
        if (!play_card_core(w, a)) {   // progress_next_card_or_announcement (state.rs:184-206)
            w.ann_turns = 0;
            w.ann_start = w.cur;
            start = w.cur;
        }
    } else if (a <= 32) {
        // FdoAction order -> FdoReservation discriminant (nibble a-24 of 0x768543210)
        w.res = byte_set(w.res, w.res_len, (uint32_t)((0x768543210ULL >> (4 * (a - 24))) & 15));
        w.res_len += 1;
        w.cur = (uint8_t)((w.cur + 1) & 3);
        if (w.res_len == 4) {
            finish_reservations(w);
            w.trick_cards = 0; w.trick_len = 0; w.trick_start = w.cur; w.n_tricks = 1;
            w.ann_turns = 0;
            w.ann_start = w.cur;
            start = w.cur;
        }
    } else {
        const int cp = w.cur;
        internal_play_announcement(w, cp, a < A_NOANN ? (1u << (a - 33)) : 0u);
        start = (cp + 1) & 3;
    }
    if (start >= 0) w.phase = internal_progress(w, start) ? PH_PLAYCARD : PH_ANNOUNCEMENT;
}

// ---- DKV scoring (stats/stats.rs:46-243 and stats/**) -------------------------
#ifndef DK_SCORE_FAST
#define DK_SCORE_FAST 0     // (measurement switch) score() without announcements takes a short path
#endif
struct Flags { bool ann, u90, u60, u30, black, none, o_ann, o_90, o_60, o_30, o_black; };
DK_HD Flags ann_flags(uint32_t prev) {
    Flags f;
    f.ann = (prev & (AN_RE | AN_COUNTER)) != 0; f.u90 = prev & AN_90; f.u60 = prev & AN_60; f.u30 = prev & AN_30;
    f.black = prev & AN_BLACK; f.none = prev == 0;
    f.o_ann = f.ann && !f.u90; f.o_90 = f.u90 && !f.u60; f.o_60 = f.u60 && !f.u30; f.o_30 = f.u30 && !f.black; f.o_black = f.black;
    return f;
}
// player_points into pts[4]
DK_HD void score(const Work& w, int pts[4]) {
    const uint32_t re = w.re_players;
    uint32_t re_eyes = 0, ko_eyes = 0, re_t = 0, ko_t = 0;
    int doko_re = 0, doko_ko = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const bool r = (re >> p) & 1;
        const uint32_t e = byte_get(w.eyes, p), t = byte_get(w.ntricks, p), d = byte_get(w.doko, p);
        re_eyes += r ? e : 0; ko_eyes += r ? 0 : e; re_t += r ? t : 0; ko_t += r ? 0 : t;
        doko_re += r ? (int)d : 0; doko_ko += r ? 0 : (int)d;
    }
    const bool re_all = re_t == 12, ko_all = ko_t == 12;
    const uint32_t rp = all_higher_than(w.re_lowest), kp = all_higher_than(w.contra_lowest);
#if DK_SCORE_FAST
    // Neither team announced (every lane of the wave: the rollouts' usual case, nobody announces
    // in them): of the winning conditions only `eyes >= 121 && R.none && K.none` (Re) and
    // `eyes >= 120 && ...` (Kontra) remain, and as re_eyes + ko_eyes = 240 exactly one holds; the
    // game value is the loser's thresholds plus "schwarz" -- the general path below gives the same.
    if (!wave_any(rp != 0u || kp != 0u)) {
        const bool rw = re_eyes >= 121;
        const bool is_solo = popc32(re) == 1;
        int ra = 0, ka = 0;
        if (!is_solo) {
            if (!rw) { ka += 1; ra -= 1; }                      // team_win == Kontra
            ra += doko_re - doko_ko; ka += doko_ko - doko_re;
            int fre = 0, fko = 0;
            for (int i = 0; i < 2; ++i) {
                if (i >= w.fox_n) break;
                const uint8_t ev = i == 0 ? w.fox0 : w.fox1;
                const bool by_re = (re >> (ev >> 2)) & 1, win_re = (re >> (ev & 3)) & 1;
                if (by_re != win_re) { if (win_re) fre++; else fko++; }
            }
            ra += fre - fko; ka += fko - fre;
            if (w.karl) { if ((re >> (w.karl - 1)) & 1) { ra += 1; ka -= 1; } else { ra -= 1; ka += 1; } }
        }
        const uint32_t loser = rw ? ko_eyes : re_eyes;
        const int v = 1 + (loser < 90) + (loser < 60) + (loser < 30) + ((rw ? re_all : ko_all) ? 1 : 0);
        int re_pts = (rw ? v : -v) + ra;
        const int ko_pts = (rw ? -v : v) + ka;
        if (is_solo) re_pts *= 3;
#pragma unroll
        for (int p = 0; p < 4; ++p) pts[p] = ((re >> p) & 1) ? re_pts : ko_pts;
        return;
    }
#endif
    const Flags R = ann_flags(rp), K = ann_flags(kp);
    const bool rw =
        (re_eyes >= 121 && R.none && K.none) || (re_eyes >= 121 && R.o_ann && !K.ann) || (re_eyes >= 121 && R.o_ann && K.o_ann) ||
        (re_eyes >= 120 && !R.ann && K.o_ann) || (re_eyes >= 151 && R.o_90) || (re_eyes >= 181 && R.o_60) ||
        (re_eyes >= 211 && R.o_30) || (re_all && R.o_black) || (re_eyes >= 90 && K.o_90 && !R.u90) ||
        (re_eyes >= 60 && K.o_60 && !R.u90) || (re_eyes >= 30 && K.o_30 && !R.u90) || (!ko_all && K.o_black && !R.u90);
    const bool kw =
        (ko_eyes >= 120 && R.none && K.none) || (ko_eyes >= 120 && R.o_ann && !K.ann) || (ko_eyes >= 120 && R.o_ann && K.o_ann) ||
        (ko_eyes >= 121 && !R.ann && K.o_ann) || (ko_eyes >= 151 && K.o_90) || (ko_eyes >= 181 && K.o_60) ||
        (ko_eyes >= 211 && K.o_30) || (ko_all && K.o_black) || (ko_eyes >= 90 && R.o_90 && !K.u90) ||
        (ko_eyes >= 60 && R.o_60 && !K.u90) || (ko_eyes >= 30 && R.o_30 && !K.u90) || (!re_all && R.o_black && !K.u90);
    const bool is_solo = popc32(re) == 1;
    int ra = 0, ka = 0;
    if (!is_solo) {
        const int team_win = rw ? 0 : (kw ? 1 : -1);
        if (team_win == 1) { ka += 1; ra -= 1; }
        ra += doko_re - doko_ko; ka += doko_ko - doko_re;
        int fre = 0, fko = 0;
        for (int i = 0; i < 2; ++i) {
            if (i >= w.fox_n) break;
            const uint8_t ev = i == 0 ? w.fox0 : w.fox1;
            const bool by_re = (re >> (ev >> 2)) & 1, win_re = (re >> (ev & 3)) & 1;
            if (by_re != win_re) { if (win_re) fre++; else fko++; }
        }
        ra += fre - fko; ka += fko - fre;
        if (w.karl) { if ((re >> (w.karl - 1)) & 1) { ra += 1; ka -= 1; } else { ra -= 1; ka += 1; } }
    }
    int re_pts, ko_pts;
    if (!rw && !kw) {
        int r = 0, k = 0;
        if (re_eyes < 90) { k++; r--; }
        if (ko_eyes < 90) { r++; k--; }
        if (re_eyes < 60) { k++; r--; }
        if (ko_eyes < 60) { r++; k--; }
        if (re_eyes < 30) { k++; r--; }
        if (ko_eyes < 30) { r++; k--; }
        if (re_eyes >= 120 && K.u90) { r++; k--; }
        if (re_eyes >= 90 && K.u60) { r++; k--; }
        if (re_eyes >= 60 && K.u30) { r++; k--; }
        if (re_eyes >= 30 && K.black) { r++; k--; }
        if (ko_eyes >= 120 && R.u90) { k++; r--; }
        if (ko_eyes >= 90 && R.u60) { k++; r--; }
        if (ko_eyes >= 60 && R.u30) { k++; r--; }
        if (ko_eyes >= 30 && R.black) { k++; r--; }
        re_pts = r + ra; ko_pts = k + ka;
    } else {
        const uint32_t loser = rw ? ko_eyes : re_eyes;
        const bool winner_all = rw ? re_all : ko_all;
        int v = 1 + (loser < 90) + (loser < 60) + (loser < 30) + (winner_all ? 1 : 0);
        v += (R.ann ? 2 : 0) + (K.ann ? 2 : 0);
        v += (int)R.u90 + (int)R.u60 + (int)R.u30 + (int)R.black + (int)K.u90 + (int)K.u60 + (int)K.u30 + (int)K.black;
        v += (re_eyes >= 120 && K.u90) + (re_eyes >= 90 && K.u60) + (re_eyes >= 60 && K.u30) + (re_eyes >= 30 && K.black);
        v += (ko_eyes >= 120 && R.u90) + (ko_eyes >= 90 && R.u60) + (ko_eyes >= 60 && R.u30) + (ko_eyes >= 30 && R.black);
        re_pts = (rw ? v : -v) + ra;
        ko_pts = (kw ? v : -v) + ka;
    }
    if (is_solo) re_pts *= 3;
#pragma unroll
    for (int p = 0; p < 4; ++p) pts[p] = ((re >> p) & 1) ? re_pts : ko_pts;
}

// ---- rollout (random_action_for_current_player_no_announcement until finished) -----
// Number of players asked in an announcement round whose offer set is non-empty:
// each of them consumes exactly one RNG draw (forced NoAnnouncement).
DK_HD int round_draws(const Work& w) {
    if (w.team_kind == TK_WED_UNSOLVED) return 0;
    int d = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) d += allowed_announcements(w, p, hand_len(w, p)) != 0 ? 1 : 0;
    return d;
}

// ---- speculative trick draw (DK_TRICK_SPEC) ------------------------------------------
// The four plies of a trick whose hands (relative to the leader) are a0..a3, as one
// straight-line block: the four draws are taken up front, skipping range_u32's rejection
// branch, the led class comes from the first card by arithmetic, so the three followers'
// legal sets, ranks and table lookups are independent of each other and issue together.
// Returns false -- generator untouched -- when any lane of the wave drew into a rejection
// zone (probability < 12 / 2^32 per ply); the caller then plays the trick by the exact
// per-ply path.  On true, rng has advanced by the trick's four draws, exactly as the per-ply
// path would have.
struct TrickDraw { uint32_t c[4]; CardInfo i[4]; uint32_t ld; };
DK_HD bool draw_trick(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, Rng& rng, uint32_t gt, uint32_t tm,
                      TrickDraw& t) {
    Rng q = rng;
    const uint32_t x0 = q.next_u32(), x1 = q.next_u32(), x2 = q.next_u32(), x3 = q.next_u32();
    const uint32_t n0 = (uint32_t)popc32(a0);
    const uint64_t m0 = (uint64_t)x0 * (uint64_t)n0;
    const uint32_t c0 = nth_set_bit24(a0, n0 - 1u - (uint32_t)(m0 >> 32));
    const uint32_t ld = class_mask(c0, tm);
    const uint32_t f1 = a1 & ld, f2 = a2 & ld, f3 = a3 & ld;
    const uint32_t l1 = f1 ? f1 : a1, l2 = f2 ? f2 : a2, l3 = f3 ? f3 : a3;
    const uint32_t n1 = (uint32_t)popc32(l1), n2 = (uint32_t)popc32(l2), n3 = (uint32_t)popc32(l3);
    const uint64_t m1 = (uint64_t)x1 * (uint64_t)n1, m2 = (uint64_t)x2 * (uint64_t)n2, m3 = (uint64_t)x3 * (uint64_t)n3;
    const bool rej = (uint32_t)m0 > 0u - n0 || (uint32_t)m1 > 0u - n1 || (uint32_t)m2 > 0u - n2 || (uint32_t)m3 > 0u - n3;
#ifdef DK_TRICK_REPLAY_ALL
    if (wave_any(rej || true)) return false;   // (test builds: every trick takes the exact path)
#else
    if (wave_any(rej)) return false;
#endif
    t.c[0] = c0;
    t.c[1] = nth_set_bit24(l1, n1 - 1u - (uint32_t)(m1 >> 32));
    t.c[2] = nth_set_bit24(l2, n2 - 1u - (uint32_t)(m2 >> 32));
    t.c[3] = nth_set_bit24(l3, n3 - 1u - (uint32_t)(m3 >> 32));
#pragma unroll
    for (int k = 0; k < 4; ++k) t.i[k] = card_info(gt, t.c[k]);
    t.ld = ld;
    rng = q;
    return true;
}

// Card phase to the end (w.phase == PH_PLAYCARD).  Returns plies played.
// The trick is evaluated incrementally as its cards are played (running best key = first
// strict maximum, eyes, Diamond-Ace players).  Hands are kept relative to the leader: after
// the partial first trick (at most three plies, played with the absolute hands), A_k / T_k
// hold the hand of player (trick_start + k) & 3 and the loop plays one whole trick per trip
// -- four plies unrolled, so each ply's hand is a register known at compile time, no
// per-ply player select or masked four-way update -- and rotates the hands by the winner's
// position once per trick.  The lanes of a wave then complete their tricks in the same trip,
// so the wave pays one trick completion per four plies.  Draw order, rewards and plies are
// the reference's (state.rs:401-431; host check fdo_engine_check).
#ifndef DK_ROLLOUT_FAST
#define DK_ROLLOUT_FAST 1   // tricks without announcement offers skip the per-card offer tests
#endif
#ifndef DK_TRICK_SPEC
#define DK_TRICK_SPEC 1     // fast tricks drawn speculatively as one block, replayed on a rejection
#endif
#ifndef DK_FOX_SKIP
#define DK_FOX_SKIP 0       // (measurement switch) fast tricks skip the fox tracking once no lane holds a Diamond Ace
#endif
DK_HD int rollout_cards(const Work& w0, Rng& rng, int pts[4]) {
    uint32_t any0, any1, any2, any3, two0, two1, two2, two3;
    {
        const uint64_t h0 = w0.h[0], h1 = w0.h[1], h2 = w0.h[2], h3 = w0.h[3];
        const uint32_t M = 0xFFFFFFu;
        any0 = ((uint32_t)h0 | (uint32_t)(h0 >> 24)) & M; two0 = ((uint32_t)h0 & (uint32_t)(h0 >> 24)) & M;
        any1 = ((uint32_t)h1 | (uint32_t)(h1 >> 24)) & M; two1 = ((uint32_t)h1 & (uint32_t)(h1 >> 24)) & M;
        any2 = ((uint32_t)h2 | (uint32_t)(h2 >> 24)) & M; two2 = ((uint32_t)h2 & (uint32_t)(h2 >> 24)) & M;
        any3 = ((uint32_t)h3 | (uint32_t)(h3 >> 24)) & M; two3 = ((uint32_t)h3 & (uint32_t)(h3 >> 24)) & M;
    }
    uint32_t nb = (uint32_t)(popc32(any0) + popc32(two0)) | (uint32_t)(popc32(any1) + popc32(two1)) << 8 |
                  (uint32_t)(popc32(any2) + popc32(two2)) << 16 | (uint32_t)(popc32(any3) + popc32(two3)) << 24;
    const uint32_t tm = trump_mask(w0.game_type);
    const uint32_t gt = w0.game_type;
    uint32_t team_kind = w0.team_kind, re_players = w0.re_players, solved = w0.solved_trick;
    const uint32_t wedding_player = w0.wedding_player;
    uint32_t theta = ann_thetas(team_kind, solved, re_players, w0.re_lowest, w0.contra_lowest);
    uint32_t cur = w0.cur, trick_start = w0.trick_start, trick_len = w0.trick_len, n_tricks = w0.n_tricks;
    uint32_t eyes = w0.eyes, ntr = w0.ntricks, doko = w0.doko;
    uint32_t fox_n = w0.fox_n, fox0 = w0.fox0, fox1 = w0.fox1, karl = w0.karl;
    uint32_t lead = 0xFFFFFFu, best_pos = 0, win_card = 0, t_eyes = 0, da_bits = 0;
    uint32_t lt = 0;   // lead | tm of the running trick (DK_ROLLOUT_FAST)
    int best_key = -2;
    for (uint32_t i = 0; i < trick_len; ++i) {
        const uint32_t c = (w0.trick_cards >> (8u * i)) & 0xFFu;
        if (i == 0) lead = class_mask(c, tm);
        const int k = key_fast(c, tm, lead);
        if (k > best_key) { best_key = k; best_pos = i; win_card = c; }
        t_eyes += eyes_fast(c);
        if (c == (uint32_t)DIAMOND_ACE) da_bits |= 1u << ((trick_start + i) & 3u);
    }
    lt = lead | tm;
    auto complete = [&](uint32_t winner) {
        const uint32_t sh = 8u * winner;
        eyes += t_eyes << sh;
        ntr += 1u << sh;
        doko += (t_eyes >= 40u ? 1u : 0u) << sh;
        if (da_bits != 0u) {
            const uint32_t rest = da_bits & (da_bits - 1u);
            const uint32_t e0 = ((uint32_t)ctz32(da_bits) << 2) | winner;
            fox0 = fox_n == 0u ? e0 : fox0;
            fox1 = fox_n == 1u ? e0 : fox1;
            fox_n += 1u;
            if (rest != 0u) { fox1 = fox_n == 1u ? (((uint32_t)ctz32(rest) << 2) | winner) : fox1; fox_n += 1u; }
        }
        const uint32_t t = n_tricks - 1u;
        karl = (t == 11u && win_card == (uint32_t)CLUB_JACK) ? 1u + winner : karl;
        if (team_kind == TK_WED_UNSOLVED && t < 3u && (winner != wedding_player || t == 2u)) {
            team_kind = TK_WED_SOLVED;
            solved = winner != wedding_player ? t : 2u;
            re_players = (1u << wedding_player) | (winner != wedding_player ? 1u << winner : 0u);
            theta = ann_thetas(team_kind, solved, re_players, w0.re_lowest, w0.contra_lowest);
        }
    };
    int plies = 0;
    // one card of player p, whose hand is (a, t2), at position `pos` of the trick; updates the
    // hand and the running trick.  `track` keeps the hand sizes (nb) per card, which only the
    // announcement offers read (draws).
    auto play = [&](uint32_t& a, uint32_t& t2, uint32_t p, bool first, uint32_t pos, bool track, bool fox = true) {
        const uint32_t f = a & lead;
        const uint32_t legal = f ? f : a;
        const uint32_t r = rng.range_u32((uint32_t)popc32(legal));
        const uint32_t card = nth_set_bit24(legal, (uint32_t)popc32(legal) - 1u - r), bit = 1u << card;
#if DK_ROLLOUT_FAST
        // the second copy goes first: t2 loses the bit if it holds it, a otherwise (no selects)
        const uint32_t second = t2 & bit;
        t2 ^= second;
        a ^= bit ^ second;
#else
        const bool dup = (t2 & bit) != 0u;
        a = dup ? a : (a ^ bit);
        t2 = dup ? (t2 ^ bit) : t2;
#endif
        if (track) nb -= 1u << (8u * p);
        const CardInfo ci = card_info(gt, card);
        lead = first ? (ci.x & 0xFFFFFFu) : lead;
#if DK_ROLLOUT_FAST
        // a card can win the trick iff it is a trump or of the led class: one bit of lead | tm
        lt = first ? (lead | tm) : lt;
        const int key = ((lt >> card) & 1u) ? (int)ci.y : -1;
#else
        const int key = (((ci.x >> 28) & 1u) || ((lead >> card) & 1u)) ? (int)ci.y : -1;
#endif
        const bool better = first || key > best_key;
        best_key = better ? key : best_key;
        best_pos = better ? pos : best_pos;
        win_card = better ? card : win_card;
        t_eyes = (first ? 0u : t_eyes) + ((ci.x >> 24) & 15u);
        // (fox = false: no lane of the wave holds a Diamond Ace, so none is played: nothing to track)
        da_bits = fox ? (first ? 0u : da_bits) | (card == (uint32_t)DIAMOND_ACE ? 1u << p : 0u) : 0u;
        plies += 1;
    };
    // collapsed announcement round after a card: one forced draw per offered player
    auto draws = [&]() {
        const uint32_t d = (uint32_t)popc32(((nb | 0x80808080u) - theta) & 0x80808080u);
        for (uint32_t i = 0; i < d; ++i) rng.advance();
        plies += (int)d;
    };
    bool done = false;
    // the partial first trick, absolute hands (a wave runs at most three of these plies)
    while (trick_len != 0u) {
        uint32_t a = sel4u(any0, any1, any2, any3, cur), t2 = sel4u(two0, two1, two2, two3, cur);
        play(a, t2, cur, false, trick_len, true);
        trick_len += 1u;
        any0 = cur == 0u ? a : any0; any1 = cur == 1u ? a : any1; any2 = cur == 2u ? a : any2; any3 = cur == 3u ? a : any3;
        two0 = cur == 0u ? t2 : two0; two1 = cur == 1u ? t2 : two1; two2 = cur == 2u ? t2 : two2; two3 = cur == 3u ? t2 : two3;
        cur = (cur + 1u) & 3u;
        if (trick_len == 4u) {
            const uint32_t winner = (trick_start + best_pos) & 3u;
            complete(winner);
            if (n_tricks == 12u) { done = true; break; }   // the rollout started within the last trick
            cur = winner; trick_start = winner; trick_len = 0; n_tricks += 1u; lead = 0xFFFFFFu;
            if (n_tricks == 12u) break;                   // forced tail below
        }
        draws();
    }
    if (!done) {
        // hands relative to trick_start (== cur between tricks)
        const uint32_t s0 = trick_start;
        uint32_t A0 = sel4u(any0, any1, any2, any3, s0), A1 = sel4u(any0, any1, any2, any3, (s0 + 1u) & 3u);
        uint32_t A2 = sel4u(any0, any1, any2, any3, (s0 + 2u) & 3u), A3 = sel4u(any0, any1, any2, any3, (s0 + 3u) & 3u);
        uint32_t T0 = sel4u(two0, two1, two2, two3, s0), T1 = sel4u(two0, two1, two2, two3, (s0 + 1u) & 3u);
        uint32_t T2 = sel4u(two0, two1, two2, two3, (s0 + 2u) & 3u), T3 = sel4u(two0, two1, two2, two3, (s0 + 3u) & 3u);
        while (n_tricks < 12u) {
            const uint32_t s = trick_start;
            // Announcement offers need n_p >= theta_p; hand sizes only fall and theta changes only
            // when a trick completes (a wedding resolved), so a trick that starts with no offer
            // for any lane of the wave has none before its last card: it skips the per-card
            // offer tests and hand-size updates (one trick's worth of sizes at its end).
            // (With nobody announcing, offers end within the first trick: theta = 11 - ws.)
            if (!DK_ROLLOUT_FAST || wave_any((((nb | 0x80808080u) - theta) & 0x80808080u) != 0u)) {
                play(A0, T0, s, true, 0u, true);
                draws();
                play(A1, T1, (s + 1u) & 3u, false, 1u, true);
                draws();
                play(A2, T2, (s + 2u) & 3u, false, 2u, true);
                draws();
                play(A3, T3, (s + 3u) & 3u, false, 3u, true);
            } else {
#if defined(DK_TRICK_DOUBLE) && defined(__HIP_DEVICE_COMPILE__)
                // measurement builds: a fast-path trick whose wave has at most DK_TRICK_DOUBLE active
                // lanes is played once more on copies (result discarded, kept alive): the time it adds
                // prices the rollout's sparse trips (the wave runs its longest lane's tricks)
                if (popc64(__builtin_amdgcn_ballot_w64(true)) <= DK_TRICK_DOUBLE) {
                    const Rng rs = rng;
                    uint32_t a0 = A0, a1 = A1, a2 = A2, a3 = A3, t0 = T0, t1 = T1, t2 = T2, t3 = T3;
                    const uint32_t sl = lead, sb = best_pos, sw = win_card, se = t_eyes, sd = da_bits, slt = lt;
                    const int sk = best_key, spl = plies;
                    play(a0, t0, s, true, 0u, false);
                    play(a1, t1, (s + 1u) & 3u, false, 1u, false);
                    play(a2, t2, (s + 2u) & 3u, false, 2u, false);
                    play(a3, t3, (s + 3u) & 3u, false, 3u, false);
                    asm volatile("" :: "v"(a0 ^ a1 ^ a2 ^ a3), "v"(t0 ^ t1 ^ t2 ^ t3), "v"(best_pos), "v"(t_eyes), "v"(da_bits),
                                 "v"(win_card), "v"((uint32_t)rng.s0));
                    rng = rs; lead = sl; best_pos = sb; win_card = sw; t_eyes = se; da_bits = sd; lt = slt; best_key = sk;
                    plies = spl;
                }
#endif
#if DK_FOX_SKIP
                // once no lane of the wave holds a Diamond Ace (the fox, stats/**), its per-card tracking is skipped
                if (!wave_any((((A0 | A1 | A2 | A3) >> (uint32_t)DIAMOND_ACE) & 1u) != 0u)) {
                    play(A0, T0, s, true, 0u, false, false);
                    play(A1, T1, (s + 1u) & 3u, false, 1u, false, false);
                    play(A2, T2, (s + 2u) & 3u, false, 2u, false, false);
                    play(A3, T3, (s + 3u) & 3u, false, 3u, false, false);
                } else
#endif
#if DK_TRICK_SPEC
                {
                    // the four plies as one block (draw_trick); the exact per-ply path on a rejection
                    TrickDraw td;
                    if (draw_trick(A0, A1, A2, A3, rng, gt, tm, td)) {
                        const uint32_t c0 = td.c[0], c1 = td.c[1], c2 = td.c[2], c3 = td.c[3], ld = td.ld;
                        const CardInfo i0 = td.i[0], i1 = td.i[1], i2 = td.i[2], i3 = td.i[3];
                        const uint32_t b0 = 1u << c0, b1 = 1u << c1, b2 = 1u << c2, b3 = 1u << c3;
                        const uint32_t d0 = T0 & b0, d1 = T1 & b1, d2 = T2 & b2, d3 = T3 & b3;
                        T0 ^= d0; A0 ^= b0 ^ d0; T1 ^= d1; A1 ^= b1 ^ d1;
                        T2 ^= d2; A2 ^= b2 ^ d2; T3 ^= d3; A3 ^= b3 ^ d3;
                        lead = ld; lt = ld | tm;
                        const int k1 = ((lt >> c1) & 1u) ? (int)i1.y : -1;
                        const int k2 = ((lt >> c2) & 1u) ? (int)i2.y : -1;
                        const int k3 = ((lt >> c3) & 1u) ? (int)i3.y : -1;
                        best_key = (int)i0.y; best_pos = 0u; win_card = c0;
                        if (k1 > best_key) { best_key = k1; best_pos = 1u; win_card = c1; }
                        if (k2 > best_key) { best_key = k2; best_pos = 2u; win_card = c2; }
                        if (k3 > best_key) { best_key = k3; best_pos = 3u; win_card = c3; }
                        t_eyes = ((i0.x >> 24) & 15u) + ((i1.x >> 24) & 15u) + ((i2.x >> 24) & 15u) + ((i3.x >> 24) & 15u);
                        da_bits = (c0 == (uint32_t)DIAMOND_ACE ? 1u << s : 0u) |
                                  (c1 == (uint32_t)DIAMOND_ACE ? 1u << ((s + 1u) & 3u) : 0u) |
                                  (c2 == (uint32_t)DIAMOND_ACE ? 1u << ((s + 2u) & 3u) : 0u) |
                                  (c3 == (uint32_t)DIAMOND_ACE ? 1u << ((s + 3u) & 3u) : 0u);
                        plies += 4;
                    } else {
                        play(A0, T0, s, true, 0u, false);
                        play(A1, T1, (s + 1u) & 3u, false, 1u, false);
                        play(A2, T2, (s + 2u) & 3u, false, 2u, false);
                        play(A3, T3, (s + 3u) & 3u, false, 3u, false);
                    }
                }
#else
                {
                    play(A0, T0, s, true, 0u, false);
                    play(A1, T1, (s + 1u) & 3u, false, 1u, false);
                    play(A2, T2, (s + 2u) & 3u, false, 2u, false);
                    play(A3, T3, (s + 3u) & 3u, false, 3u, false);
                }
#endif
                nb -= 0x01010101u;
            }
            const uint32_t bp = best_pos;
            const uint32_t winner = (s + bp) & 3u;
            complete(winner);
            trick_start = winner; trick_len = 0; n_tricks += 1u; lead = 0xFFFFFFu;
            // the winner leads: rotate the hands left by its position in the trick
            const bool r1 = (bp & 1u) != 0u, r2 = (bp & 2u) != 0u;
            uint32_t b0 = r1 ? A1 : A0, b1 = r1 ? A2 : A1, b2 = r1 ? A3 : A2, b3 = r1 ? A0 : A3;
            A0 = r2 ? b2 : b0; A1 = r2 ? b3 : b1; A2 = r2 ? b0 : b2; A3 = r2 ? b1 : b3;
            b0 = r1 ? T1 : T0; b1 = r1 ? T2 : T1; b2 = r1 ? T3 : T2; b3 = r1 ? T0 : T3;
            T0 = r2 ? b2 : b0; T1 = r2 ? b3 : b1; T2 = r2 ? b0 : b2; T3 = r2 ? b1 : b3;
            if (n_tricks == 12u) break;   // every hand holds one card: no offer, forced tail below
            draws();
        }
        // ---- the last trick: four forced plays from `trick_start`, one range(0..1) draw each
        const uint32_t s = trick_start;
        uint32_t best = 0;
        const uint32_t hs[4] = {A0, A1, A2, A3};
#pragma unroll
        for (uint32_t i = 0; i < 4u; ++i) {
            const uint32_t p = (s + i) & 3u;
            const uint32_t card = (uint32_t)ctz32(hs[i]);
            rng.advance();
            const CardInfo ci = card_info(gt, card);
            if (i == 0u) {
                lead = ci.x & 0xFFFFFFu;
                best_key = (int)ci.y; best = 0; win_card = card;
                t_eyes = (ci.x >> 24) & 15u; da_bits = 0;
            } else {
                const int key = (((ci.x >> 28) & 1u) || ((lead >> card) & 1u)) ? (int)ci.y : -1;
                const bool better = key > best_key;
                best_key = better ? key : best_key;
                best = better ? i : best;
                win_card = better ? card : win_card;
                t_eyes += (ci.x >> 24) & 15u;
            }
            da_bits |= card == (uint32_t)DIAMOND_ACE ? 1u << p : 0u;
        }
        plies += 4;
        complete((s + best) & 3u);
    }
    Work fin = w0;
    fin.eyes = eyes; fin.ntricks = ntr; fin.doko = doko;
    fin.fox_n = (uint8_t)fox_n; fin.fox0 = (uint8_t)fox0; fin.fox1 = (uint8_t)fox1; fin.karl = (uint8_t)karl;
    fin.re_players = (uint8_t)re_players;
    score(fin, pts);
    return plies;
}

// The rest of a pending announcement round when nobody announces: the asked
// player and each later player of the round (4 - ann_turns asks in all) with a
// non-empty offer take one forced NoAnnouncement draw; then the card phase
// resumes with the player who started the round (announcement.rs:137-180).
DK_HD int collapse_announcement_round(Work& w, Rng& rng) {
    const uint32_t theta = ann_thetas(w.team_kind, w.solved_trick, w.re_players, w.re_lowest, w.contra_lowest);
    const uint32_t asks = 4u - (uint32_t)w.ann_turns;
    int draws = 1;   // the asked player (its offer is non-empty)
#pragma unroll
    for (uint32_t i = 1; i < 4; ++i) {
        const uint32_t p = ((uint32_t)w.cur + i) & 3u;
        const bool offered = (uint32_t)hand_len(w, (int)p) >= ((theta >> (8u * p)) & 0xFFu);
        draws += (i < asks && offered) ? 1 : 0;
    }
    for (int i = 0; i < draws; ++i) rng.advance();
    w.ann_turns = 4; w.ann_allowed = 0; w.cur = w.ann_start; w.phase = PH_PLAYCARD;
    return draws;
}

// Returns the rewards (player_points) and the number of plies played.
DK_HD int rollout(Work w, Rng& rng, int pts[4]) {
    int plies = 0;
    // Generic steps through the reservation round.
    while (w.phase == PH_RESERVATION) {
        const uint64_t a = legal_actions(w) & ~ANN_ACTIONS;
        const int act = ctz64(random_single(a, rng));
        play_action(w, act);
        plies++;
    }
    if (w.phase == PH_ANNOUNCEMENT) plies += collapse_announcement_round(w, rng);
    if (w.phase == PH_FINISHED) { score(w, pts); return plies; }
    return plies + rollout_cards(w, rng, pts);
}

// Reference restatement of the card phase on the full Work state, step by step
// (kept as the host-side cross-check of rollout_cards).
DK_HD int rollout_stepwise(Work w, Rng& rng, int pts[4]) {
    int plies = 0;
    while (w.phase != PH_PLAYCARD && w.phase != PH_FINISHED) {
        const uint64_t a = legal_actions(w) & ~ANN_ACTIONS;
        const int act = ctz64(random_single(a, rng));
        play_action(w, act);
        plies++;
    }
    while (w.phase != PH_FINISHED) {
        const uint64_t a = legal_actions(w);
        const int card = ctz64(random_single(a, rng));
        plies++;
        if (play_card_core(w, card)) break;
        const int d = round_draws(w);
        for (int i = 0; i < d; ++i) (void)rng.next_u64();
        plies += d;
    }
    score(w, pts);
    return plies;
}

// ---- node-state record of the search pools (64 B) --------------------------------
// The search stores one state per expanded tree node; 64 B aligned to 64 is one memory
// sector and four 16-B accesses, against 88 B (eleven 8-B accesses, up to two lines) for
// Work itself.  Hands are 48-bit masks; per-player trick and >= 40-eye trick counts are
// <= 12 (nibbles); twelve small fields are nibbles (trick_len <= 4, trick_start /
// ann_start / res_start < 4, phase / team_kind < 4, ann_turns / res_len / karl <= 4,
// fox events < 16, n_tricks <= 12).  States the engine reaches keep these ranges; a
// search root is checked (node_ok) before it is stored.
struct alignas(16) Node { uint32_t w[16]; };
DK_HD uint32_t nib4(uint32_t x) { return (x & 0xFu) | ((x >> 4) & 0xF0u) | ((x >> 8) & 0xF00u) | ((x >> 12) & 0xF000u); }
DK_HD uint32_t unnib4(uint32_t y) { return (y & 0xFu) | ((y & 0xF0u) << 4) | ((y & 0xF00u) << 8) | ((y & 0xF000u) << 12); }
DK_HD Node pack_node(const Work& x) {
    Node n;
    n.w[0] = (uint32_t)x.h[0];
    n.w[1] = (uint32_t)(x.h[0] >> 32) | (uint32_t)x.h[1] << 16;
    n.w[2] = (uint32_t)(x.h[1] >> 16);
    n.w[3] = (uint32_t)x.h[2];
    n.w[4] = (uint32_t)(x.h[2] >> 32) | (uint32_t)x.h[3] << 16;
    n.w[5] = (uint32_t)(x.h[3] >> 16);
    n.w[6] = x.trick_cards;
    n.w[7] = x.trick_winners | (uint32_t)x.fox_n << 24;
    n.w[8] = x.eyes;
    n.w[9] = nib4(x.ntricks) | nib4(x.doko) << 16;
    n.w[10] = x.res;
    n.w[11] = (uint32_t)x.trick_len | (uint32_t)x.trick_start << 4 | (uint32_t)x.phase << 8 | (uint32_t)x.team_kind << 12 |
              (uint32_t)x.ann_turns << 16 | (uint32_t)x.ann_start << 20 | (uint32_t)x.res_start << 24 | (uint32_t)x.res_len << 28;
    n.w[12] = (uint32_t)x.karl | (uint32_t)x.fox0 << 4 | (uint32_t)x.fox1 << 8 | (uint32_t)x.n_tricks << 12 |
              (uint32_t)x.card_index << 16 | (uint32_t)x.game_type << 24;
    n.w[13] = (uint32_t)x.rr_kind | (uint32_t)x.rr_player << 8 | (uint32_t)x.rr_res << 16 | (uint32_t)x.wedding_player << 24;
    n.w[14] = (uint32_t)x.solved_trick | (uint32_t)x.re_players << 8 | (uint32_t)x.re_lowest << 16 | (uint32_t)x.contra_lowest << 24;
    n.w[15] = (uint32_t)x.ann_allowed | (uint32_t)x.ann_count << 8 | (uint32_t)x.ann_players << 16 | (uint32_t)x.cur << 24;
    return n;
}
DK_HD Work unpack_node(const Node& n) {
    Work x;
    const uint64_t M48 = 0xFFFFFFFFFFFFULL;
    x.h[0] = ((uint64_t)n.w[0] | (uint64_t)n.w[1] << 32) & M48;
    x.h[1] = (uint64_t)(n.w[1] >> 16) | (uint64_t)n.w[2] << 16;
    x.h[2] = ((uint64_t)n.w[3] | (uint64_t)n.w[4] << 32) & M48;
    x.h[3] = (uint64_t)(n.w[4] >> 16) | (uint64_t)n.w[5] << 16;
    x.trick_cards = n.w[6];
    x.trick_winners = n.w[7] & 0xFFFFFFu; x.fox_n = (uint8_t)(n.w[7] >> 24);
    x.eyes = n.w[8];
    x.ntricks = unnib4(n.w[9] & 0xFFFFu); x.doko = unnib4(n.w[9] >> 16);
    x.res = n.w[10];
    const uint32_t a = n.w[11], b = n.w[12], c = n.w[13], d = n.w[14], e = n.w[15];
    x.trick_len = (uint8_t)(a & 15u); x.trick_start = (uint8_t)((a >> 4) & 15u); x.phase = (uint8_t)((a >> 8) & 15u);
    x.team_kind = (uint8_t)((a >> 12) & 15u); x.ann_turns = (uint8_t)((a >> 16) & 15u); x.ann_start = (uint8_t)((a >> 20) & 15u);
    x.res_start = (uint8_t)((a >> 24) & 15u); x.res_len = (uint8_t)(a >> 28);
    x.karl = (uint8_t)(b & 15u); x.fox0 = (uint8_t)((b >> 4) & 15u); x.fox1 = (uint8_t)((b >> 8) & 15u);
    x.n_tricks = (uint8_t)((b >> 12) & 15u); x.card_index = (uint8_t)(b >> 16); x.game_type = (uint8_t)(b >> 24);
    x.rr_kind = (uint8_t)c; x.rr_player = (uint8_t)(c >> 8); x.rr_res = (uint8_t)(c >> 16); x.wedding_player = (uint8_t)(c >> 24);
    x.solved_trick = (uint8_t)d; x.re_players = (uint8_t)(d >> 8); x.re_lowest = (uint8_t)(d >> 16); x.contra_lowest = (uint8_t)(d >> 24);
    x.ann_allowed = (uint8_t)e; x.ann_count = (uint8_t)(e >> 8); x.ann_players = (uint8_t)(e >> 16); x.cur = (uint8_t)(e >> 24);
    x.pad0 = 0; x.pad1 = 0;
    return x;
}
// the record holds this state exactly (the search checks every root)
DK_HD bool node_ok(const Work& x) {
    const Work y = unpack_node(pack_node(x));
    bool ok = x.h[0] == y.h[0] && x.h[1] == y.h[1] && x.h[2] == y.h[2] && x.h[3] == y.h[3];
    ok = ok && x.trick_cards == y.trick_cards && x.trick_winners == y.trick_winners && x.eyes == y.eyes;
    ok = ok && x.ntricks == y.ntricks && x.doko == y.doko && x.res == y.res;
    ok = ok && x.fox_n == y.fox_n && x.fox0 == y.fox0 && x.fox1 == y.fox1 && x.karl == y.karl;
    ok = ok && x.trick_len == y.trick_len && x.trick_start == y.trick_start && x.n_tricks == y.n_tricks && x.card_index == y.card_index;
    ok = ok && x.phase == y.phase && x.cur == y.cur && x.game_type == y.game_type && x.rr_kind == y.rr_kind;
    ok = ok && x.rr_player == y.rr_player && x.rr_res == y.rr_res && x.team_kind == y.team_kind && x.wedding_player == y.wedding_player;
    ok = ok && x.solved_trick == y.solved_trick && x.re_players == y.re_players && x.re_lowest == y.re_lowest &&
         x.contra_lowest == y.contra_lowest;
    ok = ok && x.ann_turns == y.ann_turns && x.ann_start == y.ann_start && x.ann_allowed == y.ann_allowed &&
         x.ann_count == y.ann_count;
    ok = ok && x.ann_players == y.ann_players && x.res_start == y.res_start && x.res_len == y.res_len;
    return ok;
}

// ---- wire format ----------------------------------------------------------------
DK_HD void unpack(const dk_fdo_state& s, Work& w) {
    for (int p = 0; p < 4; ++p) w.h[p] = s.hands[p];
    w.eyes = (uint32_t)s.eyes[0] | (uint32_t)s.eyes[1] << 8 | (uint32_t)s.eyes[2] << 16 | (uint32_t)s.eyes[3] << 24;
    w.ntricks = (uint32_t)s.ntricks[0] | (uint32_t)s.ntricks[1] << 8 | (uint32_t)s.ntricks[2] << 16 | (uint32_t)s.ntricks[3] << 24;
    w.trick_winners = s.trick_winners;
    w.res = (uint32_t)s.res[0] | (uint32_t)s.res[1] << 8 | (uint32_t)s.res[2] << 16 | (uint32_t)s.res[3] << 24;
    w.res_start = s.res_start; w.res_len = s.res_len; w.card_index = s.card_index; w.phase = s.phase;
    w.cur = s.current_player; w.game_type = s.game_type;
    w.rr_kind = s.rr_kind == DK_NONE ? (uint8_t)RR_NONE : (s.rr_kind == 0 ? (uint8_t)RR_NONE : s.rr_kind);
    w.rr_player = s.rr_player; w.rr_res = s.rr_reservation;
    w.team_kind = s.team_kind; w.wedding_player = s.wedding_player; w.solved_trick = s.solved_trick; w.re_players = s.re_players;
    w.re_lowest = s.re_lowest; w.contra_lowest = s.contra_lowest; w.ann_turns = s.ann_turns; w.ann_start = s.ann_start;
    w.ann_allowed = s.ann_allowed; w.ann_count = s.ann_count; w.ann_players = s.ann_players; w.n_tricks = s.n_tricks;
    w.pad0 = 0;
    // current trick and scoring accumulators from the card history
    w.doko = 0; w.fox_n = 0; w.fox0 = 0; w.fox1 = 0; w.karl = 0;
    const int completed = s.card_index / 4;
    for (int t = 0; t < completed && t < 12; ++t) {
        const int winner = (int)((s.trick_winners >> (2 * t)) & 3);
        const int start = t == 0 ? s.res_start : (int)((s.trick_winners >> (2 * (t - 1))) & 3);
        uint32_t e = 0; int best_key = -2, best_i = 0;
        const uint32_t tc = card_color(s.cards[4 * t], s.game_type);
        for (int i = 0; i < 4; ++i) {
            const int c = s.cards[4 * t + i];
            e += card_eyes(c);
            const int k = trick_key(c, tc, s.game_type);
            if (k > best_key) { best_key = k; best_i = i; }
            if (c == DIAMOND_ACE) {
                const uint8_t ev = (uint8_t)((((start + i) & 3) << 2) | winner);
                if (w.fox_n == 0) w.fox0 = ev; else w.fox1 = ev;
                w.fox_n += 1;
            }
        }
        if (e >= 40) w.doko = byte_add(w.doko, winner, 1);
        if (t == 11 && s.cards[4 * t + best_i] == CLUB_JACK) w.karl = (uint8_t)(1 + winner);
    }
    w.trick_cards = 0; w.trick_len = 0;
    w.trick_start = (uint8_t)(completed == 0 ? s.res_start : (int)((s.trick_winners >> (2 * (completed - 1))) & 3));
    if (s.n_tricks > 0 && s.phase != PH_FINISHED) {
        const int in_trick = s.card_index - 4 * (s.n_tricks - 1);
        for (int i = 0; i < in_trick; ++i) w.trick_cards |= (uint32_t)s.cards[4 * (s.n_tricks - 1) + i] << (8 * i);
        w.trick_len = (uint8_t)in_trick;
    }
}

DK_HD void pack_fields(const Work& w, dk_fdo_state& s) {
    for (int p = 0; p < 4; ++p) { s.hands[p] = w.h[p]; s.eyes[p] = (uint8_t)byte_get(w.eyes, p); s.ntricks[p] = (uint8_t)byte_get(w.ntricks, p); }
    s.trick_winners = w.trick_winners;
    for (int i = 0; i < 4; ++i) s.res[i] = i < w.res_len ? (uint8_t)byte_get(w.res, i) : (uint8_t)DK_NONE;
    s.res_start = w.res_start; s.res_len = w.res_len; s.card_index = w.card_index; s.phase = w.phase;
    s.current_player = w.phase == PH_FINISHED ? (uint8_t)DK_NONE : w.cur;
    s.game_type = w.game_type;
    s.rr_kind = w.res_len < 4 ? (uint8_t)DK_NONE : (w.rr_kind == RR_NONE ? (uint8_t)0 : w.rr_kind);
    s.rr_player = w.rr_player; s.rr_reservation = w.rr_res;
    s.team_kind = w.team_kind; s.wedding_player = w.wedding_player; s.solved_trick = w.solved_trick; s.re_players = w.re_players;
    s.re_lowest = w.re_lowest; s.contra_lowest = w.contra_lowest; s.ann_turns = w.ann_turns; s.ann_start = w.ann_start;
    s.ann_allowed = w.ann_allowed; s.ann_count = w.ann_count; s.ann_players = w.ann_players; s.n_tricks = w.n_tricks;
    s.game = DK_GAME_FULL_DOKO;
}

// McEnvState::by_action on the wire format (keeps the card history).
DK_HD void step_packed(dk_fdo_state& s, int a) {
    Work w; unpack(s, w);
    const uint8_t ci = w.card_index;
    play_action(w, a);
    if (a <= 23) s.cards[ci] = (uint8_t)a;
    pack_fields(w, s);
}

// rewards_or_none / finished check on the working state
DK_HD bool is_terminal(const Work& w) { return w.phase == PH_FINISHED; }
DK_HD int env_current_player(const Work& w) { return w.phase == PH_FINISHED ? 0 : (int)w.cur; }

}  // namespace fdo
}  // namespace dk
