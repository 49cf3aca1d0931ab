// rs-doko (simplified Doppelkopf: normal game, wedding, silent solo; no
// announcements) as a register-resident state machine.
// Reference: rs-doko/src/state/state.rs:159-334, action/allowed_actions.rs:131-198,
// trick/trick_winning_player_logic.rs:11-34, teams/team_logic.rs:69-143,
// stats/stats.rs:25-135, hand/hand.rs:38-46 (removes the FIRST copy),
// env adapter rs-doko-mcts/src/env/envs/env_state_doko.rs (allowed_actions /
// by_action are todo!() there; DoAction bits 0-25 == FdoAction bits 0-25).
#pragma once
#include "../../../include/doko_amd.h"
#include "common.h"
#include "fdo_engine.h"
#include "rng.h"

namespace dk {
namespace dko {

enum : uint32_t { PH_RESERVATION = 0, PH_PLAYCARD = 1, PH_FINISHED = 2 };
enum : uint32_t { RES_WEDDING = 0, RES_HEALTHY = 1 };

struct Work {
    uint64_t h[4];
    uint32_t trick_cards, trick_winners, eyes, ntricks, res;
    uint8_t trick_len, trick_start, trick_index, card_index;
    uint8_t phase, cur, res_len, res_start;
    uint8_t rr_wedding, team_kind, wedding_player, solved_trick;  // rr_wedding: 0xFF = NoReservation
    uint8_t re_players, pad0, pad1, pad2;
};

DK_HD uint64_t legal_actions(const Work& w) {
    const uint64_t h = sel4(w.h, w.cur);
    if (w.phase == PH_RESERVATION) {
        uint64_t a = 1ULL << 24;
        if ((h >> 15 & 1) && (h >> 39 & 1)) a |= 1ULL << 25;
        return a;
    }
    if (w.phase != PH_PLAYCARD) return 0;
    const uint64_t single = (h | (h >> 24)) & 0xFFFFFFULL;
    if (w.trick_len == 0) return single;
    const uint32_t tc = fdo::card_color((int)(w.trick_cards & 0xFF), fdo::GT_NORMAL);
    const uint64_t follow = single & fdo::color_mask(tc, fdo::GT_NORMAL);
    return follow ? follow : single;
}

DK_HD void finish_reservations(Work& w) {
    int wi = -1;
    for (int i = 0; i < 4; ++i) if (byte_get(w.res, i) == RES_WEDDING) wi = i;
    w.rr_wedding = wi < 0 ? 0xFF : (uint8_t)((wi + w.res_start) & 3);
    if (wi < 0) {
        uint8_t re = 0;
        for (int p = 0; p < 4; ++p) { const uint64_t h = sel4(w.h, p); if ((h >> 15 & 1) || (h >> 39 & 1)) re |= (uint8_t)(1u << p); }
        w.team_kind = fdo::TK_NOWEDDING; w.re_players = re;
    } else {
        w.team_kind = fdo::TK_WED_UNSOLVED; w.wedding_player = w.rr_wedding; w.re_players = 0;
    }
}

DK_HD int complete_trick(Work& w) {
    const uint32_t tc = fdo::card_color((int)(w.trick_cards & 0xFF), fdo::GT_NORMAL);
    int best_key = -2, best_i = 0; uint32_t e = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int c = (int)((w.trick_cards >> (8 * i)) & 0xFF);
        const int k = fdo::trick_key(c, tc, fdo::GT_NORMAL);
        const bool better = k > best_key;
        best_key = better ? k : best_key; best_i = better ? i : best_i;
        e += fdo::card_eyes(c);
    }
    const int winner = (w.trick_start + best_i) & 3;
    const int t = w.trick_index;
    w.trick_winners |= (uint32_t)winner << (2 * t);
    w.eyes = byte_add(w.eyes, winner, e);
    w.ntricks = byte_add(w.ntricks, winner, 1);
    if (w.team_kind == fdo::TK_WED_UNSOLVED && t < 3) {
        if (winner != w.wedding_player) {
            w.team_kind = fdo::TK_WED_SOLVED; w.solved_trick = (uint8_t)t;
            w.re_players = (uint8_t)((1u << w.wedding_player) | (1u << winner));
        } else if (t == 2) {
            w.team_kind = fdo::TK_WED_SOLVED; w.solved_trick = 2; w.re_players = (uint8_t)(1u << w.wedding_player);
        }
    }
    return winner;
}

// DoState::play_action (state.rs:189-309)
DK_HD void play_action(Work& w, int a) {
    const int cp = w.cur;
    if (a <= 23) {
        const uint64_t h = sel4(w.h, cp);
        const uint64_t lo = 1ULL << a;
        set4(w.h, cp, (h & lo) ? (h & ~lo) : (h & ~(1ULL << (a + 24))));
        w.trick_cards |= (uint32_t)a << (8 * w.trick_len);
        w.trick_len += 1; w.card_index += 1;
        if (w.trick_len == 4) {
            const int winner = complete_trick(w);
            w.trick_index += 1;
            if (w.trick_index == 12) { w.phase = PH_FINISHED; w.cur = 0xFF; return; }
            w.trick_cards = 0; w.trick_len = 0; w.trick_start = (uint8_t)winner; w.cur = (uint8_t)winner;
            return;
        }
        w.cur = (uint8_t)((cp + 1) & 3);
    } else {
        w.res = byte_set(w.res, w.res_len, a == 25 ? RES_WEDDING : RES_HEALTHY);
        w.res_len += 1;
        w.cur = (uint8_t)((cp + 1) & 3);
        if (w.res_len == 4) {
            w.phase = PH_PLAYCARD;
            w.trick_index = 0; w.trick_cards = 0; w.trick_len = 0; w.trick_start = w.cur;
            finish_reservations(w);
        }
    }
}

// stats.rs:25-135 -> player points (env_state_doko.rs:36-97 rewards)
DK_HD void score(const Work& w, int pts[4]) {
    uint32_t re_e = 0, ko_e = 0, re_t = 0, ko_t = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const bool r = (w.re_players >> p) & 1;
        re_e += r ? byte_get(w.eyes, p) : 0; ko_e += r ? 0 : byte_get(w.eyes, p);
        re_t += r ? byte_get(w.ntricks, p) : 0; ko_t += r ? 0 : byte_get(w.ntricks, p);
    }
    const bool re_wins = re_e > ko_e;
    const uint32_t we = re_wins ? re_e : ko_e, wt = re_wins ? re_t : ko_t;
    const int v = (we >= 120) + (we >= 150) + (we >= 180) + (we >= 210) + (wt == 12);
    int rp = re_wins ? v : -v;
    const int kp = re_wins ? -v : v;
    if (popc32(w.re_players) == 1) rp *= 3;
#pragma unroll
    for (int p = 0; p < 4; ++p) pts[p] = ((w.re_players >> p) & 1) ? rp : kp;
}

// Generic stepwise rollout (random_action_for_current_player until finished,
// state.rs:315-334); kept as the host-side cross-check of rollout_cards.
DK_HD int rollout_stepwise(Work w, Rng& rng, int pts[4]) {
    int plies = 0;
    while (w.phase != PH_FINISHED) {
        const uint64_t a = legal_actions(w);
        play_action(w, ctz64(random_single(a, rng)));
        plies++;
    }
    score(w, pts);
    return plies;
}

// Card phase to the end (w.phase == PH_PLAYCARD), the rs-doko counterpart of
// fdo::rollout_cards: hands as "kinds held" / "kinds held twice" 24-bit masks
// (which copy a removal takes is invisible to the rewards), the trick evaluated
// incrementally as its cards are played (first strict maximum, eyes), and after the
// partial first trick one whole trick per loop trip with the hands relative to the
// leader (four plies unrolled, one rotation by the winner per trick).  One range draw
// per card, as random_single draws one even for a single option.
DK_HD int rollout_cards(const Work& w0, Rng& rng, int pts[4]) {
    uint32_t any0, any1, any2, any3, two0, two1, two2, two3;
    {
        const uint32_t M = 0xFFFFFFu;
        const uint64_t h0 = w0.h[0], h1 = w0.h[1], h2 = w0.h[2], h3 = w0.h[3];
        any0 = ((uint32_t)h0 | (uint32_t)(h0 >> 24)) & M; two0 = ((uint32_t)h0 & (uint32_t)(h0 >> 24)) & M;
        any1 = ((uint32_t)h1 | (uint32_t)(h1 >> 24)) & M; two1 = ((uint32_t)h1 & (uint32_t)(h1 >> 24)) & M;
        any2 = ((uint32_t)h2 | (uint32_t)(h2 >> 24)) & M; two2 = ((uint32_t)h2 & (uint32_t)(h2 >> 24)) & M;
        any3 = ((uint32_t)h3 | (uint32_t)(h3 >> 24)) & M; two3 = ((uint32_t)h3 & (uint32_t)(h3 >> 24)) & M;
    }
    const uint32_t tm = fdo::trump_mask(fdo::GT_NORMAL);
    uint32_t team_kind = w0.team_kind, re_players = w0.re_players;
    const uint32_t wedding_player = w0.wedding_player;
    uint32_t cur = w0.cur, trick_start = w0.trick_start, trick_len = w0.trick_len, t_idx = w0.trick_index;
    uint32_t eyes = w0.eyes, ntr = w0.ntricks;
    uint32_t lead = 0xFFFFFFu, best_pos = 0, t_eyes = 0;
    int best_key = -2;
    for (uint32_t i = 0; i < trick_len; ++i) {
        const uint32_t c = (w0.trick_cards >> (8u * i)) & 0xFFu;
        if (i == 0) lead = fdo::class_mask(c, tm);
        const int k = fdo::key_fast(c, tm, lead);
        if (k > best_key) { best_key = k; best_pos = i; }
        t_eyes += fdo::eyes_fast(c);
    }
    uint32_t lt = lead | tm;   // a card can win the trick iff it is a trump or of the led class
    int plies = 0;
    // one card of the player whose hand is (a, t2), at position `pos` of the trick; updates the
    // hand (the second copy first: no selects) and the running trick
    auto play = [&](uint32_t& a, uint32_t& t2, bool first, uint32_t pos) {
        const uint32_t f = a & lead;
        const uint32_t legal = f ? f : a;
        const uint32_t r = rng.range_u32((uint32_t)popc32(legal));
        const uint32_t card = fdo::nth_set_bit24(legal, (uint32_t)popc32(legal) - 1u - r), bit = 1u << card;
#if DK_ROLLOUT_FAST
        const uint32_t second = t2 & bit;
        t2 ^= second;
        a ^= bit ^ second;
#else
        const bool dup = (t2 & bit) != 0u;
        a = dup ? a : (a ^ bit);
        t2 = dup ? (t2 ^ bit) : t2;
#endif
        const fdo::CardInfo ci = fdo::card_info(fdo::GT_NORMAL, card);
        lead = first ? (ci.x & 0xFFFFFFu) : lead;
#if DK_ROLLOUT_FAST
        lt = first ? (lead | tm) : lt;
        const int key = ((lt >> card) & 1u) ? (int)ci.y : -1;
#else
        const int key = (((ci.x >> 28) & 1u) || ((lead >> card) & 1u)) ? (int)ci.y : -1;
#endif
        const bool better = first || key > best_key;
        best_key = better ? key : best_key;
        best_pos = better ? pos : best_pos;
        t_eyes = (first ? 0u : t_eyes) + ((ci.x >> 24) & 15u);
        plies += 1;
    };
    auto complete = [&](uint32_t winner) {
        eyes += t_eyes << (8u * winner);
        ntr += 1u << (8u * winner);
        if (team_kind == fdo::TK_WED_UNSOLVED && t_idx < 3u && (winner != wedding_player || t_idx == 2u)) {
            team_kind = fdo::TK_WED_SOLVED;
            re_players = (1u << wedding_player) | (winner != wedding_player ? 1u << winner : 0u);
        }
        t_idx += 1u;
    };
    bool done = false;
    // the partial first trick, absolute hands (a wave runs at most three of these plies)
    while (trick_len != 0u) {
        uint32_t a = fdo::sel4u(any0, any1, any2, any3, cur), t2 = fdo::sel4u(two0, two1, two2, two3, cur);
        play(a, t2, false, trick_len);
        trick_len += 1u;
        any0 = cur == 0u ? a : any0; any1 = cur == 1u ? a : any1; any2 = cur == 2u ? a : any2; any3 = cur == 3u ? a : any3;
        two0 = cur == 0u ? t2 : two0; two1 = cur == 1u ? t2 : two1; two2 = cur == 2u ? t2 : two2; two3 = cur == 3u ? t2 : two3;
        cur = (cur + 1u) & 3u;
        if (trick_len == 4u) {
            const uint32_t winner = (trick_start + best_pos) & 3u;
            complete(winner);
            if (t_idx == 12u) { done = true; break; }
            cur = winner; trick_start = winner; trick_len = 0; lead = 0xFFFFFFu;
        }
    }
    if (!done) {
        const uint32_t s0 = trick_start;
        uint32_t A0 = fdo::sel4u(any0, any1, any2, any3, s0), A1 = fdo::sel4u(any0, any1, any2, any3, (s0 + 1u) & 3u);
        uint32_t A2 = fdo::sel4u(any0, any1, any2, any3, (s0 + 2u) & 3u), A3 = fdo::sel4u(any0, any1, any2, any3, (s0 + 3u) & 3u);
        uint32_t T0 = fdo::sel4u(two0, two1, two2, two3, s0), T1 = fdo::sel4u(two0, two1, two2, two3, (s0 + 1u) & 3u);
        uint32_t T2 = fdo::sel4u(two0, two1, two2, two3, (s0 + 2u) & 3u), T3 = fdo::sel4u(two0, two1, two2, two3, (s0 + 3u) & 3u);
        for (;;) {
            fdo::TrickDraw td;
            if (DK_TRICK_SPEC && fdo::draw_trick(A0, A1, A2, A3, rng, fdo::GT_NORMAL, tm, td)) {
                // the four plies as one block (fdo::draw_trick); the exact per-ply path on a rejection
                const uint32_t b0 = 1u << td.c[0], b1 = 1u << td.c[1], b2 = 1u << td.c[2], b3 = 1u << td.c[3];
                const uint32_t d0 = T0 & b0, d1 = T1 & b1, d2 = T2 & b2, d3 = T3 & b3;
                T0 ^= d0; A0 ^= b0 ^ d0; T1 ^= d1; A1 ^= b1 ^ d1;
                T2 ^= d2; A2 ^= b2 ^ d2; T3 ^= d3; A3 ^= b3 ^ d3;
                lead = td.ld; lt = td.ld | tm;
                const int k1 = ((lt >> td.c[1]) & 1u) ? (int)td.i[1].y : -1;
                const int k2 = ((lt >> td.c[2]) & 1u) ? (int)td.i[2].y : -1;
                const int k3 = ((lt >> td.c[3]) & 1u) ? (int)td.i[3].y : -1;
                best_key = (int)td.i[0].y; best_pos = 0u;
                if (k1 > best_key) { best_key = k1; best_pos = 1u; }
                if (k2 > best_key) { best_key = k2; best_pos = 2u; }
                if (k3 > best_key) { best_key = k3; best_pos = 3u; }
                t_eyes = ((td.i[0].x >> 24) & 15u) + ((td.i[1].x >> 24) & 15u) + ((td.i[2].x >> 24) & 15u) +
                         ((td.i[3].x >> 24) & 15u);
                plies += 4;
            } else {
                play(A0, T0, true, 0u);
                play(A1, T1, false, 1u);
                play(A2, T2, false, 2u);
                play(A3, T3, false, 3u);
            }
            const uint32_t bp = best_pos;
            const uint32_t winner = (trick_start + bp) & 3u;
            complete(winner);
            if (t_idx == 12u) break;
            trick_start = winner; trick_len = 0; lead = 0xFFFFFFu;
            // the winner leads: rotate the hands left by its position in the trick
            const bool r1 = (bp & 1u) != 0u, r2 = (bp & 2u) != 0u;
            uint32_t b0 = r1 ? A1 : A0, b1 = r1 ? A2 : A1, b2 = r1 ? A3 : A2, b3 = r1 ? A0 : A3;
            A0 = r2 ? b2 : b0; A1 = r2 ? b3 : b1; A2 = r2 ? b0 : b2; A3 = r2 ? b1 : b3;
            b0 = r1 ? T1 : T0; b1 = r1 ? T2 : T1; b2 = r1 ? T3 : T2; b3 = r1 ? T0 : T3;
            T0 = r2 ? b2 : b0; T1 = r2 ? b3 : b1; T2 = r2 ? b0 : b2; T3 = r2 ? b1 : b3;
        }
    }
    Work fin = w0;
    fin.eyes = eyes; fin.ntricks = ntr; fin.re_players = (uint8_t)re_players;
    score(fin, pts);
    return plies;
}

DK_HD int rollout(Work w, Rng& rng, int pts[4]) {
    int plies = 0;
    while (w.phase == PH_RESERVATION) {
        const uint64_t a = legal_actions(w);
        play_action(w, ctz64(random_single(a, rng)));
        plies++;
    }
    if (w.phase == PH_FINISHED) { score(w, pts); return plies; }
    return plies + rollout_cards(w, rng, pts);
}

// node-state record of the search pools: 64 B (hands as 48-bit masks), lossless
struct alignas(16) Node { uint32_t w[16]; };
DK_HD Node pack_node(const Work& x) {
    Node n;
    n.w[0] = (uint32_t)x.h[0];
    n.w[1] = (uint32_t)(x.h[0] >> 32) | (uint32_t)x.h[1] << 16;
    n.w[2] = (uint32_t)(x.h[1] >> 16);
    n.w[3] = (uint32_t)x.h[2];
    n.w[4] = (uint32_t)(x.h[2] >> 32) | (uint32_t)x.h[3] << 16;
    n.w[5] = (uint32_t)(x.h[3] >> 16);
    n.w[6] = x.trick_cards; n.w[7] = x.trick_winners; n.w[8] = x.eyes; n.w[9] = x.ntricks; n.w[10] = x.res;
    n.w[11] = (uint32_t)x.trick_len | (uint32_t)x.trick_start << 8 | (uint32_t)x.trick_index << 16 | (uint32_t)x.card_index << 24;
    n.w[12] = (uint32_t)x.phase | (uint32_t)x.cur << 8 | (uint32_t)x.res_len << 16 | (uint32_t)x.res_start << 24;
    n.w[13] = (uint32_t)x.rr_wedding | (uint32_t)x.team_kind << 8 | (uint32_t)x.wedding_player << 16 | (uint32_t)x.solved_trick << 24;
    n.w[14] = (uint32_t)x.re_players;
    n.w[15] = 0;
    return n;
}
DK_HD Work unpack_node(const Node& n) {
    Work x;
    const uint64_t M48 = 0xFFFFFFFFFFFFULL;
    x.h[0] = ((uint64_t)n.w[0] | (uint64_t)n.w[1] << 32) & M48;
    x.h[1] = (uint64_t)(n.w[1] >> 16) | (uint64_t)n.w[2] << 16;
    x.h[2] = ((uint64_t)n.w[3] | (uint64_t)n.w[4] << 32) & M48;
    x.h[3] = (uint64_t)(n.w[4] >> 16) | (uint64_t)n.w[5] << 16;
    x.trick_cards = n.w[6]; x.trick_winners = n.w[7]; x.eyes = n.w[8]; x.ntricks = n.w[9]; x.res = n.w[10];
    x.trick_len = (uint8_t)n.w[11]; x.trick_start = (uint8_t)(n.w[11] >> 8); x.trick_index = (uint8_t)(n.w[11] >> 16);
    x.card_index = (uint8_t)(n.w[11] >> 24);
    x.phase = (uint8_t)n.w[12]; x.cur = (uint8_t)(n.w[12] >> 8); x.res_len = (uint8_t)(n.w[12] >> 16); x.res_start = (uint8_t)(n.w[12] >> 24);
    x.rr_wedding = (uint8_t)n.w[13]; x.team_kind = (uint8_t)(n.w[13] >> 8); x.wedding_player = (uint8_t)(n.w[13] >> 16);
    x.solved_trick = (uint8_t)(n.w[13] >> 24);
    x.re_players = (uint8_t)n.w[14]; x.pad0 = 0; x.pad1 = 0; x.pad2 = 0;
    return x;
}
// the record holds this state exactly (the search checks every root, as for rs-full-doko):
// everything but the hands is stored whole, the hands as 48-bit masks
DK_HD bool node_ok(const Work& x) {
    const Work y = unpack_node(pack_node(x));
    return x.h[0] == y.h[0] && x.h[1] == y.h[1] && x.h[2] == y.h[2] && x.h[3] == y.h[3];
}

DK_HD void unpack(const dk_do_state& s, Work& w) {
    for (int p = 0; p < 4; ++p) w.h[p] = s.hands[p];
    w.eyes = (uint32_t)s.eyes[0] | (uint32_t)s.eyes[1] << 8 | (uint32_t)s.eyes[2] << 16 | (uint32_t)s.eyes[3] << 24;
    w.ntricks = (uint32_t)s.ntricks[0] | (uint32_t)s.ntricks[1] << 8 | (uint32_t)s.ntricks[2] << 16 | (uint32_t)s.ntricks[3] << 24;
    w.trick_winners = s.trick_winners;
    w.res = 0;
    for (int i = 0; i < 4; ++i) if (i < s.res_len) w.res = byte_set(w.res, i, s.res[i]);
    w.res_len = s.res_len; w.res_start = s.res_start; w.card_index = s.card_index; w.phase = s.phase;
    w.cur = s.current_player; w.trick_index = s.trick_index;
    w.rr_wedding = s.rr_kind == 2 ? s.rr_player : (uint8_t)0xFF;
    w.team_kind = s.team_kind; w.wedding_player = s.wedding_player; w.solved_trick = s.solved_trick; w.re_players = s.re_players;
    w.pad0 = w.pad1 = w.pad2 = 0;
    w.trick_cards = 0; w.trick_len = 0;
    const int completed = s.card_index / 4;
    w.trick_start = (uint8_t)(completed == 0 ? s.res_start : (int)((s.trick_winners >> (2 * (completed - 1))) & 3));
    if (s.phase == PH_PLAYCARD) {
        const int in_trick = s.card_index - 4 * completed;
        for (int i = 0; i < in_trick; ++i) w.trick_cards |= (uint32_t)s.cards[4 * completed + i] << (8 * i);
        w.trick_len = (uint8_t)in_trick;
    }
}

DK_HD void pack_fields(const Work& w, dk_do_state& s) {
    for (int p = 0; p < 4; ++p) { s.hands[p] = w.h[p]; s.eyes[p] = (uint8_t)byte_get(w.eyes, p); s.ntricks[p] = (uint8_t)byte_get(w.ntricks, p); }
    s.trick_winners = w.trick_winners;
    for (int i = 0; i < 4; ++i) s.res[i] = i < w.res_len ? (uint8_t)byte_get(w.res, i) : (uint8_t)DK_NONE;
    s.res_start = w.res_start; s.res_len = w.res_len; s.card_index = w.card_index; s.phase = w.phase;
    s.current_player = w.phase == PH_FINISHED ? (uint8_t)DK_NONE : w.cur;
    s.rr_kind = w.res_len < 4 ? (uint8_t)DK_NONE : (w.rr_wedding == 0xFF ? (uint8_t)0 : (uint8_t)2);
    s.rr_player = w.rr_wedding == 0xFF ? 0 : w.rr_wedding;
    s.team_kind = w.team_kind; s.wedding_player = w.wedding_player; s.solved_trick = w.solved_trick; s.re_players = w.re_players;
    s.trick_index = w.trick_index; s.game = DK_GAME_DOKO;
}

DK_HD void step_packed(dk_do_state& s, int a) {
    Work w; unpack(s, w);
    const uint8_t ci = w.card_index;
    play_action(w, a);
    if (a <= 23) s.cards[ci] = (uint8_t)a;
    pack_fields(w, s);
}

DK_HD bool is_terminal(const Work& w) { return w.phase == PH_FINISHED; }
DK_HD int env_current_player(const Work& w) { return w.phase == PH_FINISHED ? 0 : (int)w.cur; }
DK_HD uint64_t env_allowed(const Work& w, bool) { return legal_actions(w); }

}  // namespace dko

// ---------------------------------------------------------------------------
// Tic-tac-toe (rs-doko-mcts/src/example/tic_tac_toe.rs:29-193): X and O as
// 9-bit masks.
namespace ttt {

struct Work { uint32_t x, o; uint8_t finish, last, pad0, pad1; };

DK_HD uint32_t finish_state(uint32_t x, uint32_t o) {
    const uint32_t L[8] = {0x007, 0x038, 0x1C0, 0x049, 0x092, 0x124, 0x111, 0x054};
    for (int i = 0; i < 8; ++i) {
        if ((x & L[i]) == L[i]) return 1;
        if ((o & L[i]) == L[i]) return 2;
    }
    return ((x | o) == 0x1FF) ? 3u : 0u;
}
DK_HD int current_player(const Work& w) { return popc32(w.x) == popc32(w.o) ? 0 : 1; }
DK_HD uint64_t env_allowed(const Work& w, bool) { return w.finish ? 0ULL : (uint64_t)(~(w.x | w.o) & 0x1FFu); }
DK_HD void play_action(Work& w, int a) {
    if (current_player(w) == 0) w.x |= 1u << a; else w.o |= 1u << a;
    w.finish = (uint8_t)finish_state(w.x, w.o);
    w.last = (uint8_t)a;
}
DK_HD void score(const Work& w, int pts[4]) {
    pts[0] = w.finish == 1 ? 1 : (w.finish == 2 ? -1 : 0);
    pts[1] = -pts[0]; pts[2] = 0; pts[3] = 0;
}
// random_state: gen_range(0..empties) over the empty cells in ascending order
DK_HD int rollout(Work w, Rng& rng, int pts[4]) {
    int plies = 0;
    while (w.finish == 0) {
        const uint32_t empt = ~(w.x | w.o) & 0x1FFu;
        const uint32_t n = (uint32_t)popc32(empt);
        const uint32_t r = rng.range_u32(n);
        const uint64_t bit = select_msb_rank((uint64_t)empt, n - 1u - r);  // r-th from the LSB
        const int cell = ctz64(bit);
        if (current_player(w) == 0) w.x |= 1u << cell; else w.o |= 1u << cell;
        w.finish = (uint8_t)finish_state(w.x, w.o);
        plies++;
    }
    score(w, pts);
    return plies;
}
DK_HD void unpack(const dk_ttt_state& s, Work& w) {
    w.x = 0; w.o = 0;
    for (int i = 0; i < 9; ++i) { if (s.board[i] == 1) w.x |= 1u << i; if (s.board[i] == 2) w.o |= 1u << i; }
    w.finish = (uint8_t)finish_state(w.x, w.o); w.last = s.last_action; w.pad0 = w.pad1 = 0;
}
DK_HD void pack_fields(const Work& w, dk_ttt_state& s) {
    for (int i = 0; i < 9; ++i) s.board[i] = (w.x >> i & 1) ? 1 : ((w.o >> i & 1) ? 2 : 0);
    s.finish = w.finish; s.last_action = w.last; s.game = DK_GAME_TTT;
}
DK_HD void step_packed(dk_ttt_state& s, int a) { Work w; unpack(s, w); play_action(w, a); pack_fields(w, s); }
DK_HD bool is_terminal(const Work& w) { return w.finish != 0; }
DK_HD int env_current_player(const Work& w) { return current_player(w); }

}  // namespace ttt
}  // namespace dk
