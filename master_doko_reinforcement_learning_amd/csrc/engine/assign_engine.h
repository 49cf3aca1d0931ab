// rs-doko rule-based determinization (sample_assignment_full) on the GPU, one
// lane per sample.  Reference: rs-doko-assignment/src/assignment.rs:12-581,
// observation from rs-doko/src/state/state.rs:336-410.
//
// The reference keeps every player's possible cards as a Vec<DoCard> and
// edits it with find/remove.  Only multiplicities are ever observable (the
// lists are tested with `contains`, compared by `len`, and drained card by
// card), so here each list is a multiset of card kinds held in two 24-bit
// masks: `one` = count >= 1, `two` = count == 2.  One rule step is then a few
// mask operations instead of O(48) list scans:
//
//   allowed_i  = remaining minus the colours i failed to follow and, with an
//                announced wedding, minus the club queens of everyone but the
//                wedding player (assignment.rs:79-287 reduce to exactly this:
//                every removal saturates and the starting count of a card is
//                2 - played - own = its count in `remaining`);
//   rule 1     = lowest kind with exactly one eligible player (:337-371);
//   rule 2     = first player whose open slots equal |allowed| (:373-408);
//   rule 3     = element r of `remaining` in hand_to_vec order, then the j-th
//                eligible player; exact-size `choose` draws only for >= 2
//                candidates (:410-446).
#pragma once
#include "do_engine.h"

namespace dk {
namespace asg {

struct MS { uint32_t one, two; };

DK_HD MS ms_of_hand(uint64_t h) {
    const uint32_t lo = (uint32_t)(h & 0xFFFFFFu), hi = (uint32_t)((h >> 24) & 0xFFFFFFu);
    return MS{lo | hi, lo & hi};
}
// hand_from_vec (rs-doko/src/hand/hand.rs:183-195): first copy low, second high.
DK_HD uint64_t hand_of_ms(MS m) { return (uint64_t)m.one | ((uint64_t)m.two << 24); }
DK_HD int ms_count(MS m) { return popc32(m.one) + popc32(m.two); }
DK_HD MS ms_mask(MS m, uint32_t keep) { return MS{m.one & keep, m.two & keep}; }
// saturating a - b
DK_HD MS ms_sub(MS a, MS b) { return MS{(a.one & ~b.one) | (a.two & b.one & ~b.two), a.two & ~b.one}; }
// a + b (total <= 2 per kind)
DK_HD MS ms_add(MS a, MS b) { return MS{a.one | b.one, a.two | b.two | (a.one & b.one)}; }
// remove one copy of kind bit `k` if present
DK_HD MS ms_remove_one(MS a, uint32_t k) {
    const bool two = (a.two & k) != 0;
    return MS{two ? a.one : (a.one & ~k), a.two & ~k};
}
DK_HD MS ms_add_one(MS a, uint32_t k) {
    const bool has = (a.one & k) != 0;
    return MS{a.one | k, has ? (a.two | k) : a.two};
}
// kind of element `idx` of the multiset listed in ascending kind order, both
// copies adjacent (hand_to_vec, hand.rs:135-181): the largest c with
// |{elements of kinds < c}| <= idx.
DK_HD int ms_kind_at(MS m, uint32_t idx) {
    int c = 0;
#pragma unroll
    for (int step = 16; step >= 1; step >>= 1) {
        const int t = c + step;
        const uint32_t below = t >= 24 ? 0xFFFFFFu : ((1u << t) - 1u);
        const uint32_t cum = (uint32_t)(popc32(m.one & below) + popc32(m.two & below));
        c = (t <= 23 && cum <= idx) ? t : c;
    }
    return c;
}

// distribute_card (:289-318). Its last step (drop `remaining` from the lists of
// players without open slots) is unobservable: every rule skips such players.
// The per-player arrays are indexed only by unrolled compile-time indices.
DK_HD void distribute(int p, uint32_t k, MS hands[4], int len[4], MS allowed[4], MS& rem) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        hands[i] = i == p ? ms_add_one(hands[i], k) : hands[i];
        len[i] -= i == p ? 1 : 0;
        allowed[i] = ms_remove_one(allowed[i], k);
    }
    rem = ms_remove_one(rem, k);
}

// Returns 0 on success, 1 where the reference panics (a card that no player
// with open slots may hold: `choose(..).unwrap()` on an empty list, :430-433).
DK_HD int sample_assignment_full(const dk_do_state& in, Rng& rng, dk_do_state& out) {
    out = in;
    const int obs = in.current_player == DK_NONE ? 0 : (int)in.current_player;   // state.rs:337-339
    const int marriage = (in.team_kind == fdo::TK_WED_UNSOLVED || in.team_kind == fdo::TK_WED_SOLVED)
                             ? (int)in.wedding_player : -1;                          // state.rs:349-353
    const MS own = ms_of_hand(sel4(in.hands, obs));

    // calc_remaining_cards (:13-39) and the colour-void part of :197-243
    MS played = MS{0u, 0u};
    uint32_t zero[4] = {0u, 0u, 0u, 0u};
    const int nc = in.card_index;
    int start = in.res_start;
    for (int t = 0; 4 * t < nc; ++t) {
        if (t > 0) start = (int)((in.trick_winners >> (2 * (t - 1))) & 3u);
        const int c0 = in.cards[4 * t];
        const uint32_t tc = fdo::card_color(c0, fdo::GT_NORMAL);
        const uint32_t void_mask = fdo::color_mask(tc, fdo::GT_NORMAL);
        for (int k = 0; k < 4 && 4 * t + k < nc; ++k) {
            const int c = in.cards[4 * t + k];
            played = ms_add_one(played, 1u << c);
            const uint32_t vm = fdo::card_color(c, fdo::GT_NORMAL) != tc ? void_mask : 0u;
            const int p = (start + k) & 3;
            zero[0] |= p == 0 ? vm : 0u; zero[1] |= p == 1 ? vm : 0u;
            zero[2] |= p == 2 ? vm : 0u; zero[3] |= p == 3 ? vm : 0u;
        }
    }
    MS rem = ms_sub(ms_sub(MS{0xFFFFFFu, 0xFFFFFFu}, played), own);

    MS allowed[4], hands[4];
    int len[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint32_t z = zero[i] | ((marriage >= 0 && i != marriage) ? (1u << 15) : 0u);   // :246-263 club queen
        z = i == obs ? 0xFFFFFFu : z;                                                  // :266-273 empties the observer's list
        allowed[i] = ms_mask(rem, ~z);
        hands[i] = MS{0u, 0u};
        len[i] = popc64(in.hands[i]);
    }

    // :532-577 — every pass assigns at least one card, so 48 passes always drain
    for (int pass = 0; pass < 49; ++pass) {
        // eligible players (open slots) per card kind
        uint32_t e[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) e[i] = len[i] > 0 ? allowed[i].one : 0u;
        uint32_t once = 0u, twice = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) { twice |= once & e[i]; once |= e[i]; }
        const uint32_t single = once & ~twice & rem.one;
        if (single) {                                         // rule 1
            const uint32_t k = single & (0u - single);
            const int p = (e[0] & k) ? 0 : ((e[1] & k) ? 1 : ((e[2] & k) ? 2 : 3));
            distribute(p, k, hands, len, allowed, rem);
            continue;
        }
        int full = -1;                                        // rule 2
#pragma unroll
        for (int i = 3; i >= 0; --i)
            if (len[i] > 0 && len[i] == ms_count(allowed[i])) full = i;
        if (full >= 0) {
            MS a = MS{0u, 0u};
#pragma unroll
            for (int i = 0; i < 4; ++i) a = i == full ? allowed[i] : a;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                hands[i] = i == full ? ms_add(hands[i], a) : hands[i];
                len[i] = i == full ? 0 : len[i];
                allowed[i] = i == full ? MS{0u, 0u} : ms_sub(allowed[i], a);
            }
            rem = ms_sub(rem, a);
            continue;
        }
        const int n = ms_count(rem);                          // rule 3
        if (n == 0) break;
        const uint32_t idx = n >= 2 ? rng.range_u32((uint32_t)n) : 0u;
        const uint32_t k = 1u << ms_kind_at(rem, idx);
        const uint32_t elig = ((e[0] & k) ? 1u : 0u) | ((e[1] & k) ? 2u : 0u) | ((e[2] & k) ? 4u : 0u) |
                              ((e[3] & k) ? 8u : 0u);
        const int m = popc32(elig);
        if (m == 0) return 1;
        uint32_t j = m >= 2 ? rng.range_u32((uint32_t)m) : 0u;
        uint32_t bits = elig;
        for (; j > 0; --j) bits &= bits - 1u;
        distribute(ctz64(bits), k, hands, len, allowed, rem);
    }
    // :579, then hand_from_vec for all four hands (:496-501)
#pragma unroll
    for (int i = 0; i < 4; ++i) out.hands[i] = hand_of_ms(i == obs ? own : hands[i]);
    return 0;
}

}  // namespace asg
}  // namespace dk
