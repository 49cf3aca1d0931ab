// CAP determinization (card_matching_full) on the GPU, one lane per sample.
// Reference: rs-full-doko/src/matching/card_matching.rs:30-497 and
// gather_impossible_colors.rs:11-43; visible reservations from
// reservation/visible_reservations_logic.rs:7-66.
//
// Everything the reference reads from the observation is derived from the
// packed state's card history: per-player impossible colours, played club
// queens, announcing players (dk_fdo_state.ann_players).
#pragma once
#include "fdo_engine.h"

namespace dk {
namespace cap {

// FdoHand add/remove semantics on raw bits (hand.rs:215-266)
DK_HD bool h_contains(uint64_t h, int c) { return ((h >> c) & 1) || ((h >> (c + 24)) & 1); }
DK_HD bool h_both(uint64_t h, int c) { return ((h >> c) & 1) && ((h >> (c + 24)) & 1); }
DK_HD uint64_t h_add(uint64_t h, int c) { return ((h >> c) & 1) ? (h | (1ULL << (c + 24))) : (h | (1ULL << c)); }
DK_HD uint64_t h_remove(uint64_t h, int c) {
    if ((h >> (c + 24)) & 1) return h & ~(1ULL << (c + 24));
    return h & ~(1ULL << c);
}
DK_HD uint64_t h_remove_ignore(uint64_t h, int c) { return h_contains(h, c) ? h_remove(h, c) : h; }
DK_HD int occ_card(int pos) { return pos < 24 ? pos : pos - 24; }

// Per-player state as four compile-time-indexed words (every loop over the players is unrolled,
// and the one runtime player index, assign_card's, is applied by selects), so nothing lives in
// scratch memory: a runtime-indexed private array is scratch on the GPU.
struct CM {
    int observing;
    uint64_t available;
    uint64_t assign[4], possible[4];
    int slots[4];
    bool must_q[4];

    DK_HD void assign_card(int p, int c) {
        available = h_remove(available, c);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (q == p) {
                assign[q] = h_add(assign[q], c);
                slots[q] -= 1;
                possible[q] = slots[q] == 0 ? 0 : h_remove(possible[q], c);
                if (c == fdo::CLUB_QUEEN) must_q[q] = false;
            } else {
                possible[q] = h_remove_ignore(possible[q], c);
            }
        }
    }
    DK_HD void rule1() {
        // No available card with exactly one possible taker: nothing to assign (the loop below
        // assigns only such cards, and nothing changes until it does), so skip the scan.
        uint32_t k1 = 0, k2 = 0;   // card kinds possible for >= 1 / >= 2 of the hidden players
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const uint32_t kp = p != observing ? (uint32_t)(possible[p] | (possible[p] >> 24)) & 0xFFFFFFu : 0u;
            k2 |= k1 & kp;
            k1 |= kp;
        }
        if ((k1 & ~k2 & ((uint32_t)(available | (available >> 24)) & 0xFFFFFFu)) == 0u) return;
        uint64_t snap = available;
        while (snap) {
            const int c = occ_card(ctz64(snap));
            snap &= snap - 1;
            int single = -1;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                if (p != observing && single != -2 && h_contains(possible[p], c)) single = single >= 0 ? -2 : p;
            }
            if (single >= 0) assign_card(single, c);
        }
    }
    DK_HD bool rule2() {
        bool changed = false;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (p == observing) continue;
            if (slots[p] > 0 && slots[p] == popc64(possible[p])) {
                changed = true;
                uint64_t snap = possible[p];
                while (snap) { const int c = occ_card(ctz64(snap)); snap &= snap - 1; assign_card(p, c); }
            }
        }
        return changed;
    }
    DK_HD bool rule3() {
        bool changed = false;
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (p == observing) continue;
            if (must_q[p] && h_contains(possible[p], fdo::CLUB_QUEEN)) { changed = true; assign_card(p, fdo::CLUB_QUEEN); }
        }
        return changed;
    }
    DK_HD void rule4(Rng& rng) {
        const uint64_t snap = available;
        const int cnt = popc64(snap);
#ifdef DK_CAP_SOL_NOCOIN
        const int idx = (int)(rng.next_u32() % (uint32_t)cnt);   // (speed-of-light measurement build: no CoinFlipper)
#else
        const int idx = choose_unsized(cnt, rng);
#endif
        // the idx-th available position from the lowest (select by rank, no per-lane loop)
        const int c = occ_card(ctz64(select_msb_rank(snap, (uint32_t)(cnt - 1 - idx))));
        int taker = -1;
#pragma unroll
        for (int p = 0; p < 4; ++p)
            if (taker < 0 && p != observing && h_contains(possible[p], c)) taker = p;
        if (taker >= 0) assign_card(taker, c);
    }
    DK_HD void execute(Rng& rng) {
        for (int guard = 0; guard < 256; ++guard) {
            if (available == 0) break;
            rule1();
            if (rule2()) continue;
            if (rule3()) continue;
            if (available == 0) break;
            rule4(rng);
        }
    }
};

// byte p of a word of four per-player bytes
DK_HD uint32_t byte4(uint32_t w, int p) { return (w >> (8 * p)) & 0xFFu; }
DK_HD uint32_t set_byte4(uint32_t w, int p, uint32_t v) { return (w & ~(0xFFu << (8 * p))) | (v << (8 * p)); }

// trick start player of trick t from the history
DK_HD int trick_start(const dk_fdo_state& s, int t) {
    return t == 0 ? (int)s.res_start : (int)((s.trick_winners >> (2 * (t - 1))) & 3);
}

// Per-player facts of the card history: club queens played, and the colours a
// player failed to follow (gather_impossible_colors.rs:11-43; bit = FdoColor), one byte per
// player (byte4).
DK_HD void history_facts(const dk_fdo_state& s, uint32_t& played_q, uint32_t& impossible) {
    played_q = 0; impossible = 0;
    const int gt = s.game_type;
    for (int t = 0; t < s.n_tricks; ++t) {
        const int start = trick_start(s, t);
        const int first = 4 * t;
        const int len = s.card_index - first < 4 ? s.card_index - first : 4;
        if (len <= 0) continue;
        const uint32_t tc = gt == DK_NONE ? 0xFF : fdo::card_color(s.cards[first], (uint32_t)gt);
        for (int i = 0; i < len; ++i) {
            const int c = s.cards[first + i];
            const uint32_t sh = 8u * (uint32_t)((start + i) & 3);
            if (c == fdo::CLUB_QUEEN) played_q += 1u << sh;
            if (gt != DK_NONE && fdo::card_color(c, (uint32_t)gt) != tc) impossible |= (1u << tc) << sh;
        }
    }
}

// visible_reservations_logic.rs:7-66 (zero-oriented result, one byte per player)
DK_HD uint32_t visible_reservations(const dk_fdo_state& s, int observing) {
    enum { V_WEDDING = 0, V_HEALTHY = 1, V_NOTREV = 2, V_NONE = 10 };
    uint32_t out = 0x0A0A0A0Au;   // V_NONE
    const bool completed = s.res_len == 4;
    bool higher = false;
    for (int i = 0; i < 4; ++i) {
        if (i >= s.res_len) break;
        const int p = (s.res_start + i) & 3;
        const uint32_t r = s.res[i];
        uint32_t v;
        if (r == fdo::R_HEALTHY) v = V_HEALTHY;
        else if (r == fdo::R_WEDDING) v = (completed || p == observing) ? V_WEDDING : V_NOTREV;
        else if (completed && !higher) { v = 3 + (r - 2); higher = true; }  // DiamondsSolo=3 ... TrumplessSolo=9
        else v = V_NOTREV;
        out = set_byte4(out, p, v);
    }
    return out;
}

// card_matching_full (card_matching.rs:241-497).  `out` receives a copy of
// `s` with new hands and (possibly) re-drawn hidden reservations.
DK_HD void card_matching_full(const dk_fdo_state& s, Rng& rng, dk_fdo_state& out) {
    out = s;
    const int cur = s.current_player;
    uint64_t available = 0;
    for (int p = 0; p < 4; ++p) {
        if (p == cur) continue;
        // plus_hand in FdoCard order
        for (int c = 0; c < 24; ++c) {
            if (h_both(s.hands[p], c)) { available = h_add(available, c); available = h_add(available, c); }
            else if (h_contains(s.hands[p], c)) available = h_add(available, c);
        }
    }
    CM st;
    st.observing = cur;
    st.available = available;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        st.slots[p] = p == cur ? 0 : popc64(s.hands[p]);
        st.possible[p] = available;
        st.assign[p] = 0;
        st.must_q[p] = false;
    }
    const uint32_t vis = visible_reservations(s, cur);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        if (byte4(vis, p) == 0) {  // V_WEDDING
#pragma unroll
            for (int o = 0; o < 4; ++o) if (o != p) {
                st.possible[o] = h_remove_ignore(st.possible[o], fdo::CLUB_QUEEN);
                st.possible[o] = h_remove_ignore(st.possible[o], fdo::CLUB_QUEEN);
            }
        }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) if (p == cur) st.possible[p] = 0;
    // per-player history facts
    uint32_t played_q, impossible;
    history_facts(s, played_q, impossible);
    const int gt = s.game_type;
    if (gt != DK_NONE) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            if (p == cur) continue;
            for (int col = 0; col < 5; ++col) {
                if (!((byte4(impossible, p) >> col) & 1)) continue;
                const uint64_t m = fdo::color_mask((uint32_t)col, (uint32_t)gt);
                st.possible[p] &= ~(m | (m << 24));
            }
        }
        if (gt == fdo::GT_NORMAL) {
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                if (!((s.ann_players >> p) & 1)) continue;
                if ((s.re_players >> p) & 1) st.must_q[p] = byte4(played_q, p) == 0;
                else {
                    st.possible[p] = h_remove_ignore(st.possible[p], fdo::CLUB_QUEEN);
                    st.possible[p] = h_remove_ignore(st.possible[p], fdo::CLUB_QUEEN);
                }
            }
        }
    }
#pragma unroll
    for (int p = 0; p < 4; ++p) if (st.slots[p] == 0) st.possible[p] = 0;
    st.execute(rng);
#pragma unroll
    for (int p = 0; p < 4; ++p) out.hands[p] = p == cur ? s.hands[p] : st.assign[p];
    // hidden reservations (card_matching.rs:409-461), EnumSet order = FdoReservation discriminants;
    // one byte per player (0xFF: none)
    uint32_t res_of = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const uint32_t v = byte4(vis, p);
        uint32_t r;
        if (v == 10) {
            r = 0xFF;
        } else {
            const uint32_t q = byte4(played_q, p);
            const bool wedding_ok = h_both(out.hands[p], fdo::CLUB_QUEEN) ||
                                    (h_contains(out.hands[p], fdo::CLUB_QUEEN) && q == 1) || q == 2;
            if (v == 0) r = fdo::R_WEDDING;
            else if (v == 1) r = fdo::R_HEALTHY;
            else if (v == 2) {
                const int n = wedding_ok ? 8 : 7;
                const int i = (int)rng.range_u32((uint32_t)n);
                // set = [Wedding?] DiamondsSolo HeartsSolo SpadesSolo ClubsSolo QueensSolo JacksSolo TrumplessSolo
                r = (uint32_t)(wedding_ok ? (i == 0 ? fdo::R_WEDDING : (fdo::R_DIAMONDS + i - 1)) : (fdo::R_DIAMONDS + i));
            } else {
                r = v - 3 + 2;  // visible solo -> the same FdoReservation
            }
        }
        res_of = set_byte4(res_of, p, r);
    }
    uint32_t nl = 0, nr = 0xFFFFFFFFu;   // DK_NONE bytes
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t r = byte4(res_of, (s.res_start + i) & 3);
        if (r != 0xFF) { nr = set_byte4(nr, (int)nl, r); nl += 1; }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) out.res[i] = (uint8_t)byte4(nr, i);
    out.res_len = (uint8_t)nl;
}

}  // namespace cap
}  // namespace dk
