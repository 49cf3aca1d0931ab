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

struct CM {
    int observing;
    uint64_t available;
    uint64_t assign[4], possible[4];
    int slots[4];
    bool must_q[4];

    DK_HD void assign_card(int p, int c) {
        assign[p] = h_add(assign[p], c);
        slots[p] -= 1;
        available = h_remove(available, c);
        possible[p] = h_remove(possible[p], c);
        if (slots[p] == 0) possible[p] = 0;
        for (int o = 0; o < 4; ++o) if (o != p) possible[o] = h_remove_ignore(possible[o], c);
        if (c == fdo::CLUB_QUEEN) must_q[p] = false;
    }
    DK_HD void rule1() {
        uint64_t snap = available;
        while (snap) {
            const int c = occ_card(ctz64(snap));
            snap &= snap - 1;
            int single = -1;
            for (int p = 0; p < 4; ++p) {
                if (p == observing) continue;
                if (h_contains(possible[p], c)) {
                    if (single >= 0) { single = -2; break; }
                    single = p;
                }
            }
            if (single >= 0) assign_card(single, c);
        }
    }
    DK_HD bool rule2() {
        bool changed = false;
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
        for (int p = 0; p < 4; ++p) {
            if (p == observing) continue;
            if (must_q[p] && h_contains(possible[p], fdo::CLUB_QUEEN)) { changed = true; assign_card(p, fdo::CLUB_QUEEN); }
        }
        return changed;
    }
    DK_HD void rule4(Rng& rng) {
        uint64_t snap = available;
        const int idx = choose_unsized(popc64(snap), rng);
        for (int i = 0; i < idx; ++i) snap &= snap - 1;
        const int c = occ_card(ctz64(snap));
        for (int p = 0; p < 4; ++p) {
            if (p != observing && h_contains(possible[p], c)) { assign_card(p, c); return; }
        }
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

// trick start player of trick t from the history
DK_HD int trick_start(const dk_fdo_state& s, int t) {
    return t == 0 ? (int)s.res_start : (int)((s.trick_winners >> (2 * (t - 1))) & 3);
}

// Per-player facts of the card history: club queens played, and the colours a
// player failed to follow (gather_impossible_colors.rs:11-43; bit = FdoColor).
DK_HD void history_facts(const dk_fdo_state& s, int played_q[4], uint32_t impossible[4]) {
    for (int p = 0; p < 4; ++p) { played_q[p] = 0; impossible[p] = 0; }
    const int gt = s.game_type;
    for (int t = 0; t < s.n_tricks; ++t) {
        const int start = trick_start(s, t);
        const int first = 4 * t;
        const int len = s.card_index - first < 4 ? s.card_index - first : 4;
        if (len <= 0) continue;
        const uint32_t tc = gt == DK_NONE ? 0xFF : fdo::card_color(s.cards[first], (uint32_t)gt);
        for (int i = 0; i < len; ++i) {
            const int c = s.cards[first + i];
            const int p = (start + i) & 3;
            if (c == fdo::CLUB_QUEEN) played_q[p] += 1;
            if (gt != DK_NONE && fdo::card_color(c, (uint32_t)gt) != tc) impossible[p] |= 1u << tc;
        }
    }
}

// visible_reservations_logic.rs:7-66 (zero-oriented result in out[4])
DK_HD void visible_reservations(const dk_fdo_state& s, int observing, uint8_t out[4]) {
    enum { V_WEDDING = 0, V_HEALTHY = 1, V_NOTREV = 2, V_NONE = 10 };
    for (int p = 0; p < 4; ++p) out[p] = V_NONE;
    const bool completed = s.res_len == 4;
    bool higher = false;
    for (int i = 0; i < 4; ++i) {
        if (i >= s.res_len) break;
        const int p = (s.res_start + i) & 3;
        const uint32_t r = s.res[i];
        if (r == fdo::R_HEALTHY) out[p] = V_HEALTHY;
        else if (r == fdo::R_WEDDING) out[p] = (completed || p == observing) ? V_WEDDING : V_NOTREV;
        else if (completed && !higher) { out[p] = (uint8_t)(3 + (r - 2)); higher = true; }  // DiamondsSolo=3 ... TrumplessSolo=9
        else out[p] = V_NOTREV;
    }
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
    for (int p = 0; p < 4; ++p) {
        st.slots[p] = p == cur ? 0 : popc64(s.hands[p]);
        st.possible[p] = available;
        st.assign[p] = 0;
        st.must_q[p] = false;
    }
    uint8_t vis[4];
    visible_reservations(s, cur, vis);
    for (int p = 0; p < 4; ++p) {
        if (vis[p] == 0) {  // V_WEDDING
            for (int o = 0; o < 4; ++o) if (o != p) {
                st.possible[o] = h_remove_ignore(st.possible[o], fdo::CLUB_QUEEN);
                st.possible[o] = h_remove_ignore(st.possible[o], fdo::CLUB_QUEEN);
            }
        }
    }
    st.possible[cur] = 0;
    // per-player history facts
    int played_q[4];
    uint32_t impossible[4];
    history_facts(s, played_q, impossible);
    const int gt = s.game_type;
    if (gt != DK_NONE) {
        for (int p = 0; p < 4; ++p) {
            if (p == cur) continue;
            for (int col = 0; col < 5; ++col) {
                if (!((impossible[p] >> col) & 1)) continue;
                const uint64_t m = fdo::color_mask((uint32_t)col, (uint32_t)gt);
                st.possible[p] &= ~(m | (m << 24));
            }
        }
        if (gt == fdo::GT_NORMAL) {
            for (int p = 0; p < 4; ++p) {
                if (!((s.ann_players >> p) & 1)) continue;
                if ((s.re_players >> p) & 1) st.must_q[p] = played_q[p] == 0;
                else {
                    st.possible[p] = h_remove_ignore(st.possible[p], fdo::CLUB_QUEEN);
                    st.possible[p] = h_remove_ignore(st.possible[p], fdo::CLUB_QUEEN);
                }
            }
        }
    }
    for (int p = 0; p < 4; ++p) if (st.slots[p] == 0) st.possible[p] = 0;
    st.execute(rng);
    for (int p = 0; p < 4; ++p) out.hands[p] = p == cur ? s.hands[p] : st.assign[p];
    // hidden reservations (card_matching.rs:409-461), EnumSet order = FdoReservation discriminants
    uint8_t res_of[4];
    for (int p = 0; p < 4; ++p) {
        const uint8_t v = vis[p];
        if (v == 10) { res_of[p] = 0xFF; continue; }
        const bool wedding_ok = h_both(out.hands[p], fdo::CLUB_QUEEN) ||
                                (h_contains(out.hands[p], fdo::CLUB_QUEEN) && played_q[p] == 1) || played_q[p] == 2;
        if (v == 0) res_of[p] = fdo::R_WEDDING;
        else if (v == 1) res_of[p] = fdo::R_HEALTHY;
        else if (v == 2) {
            const int n = wedding_ok ? 8 : 7;
            const int i = (int)rng.range_u32((uint32_t)n);
            // set = [Wedding?] DiamondsSolo HeartsSolo SpadesSolo ClubsSolo QueensSolo JacksSolo TrumplessSolo
            res_of[p] = (uint8_t)(wedding_ok ? (i == 0 ? fdo::R_WEDDING : (fdo::R_DIAMONDS + i - 1)) : (fdo::R_DIAMONDS + i));
        } else {
            res_of[p] = (uint8_t)(v - 3 + 2);  // visible solo -> the same FdoReservation
        }
    }
    uint8_t nl = 0;
    uint8_t nr[4] = {DK_NONE, DK_NONE, DK_NONE, DK_NONE};
    for (int i = 0; i < 4; ++i) {
        const int p = (s.res_start + i) & 3;
        if (res_of[p] != 0xFF) nr[nl++] = res_of[p];
    }
    for (int i = 0; i < 4; ++i) out.res[i] = nr[i];
    out.res_len = nl;
}

}  // namespace cap
}  // namespace dk
