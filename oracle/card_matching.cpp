// ORACLE — test infrastructure only. Never linked into the product library.
//
// CAP determinization: restates rs-full-doko/src/matching/card_matching.rs
// (CardMatchingState :30-238, card_matching :241-467, card_matching_full
// :469-497) and gather_impossible_colors.rs:11-43, plus the consistency
// checker used by the reference's property test (card_matching.rs:548-643:
// every sample must be consistent with the observation).
// Rule 4 draws through IteratorRandom::choose on FdoHandIter, which has no size
// hint -> the CoinFlipper path of rand 0.9 (parity UNPINNED: no reference fixture).
#include "card_matching.hpp"
#include <cstdio>
#include <cstdlib>

namespace oracle {
namespace fdo {

struct CMState {
    int observing;
    Hand available;
    bool must_q[4];
    int slots[4];
    Hand assign[4];
    Hand possible[4];

    // card_matching.rs:47-76
    void assign_card(int p, int c) {
        assign[p].add(c);
        slots[p] -= 1;
        available.remove(c);
        possible[p].remove(c);
        if (slots[p] == 0) possible[p] = Hand();
        for (int o = 0; o < 4; ++o) if (o != p) possible[o].remove_ignore(c);
        if (c == ClubQueen) must_q[p] = false;
    }
    // :78-112
    void rule1() {
        int cards[48]; const int n = available.iter(cards);   // iterator over a snapshot of the bits
        for (int i = 0; i < n; ++i) {
            const int c = cards[i];
            int single = -1; bool many = false;
            for (int p = 0; p < 4; ++p) {
                if (p == observing) continue;
                if (possible[p].contains(c)) {
                    if (single >= 0) { single = -1; many = true; break; }
                    single = p;
                }
            }
            (void)many;
            if (single >= 0) assign_card(single, c);
        }
    }
    // :114-140
    bool rule2() {
        bool changed = false;
        for (int p = 0; p < 4; ++p) {
            if (p == observing) continue;
            if (slots[p] > 0 && slots[p] == possible[p].len()) {
                changed = true;
                int cards[48]; const int n = possible[p].iter(cards);
                for (int i = 0; i < n; ++i) assign_card(p, cards[i]);
            }
        }
        return changed;
    }
    // :142-166
    bool rule3() {
        bool changed = false;
        for (int p = 0; p < 4; ++p) {
            if (p == observing) continue;
            if (must_q[p] && possible[p].contains(ClubQueen)) { changed = true; assign_card(p, ClubQueen); }
        }
        return changed;
    }
    // :168-196
    void rule4(SmallRng& rng) {
        int cards[48]; const int n = available.iter(cards);
        const int idx = choose_unsized((size_t)n, rng);
        if (idx < 0) { fprintf(stderr, "oracle panic: rule4 empty\n"); abort(); }
        const int chosen = cards[idx];
        int player = -1;
        for (int p = 0; p < 4; ++p) if (p != observing && possible[p].contains(chosen)) { player = p; break; }
        if (player < 0) { fprintf(stderr, "oracle panic: rule4 no player\n"); abort(); }
        if (possible[player].contains(chosen)) assign_card(player, chosen);
    }
    // :198-237
    void execute(SmallRng& rng) {
        for (;;) {
            if (available.len() == 0) break;
            rule1();
            if (rule2()) continue;
            if (rule3()) continue;
            if (available.len() == 0) break;
            rule4(rng);
        }
    }
};

// gather_impossible_colors.rs:11-43 (bit i of out[p] = color i impossible)
void gather_impossible_colors(const State& s, uint32_t out[4]) {
    for (int p = 0; p < 4; ++p) out[p] = 0;
    if (s.game_type < 0) return;
    for (int t = 0; t < s.n_tricks; ++t) {
        const Trick& tr = s.tricks[t];
        const int tc = trick_color(tr, s.game_type);
        if (tc < 0) continue;
        for (int i = 0; i < tr.len; ++i) {
            if (card_to_color(tr.cards[i], s.game_type) != tc) out[tr.player_at(i)] |= 1u << tc;
        }
    }
}

void played_club_queens(const State& s, int out[4]) {
    for (int p = 0; p < 4; ++p) out[p] = 0;
    for (int t = 0; t < s.n_tricks; ++t)
        for (int i = 0; i < s.tricks[t].len; ++i) if (s.tricks[t].cards[i] == ClubQueen) out[s.tricks[t].player_at(i)]++;
}

// card_matching.rs:241-467
void card_matching(const State& s, SmallRng& rng, Hand out_hands[4], int out_res[4]) {
    if (s.current_player < 0) { fprintf(stderr, "oracle panic: card matching on finished game\n"); abort(); }
    const int cur = s.current_player;
    Hand available;
    for (int p = 0; p < 4; ++p) if (p != cur) available = available.plus_hand(s.hands[p]);
    int slots[4];
    for (int p = 0; p < 4; ++p) slots[p] = s.hands[p].len();
    slots[cur] = 0;
    Hand possible[4] = {available, available, available, available};
    int vis[4]; visible_reservations(s, cur, vis);
    // iter_with_player over the visible reservations (starting at the round's start player)
    for (int i = 0; i < 4; ++i) {
        const int p = (s.res_start + i) % 4;
        if (vis[p] == V_Wedding) {
            for (int o = 0; o < 4; ++o) if (o != p) { possible[o].remove_ignore(ClubQueen); possible[o].remove_ignore(ClubQueen); }
        }
    }
    possible[cur] = Hand();
    int played_q[4]; played_club_queens(s, played_q);
    bool must_q[4] = {false, false, false, false};
    if (s.game_type >= 0) {
        uint32_t imp[4]; gather_impossible_colors(s, imp);
        for (int p = 0; p < 4; ++p) {
            if (p == cur) continue;
            // EnumSet iteration order = FdoColor discriminant order
            for (int col = 0; col < 5; ++col) if (imp[p] >> col & 1) possible[p].remove_color(col, s.game_type);
        }
        if (s.game_type == Normal) {
            if (!s.team_state.has_re()) { fprintf(stderr, "oracle panic: normal game without re players\n"); abort(); }
            const uint8_t re = s.team_state.re_players;
            for (int k = 0; k < s.announcements.n; ++k) {
                const int ap = s.announcements.list[k].player;
                if (re >> ap & 1) must_q[ap] = played_q[ap] > 0 ? false : true;
                else { possible[ap].remove_ignore(ClubQueen); possible[ap].remove_ignore(ClubQueen); }
            }
        }
    }
    for (int p = 0; p < 4; ++p) if (slots[p] == 0) possible[p] = Hand();
    CMState st;
    st.observing = cur; st.available = available;
    for (int p = 0; p < 4; ++p) { st.must_q[p] = must_q[p]; st.slots[p] = slots[p]; st.assign[p] = Hand(); st.possible[p] = possible[p]; }
    st.execute(rng);
    for (int p = 0; p < 4; ++p) out_hands[p] = st.assign[p];
    out_hands[cur] = s.hands[cur];
    // reservations (:409-461): EnumSet<FdoReservation> iterates in discriminant order
    for (int p = 0; p < 4; ++p) {
        const int v = vis[p];
        if (v == V_NoneYet) { out_res[p] = -1; continue; }
        int set[9]; int n = 0;
        const bool wedding_ok = out_hands[p].contains_both(ClubQueen) ||
                                (out_hands[p].contains(ClubQueen) && played_q[p] == 1) || played_q[p] == 2;
        if (wedding_ok) set[n++] = Wedding;
        set[n++] = DiamondsSolo; set[n++] = HeartsSolo; set[n++] = SpadesSolo; set[n++] = ClubsSolo;
        set[n++] = QueensSolo; set[n++] = JacksSolo; set[n++] = TrumplessSolo;
        switch (v) {
            case V_Wedding: out_res[p] = Wedding; break;
            case V_Healthy: out_res[p] = Healthy; break;
            case V_NotRevealed: { const int i = choose_sized((size_t)n, rng); out_res[p] = set[i]; break; }
            case V_DiamondsSolo: out_res[p] = DiamondsSolo; break;
            case V_HeartsSolo: out_res[p] = HeartsSolo; break;
            case V_SpadesSolo: out_res[p] = SpadesSolo; break;
            case V_ClubsSolo: out_res[p] = ClubsSolo; break;
            case V_QueensSolo: out_res[p] = QueensSolo; break;
            case V_JacksSolo: out_res[p] = JacksSolo; break;
            case V_TrumplessSolo: out_res[p] = TrumplessSolo; break;
            default: fprintf(stderr, "oracle panic: unknown reservation\n"); abort();
        }
    }
}

// card_matching.rs:469-497
State card_matching_full(const State& s, SmallRng& rng) {
    Hand hands[4]; int res[4];
    card_matching(s, rng, hands, res);
    State n = s;
    for (int p = 0; p < 4; ++p) n.hands[p] = hands[p];
    // FdoReservationRound::existing(start, rotate_to(start).all_present())
    n.res_len = 0;
    for (int i = 0; i < 4; ++i) {
        const int p = (s.res_start + i) % 4;
        if (res[p] >= 0) n.res[n.res_len++] = res[p];
    }
    return n;
}

// Property used by the reference's card_matching test: the sample keeps the
// observer's hand, every other hand has the same size, the multiset of hidden
// cards is unchanged, no player holds a colour he failed to follow, and the
// re/kontra club-queen constraints of a normal game hold.
bool sample_consistent(const State& orig, const State& sample) {
    const int cur = orig.current_player;
    if (sample.hands[cur].bits != orig.hands[cur].bits) return false;
    int cnt_a[24] = {0}, cnt_b[24] = {0};
    for (int p = 0; p < 4; ++p) {
        if (sample.hands[p].len() != orig.hands[p].len()) return false;
        if (p == cur) continue;
        for (int c = 0; c < 24; ++c) {
            cnt_a[c] += (int)(orig.hands[p].bits >> c & 1) + (int)(orig.hands[p].bits >> (c + 24) & 1);
            cnt_b[c] += (int)(sample.hands[p].bits >> c & 1) + (int)(sample.hands[p].bits >> (c + 24) & 1);
        }
    }
    for (int c = 0; c < 24; ++c) if (cnt_a[c] != cnt_b[c]) return false;
    if (orig.game_type >= 0) {
        uint32_t imp[4]; gather_impossible_colors(orig, imp);
        for (int p = 0; p < 4; ++p) {
            if (p == cur) continue;
            for (int col = 0; col < 5; ++col) {
                if (!(imp[p] >> col & 1)) continue;
                uint64_t m[5]; color_masks(orig.game_type, m);
                if (sample.hands[p].bits & (m[col] | m[col] << 24)) return false;
            }
        }
        if (orig.game_type == Normal) {
            int played_q[4]; played_club_queens(orig, played_q);
            const uint8_t re = orig.team_state.re_players;
            for (int k = 0; k < orig.announcements.n; ++k) {
                const int ap = orig.announcements.list[k].player;
                if (ap == cur) continue;
                const bool holds = sample.hands[ap].contains(ClubQueen);
                if ((re >> ap & 1) && played_q[ap] == 0 && !holds) return false;
                if (!(re >> ap & 1) && holds) return false;
            }
        }
    }
    return true;
}

}  // namespace fdo
}  // namespace oracle
