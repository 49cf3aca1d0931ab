// ORACLE — test infrastructure only. Never linked into the product library.
// Restatement of rs-doko-assignment/src/assignment.rs (see assignment.hpp).
#include "assignment.hpp"

#include <algorithm>

namespace oracle {
namespace dko {

CardVec hand_to_vec(uint64_t hand) {
    CardVec v;
    for (int c = 0; c < 24; ++c) {
        const bool lo = hand >> c & 1, hi = hand >> (c + 24) & 1;
        if (lo && hi) { v.push_back(c); v.push_back(c); }
        else if (lo || hi) v.push_back(c);
    }
    return v;
}

uint64_t hand_from_vec(const CardVec& cards) {
    uint64_t h = 0;
    for (int c : cards) h = hand_add(h, c);
    return h;
}

// assignment.rs:13-39
uint64_t calc_remaining_cards(const Trick tricks[12], uint64_t observing_hand) {
    uint64_t available = (1ULL << 48) - 1;
    for (int i = 0; i < 12; ++i) {
        if (!tricks[i].present) break;
        for (int j = 0; j < 4; ++j) {
            if (tricks[i].cards[j] < 0) break;
            available = hand_remove(available, tricks[i].cards[j]);
        }
    }
    for (int c : hand_to_vec(observing_hand)) available = hand_remove(available, c);
    return available;
}

// assignment.rs:41-58: every listed card removes up to two copies.
static void remove_all_of(CardVec& v, const CardVec& cards) {
    for (int c : cards)
        for (int k = 0; k < 2; ++k) {
            auto it = std::find(v.begin(), v.end(), c);
            if (it != v.end()) v.erase(it);
        }
}
// assignment.rs:60-77
static void remove_one_of(CardVec& v, int c) {
    auto it = std::find(v.begin(), v.end(), c);
    if (it != v.end()) v.erase(it);
}

// assignment.rs:79-287
void player_allowed_to_have(int marriage, const Trick tricks[12], uint64_t observing_hand, int observing_player,
                            CardVec out[4]) {
    // :95-111 (DiamondJack and DiamondQueen are listed twice, as in the reference)
    static const CardVec trump = {0, 1, 2, 3, 4, 5, 2, 8, 20, 14, 3, 9, 21, 15, 7};
    static const CardVec heart = {6, 10, 11};
    static const CardVec spade = {18, 19, 22, 23};
    static const CardVec club = {12, 13, 16, 17};
    // :133-185 — Diamonds, Hearts, Spades, Clubs; every card twice
    CardVec all_two;
    for (int c = 0; c < 12; ++c) { all_two.push_back(c); all_two.push_back(c); }
    for (int c = 18; c < 24; ++c) { all_two.push_back(c); all_two.push_back(c); }
    for (int c = 12; c < 18; ++c) { all_two.push_back(c); all_two.push_back(c); }

    for (int i = 0; i < 4; ++i) out[i] = all_two;
    out[observing_player] = hand_to_vec(observing_hand);

    // :197-243
    for (int j = 0; j < 12; ++j) {
        const Trick& t = tricks[j];
        if (!t.present || t.cards[0] < 0) break;   // trick_color_in_normal_game == None
        const int tc = card_color(t.cards[0]);
        int p = t.start;
        for (int k = 0; k < 4; ++k) {
            const int c = t.cards[k];
            if (c < 0) break;
            for (int i = 0; i < 4; ++i) remove_one_of(out[i], c);
            if (card_color(c) != tc) {
                const CardVec& rm = tc == Trump ? trump : (tc == Heart ? heart : (tc == Spade ? spade : club));
                remove_all_of(out[p], rm);
            }
            p = (p + 1) % 4;
        }
    }
    // :246-263 — nobody but the wedding player holds a club queen
    if (marriage >= 0)
        for (int i = 0; i < 4; ++i)
            if (i != marriage) remove_all_of(out[i], CardVec{15});
    // :266-273
    const CardVec own = hand_to_vec(observing_hand);
    for (int i = 0; i < 4; ++i)
        for (int c : own) remove_one_of(out[i], c);
}

// assignment.rs:289-318
static void distribute_card(int player, int card, CardVec hands[4], int len[4], CardVec allowed[4], CardVec& remaining) {
    hands[player].push_back(card);
    len[player] -= 1;
    for (int i = 0; i < 4; ++i) remove_one_of(allowed[i], card);
    remove_one_of(remaining, card);
    for (int i = 0; i < 4; ++i)
        if (len[i] == 0) remove_all_of(allowed[i], remaining);
}

// assignment.rs:320-335
static std::vector<int> players_for(int card, const CardVec allowed[4], const int len[4]) {
    std::vector<int> ps;
    for (int i = 0; i < 4; ++i)
        if (std::find(allowed[i].begin(), allowed[i].end(), card) != allowed[i].end() && len[i] > 0) ps.push_back(i);
    return ps;
}

// assignment.rs:337-371
static bool distribute_single_cards(CardVec& remaining, CardVec hands[4], int len[4], CardVec allowed[4]) {
    for (int c : remaining) {
        const auto ps = players_for(c, allowed, len);
        if (ps.size() == 1) {
            distribute_card(ps[0], c, hands, len, allowed, remaining);
            return true;
        }
    }
    return false;
}

// assignment.rs:373-408
static bool distribute_exactly_as_per_hand(CardVec hands[4], int len[4], CardVec allowed[4], CardVec& remaining) {
    for (int i = 0; i < 4; ++i) {
        if (len[i] == 0) continue;
        if ((size_t)len[i] == allowed[i].size()) {
            const CardVec copy = allowed[i];
            for (int c : copy) distribute_card(i, c, hands, len, allowed, remaining);
            return true;
        }
    }
    return false;
}

// assignment.rs:410-446. `iter().choose` and `into_iter().choose` see exact
// size hints: 0 -> None, 1 -> the element without a draw, else random_range(..n).
// Returns 0 = nothing left, 1 = assigned, -1 = no player may hold the card (panic).
static int distribute_single_card_randomly(CardVec& remaining, CardVec hands[4], int len[4], CardVec allowed[4],
                                           SmallRng& rng) {
    const int ci = choose_sized(remaining.size(), rng);
    if (ci < 0) return 0;
    const int card = remaining[(size_t)ci];
    const auto ps = players_for(card, allowed, len);
    const int pi = choose_sized(ps.size(), rng);
    if (pi < 0) return -1;
    distribute_card(ps[(size_t)pi], card, hands, len, allowed, remaining);
    return 1;
}

// assignment.rs:507-580
bool sample_assignment(int marriage, const Trick tricks[12], uint64_t observing_hand, const int lengths[4],
                       int observing_player, SmallRng& rng, CardVec out[4]) {
    CardVec remaining = hand_to_vec(calc_remaining_cards(tricks, observing_hand));
    CardVec hands[4];
    CardVec allowed[4];
    player_allowed_to_have(marriage, tricks, observing_hand, observing_player, allowed);
    int len[4] = {lengths[0], lengths[1], lengths[2], lengths[3]};
    for (;;) {
        if (distribute_single_cards(remaining, hands, len, allowed)) continue;
        if (distribute_exactly_as_per_hand(hands, len, allowed, remaining)) continue;
        const int r = distribute_single_card_randomly(remaining, hands, len, allowed, rng);
        if (r < 0) return false;
        if (r == 0) break;
    }
    hands[observing_player] = hand_to_vec(observing_hand);
    for (int i = 0; i < 4; ++i) out[i] = hands[i];
    return true;
}

bool sample_assignment_full(const State& s, SmallRng& rng, State& out) {
    const int obs = s.current_player < 0 ? 0 : s.current_player;
    const int marriage = (s.team.kind == WeddingUnsolved || s.team.kind == WeddingSolved) ? s.team.wedding_player : -1;
    int lengths[4];
    for (int i = 0; i < 4; ++i) lengths[i] = __builtin_popcountll(s.hands[i]);
    CardVec hv[4];
    if (!sample_assignment(marriage, s.tricks, s.hands[obs], lengths, obs, rng, hv)) return false;
    out = s;
    for (int i = 0; i < 4; ++i) out.hands[i] = hand_from_vec(hv[i]);
    return true;
}

}  // namespace dko
}  // namespace oracle
