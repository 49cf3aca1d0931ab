// ORACLE — test infrastructure only. Never linked into the product library.
//
// Restatement of the perfect-information state encoder of the AlphaZero
// network, encode_state_pi (rs-doko-networks/src/full_doko/var1/encode_pi.rs:27-214),
// with its token helpers:
//   encode_position_or_unknown_{hand,int}        var2/encode_position_or_unknown.rs:6-33
//   encode_reservation_or_card_or_pi_{announcement,reservation}, _none_card
//                                                var2/encode_reservation_or_card_or_none.rs:6-117
//   encode_subposition_{card,pos}                var2/encode_subposition.rs:3-21
//   encode_announcement_team                     var2/encode_annoucnement_team.rs:3-14
//   encode_player_or_none                        var1/player.rs:5-28
//   encode_phase                                 var1/phase.rs:5-15
// Output: 311 tokens = [object 62][position 62][player 62][subposition 62][team 62][phase 1].
#pragma once
#include <cstdint>

#include "full_doko.hpp"

namespace oracle {
namespace enc {

inline int64_t rel_player(int p, int to) { return (int64_t)(((p - to) % 4 + 4) % 4); }
inline int64_t position_hand(int player, int to) { return player < 0 ? 0 : rel_player(player, to) + 1 + 52; }
inline int64_t position_int(int pos) { return (int64_t)pos + 1; }   // asserts pos < 52
inline int64_t player_or_none(int player, int to) { return player < 0 ? 0 : rel_player(player, to) + 1; }
inline int64_t subposition_card(int sub) { return sub < 0 ? 0 : (sub == 0 ? 11 : 12); }
inline int64_t subposition_pos(int pos) { return pos < 0 ? 0 : (int64_t)pos + 1; }
inline int64_t team(int t) { return t < 0 ? 0 : (t == 0 ? 1 : 2); }   // 0 Re, 1 Kontra
inline int64_t pi_reservation(int r) { return r < 0 ? 36 : 25 + (int64_t)r; }   // FdoReservation order
inline int64_t pi_announcement(int a_bit) {
    switch (a_bit) {
        case -1: return 37;
        case fdo::ReContra: case fdo::CounterReContra: return 38;
        case fdo::No90: return 39;
        case fdo::No60: return 40;
        case fdo::No30: return 41;
        default: return 42;   // Black
    }
}
inline int64_t card_token(int c) {
    // HeartTen, the queens, the jacks, then diamonds, clubs, spades, hearts (A, 10, K, 9)
    static const int64_t t[24] = {13, 11, 9, 5, 12, 10,     // Diamond 9 10 J Q K A
                                  24, 1, 8, 4, 23, 22,      // Heart   9 10 J Q K A
                                  17, 15, 6, 2, 16, 14,     // Club
                                  21, 19, 7, 3, 20, 18};    // Spade
    return c < 0 ? 0 : t[c];
}

inline void encode_state_pi(const fdo::State& s, int64_t out[311]) {
    const int cp = s.current_player < 0 ? 0 : s.current_player;
    int64_t obj[62], pos[62], ply[62], sub[62], tm[62];
    int n = 0, card_index = 0;
    auto push = [&](int64_t p, int64_t o, int64_t pl, int64_t su, int64_t t) {   // position first, as at the call sites
        obj[n] = o; pos[n] = p; ply[n] = pl; sub[n] = su; tm[n] = t; ++n;
    };
    // reservations in round order (to_array_remaining_option().iter_with_player())
    for (int k = 0; k < 4; ++k) {
        const int player = (s.res_start + k) % 4;
        if (k >= s.res_len) push(position_hand(-1, cp), pi_reservation(-1), player_or_none(-1, cp), subposition_pos(-1), team(-1));
        else push(position_int(card_index), pi_reservation(s.res[k]), player_or_none(player, cp), subposition_pos(-1), team(-1));
        card_index += 1;
    }
    // played cards, trick by trick
    for (int t = 0; t < s.n_tricks; ++t)
        for (int i = 0; i < s.tricks[t].len; ++i) {
            push(position_int(card_index), card_token(s.tricks[t].cards[i]), player_or_none(s.tricks[t].player_at(i), cp),
                 subposition_pos(-1), team(-1));
            card_index += 1;
        }
    // real hands, starting with the current player (rotate_to(current_player))
    for (int k = 0; k < 4; ++k) {
        const int player = (cp + k) % 4;
        fdo::Hand seen;
        int cards[48];
        const int m = s.hands[player].iter(cards);
        for (int i = 0; i < m; ++i) {
            push(position_hand(player, cp), card_token(cards[i]), player_or_none(-1, cp),
                 subposition_card(seen.contains(cards[i]) ? 1 : 0), team(-1));
            seen.add(cards[i]);
        }
    }
    // announcements (subposition counts announcements at the same card index)
    int sub_i = 0, last = -1;
    for (int k = 0; k < s.announcements.n; ++k) {
        const fdo::AnnOccurrence& a = s.announcements.list[k];
        if (a.card_index != last) { last = a.card_index; sub_i = 0; }
        const int t = (s.team_state.re_players >> a.player & 1) ? 0 : 1;
        push(position_int(a.card_index), pi_announcement((int)a.announcement), player_or_none(a.player, cp),
             subposition_pos(sub_i), team(t));
        sub_i += 1;
    }
    for (int k = s.announcements.n; k < 10; ++k)
        push(position_hand(-1, cp), pi_announcement(-1), player_or_none(-1, cp), subposition_pos(-1), team(-1));
    for (int i = 0; i < 62; ++i) {
        out[i] = obj[i]; out[62 + i] = pos[i]; out[124 + i] = ply[i]; out[186 + i] = sub[i]; out[248 + i] = tm[i];
    }
    out[310] = (int64_t)s.phase;
}

}  // namespace enc
}  // namespace oracle
