// The AlphaZero network's input: encode_state_pi
// (rs-doko-networks/src/full_doko/var1/encode_pi.rs:27-214) of a dk_az_state,
// one lane per state.  311 tokens = [object 62][position 62][player 62]
// [subposition 62][team 62][phase 1]:
//   4 reservation entries in round order (position k+1, or 0 / token 36 when
//   not made yet), every played card (position = its index + 5), the four real
//   hands from the current player on (position 53 + relative player,
//   subposition 11 / 12 for the first / second copy), the announcement
//   occurrences (position card_index + 1, subposition = rank among the
//   occurrences at the same card index + 1, team 1 Re / 2 Kontra), padded to
//   ten entries with token 37.
// Token tables: var2/encode_reservation_or_card_or_none.rs:6-117,
// var2/encode_position_or_unknown.rs:6-33, var2/encode_subposition.rs:3-21,
// var2/encode_annoucnement_team.rs:3-14, var1/player.rs:5-28, var1/phase.rs:5-15.
#pragma once
#include "fdo_engine.h"

namespace dk {
namespace enc {

// card token by FdoCard index: HeartTen 1, queens 2-5, jacks 6-9, then
// diamonds, clubs, spades, hearts (A, 10, K, 9); 5 bits per card, one u32 per suit
DK_HD uint32_t card_token(uint32_t c) {
    const uint32_t w = c < 6u ? (13u | 11u << 5 | 9u << 10 | 5u << 15 | 12u << 20 | 10u << 25)
                     : c < 12u ? (24u | 1u << 5 | 8u << 10 | 4u << 15 | 23u << 20 | 22u << 25)
                     : c < 18u ? (17u | 15u << 5 | 6u << 10 | 2u << 15 | 16u << 20 | 14u << 25)
                               : (21u | 19u << 5 | 7u << 10 | 3u << 15 | 20u << 20 | 18u << 25);
    return (w >> (5u * (c % 6u))) & 31u;
}

template <class Out>
DK_HD void encode_state_pi(const dk_az_state& r, Out& out) {
    const dk_fdo_state& s = r.state.fdo;
    const uint32_t cp = s.current_player == DK_NONE ? 0u : (uint32_t)s.current_player;
    uint32_t n = 0;
    auto put = [&](uint32_t obj, uint32_t pos, uint32_t ply, uint32_t sub, uint32_t team) {
        out(n, obj); out(62 + n, pos); out(124 + n, ply); out(186 + n, sub); out(248 + n, team);
        ++n;
    };
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t p = (s.res_start + k) & 3u;
        if (k < s.res_len) put(25u + s.res[k], k + 1u, ((p - cp) & 3u) + 1u, 0u, 0u);
        else put(36u, 0u, 0u, 0u, 0u);
    }
    for (uint32_t i = 0; i < s.card_index; ++i) {
        const uint32_t t = i >> 2;
        const uint32_t start = t == 0 ? (uint32_t)s.res_start : (s.trick_winners >> (2u * (t - 1u))) & 3u;
        const uint32_t p = (start + (i & 3u)) & 3u;
        put(card_token(s.cards[i]), i + 5u, ((p - cp) & 3u) + 1u, 0u, 0u);
    }
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t p = (cp + k) & 3u;
        const uint64_t h = s.hands[p];
        uint64_t b = h;
        while (b) {   // FdoHandIter: ascending bits, first copies (0..23) before second copies
            const uint32_t pos = (uint32_t)ctz64(b);
            b &= b - 1;
            const uint32_t c = pos < 24u ? pos : pos - 24u;
            const bool second = pos >= 24u && ((h >> c) & 1u);
            put(card_token(c), 53u + k, 0u, second ? 12u : 11u, 0u);
        }
    }
    uint32_t sub = 0, last = 0xFFFFFFFFu;
    const uint32_t na = r.ann_n < 10 ? r.ann_n : 10u;
    for (uint32_t k = 0; k < na; ++k) {
        const uint32_t ci = r.ann_card[k], p = r.ann_code[k] >> 4, a = r.ann_code[k] & 15u;
        sub = ci == last ? sub + 1u : 0u;
        last = ci;
        put(38u + a, ci + 1u, ((p - cp) & 3u) + 1u, sub + 1u, ((s.re_players >> p) & 1u) ? 1u : 2u);
    }
    for (uint32_t k = na; k < 10; ++k) put(37u, 0u, 0u, 0u, 0u);
    out(310, (uint32_t)s.phase);
}

}  // namespace enc
}  // namespace dk
