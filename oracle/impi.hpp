// ORACLE — test infrastructure only. Never linked into the product library.
//
// Restatement of the autoregressive (IMPI) determinization of rs-doko-impi:
//   forward_pred_process_with_mask   rs-doko-impi/src/forward.rs:392-661
//   stochastic_next (mask, softmax,  forward.rs:33-121 (apply_mask_inplace, softmax_inplace,
//     normalize, choose_weighted)      normalize_float; IndexedRandom::choose_weighted =
//                                      WeightedIndex<f32> + UniformFloat<f32>, rand 0.9)
//   next_possible_card               rs-doko-impi/src/next_consistent.rs:25-139
//   next_possible_reservation        next_consistent.rs:141-193
//   encode_state_ipi                 rs-doko-networks/src/full_doko/var1/encode_ipi.rs:48-282
//   output classes                   rs-doko-networks/src/full_doko/var1/ipi_output.rs:13-83
//                                    (0..8 = FdoReservation order, 9 + FdoCard for cards)
//   _is_consistent                   rs-full-doko/src/matching/is_consistent.rs:38-305
//   clone_with_different_hands_
//     and_reservations               rs-full-doko/src/state/state.rs:96-118
// The network is a callback (EvaluateNetFn::evaluate: 311 tokens -> 33 logits).
// f32 exp is (float)exp((double)x), which equals glibc expf except in
// double-rounding cases (parity unpinned at that level, as for the AZ softmax).
// The log-file draws (rng.random_bool(log_chance) / (log_chance * 4)) at the end
// are kept: one u64 each.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>

#include "card_matching.hpp"
#include "full_doko.hpp"
#include "rand09.hpp"

namespace oracle {
namespace impi {

using fdo::Hand;
using fdo::State;

static constexpr int IPI_TOKENS = 311;
static constexpr int IPI_OUT = 33;     // ImperfectInformationOutput::COUNT
static constexpr int OUT_CARD0 = 9;    // ipi_output.rs:27: DiamondNine = 9 ... SpadeAce = 32

// NotConsistentReason (is_consistent.rs:26-36)
enum Reason : int {
    HandSizeMismatch = 0, NotInRemainingCards, RemainingCardsLeft, AlreadyDiscardedColor,
    HasClubQueenButSomeoneElseAnnouncedWedding, HasNoClubQueenButAnnouncedRe, HasClubQueenButAnnouncedKontra,
    WrongReservation, WrongReservationClubQ,
};

inline int rel1(int p, int cp) { return ((p - cp + 4) % 4) + 1; }   // encode_player_or_none(Some(p), cp)

// union of the real hands (obs.phi_real_hands), plus_hand order BOTTOM..RIGHT
inline Hand real_union(const State& s) {
    Hand r;
    for (int p = 0; p < 4; ++p) r = r.plus_hand(s.hands[p]);
    return r;
}
// FdoHand::minus_hand (hand.rs:85-100)
inline Hand minus_hand(Hand h, const Hand& o) {
    for (int c = 0; c < 24; ++c) {
        if (o.contains_both(c)) h.remove_both(c);
        else if (o.contains(c)) h.remove(c);
    }
    return h;
}

// next_consistent.rs:25-139
inline Hand next_possible_card(const State& s, const Hand assumed[4], const int assumed_res[4], int for_player) {
    Hand remaining = real_union(s);
    for (int p = 0; p < 4; ++p) remaining = minus_hand(remaining, assumed[p]);
    Hand possible = remaining;
    if (s.game_type >= 0) {
        uint32_t imp[4]; fdo::gather_impossible_colors(s, imp);
        for (int col = 0; col < 5; ++col) if (imp[for_player] >> col & 1) possible.remove_color(col, s.game_type);
    }
    for (int p = 0; p < 4; ++p) {   // FdoPlayerSet::all(): BOTTOM..RIGHT
        if (p == for_player) continue;
        if (assumed_res[p] == fdo::Wedding) { possible.remove_ignore(fdo::ClubQueen); possible.remove_ignore(fdo::ClubQueen); }
    }
    if (s.team_state.has_re() && s.game_type == fdo::Normal) {
        const uint8_t re = s.team_state.re_players;
        int played[4]; fdo::played_club_queens(s, played);
        bool removed[4] = {false, false, false, false};
        for (int k = 0; k < s.announcements.n; ++k) {
            const int ap = s.announcements.list[k].player;
            if ((re >> ap & 1) && ap != for_player && !assumed[ap].contains(fdo::ClubQueen) && !removed[ap]) {
                if (played[ap] == 0) { possible.remove_ignore(fdo::ClubQueen); removed[ap] = true; }
            }
            if (!(re >> ap & 1) && ap == for_player) {
                possible.remove_ignore(fdo::ClubQueen); possible.remove_ignore(fdo::ClubQueen);
            }
        }
    }
    return possible;
}

// next_consistent.rs:141-193: bit r = FdoReservation r allowed
inline uint32_t next_possible_reservation(const State& s, const Hand assumed[4], int for_player) {
    int played[4]; fdo::played_club_queens(s, played);
    const bool wedding = assumed[for_player].contains_both(fdo::ClubQueen) ||
                         (assumed[for_player].contains(fdo::ClubQueen) && played[for_player] == 1) || played[for_player] == 2;
    uint32_t set = 0x1FFu & ~(1u << fdo::Wedding);
    if (wedding) set |= 1u << fdo::Wedding;
    return set;
}

// reservation_to_visible_reservation + encode_reservation_or_card_or_reservation
// (encode_ipi.rs:29-46; var2/encode_reservation_or_card_or_none.rs:48-70)
inline int64_t visible_token(int v) {
    switch (v) {
        case fdo::V_Healthy: return 25;
        case fdo::V_Wedding: return 26;
        case fdo::V_NotRevealed: return 34;
        case fdo::V_NoneYet: return 35;
        default: return 27 + (v - fdo::V_DiamondsSolo);   // DiamondsSolo 27 ... TrumplessSolo 33
    }
}
// var2/encode_reservation_or_card_or_none.rs:72-110
inline int64_t card_token(int c) {
    static const int64_t t[24] = {13, 11, 9, 5, 12, 10, 24, 1, 8, 4, 23, 22, 17, 15, 6, 2, 16, 14, 21, 19, 7, 3, 20, 18};
    return t[c];
}
inline int64_t ann_token(uint32_t a) {   // encode_reservation_or_card_or_pi_announcement
    switch (a) {
        case fdo::ReContra: case fdo::CounterReContra: return 38;
        case fdo::No90: return 39;
        case fdo::No60: return 40;
        case fdo::No30: return 41;
        default: return 42;   // Black
    }
}

// encode_ipi.rs:48-282.  Returns false where the reference panics.
inline bool encode_state_ipi(const State& s, const Hand assumed[4], const int assumed_res[4], int guess, int64_t out[IPI_TOKENS]) {
    const int cp = s.current_player < 0 ? 0 : s.current_player;
    int64_t obj[62], pos[62], ply[62], sub[62], team[62];
    int n = 0;
    auto push = [&](int64_t o, int64_t ps, int64_t pl, int64_t sb, int64_t tm) {
        if (n >= 62) return false;
        obj[n] = o; pos[n] = ps; ply[n] = pl; sub[n] = sb; team[n] = tm; ++n;
        return true;
    };
    int vis[4]; fdo::visible_reservations(s, cp, vis);
    int index = 0;
    for (int k = 0; k < 4; ++k) {   // PlayerOrientedArr::iter_with_player from the round's start player
        const int p = (s.res_start + k) % 4;
        int v = vis[p];
        if (v == fdo::V_NotRevealed && assumed_res[p] >= 0) {
            static const int r2v[9] = {fdo::V_Healthy, fdo::V_Wedding, fdo::V_DiamondsSolo, fdo::V_HeartsSolo, fdo::V_SpadesSolo,
                                       fdo::V_ClubsSolo, fdo::V_QueensSolo, fdo::V_JacksSolo, fdo::V_TrumplessSolo};
            v = r2v[assumed_res[p]];
        }
        push(visible_token(v), index + 1, rel1(p, cp), 0, 0);
        ++index;
    }
    for (int t = 0; t < s.n_tricks; ++t) {
        for (int i = 0; i < s.tricks[t].len; ++i) {
            push(card_token(s.tricks[t].cards[i]), index + 1, rel1(s.tricks[t].player_at(i), cp), 0, 0);
            ++index;
        }
    }
    {   // the current player's real hand (position 53, subposition 11 / 12)
        int cards[48]; const int m = s.hands[cp].iter(cards);
        Hand done;
        for (int i = 0; i < m; ++i) {
            push(card_token(cards[i]), 53, 0, done.contains(cards[i]) ? 12 : 11, 0);
            done.add(cards[i]);
        }
    }
    for (int k = 1; k < 4; ++k) {   // rotate_to(cp): the other players in turn order
        const int p = (cp + k) % 4;
        int cards[48]; const int m = assumed[p].iter(cards);
        Hand done;
        for (int i = 0; i < m; ++i) {
            push(card_token(cards[i]), 52 + rel1(p, cp), 0, done.contains(cards[i]) ? 12 : 11, 0);
            done.add(cards[i]);
        }
        const int diff = s.hands[p].len() - assumed[p].len();
        for (int i = 0; i < diff; ++i) push(0, 52 + rel1(p, cp), 0, 0, 0);
    }
    int subi = 0, last = -1;
    for (int k = 0; k < s.announcements.n; ++k) {
        const fdo::AnnOccurrence& a = s.announcements.list[k];
        if (a.card_index != last) { last = a.card_index; subi = 0; }
        if (!s.team_state.has_re()) return false;   // get_team_for_announcement: panic!("not possible")
        const int64_t tm = (s.team_state.re_players >> a.player & 1) ? 1 : 2;
        if (!push(ann_token(a.announcement), a.card_index + 1, rel1(a.player, cp), subi + 1, tm)) return false;
        ++subi;
    }
    if (s.announcements.n > 10) return false;        // 10 - len underflows
    for (int k = s.announcements.n; k < 10; ++k) push(37, 0, 0, 0, 0);
    if (n != 62) return false;                        // try_into::<[i64; 62]>().unwrap()
    for (int i = 0; i < 62; ++i) {
        out[i] = obj[i]; out[62 + i] = pos[i]; out[124 + i] = ply[i]; out[186 + i] = sub[i]; out[248 + i] = team[i];
    }
    out[310] = rel1(guess, cp);
    return true;
}

// is_consistent.rs:38-305; -1 = consistent
inline int is_consistent_reason(const State& s, const Hand assumed[4], const int assumed_res[4]) {
    const int cp = s.current_player;
    for (int p = 0; p < 4; ++p) if (assumed[p].len() != s.hands[p].len()) return HandSizeMismatch;
    Hand remaining = real_union(s);
    for (int p = 0; p < 4; ++p) {
        int cards[48]; const int m = assumed[p].iter(cards);
        for (int i = 0; i < m; ++i) {
            if (!remaining.contains(cards[i])) return NotInRemainingCards;
            remaining.remove(cards[i]);
        }
    }
    if (remaining.len() != 0) return RemainingCardsLeft;
    if (s.game_type >= 0) {
        uint32_t imp[4]; fdo::gather_impossible_colors(s, imp);
        uint64_t m[5]; fdo::color_masks(s.game_type, m);
        for (int p = 0; p < 4; ++p)
            for (int col = 0; col < 5; ++col)
                if ((imp[p] >> col & 1) && (assumed[p].bits & (m[col] | m[col] << 24))) return AlreadyDiscardedColor;
    }
    int wedding_player = -1;
    for (int p = 0; p < 4; ++p) if (assumed_res[p] == fdo::Wedding) wedding_player = p;   // to_oriented_arr: from BOTTOM
    if (wedding_player >= 0)
        for (int p = 0; p < 4; ++p)
            if (p != wedding_player && assumed[p].contains(fdo::ClubQueen)) return HasClubQueenButSomeoneElseAnnouncedWedding;
    int played[4]; fdo::played_club_queens(s, played);
    if (s.team_state.has_re() && s.game_type == fdo::Normal) {
        const uint8_t re = s.team_state.re_players;
        for (int k = 0; k < s.announcements.n; ++k) {
            const int ap = s.announcements.list[k].player;
            const bool q = assumed[ap].contains(fdo::ClubQueen);
            if (re >> ap & 1) { if (!q && played[ap] == 0) return HasNoClubQueenButAnnouncedRe; }
            else if (q) return HasClubQueenButAnnouncedKontra;
        }
    }
    int qcount[4];
    for (int p = 0; p < 4; ++p)
        qcount[p] = played[p] + (assumed[p].contains_both(fdo::ClubQueen) ? 2 : assumed[p].contains(fdo::ClubQueen) ? 1 : 0);
    int vis[4]; fdo::visible_reservations(s, cp, vis);
    for (int p = 0; p < 4; ++p) {
        const int v = vis[p], r = assumed_res[p];
        if (v != fdo::V_NoneYet && r < 0) return WrongReservation;
        if (v == fdo::V_NoneYet && r >= 0) return WrongReservation;
        if (v == fdo::V_Healthy && r != fdo::Healthy) return WrongReservation;
        if (v == fdo::V_Wedding && r != fdo::Wedding) return WrongReservation;
        if (v >= fdo::V_DiamondsSolo && v <= fdo::V_TrumplessSolo) {
            static const int v2r[11] = {0, 0, 0, fdo::DiamondsSolo, fdo::HeartsSolo, fdo::SpadesSolo, fdo::ClubsSolo,
                                        fdo::QueensSolo, fdo::JacksSolo, fdo::TrumplessSolo, 0};
            if (r != v2r[v]) return WrongReservation;
        }
        if (r == fdo::Wedding && qcount[p] < 2) return WrongReservationClubQ;
    }
    return -1;
}

// forward.rs:33-121: mask, softmax with temperature, normalize, choose_weighted.
// Returns the class index, or -1 where the reference panics (WeightedIndex error).
inline int stochastic_next(float logits[IPI_OUT], const bool mask[IPI_OUT], float temperature, SmallRng& rng) {
    for (int i = 0; i < IPI_OUT; ++i) if (!mask[i]) logits[i] = -3.40282347e+38f;   // f32::MIN
    const float temp = std::fmax(temperature, 1e-6f);
    float mx = -INFINITY;
    for (int i = 0; i < IPI_OUT; ++i) mx = std::fmax(mx, logits[i]);   // fold(NEG_INFINITY, f32::max)
    for (int i = 0; i < IPI_OUT; ++i) logits[i] = (float)std::exp((double)((logits[i] - mx) / temp));
    float sum = 0.0f;
    for (int i = 0; i < IPI_OUT; ++i) sum += logits[i];
    if (std::isfinite(sum) && sum > 0.0f) { for (int i = 0; i < IPI_OUT; ++i) logits[i] /= sum; }
    else { for (int i = 0; i < IPI_OUT; ++i) logits[i] = 1.0f / (float)IPI_OUT; }
    float w[IPI_OUT];
    for (int i = 0; i < IPI_OUT; ++i) {
        const float x = logits[i];
        w[i] = (std::isnan(x) || std::isinf(x) || std::signbit(x)) ? 0.0f : x;   // normalize_float (twice)
        if (w[i] == 0.0f) w[i] = 0.0f;   // -0.0 is "negative": normalize_float maps it to +0.0
    }
    // WeightedIndex::new (rand 0.9 distr/weighted/weighted_index.rs) + sample
    float cum[IPI_OUT]; float total = w[0];
    for (int i = 1; i < IPI_OUT; ++i) { cum[i - 1] = total; total += w[i]; }
    if (!(total > 0.0f)) return -1;   // InsufficientNonZero -> unwrap panic
    const float max_rand = 1.0f - 1.1920929e-07f;
    float scale = total;
    while (scale * max_rand >= total) scale = std::nextafter(scale, 0.0f);
    const uint32_t bits = (rng.next_u32() >> 9) | 0x3F800000u;
    float v12; std::memcpy(&v12, &bits, 4);
    const float chosen = (v12 - 1.0f) * scale + 0.0f;
    int k = 0;
    while (k < IPI_OUT - 1 && cum[k] <= chosen) ++k;
    return k;
}

struct ArResult {
    int status = 0;   // 0 consistent, 1 not consistent, 2 the reference panics
    int reason = -1;
    State state;
    int guesses = 0;  // network evaluations
};

using EvalFn = std::function<void(const int64_t tokens[IPI_TOKENS], float logits[IPI_OUT])>;

// forward.rs:392-661 (forward_pred_process_with_mask)
inline ArResult forward_pred_process_with_mask(const State& s, float temperature, float log_chance, const EvalFn& eval,
                                               SmallRng& rng) {
    ArResult res;
    if (s.current_player < 0) { res.status = 2; return res; }   // obs.current_player.unwrap()
    const int cp = s.current_player;
    int slots[4];
    for (int p = 0; p < 4; ++p) slots[p] = s.hands[p].len();
    Hand hands[4];
    int ares[4] = {-1, -1, -1, -1};
    hands[cp] = s.hands[cp];
    auto real_res = [&](int p) {   // phi_real_reservations.reservations.get(p)
        const int i = (p - s.res_start + 4) % 4;
        return i < s.res_len ? s.res[i] : -1;
    };
    ares[cp] = real_res(cp);
    int64_t tok[IPI_TOKENS];
    float logits[IPI_OUT];
    bool mask[IPI_OUT];
    for (int hci = 0; hci < 12; ++hci) {
        for (int i = 1; i <= 3; ++i) {
            const int p = (cp + i) % 4;
            if (slots[p] == 0) continue;
            if (!encode_state_ipi(s, hands, ares, p, tok)) { res.status = 2; return res; }
            const Hand np = next_possible_card(s, hands, ares, p);
            if (np.len() == 0) { res.status = 1; res.reason = RemainingCardsLeft; return res; }
            for (int k = 0; k < IPI_OUT; ++k) mask[k] = k >= OUT_CARD0 && np.contains(k - OUT_CARD0);
            eval(tok, logits);
            res.guesses++;
            const int k = stochastic_next(logits, mask, temperature, rng);
            if (k < OUT_CARD0) { res.status = 2; return res; }   // panic / to_card().unwrap()
            const int card = k - OUT_CARD0;
            if (hands[p].contains_both(card)) { res.status = 1; res.reason = NotInRemainingCards; return res; }
            hands[p].add(card);
            slots[p] -= 1;
        }
    }
    int vis[4]; fdo::visible_reservations(s, cp, vis);
    for (int i = 1; i <= 3; ++i) {
        const int p = (cp + i) % 4;
        if (vis[p] != fdo::V_NotRevealed) { ares[p] = real_res(p); continue; }
        if (!encode_state_ipi(s, hands, ares, p, tok)) { res.status = 2; return res; }
        const uint32_t set = next_possible_reservation(s, hands, p);
        for (int k = 0; k < IPI_OUT; ++k) mask[k] = k < 9 && (set >> k & 1);
        eval(tok, logits);
        res.guesses++;
        const int k = stochastic_next(logits, mask, temperature, rng);
        if (k < 0 || k >= 9) { res.status = 2; return res; }   // to_reservation().unwrap()
        ares[p] = k;
    }
    const int reason = is_consistent_reason(s, hands, ares);
    if (reason < 0) {
        (void)rng.random_bool((double)log_chance);
        res.status = 0;
        res.state = s;
        for (int p = 0; p < 4; ++p) res.state.hands[p] = hands[p];
        // FdoReservationRound::existing(start, rotate_to(start).all_present())
        int nl = 0, nr[4] = {0, 0, 0, 0};
        for (int k = 0; k < 4; ++k) { const int p = (s.res_start + k) % 4; if (ares[p] >= 0) nr[nl++] = ares[p]; }
        for (int k = 0; k < 4; ++k) res.state.res[k] = nr[k];
        res.state.res_len = nl;
        return res;
    }
    (void)rng.random_bool((double)log_chance * 4.0);
    res.status = 1;
    res.reason = reason;
    return res;
}

// Synthetic network for parity tests: FNV-1a over the 311 tokens, 33 logits in
// [-8, 7.75] from splitmix64 of (hash + class).
inline void hash_eval(const int64_t tok[IPI_TOKENS], float logits[IPI_OUT]) {
    uint64_t h = 0xcbf29ce484222325ULL;
    for (int i = 0; i < IPI_TOKENS; ++i) { h ^= (uint64_t)tok[i]; h *= 0x100000001b3ULL; }
    for (int a = 0; a < IPI_OUT; ++a) {
        uint64_t z = h + (uint64_t)a + 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z ^= z >> 31;
        logits[a] = ((float)(int)(z & 63) - 32.0f) * 0.25f;
    }
}

}  // namespace impi
}  // namespace oracle
