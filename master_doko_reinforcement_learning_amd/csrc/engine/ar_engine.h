// Autoregressive (IMPI) determinization, batched: one lane per (infostate, sample).
// Reference: forward_pred_process_with_mask (rs-doko-impi/src/forward.rs:392-661)
// with stochastic_next (forward.rs:33-121), next_possible_card / _reservation
// (rs-doko-impi/src/next_consistent.rs:25-193), encode_state_ipi
// (rs-doko-networks/src/full_doko/var1/encode_ipi.rs:48-282), _is_consistent
// (rs-full-doko/src/matching/is_consistent.rs:38-305) and
// clone_with_different_hands_and_reservations (rs-full-doko/src/state/state.rs:96-118).
//
// The reference samples one card per network call, awaiting each call.  Here the
// guesses of all lanes advance in lockstep rounds, each round one batched network
// evaluation between two kernels:
//   prepare: move the lane's cursor to its next guess (a card for the next player
//            with open slots, 12 x 3 steps, then the hidden reservations) and
//            write that guess's 311 tokens and class mask, or finish the lane
//            (consistency check, the log draw);
//   choose : mask, softmax with temperature, weighted draw (the lane's SmallRng).
// The per-card facts the reference recomputes from the observation at every
// call (remaining multiset, impossible colours, played club queens, visible
// reservations) are computed once per lane at begin.
//
// Card multisets (count 0..2 per FdoCard) are two 24-bit masks: `a` = count >= 1,
// `b` = count == 2.
#pragma once
#include "cap_engine.h"
#include "encode_pi.h"

namespace dk {
namespace ar {

enum : uint32_t { OUT = 33, CARD0 = 9, TOKENS = 311 };   // ipi_output.rs:13-53
enum : uint8_t { RUNNING = 0, CONSISTENT = 1, NOT_CONSISTENT = 2, PANIC = 3 };
// NotConsistentReason (is_consistent.rs:26-36)
enum : uint8_t { R_HAND_SIZE = 0, R_NOT_IN_REMAINING, R_REMAINING_LEFT, R_DISCARDED_COLOR, R_CQ_OTHER_WEDDING,
                 R_NO_CQ_RE, R_CQ_KONTRA, R_WRONG_RES, R_WRONG_RES_CQ, R_NONE = 0xFF };
enum : uint8_t { V_WEDDING = 0, V_HEALTHY = 1, V_NOTREV = 2, V_NONE = 10 };   // FdoVisibleReservation
static constexpr uint32_t M24 = 0xFFFFFFu;
static constexpr uint8_t CURSOR_RES = 36, CURSOR_END = 39;

struct alignas(16) Lane {          // 96 B
    uint64_t hands[4];             // assumed hands (hands[cp] = the real one)
    uint64_t rng[4];
    uint64_t mask;                 // classes of the pending guess
    uint32_t rem_a, rem_b;         // multiset of all unplayed cards (union of the real hands)
    uint32_t imp;                  // impossible colours, 5 bits per player
    uint8_t res[4];                // assumed reservations (DK_NONE = None)
    uint8_t slots[4];
    uint8_t vis[4];                // visible reservations for the current player
    uint8_t played_q;              // club queens played, 2 bits per player
    uint8_t cursor;                // 0..35 card steps (hand index * 3 + i - 1), 36..38 reservations, 39 end
    uint8_t guess;                 // player of the pending guess, DK_NONE = none
    uint8_t status, reason, cp;
};

DK_HD void ms_of(uint64_t h, uint32_t& a, uint32_t& b) {
    const uint32_t lo = (uint32_t)h & M24, hi = (uint32_t)(h >> 24) & M24;
    a = lo | hi; b = lo & hi;
}
DK_HD void ms_add(uint32_t& a, uint32_t& b, uint32_t a2, uint32_t b2) { b = b | b2 | (a & a2); a = a | a2; }
DK_HD void ms_sub(uint32_t& a, uint32_t& b, uint32_t a2, uint32_t b2) {   // saturating count difference
    const uint32_t na = (b & ~b2) | (a & ~a2), nb = b & ~a2;
    a = na; b = nb;
}
DK_HD void ms_remove_one(uint32_t& a, uint32_t& b, int c) {
    const uint32_t m = 1u << c;
    if (b & m) b &= ~m; else a &= ~m;
}

DK_HD int real_res(const dk_fdo_state& s, int p) {   // phi_real_reservations.reservations.get(p)
    const int i = (p - (int)s.res_start) & 3;
    return i < (int)s.res_len ? (int)s.res[i] : -1;
}
DK_HD uint32_t imp_of(const Lane& L, int p) { return (L.imp >> (5 * p)) & 31u; }
DK_HD int played_of(const Lane& L, int p) { return (L.played_q >> (2 * p)) & 3; }

// forward.rs:403-453 (set-up) plus the per-lane facts; returns the number of guesses
// (network calls) the lane makes unless it stops early.
DK_HD uint32_t init(const dk_az_state& r, uint64_t seed, Lane& L) {
    const dk_fdo_state& s = r.state.fdo;
    Rng rng = Rng::seed_from_u64(seed);
    L.rng[0] = rng.s0; L.rng[1] = rng.s1; L.rng[2] = rng.s2; L.rng[3] = rng.s3;
    L.mask = 0; L.guess = DK_NONE; L.reason = R_NONE; L.cursor = 0;
    if (s.current_player == DK_NONE) { L.status = PANIC; L.cp = 0; return 0; }   // current_player.unwrap()
    L.status = RUNNING;
    const int cp = s.current_player;
    L.cp = (uint8_t)cp;
    uint32_t ua = 0, ub = 0;
    for (int p = 0; p < 4; ++p) {
        uint32_t a, b; ms_of(s.hands[p], a, b); ms_add(ua, ub, a, b);
        L.hands[p] = p == cp ? s.hands[p] : 0;
        L.slots[p] = (uint8_t)popc64(s.hands[p]);
        L.res[p] = DK_NONE;
    }
    L.rem_a = ua; L.rem_b = ub;
    const int rc = real_res(s, cp);
    L.res[cp] = rc < 0 ? DK_NONE : (uint8_t)rc;
    uint32_t pq, imp;   // one byte per player (cap::byte4)
    cap::history_facts(s, pq, imp);
    L.imp = 0; L.played_q = 0;
    for (int p = 0; p < 4; ++p) {
        L.imp |= cap::byte4(imp, p) << (5 * p);
        L.played_q |= (uint8_t)((cap::byte4(pq, p) & 3) << (2 * p));
    }
    const uint32_t vis = cap::visible_reservations(s, cp);
    for (int p = 0; p < 4; ++p) L.vis[p] = (uint8_t)cap::byte4(vis, p);
    uint32_t n = 0;
    for (int i = 1; i <= 3; ++i) {
        const int p = (cp + i) & 3;
        n += L.slots[p] + (L.vis[p] == V_NOTREV ? 1u : 0u);
    }
    return n;
}

// next_consistent.rs:25-139 -> multiset mask `a` of the possible cards
DK_HD uint32_t next_possible_card(const dk_az_state& r, const Lane& L, int for_player) {
    const dk_fdo_state& s = r.state.fdo;
    uint32_t a = L.rem_a, b = L.rem_b;
    for (int p = 0; p < 4; ++p) { uint32_t ha, hb; ms_of(L.hands[p], ha, hb); ms_sub(a, b, ha, hb); }
    if (s.game_type != DK_NONE) {
        const uint32_t im = imp_of(L, for_player);
        for (uint32_t col = 0; col < 5; ++col)
            if ((im >> col) & 1u) { const uint32_t m = ~fdo::color_mask(col, s.game_type); a &= m; b &= m; }
    }
    const uint32_t CQ = 1u << fdo::CLUB_QUEEN;
    for (int p = 0; p < 4; ++p)
        if (p != for_player && L.res[p] == fdo::R_WEDDING) { a &= ~CQ; b &= ~CQ; }
    if ((s.team_kind == fdo::TK_WED_SOLVED || s.team_kind == fdo::TK_NOWEDDING) && s.game_type == fdo::GT_NORMAL) {
        uint32_t removed = 0;
        const uint32_t na = r.ann_n < 12 ? r.ann_n : 12u;
        for (uint32_t k = 0; k < na; ++k) {
            const int ap = r.ann_code[k] >> 4;
            const bool re = (s.re_players >> ap) & 1u;
            if (re && ap != for_player && !cap::h_contains(L.hands[ap], fdo::CLUB_QUEEN) && !((removed >> ap) & 1u)) {
                if (played_of(L, ap) == 0) { ms_remove_one(a, b, fdo::CLUB_QUEEN); removed |= 1u << ap; }
            }
            if (!re && ap == for_player) { a &= ~CQ; b &= ~CQ; }
        }
    }
    return a;
}

// next_consistent.rs:141-193 -> class mask (bit r = FdoReservation r)
DK_HD uint32_t next_possible_reservation(const Lane& L, int p) {
    const uint64_t h = L.hands[p];
    const int pq = played_of(L, p);
    const bool wedding = cap::h_both(h, fdo::CLUB_QUEEN) || (cap::h_contains(h, fdo::CLUB_QUEEN) && pq == 1) || pq == 2;
    return 0x1FDu | (wedding ? 2u : 0u);
}

// encode_ipi.rs:48-282 into out(i, token).  Returns false where the reference panics.
template <class Out>
DK_HD bool encode_state_ipi(const dk_az_state& r, const Lane& L, int guess, Out& out) {
    const dk_fdo_state& s = r.state.fdo;
    const uint32_t cp = L.cp;
    if (r.ann_n > 10) return false;   // 10 - len underflows / the 62-entry vectors overflow
    uint32_t n = 0;
    auto put = [&](uint32_t obj, uint32_t pos, uint32_t ply, uint32_t sub, uint32_t team) {
        out(n, obj); out(62 + n, pos); out(124 + n, ply); out(186 + n, sub); out(248 + n, team);
        ++n;
    };
    for (uint32_t k = 0; k < 4; ++k) {   // visible reservations from the round's start player
        const uint32_t p = (s.res_start + k) & 3u;
        uint32_t v = L.vis[p];
        const uint32_t ar = L.res[p];
        uint32_t tok;
        if (v == V_NOTREV && ar != DK_NONE) tok = 25u + ar;   // the assumed reservation (Healthy 25 ... TrumplessSolo 33)
        else tok = v == V_HEALTHY ? 25u : v == V_WEDDING ? 26u : v == V_NOTREV ? 34u : v == V_NONE ? 35u : 24u + v;
        put(tok, k + 1u, ((p - cp) & 3u) + 1u, 0u, 0u);
    }
    for (uint32_t i = 0; i < s.card_index; ++i) {
        const uint32_t t = i >> 2;
        const uint32_t start = t == 0 ? (uint32_t)s.res_start : (s.trick_winners >> (2u * (t - 1u))) & 3u;
        const uint32_t p = (start + (i & 3u)) & 3u;
        put(enc::card_token(s.cards[i]), i + 5u, ((p - cp) & 3u) + 1u, 0u, 0u);
    }
    for (uint32_t k = 0; k < 4; ++k) {
        const uint32_t p = (cp + k) & 3u;
        const uint64_t h = L.hands[p];
        uint64_t b = h;
        while (b) {   // FdoHandIter: ascending bits
            const uint32_t pos = (uint32_t)ctz64(b);
            b &= b - 1;
            const uint32_t c = pos < 24u ? pos : pos - 24u;
            const bool second = pos >= 24u && ((h >> c) & 1u);
            put(enc::card_token(c), 53u + k, 0u, second ? 12u : 11u, 0u);
        }
        if (k > 0) {   // cards not guessed yet
            const uint32_t diff = (uint32_t)popc64(s.hands[p]) - (uint32_t)popc64(h);
            for (uint32_t j = 0; j < diff; ++j) put(0u, 53u + k, 0u, 0u, 0u);
        }
    }
    uint32_t sub = 0, last = 0xFFFFFFFFu;
    const bool teams = s.team_kind == fdo::TK_WED_SOLVED || s.team_kind == fdo::TK_NOWEDDING;
    for (uint32_t k = 0; k < r.ann_n; ++k) {
        if (!teams) return false;   // get_team_for_announcement: panic!
        const uint32_t ci = r.ann_card[k], p = r.ann_code[k] >> 4, a = r.ann_code[k] & 15u;
        sub = ci == last ? sub + 1u : 0u;
        last = ci;
        put(38u + (a == 5u ? 0u : a), ci + 1u, ((p - cp) & 3u) + 1u, sub + 1u, ((s.re_players >> p) & 1u) ? 1u : 2u);
    }
    for (uint32_t k = r.ann_n; k < 10; ++k) put(37u, 0u, 0u, 0u, 0u);
    if (n != 62) return false;
    out(310, (((uint32_t)guess - cp) & 3u) + 1u);
    return true;
}

// is_consistent.rs:38-305 -> reason or R_NONE
DK_HD uint8_t consistency(const dk_az_state& r, const Lane& L) {
    const dk_fdo_state& s = r.state.fdo;
    for (int p = 0; p < 4; ++p) if (popc64(L.hands[p]) != popc64(s.hands[p])) return R_HAND_SIZE;
    bool missing = false;
    for (int c = 0; c < 24; ++c) {   // per-card counts: assumed above real -> NotInRemainingCards
        const int real = (int)((L.rem_a >> c) & 1u) + (int)((L.rem_b >> c) & 1u);
        int assumed = 0;
        for (int p = 0; p < 4; ++p) assumed += (int)((L.hands[p] >> c) & 1u) + (int)((L.hands[p] >> (c + 24)) & 1u);
        if (assumed > real) return R_NOT_IN_REMAINING;
        missing |= assumed < real;
    }
    if (missing) return R_REMAINING_LEFT;
    if (s.game_type != DK_NONE) {
        for (int p = 0; p < 4; ++p) {
            const uint32_t im = imp_of(L, p);
            for (uint32_t col = 0; col < 5; ++col) {
                if (!((im >> col) & 1u)) continue;
                const uint64_t m = fdo::color_mask(col, s.game_type);
                if (L.hands[p] & (m | (m << 24))) return R_DISCARDED_COLOR;
            }
        }
    }
    int wedding = -1;
    for (int p = 0; p < 4; ++p) if (L.res[p] == fdo::R_WEDDING) wedding = p;
    if (wedding >= 0)
        for (int p = 0; p < 4; ++p)
            if (p != wedding && cap::h_contains(L.hands[p], fdo::CLUB_QUEEN)) return R_CQ_OTHER_WEDDING;
    if ((s.team_kind == fdo::TK_WED_SOLVED || s.team_kind == fdo::TK_NOWEDDING) && s.game_type == fdo::GT_NORMAL) {
        const uint32_t na = r.ann_n < 12 ? r.ann_n : 12u;
        for (uint32_t k = 0; k < na; ++k) {
            const int ap = r.ann_code[k] >> 4;
            const bool q = cap::h_contains(L.hands[ap], fdo::CLUB_QUEEN);
            if ((s.re_players >> ap) & 1u) { if (!q && played_of(L, ap) == 0) return R_NO_CQ_RE; }
            else if (q) return R_CQ_KONTRA;
        }
    }
    for (int p = 0; p < 4; ++p) {
        const uint32_t v = L.vis[p], a = L.res[p];
        const bool some = a != DK_NONE;
        if (v != V_NONE && !some) return R_WRONG_RES;
        if (v == V_NONE && some) return R_WRONG_RES;
        if (v == V_HEALTHY && a != fdo::R_HEALTHY) return R_WRONG_RES;
        if (v == V_WEDDING && a != fdo::R_WEDDING) return R_WRONG_RES;
        if (v >= 3 && v <= 9 && a != v - 1) return R_WRONG_RES;   // visible solo v <-> FdoReservation v - 1
        if (a == fdo::R_WEDDING) {
            const uint64_t h = L.hands[p];
            const int q = played_of(L, p) + (cap::h_both(h, fdo::CLUB_QUEEN) ? 2 : cap::h_contains(h, fdo::CLUB_QUEEN) ? 1 : 0);
            if (q < 2) return R_WRONG_RES_CQ;
        }
    }
    return R_NONE;
}

// prepare: advance to the lane's next guess and write its tokens, or finish the lane.
template <class Out>
DK_HD void prepare(const dk_az_state& r, Lane& L, float log_chance, Out& out) {
    L.guess = DK_NONE;
    if (L.status != RUNNING) return;
    const int cp = L.cp;
    while (L.cursor < CURSOR_RES) {
        const int p = (cp + 1 + L.cursor % 3) & 3;
        if (L.slots[p] == 0) { ++L.cursor; continue; }
        if (!encode_state_ipi(r, L, p, out)) { L.status = PANIC; return; }
        const uint32_t np = next_possible_card(r, L, p);
        if (np == 0) { L.status = NOT_CONSISTENT; L.reason = R_REMAINING_LEFT; return; }
        L.mask = (uint64_t)np << CARD0;
        L.guess = (uint8_t)p;
        return;
    }
    while (L.cursor < CURSOR_END) {
        const int p = (cp + 1 + (L.cursor - CURSOR_RES)) & 3;
        if (L.vis[p] != V_NOTREV) {
            const int rr = real_res(r.state.fdo, p);
            L.res[p] = rr < 0 ? DK_NONE : (uint8_t)rr;
            ++L.cursor;
            continue;
        }
        if (!encode_state_ipi(r, L, p, out)) { L.status = PANIC; return; }
        L.mask = next_possible_reservation(L, p);
        L.guess = (uint8_t)p;
        return;
    }
    // forward.rs:631-660: consistency, then the log-file draw
    Rng rng; rng.s0 = L.rng[0]; rng.s1 = L.rng[1]; rng.s2 = L.rng[2]; rng.s3 = L.rng[3];
    const uint8_t reason = consistency(r, L);
    (void)rng.random_bool(reason == R_NONE ? (double)log_chance : (double)log_chance * 4.0);
    L.rng[0] = rng.s0; L.rng[1] = rng.s1; L.rng[2] = rng.s2; L.rng[3] = rng.s3;
    L.status = reason == R_NONE ? CONSISTENT : NOT_CONSISTENT;
    L.reason = reason;
}

DK_HD float exp_f32(float x) { return (float)exp((double)x); }

// forward.rs:33-121 for the pending guess: mask, softmax(temperature), normalize,
// choose_weighted (WeightedIndex<f32> + UniformFloat<f32>), then apply the guess.
DK_HD void choose(Lane& L, const float* logits, float temperature) {
    if (L.status != RUNNING || L.guess == DK_NONE) return;
    float w[OUT];
    float mx = -INFINITY;
    for (uint32_t i = 0; i < OUT; ++i) {
        w[i] = ((L.mask >> i) & 1u) ? logits[i] : -3.40282347e+38f;   // f32::MIN
        mx = fmaxf(mx, w[i]);
    }
    const float temp = fmaxf(temperature, 1e-6f);
    float sum = 0.0f;
    for (uint32_t i = 0; i < OUT; ++i) { w[i] = exp_f32((w[i] - mx) / temp); sum += w[i]; }
    if (__builtin_isfinite(sum) && sum > 0.0f) { for (uint32_t i = 0; i < OUT; ++i) w[i] /= sum; }
    else { for (uint32_t i = 0; i < OUT; ++i) w[i] = 1.0f / (float)OUT; }
    for (uint32_t i = 0; i < OUT; ++i) if (__builtin_isnan(w[i]) || __builtin_isinf(w[i]) || __builtin_signbit(w[i])) w[i] = 0.0f;   // normalize_float
    float cum[OUT];
    float total = w[0];
    for (uint32_t i = 1; i < OUT; ++i) { cum[i - 1] = total; total += w[i]; }
    if (!(total > 0.0f)) { L.status = PANIC; return; }   // WeightedIndex error -> unwrap
    Rng rng; rng.s0 = L.rng[0]; rng.s1 = L.rng[1]; rng.s2 = L.rng[2]; rng.s3 = L.rng[3];
    const float max_rand = 1.0f - 1.1920929e-07f;
    float scale = total;
    for (int g = 0; g < 64 && scale * max_rand >= total; ++g) scale = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, scale) - 1u);
    const float v12 = __builtin_bit_cast(float, (rng.next_u32() >> 9) | 0x3F800000u);
    const float chosen = (v12 - 1.0f) * scale + 0.0f;
    uint32_t k = 0;
    while (k + 1 < OUT && cum[k] <= chosen) ++k;
    L.rng[0] = rng.s0; L.rng[1] = rng.s1; L.rng[2] = rng.s2; L.rng[3] = rng.s3;
    const int p = L.guess;
    L.guess = DK_NONE;
    if (L.cursor < CURSOR_RES) {
        if (k < CARD0) { L.status = PANIC; return; }   // to_card().unwrap()
        const int c = (int)k - (int)CARD0;
        if (cap::h_both(L.hands[p], c)) { L.status = NOT_CONSISTENT; L.reason = R_NOT_IN_REMAINING; return; }
        L.hands[p] = cap::h_add(L.hands[p], c);
        L.slots[p] -= 1;
    } else {
        if (k >= CARD0) { L.status = PANIC; return; }  // to_reservation().unwrap()
        L.res[p] = (uint8_t)k;
    }
    ++L.cursor;
}

// the sample (state.rs:96-118): the infostate with the assumed hands and the
// reservation round rebuilt from the assumed reservations present, in round order
DK_HD void output(const dk_az_state& r, const Lane& L, dk_fdo_state& out) {
    out = r.state.fdo;
    if (L.status != CONSISTENT) return;
    for (int p = 0; p < 4; ++p) out.hands[p] = L.hands[p];
    uint8_t nl = 0;
    uint8_t nr[4] = {DK_NONE, DK_NONE, DK_NONE, DK_NONE};
    for (int i = 0; i < 4; ++i) {
        const int p = (r.state.fdo.res_start + i) & 3;
        if (L.res[p] != DK_NONE) nr[nl++] = L.res[p];
    }
    for (int i = 0; i < 4; ++i) out.res[i] = nr[i];
    out.res_len = nl;
}

}  // namespace ar
}  // namespace dk
