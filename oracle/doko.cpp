// ORACLE — test infrastructure only. Never linked into the product library.
// Restates rs-doko (/root/reference/rs-doko/src); each function cites its source.
#include "doko.hpp"
#include <cstdio>
#include <cstdlib>

namespace oracle {
namespace dko {

static void panic(const char* m) { fprintf(stderr, "oracle(dko) panic: %s\n", m); abort(); }

// hand/hand.rs:28-35
uint64_t hand_add(uint64_t h, int c) {
    const bool has = (h >> c & 1) || (h >> (c + 24) & 1);
    return has ? (h | 1ULL << (c + 24)) : (h | 1ULL << c);
}
// hand/hand.rs:38-46
uint64_t hand_remove(uint64_t h, int c) {
    if (h >> c & 1) return h & ~(1ULL << c);
    if (h >> (c + 24) & 1) return h & ~(1ULL << (c + 24));
    panic("Karte nicht in Hand");
    return h;
}
// card/card_to_color.rs:10-40
int card_color(int c) {
    if (c / 6 == 0 || c == 7 /*HeartTen*/ || c % 6 == 2 || c % 6 == 3) return Trump;
    switch (c / 6) { case 1: return Heart; case 2: return Club; default: return Spade; }
}
static uint32_t eyes(int c) { static const uint32_t e[6] = {0, 10, 2, 3, 4, 11}; return e[c % 6]; }
// card/card_in_trick_logic.rs:17-48
static int trump_rank(int c) {
    switch (c) {
        case 0: return 0; case 4: return 1; case 1: return 2; case 5: return 3;
        case 2: return 4; case 8: return 5; case 20: return 6; case 14: return 7;
        case 3: return 8; case 9: return 9; case 21: return 10; case 15: return 11;
        case 7: return 12;
    }
    panic("not a trump card");
    return 0;
}
// card/card_in_trick_logic.rs:57-106
static bool is_greater(int cur, int prev, int tc) {
    const int cc = card_color(cur), pc = card_color(prev);
    const bool ct = cc == Trump, pt = pc == Trump;
    if (ct && !pt) return true;
    if (!ct && pt) return false;
    if (ct && pt) return trump_rank(prev) < trump_rank(cur);
    const bool a = cc == tc, b = pc == tc;
    if (a && !b) return true;
    if (a && b) return eyes(cur) > eyes(prev);
    return false;
}
// trick/trick_winning_player_logic.rs:11-34
int winning_player_in_trick(const Trick& t) {
    const int tc = card_color(t.cards[0]);
    int wc = t.cards[0], wi = 0;
    for (int i = 0; i < 4; ++i) if (is_greater(t.cards[i], wc, tc)) { wc = t.cards[i]; wi = i; }
    return (wi + t.start) % 4;
}
static bool trick_complete(const Trick& t) { return t.cards[3] >= 0; }
static uint32_t trick_eyes(const Trick& t) { uint32_t e = 0; for (int i = 0; i < 4; ++i) if (t.cards[i] >= 0) e += eyes(t.cards[i]); return e; }

static const uint64_t TRUMP_MASK = 0b001100001100001110111111ULL;  // card_color_masks.rs (test at :33)
static const uint64_t HEART_MASK = 0b000000000000110001000000ULL;
static const uint64_t SPADE_MASK = 0b110011000000000000000000ULL;
static const uint64_t CLUB_MASK = 0b000000110011000000000000ULL;

// action/allowed_actions.rs:131-198
uint64_t calculate_allowed_actions(int phase, int tc, uint64_t hand) {
    switch (phase) {
        case Reservation: {
            uint64_t a = 1ULL << A_Healthy;
            if ((hand >> 15 & 1) && (hand >> 39 & 1)) a |= 1ULL << A_Wedding;
            return a;
        }
        case PlayCard: {
            const uint64_t single = (hand | (hand >> 24)) & 0xFFFFFFULL;
            if (tc < 0) return single;
            const uint64_t m = tc == Trump ? TRUMP_MASK : tc == Heart ? HEART_MASK : tc == Spade ? SPADE_MASK : CLUB_MASK;
            if (single & m) return single & m;
            return single;
        }
        default: return 0;
    }
}

// hand/hand_random.rs:47-63 and state/state.rs:159-168
State from_hands(const uint64_t hands[4], int start) {
    State s; s.res_start = start; s.current_player = start;
    for (int i = 0; i < 4; ++i) s.hands[i] = hands[i];
    return s;
}
State new_game(SmallRng& rng) {
    const int start = (int)rng.random_range_usize(0, 4);
    int cards[48];
    for (int i = 0; i < 24; ++i) { cards[2 * i] = i; cards[2 * i + 1] = i; }
    shuffle(cards, 48, rng);
    uint64_t h[4] = {0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 12; ++j) h[i] = hand_add(h[i], cards[i * 12 + j]);
    return from_hands(h, start);
}

// teams/team_logic.rs:69-143
TeamState resolve_team(const State& s) {
    TeamState t;
    if (s.rr_wedding < 0) {
        t.kind = NoWedding;
        for (int i = 0; i < 4; ++i) if ((s.hands[i] >> 15 & 1) || (s.hands[i] >> 39 & 1)) t.re |= 1 << i;
        return t;
    }
    const int wp = s.rr_wedding;
    int partner = -1, solved = -1, completed = 0;
    for (int i = 0; i < 3; ++i) {
        if (s.tricks[i].present) {
            if (!trick_complete(s.tricks[i])) break;
            completed += 1;
            const int w = winning_player_in_trick(s.tricks[i]);
            if (w != wp) { partner = w; solved = i; break; }
        }
    }
    t.wedding_player = wp;
    if (partner >= 0) { t.kind = WeddingSolved; t.solved = solved; t.re = (uint8_t)((1 << wp) | (1 << partner)); return t; }
    if (completed == 3) { t.kind = WeddingSolved; t.solved = 2; t.re = (uint8_t)(1 << wp); return t; }
    t.kind = WeddingUnsolved;
    return t;
}
static bool team_final(const TeamState& t) { return t.kind == WeddingSolved || t.kind == NoWedding; }

// stats/stats.rs:25-135
Stats calculate_stats(uint8_t re, const uint32_t e[4], const uint32_t nt[4]) {
    Stats s{};
    uint32_t rt = 0, kt = 0, reye = 0, keye = 0;
    for (int p = 0; p < 4; ++p) { if (re >> p & 1) { reye += e[p]; rt += nt[p]; } else { keye += e[p]; kt += nt[p]; } }
    const bool re_wins = reye > keye;
    const bool is_solo = __builtin_popcount(re) == 1;
    const uint32_t we = re_wins ? reye : keye, wt = re_wins ? rt : kt;
    int pts = 0;
    if (we >= 120) pts++;
    if (we >= 150) pts++;
    if (we >= 180) pts++;
    if (we >= 210) pts++;
    if (wt == 12) pts++;
    int rp = re_wins ? pts : -pts, kp = re_wins ? -pts : pts;
    if (is_solo) rp *= 3;
    s.winning_team = re_wins ? 0 : 1; s.re_players = re; s.is_solo = is_solo; s.re_eyes = reye; s.kontra_eyes = keye;
    s.re_points = rp; s.kontra_points = kp;
    for (int p = 0; p < 4; ++p) s.player_points[p] = (re >> p & 1) ? rp : kp;
    return s;
}

// state/state.rs:189-309
void play_action(State& s, int a) {
    if (s.phase == Finished) panic("finished");
    const int cp = s.current_player;
    if (a <= 23) {
        if (!s.has_rr) panic("no reservation result");
        s.hands[cp] = hand_remove(s.hands[cp], a);
        Trick& t = s.tricks[s.trick_index];
        for (int i = 0; i < 4; ++i) if (t.cards[i] < 0) { t.cards[i] = a; break; }
        if (trick_complete(t)) {
            s.trick_index += 1;
            const int w = winning_player_in_trick(t);
            s.eyes[w] += trick_eyes(t);
            s.ntricks[w] += 1;
            if (!team_final(s.team)) s.team = resolve_team(s);
            if (s.trick_index == 12) {
                s.phase = Finished; s.current_player = -1;
                if (!team_final(s.team)) panic("teams unknown");
                s.stats = calculate_stats(s.team.re, s.eyes, s.ntricks); s.has_stats = true;
                return;
            }
            s.tricks[s.trick_index] = Trick(); s.tricks[s.trick_index].start = w; s.tricks[s.trick_index].present = true;
            s.current_player = w;
            return;
        }
        s.current_player = (cp + 1) % 4;
    } else {
        const int r = a == A_Wedding ? Wedding : Healthy;
        for (int i = 0; i < 4; ++i) if (s.res[i] < 0) { s.res[i] = r; break; }
        const int np = (cp + 1) % 4;
        s.current_player = np;
        if (s.res[3] >= 0) {
            s.phase = PlayCard;
            // reservation/reservation_winning_logic.rs:13-36 (last wedding in round order wins)
            int wi = -1;
            for (int i = 0; i < 4; ++i) if (s.res[i] == Wedding) wi = i;
            s.has_rr = true; s.rr_wedding = wi < 0 ? -1 : (wi + s.res_start) % 4;
            s.trick_index = 0;
            s.tricks[0] = Trick(); s.tricks[0].start = np; s.tricks[0].present = true;
            if (!team_final(s.team)) s.team = resolve_team(s);
        }
    }
}

static int cur_trick_color(const State& s) {
    if (s.trick_index >= 12 || !s.tricks[s.trick_index].present) return -1;
    const Trick& t = s.tricks[s.trick_index];
    return t.cards[0] < 0 ? -1 : card_color(t.cards[0]);
}
// state/state.rs:315-334 + allowed_actions.rs:97-104
bool random_action_for_current_player(State& s, SmallRng& rng) {
    if (s.phase == Finished) return true;
    const uint64_t a = calculate_allowed_actions(s.phase, cur_trick_color(s), s.hands[s.current_player]);
    const uint32_t n = (uint32_t)__builtin_popcountll(a);
    const uint32_t idx = rng.random_range_u32(0, n);
    uint64_t r = idx; int bit = -1;
    for (int b = 63; b >= 0; --b) if (a >> b & 1) { if (r == 0) { bit = b; break; } --r; }
    play_action(s, bit);
    return false;
}
// state/state.rs:336-410
uint64_t observation_allowed(const State& s) {
    const int obs = s.current_player < 0 ? 0 : s.current_player;
    return calculate_allowed_actions(s.phase, cur_trick_color(s), s.hands[obs]);
}

// rs-doko-mcts/src/env/envs/env_state_doko.rs:36-97, :150-169
bool Env::rewards_or_none(double out[4]) const {
    if (!doko.has_stats) return false;
    for (int p = 0; p < 4; ++p) out[p] = (doko.stats.re_players >> p & 1) ? doko.stats.re_points : doko.stats.kontra_points;
    return true;
}
void Env::random_rollout(SmallRng& rng, double out[4]) const {
    State r = doko;
    for (;;) if (random_action_for_current_player(r, rng)) break;
    for (int p = 0; p < 4; ++p) out[p] = (r.stats.re_players >> p & 1) ? r.stats.re_points : r.stats.kontra_points;
}

}  // namespace dko
}  // namespace oracle
