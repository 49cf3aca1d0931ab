// ORACLE — test infrastructure only. Never linked into the product library.
//
// extern "C" surface of the CPU restatement, loaded with ctypes by tests/ and
// by bench.py's cpu_baseline leg.  Handles are heap objects of the restated
// Rust types; pack functions emit the product's dk_state wire format
// (include/doko_amd.h) so parity tests can feed identical inputs to both.
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <atomic>
#include <memory>
#include <vector>

#include "../include/doko_amd.h"
#include "card_matching.hpp"
#include "doko.hpp"
#include "assignment.hpp"
#include "az_eval.hpp"
#include "az_mcts.hpp"
#include "encode_pi.hpp"
#include "impi.hpp"
#include "full_doko.hpp"
#include "fusion.hpp"
#include "mcts.hpp"
#include "ttt.hpp"

using namespace oracle;

static_assert(sizeof(dk_fdo_state) == 128, "dk_fdo_state size");
static_assert(sizeof(dk_do_state) == 128, "dk_do_state size");
static_assert(sizeof(dk_ttt_state) == 128, "dk_ttt_state size");
static_assert(sizeof(dk_az_state) == 160, "dk_az_state size");

static SmallRng rng_from(const uint64_t* s) { SmallRng r; for (int i = 0; i < 4; ++i) r.s[i] = s[i]; return r; }
static void rng_to(const SmallRng& r, uint64_t* s) { if (s) for (int i = 0; i < 4; ++i) s[i] = r.s[i]; }

extern "C" {

void or_rng_seed(uint64_t seed, uint64_t* out) { rng_to(SmallRng::seed_from_u64(seed), out); }
uint64_t or_rng_next_u64(uint64_t* st) { SmallRng r = rng_from(st); uint64_t v = r.next_u64(); rng_to(r, st); return v; }
uint32_t or_rng_range_u32(uint64_t* st, uint32_t lo, uint32_t hi) { SmallRng r = rng_from(st); uint32_t v = r.random_range_u32(lo, hi); rng_to(r, st); return v; }
int or_rng_choose_unsized(uint64_t* st, uint32_t n) { SmallRng r = rng_from(st); int v = choose_unsized(n, r); rng_to(r, st); return v; }
uint64_t or_select_by_rank(uint64_t v, uint64_t r) { return fdo::select_by_rank(v, r); }

// ---------------------------------------------------------------- full doko
void* or_fdo_new_game(uint64_t seed) { SmallRng r = SmallRng::seed_from_u64(seed); return new fdo::State(fdo::new_game(r)); }
void* or_fdo_from_hands(const uint64_t* hands, int start) {
    fdo::Hand h[4]; for (int i = 0; i < 4; ++i) h[i].bits = hands[i];
    return new fdo::State(fdo::new_game_from_hand_and_start_player(h, start));
}
void* or_fdo_clone(void* s) { return new fdo::State(*(fdo::State*)s); }
void or_fdo_free(void* s) { delete (fdo::State*)s; }
void or_fdo_play(void* s, int a) { fdo::play_action(*(fdo::State*)s, a); }
uint64_t or_fdo_allowed(void* s) { return fdo::observation_allowed_actions(*(fdo::State*)s); }
uint64_t or_fdo_env_allowed(void* s, int first) { fdo::Env e; e.doko = *(fdo::State*)s; return e.allowed_actions(first != 0); }
void or_fdo_hands(void* s, uint64_t* out) { for (int i = 0; i < 4; ++i) out[i] = ((fdo::State*)s)->hands[i].bits; }

// info layout: [0] phase [1] current_player [2] game_type [3..6] eyes [7] re_lowest [8] contra_lowest
// [9] has_stats [10..13] player_points [14] re_eyes [15] kontra_eyes [16] re_points [17] kontra_points
// [18] is_solo [19] n_tricks [20..31] trick winners [32] re_players (-1 unknown) [33] card_index
// [34] team_kind [35] ann_turns [36] ann_allowed [37] n_announcements
void or_fdo_info(void* sp, int32_t* o) {
    const fdo::State& s = *(fdo::State*)sp;
    o[0] = s.phase; o[1] = s.current_player; o[2] = s.game_type;
    for (int p = 0; p < 4; ++p) o[3 + p] = (int32_t)s.player_eyes[p];
    o[7] = s.announcements.re_lowest; o[8] = s.announcements.contra_lowest;
    o[9] = s.has_stats;
    for (int p = 0; p < 4; ++p) o[10 + p] = s.has_stats ? s.stats.player_points[p] : 0;
    o[14] = s.has_stats ? (int32_t)s.stats.re_eyes : 0; o[15] = s.has_stats ? (int32_t)s.stats.kontra_eyes : 0;
    o[16] = s.has_stats ? s.stats.re_points : 0; o[17] = s.has_stats ? s.stats.kontra_points : 0;
    o[18] = s.has_stats ? s.stats.is_solo : 0; o[19] = s.n_tricks;
    for (int t = 0; t < 12; ++t) o[20 + t] = t < s.n_tricks ? s.tricks[t].winning_player : -1;
    o[32] = s.team_state.has_re() ? s.team_state.re_players : -1;
    o[33] = s.card_index; o[34] = s.team_state.kind; o[35] = s.announcements.turns_without;
    o[36] = (int32_t)s.announcements.allowed; o[37] = s.announcements.n;
}

// Emit the product's dk_fdo_state wire format.
void or_fdo_pack(void* sp, uint8_t* out) {
    const fdo::State& s = *(fdo::State*)sp;
    dk_fdo_state d; memset(&d, 0, sizeof(d));
    for (int p = 0; p < 4; ++p) d.hands[p] = s.hands[p].bits;
    memset(d.cards, DK_NONE, sizeof(d.cards));
    int ci = 0;
    for (int t = 0; t < s.n_tricks; ++t) for (int i = 0; i < s.tricks[t].len; ++i) d.cards[ci++] = (uint8_t)s.tricks[t].cards[i];
    for (int p = 0; p < 4; ++p) { d.eyes[p] = (uint8_t)s.player_eyes[p]; d.ntricks[p] = (uint8_t)s.player_num_tricks[p]; }
    d.trick_winners = 0;
    for (int t = 0; t < s.n_tricks; ++t) if (s.tricks[t].winning_player >= 0) d.trick_winners |= (uint32_t)s.tricks[t].winning_player << (2 * t);
    memset(d.res, DK_NONE, 4);
    for (int i = 0; i < s.res_len; ++i) d.res[i] = (uint8_t)s.res[i];
    d.res_start = (uint8_t)s.res_start; d.res_len = (uint8_t)s.res_len; d.card_index = (uint8_t)s.card_index;
    d.phase = (uint8_t)s.phase; d.current_player = s.current_player < 0 ? DK_NONE : (uint8_t)s.current_player;
    d.game_type = s.game_type < 0 ? DK_NONE : (uint8_t)s.game_type;
    d.rr_kind = s.has_reservation_result ? (uint8_t)s.reservation_result.kind : DK_NONE;
    d.rr_player = (uint8_t)s.reservation_result.player; d.rr_reservation = (uint8_t)s.reservation_result.reservation;
    d.team_kind = (uint8_t)s.team_state.kind; d.wedding_player = (uint8_t)s.team_state.wedding_player;
    d.solved_trick = (uint8_t)s.team_state.solved_trick_index; d.re_players = s.team_state.re_players;
    d.re_lowest = s.announcements.re_lowest < 0 ? 0 : (uint8_t)s.announcements.re_lowest;
    d.contra_lowest = s.announcements.contra_lowest < 0 ? 0 : (uint8_t)s.announcements.contra_lowest;
    d.ann_turns = (uint8_t)s.announcements.turns_without; d.ann_start = (uint8_t)s.announcements.starting_player;
    d.ann_allowed = (uint8_t)s.announcements.allowed; d.ann_count = (uint8_t)s.announcements.n;
    uint8_t ap = 0; for (int k = 0; k < s.announcements.n; ++k) ap |= (uint8_t)(1 << s.announcements.list[k].player);
    d.ann_players = ap; d.n_tricks = (uint8_t)s.n_tricks; d.game = DK_GAME_FULL_DOKO;
    memcpy(out, &d, sizeof(d));
}

// The reference's FdoState fields as the C-ABI's dk_fdo_fields (the input of dk_fdo_from_fields).
void or_fdo_fields(void* sp, dk_fdo_fields* f) {
    const fdo::State& s = *(fdo::State*)sp;
    memset(f, 0, sizeof(*f));
    for (int p = 0; p < 4; ++p) { f->hands[p] = s.hands[p].bits; f->player_eyes[p] = s.player_eyes[p]; f->player_num_tricks[p] = s.player_num_tricks[p]; }
    f->res_start = (int8_t)s.res_start; f->res_len = (int8_t)s.res_len;
    for (int i = 0; i < 4; ++i) f->reservations[i] = i < s.res_len ? (int8_t)s.res[i] : (int8_t)-1;
    f->n_tricks = (int8_t)s.n_tricks;
    memset(f->trick_start, -1, sizeof(f->trick_start)); memset(f->trick_cards, -1, sizeof(f->trick_cards));
    for (int t = 0; t < s.n_tricks; ++t) {
        f->trick_start[t] = (int8_t)s.tricks[t].start;
        for (int i = 0; i < s.tricks[t].len; ++i) f->trick_cards[t][i] = (int8_t)s.tricks[t].cards[i];
    }
    f->ann_n = (int8_t)s.announcements.n;
    memset(f->ann_card_index, -1, sizeof(f->ann_card_index)); memset(f->ann_player, -1, sizeof(f->ann_player));
    for (int k = 0; k < s.announcements.n; ++k) {
        f->ann_card_index[k] = (int8_t)s.announcements.list[k].card_index; f->ann_player[k] = (int8_t)s.announcements.list[k].player;
        f->ann_announcement[k] = (uint8_t)s.announcements.list[k].announcement;
    }
    f->re_lowest = s.announcements.re_lowest < 0 ? 0 : (uint8_t)s.announcements.re_lowest;
    f->contra_lowest = s.announcements.contra_lowest < 0 ? 0 : (uint8_t)s.announcements.contra_lowest;
    f->ann_turns_without = (int8_t)s.announcements.turns_without; f->ann_start = (int8_t)s.announcements.starting_player;
    f->ann_allowed = (uint8_t)s.announcements.allowed; f->card_index = (int8_t)s.card_index;
    f->current_player = (int8_t)s.current_player; f->phase = (int8_t)s.phase;
    f->rr_kind = s.has_reservation_result ? (int8_t)s.reservation_result.kind : (int8_t)-1;
    f->rr_player = (int8_t)s.reservation_result.player; f->rr_reservation = (int8_t)s.reservation_result.reservation;
    f->game_type = (int8_t)s.game_type;
    f->team_kind = (int8_t)s.team_state.kind; f->wedding_player = (int8_t)s.team_state.wedding_player;
    f->solved_trick = (int8_t)s.team_state.solved_trick_index; f->re_players = s.team_state.re_players;
}

int or_fdo_random_plies(void* sp, uint64_t* rng_state, int k, int no_announcement) {
    fdo::State& s = *(fdo::State*)sp; SmallRng r = rng_from(rng_state);
    int done = 0;
    for (int i = 0; i < k; ++i) {
        const bool fin = no_announcement ? fdo::random_action_for_current_player_no_announcement(s, r)
                                         : fdo::random_action_for_current_player(s, r);
        if (fin) break;
        done++;
    }
    rng_to(r, rng_state);
    return done;
}

void or_fdo_rollout(void* sp, uint64_t* rng_state, double* out) {
    fdo::Env e; e.doko = *(fdo::State*)sp; SmallRng r = rng_from(rng_state);
    e.random_rollout(r, out); rng_to(r, rng_state);
}
int or_fdo_rewards(void* sp, double* out) { fdo::Env e; e.doko = *(fdo::State*)sp; return e.rewards_or_none(out); }

// design data: the branching-pick child counts of one search (see SearchCounters::pick_trace)
int or_fdo_search_trace(void* sp, uint64_t* rng_state, uint32_t iters, double c, uint8_t* out, int cap) {
    fdo::Env e; e.doko = *(fdo::State*)sp; SmallRng r = rng_from(rng_state);
    Mcts<fdo::Env> m; SearchCounters ctr; std::vector<uint8_t> tr; ctr.pick_trace = &tr;
    m.search(e, c, iters, r, &ctr);
    const int n = (int)tr.size() < cap ? (int)tr.size() : cap;
    for (int i = 0; i < n; ++i) out[i] = tr[i];
    return (int)tr.size();
}
int or_fdo_search(void* sp, uint64_t* rng_state, uint32_t iters, double c, uint32_t* visits, double* values, uint64_t* counters) {
    fdo::Env e; e.doko = *(fdo::State*)sp; SmallRng r = rng_from(rng_state);
    Mcts<fdo::Env> m; SearchCounters ctr;
    auto moves = m.search(e, c, iters, r, &ctr);
    rng_to(r, rng_state);
    if (counters) {
        counters[0] = ctr.iterations; counters[1] = ctr.children_scanned; counters[2] = ctr.path_nodes;
        counters[3] = ctr.max_depth; counters[4] = ctr.nodes; counters[5] = ctr.child_slots;
        counters[6] = ctr.max_path_entries;
    }
    return moves_to_arrays(moves, visits, values, DK_NUM_ACTIONS);
}

void* or_fdo_card_matching(void* sp, uint64_t* rng_state) {
    SmallRng r = rng_from(rng_state);
    fdo::State* n = new fdo::State(fdo::card_matching_full(*(fdo::State*)sp, r));
    rng_to(r, rng_state);
    return n;
}
int or_fdo_sample_consistent(void* orig, void* sample) { return fdo::sample_consistent(*(fdo::State*)orig, *(fdo::State*)sample); }
void or_fdo_visible_reservations(void* sp, int obs, int32_t* out) { int v[4]; fdo::visible_reservations(*(fdo::State*)sp, obs, v); for (int i = 0; i < 4; ++i) out[i] = v[i]; }
int or_fdo_calc_allowed_announcements(int player, int n_cards, int team_kind, int solved, int re_players, int re_low, int contra_low) {
    fdo::TeamState t; t.kind = team_kind; t.solved_trick_index = solved; t.re_players = (uint8_t)re_players;
    return (int)fdo::calc_allowed_announcements(player, n_cards, t, re_low, contra_low);
}
int or_fdo_card_to_color(int card, int gt) { return fdo::card_to_color(card, gt); }
int or_fdo_is_greater(int cur, int prev, int tc, int gt) { return fdo::is_greater_in_trick(cur, prev, tc, gt); }

// Root-parallel CPU baseline: `threads` workers, one arena + RNG each, like
// MCTSWorkers (rs-doko-evaluator/src/full_doko/policy/mcts_policy.rs:55-126).
double or_fdo_search_many(const uint8_t* packed_unused, void** roots, const uint64_t* seeds, uint32_t n, uint32_t iters,
                          double c, uint32_t* visits, int threads) {
    (void)packed_unused;
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    auto next = std::make_shared<std::atomic<uint32_t>>(0);   // shared root queue (MCTSWorkers' MPMC channel)
    for (int t = 0; t < threads; ++t) {
        pool.emplace_back([=]() {
            Mcts<fdo::Env> m;
            for (uint32_t i; (i = next->fetch_add(1)) < n;) {
                fdo::Env e; e.doko = *(fdo::State*)roots[i];
                SmallRng r = SmallRng::seed_from_u64(seeds[i]);
                auto moves = m.search(e, c, iters, r, nullptr);
                double vals[DK_NUM_ACTIONS];
                moves_to_arrays(moves, visits + (size_t)i * DK_NUM_ACTIONS, vals, DK_NUM_ACTIONS);
            }
        });
    }
    for (auto& th : pool) th.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// ---------------------------------------------------------------- rs-doko
void* or_do_new_game(uint64_t seed) { SmallRng r = SmallRng::seed_from_u64(seed); return new dko::State(dko::new_game(r)); }
void* or_do_from_hands(const uint64_t* hands, int start) { return new dko::State(dko::from_hands(hands, start)); }
void* or_do_clone(void* s) { return new dko::State(*(dko::State*)s); }
void or_do_free(void* s) { delete (dko::State*)s; }
void or_do_play(void* s, int a) { dko::play_action(*(dko::State*)s, a); }
uint64_t or_do_allowed(void* s) { return dko::observation_allowed(*(dko::State*)s); }
void or_do_hands(void* s, uint64_t* out) { for (int i = 0; i < 4; ++i) out[i] = ((dko::State*)s)->hands[i]; }
// [0] phase [1] current [2..5] eyes [6] has_stats [7..10] points [11] re_eyes [12] kontra_eyes [13] re_points
// [14] kontra_points [15] trick_index [16..27] trick winners (-1) [28] re_players
void or_do_info(void* sp, int32_t* o) {
    const dko::State& s = *(dko::State*)sp;
    o[0] = s.phase; o[1] = s.current_player;
    for (int p = 0; p < 4; ++p) o[2 + p] = (int32_t)s.eyes[p];
    o[6] = s.has_stats;
    double rw[4]; dko::Env e; e.doko = s; const bool has = e.rewards_or_none(rw);
    for (int p = 0; p < 4; ++p) o[7 + p] = has ? (int32_t)rw[p] : 0;
    o[11] = s.has_stats ? (int32_t)s.stats.re_eyes : 0; o[12] = s.has_stats ? (int32_t)s.stats.kontra_eyes : 0;
    o[13] = s.has_stats ? s.stats.re_points : 0; o[14] = s.has_stats ? s.stats.kontra_points : 0;
    o[15] = s.trick_index;
    for (int t = 0; t < 12; ++t) {
        const dko::Trick& tr = s.tricks[t];
        o[16 + t] = (tr.present && tr.cards[3] >= 0) ? dko::winning_player_in_trick(tr) : -1;
    }
    o[28] = (s.team.kind == dko::WeddingSolved || s.team.kind == dko::NoWedding) ? s.team.re : -1;
}
void or_do_pack(void* sp, uint8_t* out) {
    const dko::State& s = *(dko::State*)sp;
    dk_do_state d; memset(&d, 0, sizeof(d));
    for (int p = 0; p < 4; ++p) d.hands[p] = s.hands[p];
    memset(d.cards, DK_NONE, sizeof(d.cards));
    int ci = 0;
    for (int t = 0; t < 12; ++t) {
        if (!s.tricks[t].present) continue;
        for (int i = 0; i < 4; ++i) if (s.tricks[t].cards[i] >= 0) d.cards[ci++] = (uint8_t)s.tricks[t].cards[i];
        if (s.tricks[t].cards[3] >= 0) d.trick_winners |= (uint32_t)dko::winning_player_in_trick(s.tricks[t]) << (2 * t);
    }
    for (int p = 0; p < 4; ++p) { d.eyes[p] = (uint8_t)s.eyes[p]; d.ntricks[p] = (uint8_t)s.ntricks[p]; }
    int rl = 0; for (int i = 0; i < 4; ++i) { d.res[i] = s.res[i] < 0 ? DK_NONE : (uint8_t)s.res[i]; rl += s.res[i] >= 0; }
    d.res_start = (uint8_t)s.res_start; d.res_len = (uint8_t)rl; d.card_index = (uint8_t)ci; d.phase = (uint8_t)s.phase;
    d.current_player = s.current_player < 0 ? DK_NONE : (uint8_t)s.current_player;
    d.rr_kind = !s.has_rr ? DK_NONE : (s.rr_wedding < 0 ? 0 : 2); d.rr_player = (uint8_t)(s.rr_wedding < 0 ? 0 : s.rr_wedding);
    d.team_kind = (uint8_t)s.team.kind; d.wedding_player = (uint8_t)s.team.wedding_player; d.solved_trick = (uint8_t)s.team.solved;
    d.re_players = s.team.re; d.trick_index = (uint8_t)s.trick_index; d.game = DK_GAME_DOKO;
    memcpy(out, &d, sizeof(d));
}
// The reference's DoState fields as the C-ABI's dk_do_fields (the input of dk_do_from_fields).
void or_do_fields(void* sp, dk_do_fields* f) {
    const dko::State& s = *(dko::State*)sp;
    memset(f, 0, sizeof(*f));
    for (int p = 0; p < 4; ++p) { f->hands[p] = s.hands[p]; f->player_eyes[p] = s.eyes[p]; f->player_num_tricks[p] = s.ntricks[p]; }
    f->res_start = (int8_t)s.res_start;
    for (int i = 0; i < 4; ++i) f->reservations[i] = (int8_t)s.res[i];
    for (int t = 0; t < 12; ++t) {
        f->trick_start[t] = s.tricks[t].present ? (int8_t)s.tricks[t].start : (int8_t)-1;
        for (int i = 0; i < 4; ++i) f->trick_cards[t][i] = s.tricks[t].present ? (int8_t)s.tricks[t].cards[i] : (int8_t)-1;
    }
    f->current_player = (int8_t)s.current_player; f->phase = (int8_t)s.phase; f->trick_index = (int8_t)s.trick_index;
    f->rr_kind = !s.has_rr ? (int8_t)-1 : (s.rr_wedding < 0 ? (int8_t)0 : (int8_t)2);
    f->rr_player = (int8_t)(s.rr_wedding < 0 ? 0 : s.rr_wedding);
    f->team_kind = (int8_t)s.team.kind; f->wedding_player = (int8_t)s.team.wedding_player;
    f->solved_trick = (int8_t)s.team.solved; f->re_players = s.team.re;
}
int or_do_random_plies(void* sp, uint64_t* rng_state, int k) {
    dko::State& s = *(dko::State*)sp; SmallRng r = rng_from(rng_state); int done = 0;
    for (int i = 0; i < k; ++i) { if (dko::random_action_for_current_player(s, r)) break; done++; }
    rng_to(r, rng_state); return done;
}
void or_do_rollout(void* sp, uint64_t* rng_state, double* out) {
    dko::Env e; e.doko = *(dko::State*)sp; SmallRng r = rng_from(rng_state); e.random_rollout(r, out); rng_to(r, rng_state);
}
int or_do_search(void* sp, uint64_t* rng_state, uint32_t iters, double c, uint32_t* visits, double* values, uint64_t* counters) {
    dko::Env e; e.doko = *(dko::State*)sp; SmallRng r = rng_from(rng_state);
    Mcts<dko::Env> m; SearchCounters ctr; auto moves = m.search(e, c, iters, r, &ctr); rng_to(r, rng_state);
    if (counters) { counters[0] = ctr.iterations; counters[1] = ctr.children_scanned; counters[2] = ctr.path_nodes;
                    counters[3] = ctr.max_depth; counters[4] = ctr.nodes; counters[5] = ctr.child_slots;
        counters[6] = ctr.max_path_entries; }
    return moves_to_arrays(moves, visits, values, DK_NUM_ACTIONS);
}
double or_do_search_many(void** roots, const uint64_t* seeds, uint32_t n, uint32_t iters, double c, uint32_t* visits, int threads) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    auto next = std::make_shared<std::atomic<uint32_t>>(0);   // shared root queue (MCTSWorkers' MPMC channel)
    for (int t = 0; t < threads; ++t) {
        pool.emplace_back([=]() {
            Mcts<dko::Env> m;
            for (uint32_t i; (i = next->fetch_add(1)) < n;) {
                dko::Env e; e.doko = *(dko::State*)roots[i];
                SmallRng r = SmallRng::seed_from_u64(seeds[i]);
                auto moves = m.search(e, c, iters, r, nullptr);
                double vals[DK_NUM_ACTIONS];
                moves_to_arrays(moves, visits + (size_t)i * DK_NUM_ACTIONS, vals, DK_NUM_ACTIONS);
            }
        });
    }
    for (auto& th : pool) th.join();
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// ---------------------------------------------------------------- rs-doko sampler
// tricks: 12 x {start player (-1 = None), card0..card3 (-1 = None)}
static void tricks_from(const int32_t* t, dko::Trick out[12]) {
    for (int i = 0; i < 12; ++i) {
        out[i] = dko::Trick();
        out[i].present = t[5 * i] >= 0;
        out[i].start = t[5 * i] < 0 ? 0 : t[5 * i];
        for (int k = 0; k < 4; ++k) out[i].cards[k] = t[5 * i + 1 + k];
    }
}
uint64_t or_do_remaining_cards(const int32_t* tricks, uint64_t hand) {
    dko::Trick t[12]; tricks_from(tricks, t); return dko::calc_remaining_cards(t, hand);
}
// out: 4 x 48 card ids (-1 padded), lens: 4
void or_do_allowed_to_have(int marriage, const int32_t* tricks, uint64_t hand, int obs, int32_t* out, int32_t* lens) {
    dko::Trick t[12]; tricks_from(tricks, t);
    dko::CardVec v[4]; dko::player_allowed_to_have(marriage, t, hand, obs, v);
    for (int i = 0; i < 4; ++i) {
        lens[i] = (int32_t)v[i].size();
        for (int k = 0; k < 48; ++k) out[48 * i + k] = k < (int)v[i].size() ? v[i][(size_t)k] : -1;
    }
}
int or_do_sample_assignment(int marriage, const int32_t* tricks, uint64_t hand, const int32_t* lengths, int obs,
                            uint64_t* rng_state, uint64_t* hands_out) {
    dko::Trick t[12]; tricks_from(tricks, t);
    int len[4] = {lengths[0], lengths[1], lengths[2], lengths[3]};
    SmallRng r = rng_from(rng_state); dko::CardVec v[4];
    const bool ok = dko::sample_assignment(marriage, t, hand, len, obs, r, v);
    rng_to(r, rng_state);
    if (ok) for (int i = 0; i < 4; ++i) hands_out[i] = dko::hand_from_vec(v[i]);
    return ok ? 1 : 0;
}
void* or_do_sample_full(void* sp, uint64_t* rng_state) {
    SmallRng r = rng_from(rng_state); dko::State out;
    const bool ok = dko::sample_assignment_full(*(dko::State*)sp, r, out);
    rng_to(r, rng_state);
    return ok ? new dko::State(out) : nullptr;
}

// ---------------------------------------------------------------- AlphaZero PUCT (synthetic network)
void or_az_hash_eval(const uint8_t* packed, float* value, float* logits) { az::hash_eval(packed, value, logits); }
// temp_mode: 0 None, 1 infinite, 2 finite `temp`.  noise NULL: the search draws
// Dirichlet([alpha; 39]) from its own SmallRng.  Returns the chosen action (-2: alpha refused).
int or_az_search(void* sp, const float* noise, float alpha, uint32_t iters, float c, float eps, int epoch, int temp_mode,
                 float temp, uint64_t* rng_state, uint32_t* visits, float* root_priors) {
    az::Env e; e.doko = *(fdo::State*)sp;
    az::Options o; o.c = c; o.dirichlet_epsilon = eps; o.epoch = epoch; o.dirichlet_alpha = alpha;
    o.has_temperature = temp_mode != 0; o.temperature = temp_mode == 1 ? INFINITY : temp;
    auto eval = [](const az::Env& st, float v[4], float l[39]) {
        uint8_t b[128]; or_fdo_pack((void*)&st.doko, b); az::hash_eval(b, v, l);
    };
    SmallRng r = rng_from(rng_state);
    az::Search s;
    const int a = s.search(e, eval, noise, iters, o, r, visits, root_priors);
    rng_to(r, rng_state);
    return a;
}
// dk_az_state record: the packed state plus the announcement occurrence list
void or_fdo_pack_az(void* sp, uint8_t* out) {
    const fdo::State& s = *(fdo::State*)sp;
    memset(out, 0, sizeof(dk_az_state));
    dk_az_state* r = (dk_az_state*)out;
    or_fdo_pack(sp, r->state.raw);
    for (int k = 0; k < s.announcements.n; ++k) {
        const fdo::AnnOccurrence& a = s.announcements.list[k];
        r->ann_card[k] = (uint8_t)a.card_index;
        r->ann_code[k] = (uint8_t)((a.player << 4) | __builtin_ctz(a.announcement));
    }
    r->ann_n = (uint8_t)s.announcements.n;
}
void or_az_take_action(void* sp, int a) { az::Env e; e.doko = *(fdo::State*)sp; *(fdo::State*)sp = e.take_action(a, true).doko; }

// rand_distr 0.5.1 draws (rand_distr05.hpp) for the moment tests and the host harness.
// Dirichlet([alpha; n]) n_draws times from one stream; returns 0 if alpha is refused.
int or_dirichlet(float alpha, int n, uint32_t n_draws, uint64_t* rng_state, float* out) {
    std::vector<float> al((size_t)n, alpha);
    SmallRng r = rng_from(rng_state);
    for (uint32_t d = 0; d < n_draws; ++d)
        if (!rdist::dirichlet(al.data(), n, r, out + (size_t)d * n)) return 0;
    rng_to(r, rng_state);
    return 1;
}
// glibc logf (fn 0) / expf (fn 1) of the f32 with bits first + i * stride (the values the device's
// restatement, engine/libm_f32.h, must reproduce)
void or_libm_f32(int fn, uint32_t first, uint32_t stride, uint64_t n, float* out) {
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t b = first + (uint32_t)i * stride;
        float x;
        std::memcpy(&x, &b, 4);
        out[i] = fn ? expf(x) : logf(x);
    }
}
void or_beta(float a, float b, uint32_t n, uint64_t* rng_state, float* out) {
    SmallRng r = rng_from(rng_state);
    const rdist::Beta g(a, b);
    for (uint32_t i = 0; i < n; ++i) out[i] = g.sample(r);
    rng_to(r, rng_state);
}
void or_gamma(float shape, uint32_t n, uint64_t* rng_state, float* out) {
    SmallRng r = rng_from(rng_state);
    const rdist::Gamma g(shape);
    for (uint32_t i = 0; i < n; ++i) out[i] = g.sample(r);
    rng_to(r, rng_state);
}
void or_normal_f64(uint32_t n, uint64_t* rng_state, double* out) {
    SmallRng r = rng_from(rng_state);
    for (uint32_t i = 0; i < n; ++i) out[i] = rdist::normal_f64(r);
    rng_to(r, rng_state);
}
void or_exp1_f64(uint32_t n, uint64_t* rng_state, double* out) {
    SmallRng r = rng_from(rng_state);
    for (uint32_t i = 0; i < n; ++i) out[i] = rdist::exp1_f64(r);
    rng_to(r, rng_state);
}
// the ziggurat tables as the oracle computed them: [NORM_X, NORM_F, EXP_X, EXP_F] x 257, R_norm, R_exp
void or_ziggurat_tables(double* out) {
    const rdist::Zig& z = rdist::zig();
    memcpy(out, z.nx, sizeof z.nx); memcpy(out + 257, z.nf, sizeof z.nf);
    memcpy(out + 514, z.ex, sizeof z.ex); memcpy(out + 771, z.ef, sizeof z.ef);
    out[1028] = z.norm_r; out[1029] = z.exp_r;
}

// ---------------------------------------------------------------- encode_state_pi
void or_encode_pi(void* sp, int64_t* out) { enc::encode_state_pi(*(fdo::State*)sp, out); }
// A state from the fields encode_state_pi reads (the reference test builds its FdoState the same way):
// f[0] res_start, f[1] res_len, f[2..5] res, f[6] n_tricks, f[7 + 6t ..] = {start, len, c0..c3} for t < 12,
// f[79] ann_n, f[80 + 3k ..] = {card_index, player, announcement bit} for k < 12,
// f[116] current_player, f[117] phase, f[118] re_players.
static fdo::State state_from_fields(const int32_t* f, const uint64_t* hands) {
    fdo::State s;
    s.res_start = f[0]; s.res_len = f[1];
    for (int i = 0; i < 4; ++i) s.res[i] = f[2 + i];
    s.n_tricks = f[6];
    for (int t = 0; t < 12; ++t) {
        const int32_t* q = f + 7 + 6 * t;
        s.tricks[t].start = q[0]; s.tricks[t].len = q[1];
        for (int i = 0; i < 4; ++i) s.tricks[t].cards[i] = q[2 + i];
    }
    for (int p = 0; p < 4; ++p) s.hands[p].bits = hands[p];
    s.announcements.n = f[79];
    for (int k = 0; k < 12; ++k) {
        s.announcements.list[k].card_index = f[80 + 3 * k];
        s.announcements.list[k].player = f[81 + 3 * k];
        s.announcements.list[k].announcement = (uint32_t)f[82 + 3 * k];
    }
    s.current_player = f[116]; s.phase = f[117];
    s.team_state.kind = fdo::NoWedding; s.team_state.re_players = (uint8_t)f[118];
    return s;
}
void or_encode_pi_fields(const int32_t* f, const uint64_t* hands, int64_t* out) {
    enc::encode_state_pi(state_from_fields(f, hands), out);
}

// ---------------------------------------------------------------- tic-tac-toe
int or_ttt_finish(const int32_t* board) { int b[9]; for (int i = 0; i < 9; ++i) b[i] = board[i]; return ttt::calc_finish_state(b); }
static ttt::Env ttt_from(const int32_t* board) {
    ttt::Env e; for (int i = 0; i < 9; ++i) e.board[i] = board[i]; e.finish = ttt::calc_finish_state(e.board); return e;
}
void or_ttt_rollout(const int32_t* board, uint64_t* rng_state, double* out) {
    ttt::Env e = ttt_from(board); SmallRng r = rng_from(rng_state); e.random_rollout(r, out); rng_to(r, rng_state);
}
int or_ttt_search(const int32_t* board, uint64_t* rng_state, uint32_t iters, double c, uint32_t* visits, double* values) {
    ttt::Env e = ttt_from(board); SmallRng r = rng_from(rng_state);
    Mcts<ttt::Env> m; auto moves = m.search(e, c, iters, r, nullptr); rng_to(r, rng_state);
    return moves_to_arrays(moves, visits, values, DK_NUM_ACTIONS);
}
void or_ttt_pack(const int32_t* board, int last_action, uint8_t* out) {
    dk_ttt_state d; memset(&d, 0, sizeof(d));
    int b[9]; for (int i = 0; i < 9; ++i) { d.board[i] = (uint8_t)board[i]; b[i] = board[i]; }
    d.finish = (uint8_t)ttt::calc_finish_state(b); d.last_action = last_action < 0 ? DK_NONE : (uint8_t)last_action;
    d.game = DK_GAME_TTT; memcpy(out, &d, sizeof(d));
}

// ---------------------------------------------------------------- fusion
int or_fuse_maxn(const uint32_t* visits, int S, uint64_t allowed, uint32_t* ranks) { return fuse_maxn(visits, S, allowed, ranks); }
int or_fuse_avg(const uint32_t* visits, int S, float* probs) { return fuse_avg(visits, S, probs); }


// ---------------------------------------------------------------- IMPI (autoregressive determinization)
static void ipi_assumed(const uint64_t* ah, const int32_t* ar, fdo::Hand h[4], int r[4]) {
    for (int p = 0; p < 4; ++p) { h[p].bits = ah[p]; r[p] = ar[p]; }
}
int or_ipi_encode(void* sp, const uint64_t* ah, const int32_t* ar, int guess, int64_t* out) {
    fdo::Hand h[4]; int r[4]; ipi_assumed(ah, ar, h, r);
    return impi::encode_state_ipi(*(fdo::State*)sp, h, r, guess, out);
}
int or_encode_ipi_fields(const int32_t* f, const uint64_t* hands, const uint64_t* ah, const int32_t* ar, int guess, int64_t* out) {
    fdo::Hand h[4]; int r[4]; ipi_assumed(ah, ar, h, r);
    return impi::encode_state_ipi(state_from_fields(f, hands), h, r, guess, out);
}
uint64_t or_ipi_next_card(void* sp, const uint64_t* ah, const int32_t* ar, int p) {
    fdo::Hand h[4]; int r[4]; ipi_assumed(ah, ar, h, r);
    return impi::next_possible_card(*(fdo::State*)sp, h, r, p).bits;
}
uint32_t or_ipi_next_reservation(void* sp, const uint64_t* ah, int p) {
    fdo::Hand h[4]; int r[4]; const int32_t none[4] = {-1, -1, -1, -1}; ipi_assumed(ah, none, h, r);
    return impi::next_possible_reservation(*(fdo::State*)sp, h, p);
}
int or_ipi_consistent(void* sp, const uint64_t* ah, const int32_t* ar) {
    fdo::Hand h[4]; int r[4]; ipi_assumed(ah, ar, h, r);
    return impi::is_consistent_reason(*(fdo::State*)sp, h, r);
}
void or_ipi_hash_eval(const int64_t* tok, float* logits) { impi::hash_eval(tok, logits); }
// forward_pred_process_with_mask with the hash network.  Returns the status (0 consistent,
// 1 not consistent, 2 reference panic); *reason, the packed sample (consistent only), and
// the number of network evaluations.
int or_ipi_sample(void* sp, uint64_t* rng_state, float temperature, float log_chance, int32_t* reason, uint8_t* out,
                  int32_t* guesses) {
    SmallRng r = rng_from(rng_state);
    const impi::ArResult a = impi::forward_pred_process_with_mask(
        *(fdo::State*)sp, temperature, log_chance, [](const int64_t* t, float* l) { impi::hash_eval(t, l); }, r);
    rng_to(r, rng_state);
    *reason = a.reason;
    *guesses = a.guesses;
    if (a.status == 0) or_fdo_pack((void*)&a.state, out);
    return a.status;
}
// the consistent sample as a new oracle state (nullptr otherwise)
void* or_ipi_sample_state(void* sp, uint64_t* rng_state, float temperature, float log_chance, int32_t* status,
                          int32_t* reason) {
    SmallRng r = rng_from(rng_state);
    const impi::ArResult a = impi::forward_pred_process_with_mask(
        *(fdo::State*)sp, temperature, log_chance, [](const int64_t* t, float* l) { impi::hash_eval(t, l); }, r);
    rng_to(r, rng_state);
    *status = a.status;
    *reason = a.reason;
    return a.status == 0 ? new fdo::State(a.state) : nullptr;
}
uint64_t or_fdo_random_single(uint64_t mask, uint64_t* rng_state) {
    SmallRng r = rng_from(rng_state); const uint64_t b = fdo::random_single(mask, r); rng_to(r, rng_state); return b;
}
}  // extern "C"
