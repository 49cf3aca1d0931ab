// TEST INFRASTRUCTURE: compiles the gfx950 engine headers for the host and
// checks them against the ORACLE on random trajectories.  Not part of the
// product (the product runs the same headers on the GPU only).
//
// Usage: fdo_engine_check <games> <seed>   -> prints "OK <checks>" or the first mismatch.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/fdo_engine.h"
#include "../../oracle/full_doko.hpp"

using namespace oracle;

static dk_fdo_state pack_oracle(const fdo::State& s);
extern "C" void or_fdo_pack(void* sp, uint8_t* out);

static dk_fdo_state pack_oracle(const fdo::State& s) {
    dk_fdo_state d;
    or_fdo_pack((void*)&s, (uint8_t*)&d);
    return d;
}

static long checks = 0;
static void fail(const char* what, int game, int step) {
    printf("MISMATCH %s game %d step %d\n", what, game, step);
    exit(1);
}

static bool same_state(const dk_fdo_state& a, const dk_fdo_state& b) {
    return memcmp(&a, &b, 117) == 0 && a.game == b.game;
}

static void check_state(const fdo::State& s, int game, int step, uint64_t seed) {
    dk_fdo_state pk = pack_oracle(s);
    dk::fdo::Work w;
    dk::fdo::unpack(pk, w);
    // round trip
    dk_fdo_state rt = pk;
    dk::fdo::pack_fields(w, rt);
    if (!same_state(rt, pk)) fail("pack/unpack roundtrip", game, step);
    if (!dk::fdo::node_ok(w)) fail("64-B node record roundtrip", game, step);
    if ((dk::fdo::env_allowed(w, false) != 0) != !dk::fdo::is_terminal(w)) fail("allowed != 0 <=> not terminal", game, step);
    {   // states the search reaches by stepping (incremental trick fields) round-trip as well
        const uint64_t la = dk::fdo::legal_actions(w);
        for (int a = 0; a < 39; ++a)
            if (la >> a & 1) { dk::fdo::Work x = w; dk::fdo::play_action(x, a); if (!dk::fdo::node_ok(x)) fail("64-B node record after step", game, step); }
    }
    if (s.phase != fdo::Finished) {
        if (dk::fdo::legal_actions(w) != fdo::observation_allowed_actions(s)) fail("legal_actions", game, step);
        fdo::Env e; e.doko = s;
        if (dk::fdo::env_allowed(w, true) != e.allowed_actions(true)) fail("env_allowed(first)", game, step);
        if (dk::fdo::env_allowed(w, false) != e.allowed_actions(false)) fail("env_allowed(non-first)", game, step);
        if (dk::fdo::env_current_player(w) != e.current_player()) fail("current_player", game, step);
        // every player's announcement offer
        if (s.team_state.kind != fdo::InReservations) {
            for (int p = 0; p < 4; ++p)
                for (int n = 0; n <= 12; ++n)
                    if (dk::fdo::allowed_announcements(w, p, n) !=
                        fdo::calc_allowed_announcements(p, n, s.team_state, s.announcements.re_lowest, s.announcements.contra_lowest))
                        fail("allowed_announcements", game, step);
            // the rollout fast path's hand-size thresholds (rollout_cards)
            const uint32_t th = dk::fdo::ann_thetas(w.team_kind, w.solved_trick, w.re_players, w.re_lowest, w.contra_lowest);
            for (int p = 0; p < 4; ++p)
                for (int n = 0; n <= 12; ++n)
                    if ((n >= (int)((th >> (8 * p)) & 0xFF)) != (dk::fdo::allowed_announcements(w, p, n) != 0))
                        fail("announcement thresholds", game, step);
        }
    }
    // rollout parity (rewards + RNG stream position)
    SmallRng r = SmallRng::seed_from_u64(seed);
    fdo::Env e; e.doko = s;
    double ref[4];
    e.random_rollout(r, ref);
    dk::Rng g = dk::Rng::seed_from_u64(seed);
    int pts[4];
    dk::fdo::rollout(w, g, pts);
    for (int p = 0; p < 4; ++p) if ((double)pts[p] != ref[p]) fail("rollout rewards", game, step);
    if (g.s0 != r.s[0] || g.s1 != r.s[1] || g.s2 != r.s[2] || g.s3 != r.s[3]) fail("rollout rng stream", game, step);
    if (s.phase == fdo::Finished) {
        dk::fdo::score(w, pts);
        for (int p = 0; p < 4; ++p) if (pts[p] != s.stats.player_points[p]) fail("score", game, step);
    }
    checks++;
}

int main(int argc, char** argv) {
    const int games = argc > 1 ? atoi(argv[1]) : 200;
    const uint64_t seed = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    std::mt19937_64 pol(seed * 7919 + 13);
    for (int g = 0; g < games; ++g) {
        SmallRng deal = SmallRng::seed_from_u64(seed * 1000003ULL + g);
        fdo::State s = fdo::new_game(deal);
        // reservation policy mix: mostly healthy so that normal games, weddings,
        // silent solos and real solos all appear
        const int mode = (int)(pol() % 10);
        int step = 0;
        while (true) {
            check_state(s, g, step, pol());
            if (s.phase == fdo::Finished) break;
            uint64_t legal = fdo::observation_allowed_actions(s);
            int a;
            if (s.phase == fdo::Reservation) {
                uint64_t pick = 1ULL << fdo::A_ReservationHealthy;
                if (mode >= 6 && (legal >> fdo::A_ReservationWedding & 1)) pick = 1ULL << fdo::A_ReservationWedding;
                if (mode >= 8 && (pol() % 4 == 0)) {
                    uint64_t solos = legal & (0x7FULL << 26);
                    int k = (int)(pol() % (uint64_t)__builtin_popcountll(solos));
                    for (int b = 0; b < 64; ++b) if (solos >> b & 1) { if (k-- == 0) { pick = 1ULL << b; break; } }
                }
                a = __builtin_ctzll(pick);
            } else if (s.phase == fdo::Announcement) {
                // announce with probability 1/3 so that all announcement paths get exercised
                uint64_t anns = legal & (0x1FULL << 33);
                if (anns && pol() % 3 == 0) {
                    int k = (int)(pol() % (uint64_t)__builtin_popcountll(anns));
                    a = -1;
                    for (int b = 0; b < 64; ++b) if (anns >> b & 1) { if (k-- == 0) { a = b; break; } }
                } else a = fdo::A_NoAnnouncement;
            } else {
                int k = (int)(pol() % (uint64_t)__builtin_popcountll(legal));
                a = -1;
                for (int b = 0; b < 64; ++b) if (legal >> b & 1) { if (k-- == 0) { a = b; break; } }
            }
            // step parity on the wire format
            dk_fdo_state before = pack_oracle(s);
            fdo::play_action(s, a);
            dk::fdo::step_packed(before, a);
            dk_fdo_state after = pack_oracle(s);
            if (!same_state(before, after)) {
                const uint8_t* x = (const uint8_t*)&before; const uint8_t* y = (const uint8_t*)&after;
                for (int i = 0; i < 128; ++i) if (x[i] != y[i]) printf("  byte %d engine %d oracle %d\n", i, x[i], y[i]);
                fail("step_packed", g, step);
            }
            step++;
        }
    }
    printf("OK %ld\n", checks);
    return 0;
}
