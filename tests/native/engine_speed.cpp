// Host-build throughput probe of the engine (not a test): rollouts/s and
// search sims/s of the gfx950 engine headers compiled for the CPU, on C3-like
// roots.  Usage: engine_speed <roots> <iters>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/adapters.h"
#include "../../master_doko_reinforcement_learning_amd/csrc/engine/search_core.h"
#include "host_mem.h"
#include "../../oracle/full_doko.hpp"
#include "../../oracle/card_matching.hpp"

using namespace oracle;
extern "C" void or_fdo_pack(void* sp, uint8_t* out);


int main(int argc, char** argv) {
    const int nroots = argc > 1 ? atoi(argv[1]) : 64;
    const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 1000;
    std::vector<dk::fdo::Work> roots;
    for (int j = 0; j < nroots; ++j) {
        SmallRng deal = SmallRng::seed_from_u64(0xC3000000ULL + j);
        fdo::State s = fdo::new_game(deal);
        for (int k = 0; k < 4; ++k) fdo::play_action(s, fdo::A_ReservationHealthy);
        SmallRng pl = SmallRng::seed_from_u64(0xC3100000ULL + j);
        const int plies = (int[]){0, 8, 20, 32}[j % 4];
        for (int k = 0; k < plies; ++k) if (fdo::random_action_for_current_player_no_announcement(s, pl)) break;
        SmallRng cm = SmallRng::seed_from_u64(0xC3200000ULL + j);
        fdo::State smp = card_matching_full(s, cm);
        dk_state p; or_fdo_pack(&smp, p.raw);
        dk::fdo::Work w; dk::fdo::unpack(p.fdo, w);
        roots.push_back(w);
    }
    // rollouts
    dk::Rng rng = dk::Rng::seed_from_u64(7);
    long plies = 0; int sink = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int j = 0; j < nroots; ++j)
        for (uint32_t i = 0; i < iters; ++i) { int r[4]; plies += dk::fdo::rollout(roots[j], rng, r); sink += r[0]; }
    double sr = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // searches
    std::vector<double> ln(iters + 2);
    for (size_t i = 0; i < ln.size(); ++i) ln[i] = std::log((double)i);
    auto t1 = std::chrono::steady_clock::now();
    uint64_t scanned = 0;
    for (int j = 0; j < nroots; ++j) {
        HostMem<dk::fdo::Node> mem(40 + 12 * iters, iters + 1, 128);
        mem.ln_table = ln.data();
        dk::Rng r2 = dk::Rng::seed_from_u64(0xC3300000ULL + j);
        uint32_t v[39]; double val[39]; uint8_t b; uint64_t sc = 0;
        dk::search_root<dk::FdoE>(roots[j], r2, iters, 2.5, mem, v, val, &b, &sc);
        scanned += sc; sink += v[0];
    }
    double ss = std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count();
    const double n = (double)nroots * iters;
    printf("rollouts/s %.0f  plies/rollout %.1f  ns/rollout %.0f | search sims/s %.0f  ns/sim %.0f  scanned/sim %.1f (%d)\n",
           n / sr, plies / n, sr / n * 1e9, n / ss, ss / n * 1e9, scanned / n, sink & 1);
    return 0;
}
