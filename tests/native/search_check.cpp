// TEST INFRASTRUCTURE: host build of the engine's search_core / rs-doko / TTT
// engines checked against the ORACLE.  Prints "OK <n>" or the first mismatch.
// Usage: search_check <roots> <iters> <seed>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/adapters.h"
#include "../../master_doko_reinforcement_learning_amd/csrc/engine/search_core.h"
#include "host_mem.h"
#include "../../oracle/doko.hpp"
#include "../../oracle/full_doko.hpp"
#include "../../oracle/mcts.hpp"
#include "../../oracle/ttt.hpp"

using namespace oracle;
extern "C" void or_fdo_pack(void* sp, uint8_t* out);
extern "C" void or_do_pack(void* sp, uint8_t* out);


static void fail(const char* w, int i) { printf("MISMATCH %s root %d\n", w, i); exit(1); }

template <class E, class OEnv>
static void compare(const dk_state& packed, const OEnv& oenv, uint64_t seed, uint32_t iters, double c,
                    const double* ln, uint32_t max_path, int idx, const char* name) {
    typename E::Work w; E::load(packed, w);
    // DK_BALIGN_LINE=1: blocks kept within 128-B lines (dk::block_base), the padding given room
    const bool line = getenv("DK_BALIGN_LINE") != nullptr;
#if DK_HOT8
    HostMem8<typename E::Node> mem(line ? std::min<uint32_t>(2 * dk::P8_SLOT_BOUND(iters), 1u << 14) : dk::P8_SLOT_BOUND(iters),
                                   iters + 1, max_path);
    if (line) mem.balign = dk::BALIGN_LINE | 16u;
#else
    HostMem<typename E::Node> mem((40 + 12 * iters) * (line ? 2 : 1), iters + 1, max_path);
    if (line) mem.balign = dk::BALIGN_LINE | 8u;
#endif
    mem.ln_table = ln;
    dk::Rng rng = dk::Rng::seed_from_u64(seed);
    uint32_t v[39]; double val[39]; uint8_t best;
    int st = dk::search_root<E>(w, rng, iters, c, mem, v, val, &best, nullptr);
    if (st != 0) fail("capacity", idx);
    SmallRng r = SmallRng::seed_from_u64(seed);
    Mcts<OEnv> m;
    auto moves = m.search(oenv, c, iters, r, nullptr);
    uint32_t ov[39]; double oval[39];
    const int ob = moves_to_arrays(moves, ov, oval, 39);
    for (int a = 0; a < 39; ++a) {
        if (v[a] != ov[a]) { printf("%s action %d visits %u vs %u\n", name, a, v[a], ov[a]); fail("visits", idx); }
        if (memcmp(&val[a], &oval[a], 8) != 0) { printf("%s action %d value %.17g vs %.17g\n", name, a, val[a], oval[a]); fail("values", idx); }
    }
    if ((ob < 0 ? 0xFF : ob) != best) fail("best", idx);
    if (rng.s0 != r.s[0] || rng.s1 != r.s[1] || rng.s2 != r.s[2] || rng.s3 != r.s[3]) fail("rng stream", idx);
}

int main(int argc, char** argv) {
    const int roots = argc > 1 ? atoi(argv[1]) : 8;
    const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 300;
    const uint64_t seed = argc > 3 ? strtoull(argv[3], 0, 10) : 1;
    const uint32_t max_path = argc > 4 ? (uint32_t)atoi(argv[4]) : 128;
    std::vector<double> ln(iters + 2);
    for (uint32_t i = 0; i < ln.size(); ++i) ln[i] = std::log((double)i);
    int n = 0;
    for (int i = 0; i < roots; ++i) {
        // full doko: seeded deal, 4x healthy (or mixed reservations), k random plies
        SmallRng deal = SmallRng::seed_from_u64(seed * 7777 + i);
        fdo::State s = fdo::new_game(deal);
        const int mode = i % 6;
        if (mode < 4) {
            for (int k = 0; k < 4; ++k) fdo::play_action(s, fdo::A_ReservationHealthy);
            SmallRng pl = SmallRng::seed_from_u64(seed + i);
            const int plies = (int[]){0, 8, 20, 32}[mode];
            for (int k = 0; k < plies; ++k) if (fdo::random_action_for_current_player(s, pl)) break;
        } else if (mode == 4) {
            // reservation-phase root (solos allowed in the tree)
        } else {
            SmallRng pl = SmallRng::seed_from_u64(seed + 99 + i);
            for (int k = 0; k < 30; ++k) if (fdo::random_action_for_current_player(s, pl)) break;
        }
        if (s.phase == fdo::Finished) continue;
        dk_state packed; or_fdo_pack(&s, packed.raw);
        fdo::Env e; e.doko = s;
        compare<dk::FdoE>(packed, e, seed * 31 + i, iters, 2.5, ln.data(), max_path, i, "fdo");
        n++;
        // rs-doko root
        SmallRng dd = SmallRng::seed_from_u64(0xD0C00000ULL + seed * 100 + i);
        dko::State ds = dko::new_game(dd);
        for (int k = 0; k < 4; ++k) dko::play_action(ds, (i % 5 == 4 && (ds.hands[ds.current_player] >> 15 & 1) && (ds.hands[ds.current_player] >> 39 & 1)) ? dko::A_Wedding : dko::A_Healthy);
        dk_state dp; or_do_pack(&ds, dp.raw);
        dko::Env de; de.doko = ds;
        compare<dk::DoE>(dp, de, seed * 57 + i, iters, 2.5, ln.data(), max_path, i, "do");
        n++;
    }
    // tic-tac-toe from the empty board, c = 2.0 (tic_tac_toe_player.rs:18)
    {
        ttt::Env e;
        dk_state tp; memset(&tp, 0, sizeof(tp)); tp.ttt.last_action = 0xFF; tp.ttt.game = DK_GAME_TTT;
        compare<dk::TttE>(tp, e, 999, iters, 2.0, ln.data(), max_path, 0, "ttt");
        n++;
    }
    printf("OK %d\n", n);
    return 0;
}
