// TEST INFRASTRUCTURE: host build of the GPU CAP sampler (cap_engine.h)
// checked against the ORACLE card_matching_full on random infosets, including
// weddings, solos, hidden reservations and announcements.
// Usage: cap_check <games> <seed>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/cap_engine.h"
#include "../../oracle/card_matching.hpp"
#include "../../oracle/full_doko.hpp"

using namespace oracle;
extern "C" void or_fdo_pack(void* sp, uint8_t* out);

int main(int argc, char** argv) {
    const int games = argc > 1 ? atoi(argv[1]) : 100;
    const uint64_t seed = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    std::mt19937_64 pol(seed);
    long n = 0;
    for (int g = 0; g < games; ++g) {
        SmallRng deal = SmallRng::seed_from_u64(seed * 4242 + g);
        fdo::State s = fdo::new_game(deal);
        const int mode = g % 5;
        while (s.phase != fdo::Finished) {
            // sample at every decision point
            dk_fdo_state pk; or_fdo_pack(&s, (uint8_t*)&pk);
            const uint64_t sd = pol();
            SmallRng r = SmallRng::seed_from_u64(sd);
            fdo::State o = fdo::card_matching_full(s, r);
            dk::Rng dr = dk::Rng::seed_from_u64(sd);
            dk_fdo_state out;
            dk::cap::card_matching_full(pk, dr, out);
            for (int p = 0; p < 4; ++p) if (out.hands[p] != o.hands[p].bits) { printf("MISMATCH hands game %d p %d\n", g, p); return 1; }
            if (out.res_len != o.res_len) { printf("MISMATCH res_len game %d\n", g); return 1; }
            for (int i = 0; i < o.res_len; ++i) if (out.res[i] != o.res[i]) { printf("MISMATCH res game %d\n", g); return 1; }
            if (dr.s0 != r.s[0] || dr.s1 != r.s[1] || dr.s2 != r.s[2] || dr.s3 != r.s[3]) { printf("MISMATCH rng game %d\n", g); return 1; }
            if (!fdo::sample_consistent(s, o)) { printf("INCONSISTENT sample game %d\n", g); return 1; }
            n++;
            const uint64_t legal = fdo::observation_allowed_actions(s);
            int a;
            if (s.phase == fdo::Reservation) {
                a = fdo::A_ReservationHealthy;
                if (mode == 1 && (legal >> fdo::A_ReservationWedding & 1)) a = fdo::A_ReservationWedding;
                if (mode == 2 && pol() % 3 == 0) a = 26 + (int)(pol() % 7);
            } else if (s.phase == fdo::Announcement) {
                const uint64_t anns = legal & (0x1FULL << 33);
                a = fdo::A_NoAnnouncement;
                if (anns && pol() % 3 == 0) { int k = (int)(pol() % (uint64_t)__builtin_popcountll(anns)); for (int b = 33; b < 38; ++b) if (anns >> b & 1) { if (k-- == 0) { a = b; break; } } }
            } else {
                int k = (int)(pol() % (uint64_t)__builtin_popcountll(legal));
                a = 0;
                for (int b = 0; b < 24; ++b) if (legal >> b & 1) { if (k-- == 0) { a = b; break; } }
            }
            fdo::play_action(s, a);
        }
    }
    printf("OK %ld\n", n);
    return 0;
}
