// TEST INFRASTRUCTURE: host build of the GPU rs-doko sampler (assign_engine.h)
// checked against the ORACLE sample_assignment_full
// (rs-doko-assignment/src/assignment.rs:472-580) at every decision point of
// random rs-doko games, weddings included: sampled hands, the RNG stream
// position, and the panic cases must agree.
// Usage: assign_check <games> <seed>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/assign_engine.h"
#include "../../oracle/assignment.hpp"
#include "../../oracle/doko.hpp"

using namespace oracle;
extern "C" void or_do_pack(void* sp, uint8_t* out);

int main(int argc, char** argv) {
    const int games = argc > 1 ? atoi(argv[1]) : 100;
    const uint64_t seed = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    std::mt19937_64 pol(seed);
    long n = 0, panics = 0, rule3_draws = 0;
    for (int g = 0; g < games; ++g) {
        SmallRng deal = SmallRng::seed_from_u64(seed * 7331 + g);
        dko::State s = dko::new_game(deal);
        const bool wedding = g % 3 == 1;
        while (s.phase != dko::Finished) {
            dk_do_state pk; or_do_pack(&s, (uint8_t*)&pk);
            for (int rep = 0; rep < 4; ++rep) {
                const uint64_t sd = pol();
                SmallRng r = SmallRng::seed_from_u64(sd);
                dko::State o;
                const bool ok = dko::sample_assignment_full(s, r, o);
                dk::Rng dr = dk::Rng::seed_from_u64(sd);
                dk_do_state out;
                const int rc = dk::asg::sample_assignment_full(pk, dr, out);
                if (ok != (rc == 0)) { printf("MISMATCH panic game %d (oracle ok=%d device rc=%d)\n", g, ok, rc); return 1; }
                if (!ok) { panics++; continue; }
                for (int p = 0; p < 4; ++p)
                    if (out.hands[p] != o.hands[p]) {
                        printf("MISMATCH hands game %d card %d p %d: %llx vs %llx\n", g, pk.card_index, p,
                               (unsigned long long)out.hands[p], (unsigned long long)o.hands[p]);
                        return 1;
                    }
                if (dr.s0 != r.s[0] || dr.s1 != r.s[1] || dr.s2 != r.s[2] || dr.s3 != r.s[3]) {
                    printf("MISMATCH rng game %d\n", g); return 1;
                }
                // the unpacked sample is the packed input with new hands
                dk_do_state chk; or_do_pack(&o, (uint8_t*)&chk);
                if (memcmp(&chk, &out, sizeof(chk)) != 0) { printf("MISMATCH packed state game %d\n", g); return 1; }
                // sizes preserved, the observer's cards kept, the hidden cards redistributed
                int pool_true[24] = {0}, pool_smp[24] = {0};
                const int obs = s.current_player < 0 ? 0 : s.current_player;
                for (int p = 0; p < 4; ++p) {
                    if (__builtin_popcountll(o.hands[p]) != __builtin_popcountll(s.hands[p])) { printf("BAD size\n"); return 1; }
                    if (p == obs) continue;
                    for (int c = 0; c < 24; ++c) {
                        pool_true[c] += (int)(s.hands[p] >> c & 1) + (int)(s.hands[p] >> (c + 24) & 1);
                        pool_smp[c] += (int)(o.hands[p] >> c & 1) + (int)(o.hands[p] >> (c + 24) & 1);
                    }
                }
                if (memcmp(pool_true, pool_smp, sizeof(pool_true)) != 0) { printf("BAD card pool game %d\n", g); return 1; }
                n++;
                rule3_draws += (r.s[0] != SmallRng::seed_from_u64(sd).s[0]);
            }
            const uint64_t legal = dko::observation_allowed(s);
            int a;
            if (s.phase == dko::Reservation) {
                a = dko::A_Healthy;
                if (wedding && (legal >> dko::A_Wedding & 1)) a = dko::A_Wedding;
            } else {
                int k = (int)(pol() % (uint64_t)__builtin_popcountll(legal));
                a = 0;
                for (int b = 0; b < 24; ++b) if (legal >> b & 1) { if (k-- == 0) { a = b; break; } }
            }
            dko::play_action(s, a);
        }
    }
    printf("OK %ld samples (%ld with random draws), %ld panics agreed\n", n, rule3_draws, panics);
    return 0;
}
