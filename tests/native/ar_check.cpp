// TEST INFRASTRUCTURE: host build of the batched IMPI determinization (ar_engine.h)
// checked against the ORACLE forward_pred_process_with_mask (oracle/impi.hpp) with
// the synthetic hash network.  The lanes are driven exactly as the GPU drives them
// (init -> rounds of {prepare -> network -> choose} -> prepare -> output); per lane
// the status, the NotConsistentReason, the sample (hands + reservation round), the
// number of network calls and the RNG stream position must be identical.  Positions
// come from random games over all legal actions (weddings, solos, announcements).
// Usage: ar_check <positions> <samples per position> <seed>   -> "OK <lanes> <consistent> <not> <panic>"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/ar_engine.h"
#include "../../oracle/full_doko.hpp"
#include "../../oracle/impi.hpp"

using namespace oracle;
extern "C" void or_fdo_pack(void* sp, uint8_t* out);
extern "C" void or_fdo_pack_az(void* sp, uint8_t* out);

int main(int argc, char** argv) {
    const int npos = argc > 1 ? atoi(argv[1]) : 60;
    const int samples = argc > 2 ? atoi(argv[2]) : 4;
    const uint64_t seed = argc > 3 ? strtoull(argv[3], 0, 10) : 1;
    std::mt19937_64 pol(seed);
    std::vector<fdo::State> pos;
    for (int g = 0; (int)pos.size() < npos; ++g) {
        SmallRng deal = SmallRng::seed_from_u64(seed * 7919 + g);
        fdo::State s = fdo::new_game(deal);
        const int stop = (int)(pol() % 56);
        for (int ply = 0; ply < 80 && s.phase != fdo::Finished; ++ply) {
            if (ply == stop) { pos.push_back(s); break; }
            const uint64_t legal = fdo::observation_allowed_actions(s);
            int k = (int)(pol() % (uint64_t)__builtin_popcountll(legal)), a = 0;
            for (int b = 0; b < 39; ++b) if (legal >> b & 1) { if (k-- == 0) { a = b; break; } }
            fdo::play_action(s, a);
        }
    }
    const int P = (int)pos.size(), N = P * samples;
    std::vector<dk_az_state> info(P);
    for (int i = 0; i < P; ++i) or_fdo_pack_az(&pos[i], (uint8_t*)&info[i]);
    const float temps[3] = {1.0f, 0.35f, 4.0f};
    const float log_chance = 1.0f / 30000.0f;
    long cnt[3] = {0, 0, 0}, lanes_done = 0;
    for (int ti = 0; ti < 3; ++ti) {
        const float temp = temps[ti];
        std::vector<uint64_t> seeds(N);
        for (auto& x : seeds) x = pol();
        // device engine, batched rounds
        std::vector<dk::ar::Lane> L(N);
        std::vector<int32_t> tok((size_t)N * 311, 0);
        std::vector<float> logits((size_t)N * 33);
        uint32_t rounds = 0;
        for (int i = 0; i < N; ++i) { const uint32_t g = dk::ar::init(info[i / samples], seeds[i], L[i]); rounds = g > rounds ? g : rounds; }
        std::vector<int> calls(N, 0);
        for (uint32_t r = 0; r <= rounds; ++r) {
            for (int i = 0; i < N; ++i) {
                int32_t* o = tok.data() + (size_t)311 * i;
                auto put = [o](uint32_t k, uint32_t v) { o[k] = (int32_t)v; };
                dk::ar::prepare(info[i / samples], L[i], log_chance, put);
            }
            if (r == rounds) break;
            for (int i = 0; i < N; ++i) {
                if (L[i].status != dk::ar::RUNNING || L[i].guess == DK_NONE) continue;
                int64_t t64[311];
                for (int k = 0; k < 311; ++k) t64[k] = tok[(size_t)311 * i + k];
                impi::hash_eval(t64, logits.data() + (size_t)33 * i);
                calls[i]++;
                dk::ar::choose(L[i], logits.data() + (size_t)33 * i, temp);
            }
        }
        for (int i = 0; i < N; ++i) {
            const int p = i / samples;
            SmallRng rng = SmallRng::seed_from_u64(seeds[i]);
            const impi::ArResult want = impi::forward_pred_process_with_mask(
                pos[p], temp, log_chance, [](const int64_t* t, float* l) { impi::hash_eval(t, l); }, rng);
            const uint8_t st = L[i].status;
            const int got_status = st == dk::ar::CONSISTENT ? 0 : st == dk::ar::NOT_CONSISTENT ? 1 : st == dk::ar::PANIC ? 2 : 3;
            if (got_status != want.status) {
                printf("MISMATCH status lane %d (pos %d, T %g): got %d want %d (reason %d / %d)\n", i, p, temp, got_status,
                       want.status, L[i].reason, want.reason);
                return 1;
            }
            if (want.status == 1 && L[i].reason != want.reason) { printf("MISMATCH reason lane %d: %d vs %d\n", i, L[i].reason, want.reason); return 1; }
            if (want.status != 2) {
                if (calls[i] != want.guesses) { printf("MISMATCH calls lane %d: %d vs %d\n", i, calls[i], want.guesses); return 1; }
                if (L[i].rng[0] != rng.s[0] || L[i].rng[1] != rng.s[1] || L[i].rng[2] != rng.s[2] || L[i].rng[3] != rng.s[3]) {
                    printf("MISMATCH rng lane %d\n", i); return 1;
                }
            }
            if (want.status == 0) {
                dk_fdo_state got;
                dk::ar::output(info[p], L[i], got);
                uint8_t w[128]; or_fdo_pack((void*)&want.state, w);
                if (memcmp(&got, w, 117) != 0) { printf("MISMATCH sample lane %d\n", i); return 1; }
            }
            cnt[want.status < 3 ? want.status : 2]++;
            lanes_done++;
        }
    }
    if (cnt[0] == 0 || cnt[1] == 0) { printf("degenerate: consistent %ld not %ld\n", cnt[0], cnt[1]); return 1; }
    printf("OK %ld %ld %ld %ld\n", lanes_done, cnt[0], cnt[1], cnt[2]);
    return 0;
}
