// TEST INFRASTRUCTURE: host build of the batched AlphaZero PUCT core (az_core.h)
// checked against the ORACLE mcts_search restatement (oracle/az_mcts.hpp) with
// the synthetic hash network: root priors, visit counts, the chosen action and
// the RNG stream position must be identical, for greedy, infinite and T = 1
// temperatures, with caller-supplied root noise and with the noise the search draws
// from its own SmallRng (rand_distr.h as az_root_kernel runs it; alphas 0.8 / 1.0 / 0.5:
// the three Gamma paths; 0.1 / 0.05: the FromBeta construction).  The batch is driven exactly as the GPU drives it: init ->
// network(root) -> root_expand -> iterations x {select -> network(leaves) ->
// backup} -> finish, over all games at once.
// Usage: az_check <positions> <iterations> <seed>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/az_core.h"
#include "../../master_doko_reinforcement_learning_amd/csrc/engine/encode_pi.h"
#include "../../master_doko_reinforcement_learning_amd/csrc/engine/rand_distr.h"
#include "../../oracle/encode_pi.hpp"
#include "../../oracle/az_eval.hpp"
#include "../../oracle/full_doko.hpp"

using namespace oracle;
extern "C" void or_fdo_pack(void* sp, uint8_t* out);
extern "C" void or_fdo_pack_az(void* sp, uint8_t* out);
extern "C" int or_az_search(void* sp, const float* noise, float alpha, uint32_t iters, float c, float eps, int epoch,
                            int temp_mode, float temp, uint64_t* rng_state, uint32_t* visits, float* root_priors);

int main(int argc, char** argv) {
    const int npos = argc > 1 ? atoi(argv[1]) : 40;
    const uint32_t iters = argc > 2 ? (uint32_t)atoi(argv[2]) : 200;
    const uint64_t seed = argc > 3 ? strtoull(argv[3], 0, 10) : 1;
    std::mt19937_64 pol(seed);
    // exp agreement on the synthetic logits (multiples of 1/4 in [-4, 4))
    for (int k = -16; k < 16; ++k) {
        const float x = (float)k * 0.25f;
        if (std::exp(x) != dk::az::exp_f32(x)) { printf("MISMATCH exp(%g)\n", x); return 1; }
    }
    // positions from random games (all phases, with announcements).  Along every
    // trajectory the device record (step_record) must equal the oracle's packed
    // record, and encode_pi.h must equal the oracle's encode_state_pi.
    std::vector<fdo::State> pos;
    long encoded = 0;
    for (int g = 0; (int)pos.size() < npos; ++g) {
        SmallRng deal = SmallRng::seed_from_u64(seed * 5077 + g);
        fdo::State s = fdo::new_game(deal);
        dk_az_state rec; or_fdo_pack_az(&s, (uint8_t*)&rec);
        const int stop = (int)(pol() % 60);
        for (int ply = 0; ply < 80 && s.phase != fdo::Finished; ++ply) {
            if (ply == stop) pos.push_back(s);
            dk_az_state want; or_fdo_pack_az(&s, (uint8_t*)&want);
            if (memcmp(&want, &rec, 117) != 0 || memcmp(want.ann_card, rec.ann_card, 32) != 0) {
                printf("MISMATCH record game %d ply %d\n", g, ply); return 1;
            }
            int64_t eo[311]; uint32_t ed[311];
            enc::encode_state_pi(s, eo);
            auto put = [&](uint32_t i, uint32_t v) { ed[i] = v; };
            dk::enc::encode_state_pi(rec, put);
            for (int i = 0; i < 311; ++i) if ((int64_t)ed[i] != eo[i]) { printf("MISMATCH encode game %d ply %d token %d: %u vs %lld\n", g, ply, i, ed[i], (long long)eo[i]); return 1; }
            encoded++;
            const uint64_t legal = fdo::observation_allowed_actions(s);
            int k = (int)(pol() % (uint64_t)__builtin_popcountll(legal)), a = 0;
            for (int b = 0; b < 39; ++b) if (legal >> b & 1) { if (k-- == 0) { a = b; break; } }
            fdo::play_action(s, a);
            dk::az::step_record(rec, a);
        }
    }
    if (encoded < 100) { printf("too few encoded positions\n"); return 1; }
    const int G = (int)pos.size();
    const float c = 2.5f, eps = 0.25f;
    long checked = 0;
    // the Open01 tables of the context (doko_amd.hip rd_tables)
    constexpr uint32_t K = 1u << 23;
    std::vector<float> ln01(K), pw01(K);
    auto u_of = [](uint32_t k) { return __builtin_bit_cast(float, k | 0x3F800000u) - (1.0f - FLT_EPSILON / 2.0f); };
    for (uint32_t k = 0; k < K; ++k) ln01[k] = logf(u_of(k));
    for (int run = 0; run < 8; ++run) {
        const int mode = run < 6 ? run % 3 : (run == 6 ? 2 : 0);
        const bool drawn = run >= 3;
        const float alpha = run >= 6 ? (run == 6 ? 0.1f : 0.05f) : (mode == 0 ? 0.8f : (mode == 1 ? 1.0f : 0.5f));
        if (drawn && alpha < 1.0f && alpha > 0.1f)
            for (uint32_t k = 0; k < K; ++k) pw01[k] = powf(u_of(k), 1.0f / alpha);
        const dk::rd::Open01Tab tab{pw01.data(), ln01.data()};
        const int epoch = mode == 1 ? 3 : 12;
        const float temp = 1.0f;
        std::vector<float> noise((size_t)G * 39);
        for (auto& x : noise) x = (float)(pol() % 1000) / 4000.0f;
        std::vector<uint64_t> seeds(G);
        for (auto& x : seeds) x = pol();
        // device core, batched
        const uint32_t cap_nodes = 40 + 39 * (iters + 1), cap_states = iters + 2;
        std::vector<dk::az::Node> nodes((size_t)G * cap_nodes);
        std::vector<dk_az_state> states((size_t)G * cap_states);
        std::vector<dk::az::Game> games(G);
        std::vector<dk_az_state> eval(G);
        std::vector<float> val((size_t)G * 4), logit((size_t)G * 39);
        auto mem = [&](int g) { dk::az::Mem m; m.nodes = &nodes[(size_t)g * cap_nodes]; m.states = &states[(size_t)g * cap_states];
                                m.cap_nodes = cap_nodes; m.cap_states = cap_states; return m; };
        auto network = [&](int g) { az::hash_eval(eval[g].state.raw, &val[4 * g], &logit[39 * g]); };
        for (int g = 0; g < G; ++g) {
            dk_az_state r; or_fdo_pack_az(&pos[g], (uint8_t*)&r);
            dk::az::Mem m = mem(g);
            dk::az::init(r, games[g], m, seeds[g]);
            eval[g] = r;
            network(g);
            const float* nz = &noise[39 * (size_t)g];
            float dn[39];
            if (drawn) {   // az_root_kernel with d_noise == NULL
                dk::Rng r; r.s0 = games[g].rng[0]; r.s1 = games[g].rng[1]; r.s2 = games[g].rng[2]; r.s3 = games[g].rng[3];
                dk::rd::dirichlet39(alpha, r, tab, dn);
                games[g].rng[0] = r.s0; games[g].rng[1] = r.s1; games[g].rng[2] = r.s2; games[g].rng[3] = r.s3;
                nz = dn;
            }
            dk::az::root_expand(games[g], m, &val[4 * g], &logit[39 * g], nz, eps, epoch);
        }
        for (uint32_t it = 0; it < iters; ++it) {
            for (int g = 0; g < G; ++g) { dk::az::Mem m = mem(g); dk::az::select(games[g], m, c, epoch, &eval[g]); }
            for (int g = 0; g < G; ++g) if (games[g].need_eval) network(g);
            for (int g = 0; g < G; ++g) { dk::az::Mem m = mem(g); dk::az::backup(games[g], m, &val[4 * g], &logit[39 * g]); }
        }
        for (int g = 0; g < G; ++g) {
            dk::az::Mem m = mem(g);
            if (games[g].status) { printf("CAPACITY game %d\n", g); return 1; }
            uint32_t dv[39];
            const int da = dk::az::finish(games[g], m, mode, temp, dv);
            // oracle
            uint64_t rs[4];
            { const SmallRng r = SmallRng::seed_from_u64(seeds[g]); for (int i = 0; i < 4; ++i) rs[i] = r.s[i]; }
            uint32_t ov[39]; float op[39];
            for (int a = 0; a < 39; ++a) op[a] = -1.0f;
            const int oa = or_az_search(&pos[g], drawn ? nullptr : &noise[39 * (size_t)g], alpha, iters, c, eps, epoch, mode,
                                        temp, rs, ov, op);
            for (int a = 0; a < 39; ++a)
                if (dv[a] != ov[a]) { printf("MISMATCH visits run %d game %d action %d: %u vs %u\n", run, g, a, dv[a], ov[a]); return 1; }
            const dk::az::Node root = m.nodes[0];
            for (uint32_t j = 0; j < root.nchild; ++j) {
                const dk::az::Node ch = m.nodes[root.child_base + j];
                if (memcmp(&ch.prior, &op[ch.action], 4) != 0) { printf("MISMATCH root prior run %d game %d\n", run, g); return 1; }
            }
            if (da != oa) { printf("MISMATCH action run %d game %d: %d vs %d\n", run, g, da, oa); return 1; }
            for (int i = 0; i < 4; ++i) if (games[g].rng[i] != rs[i]) { printf("MISMATCH rng run %d game %d\n", run, g); return 1; }
            checked++;
        }
    }
    printf("OK %ld searches\n", checked);
    return 0;
}
