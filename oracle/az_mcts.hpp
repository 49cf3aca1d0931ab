// ORACLE — test infrastructure only. Never linked into the product library.
//
// Restatement of the AlphaZero PUCT search of rs-doko-alpha-zero over the
// full-doko AZ env:
//   env     FdoAzEnvState            rs-doko-alpha-zero/src/env/envs/full_doko/full_doko.rs:15-172
//   search  mcts_search              rs-doko-alpha-zero/src/alpha_zero/mcts/async_mcts.rs:224-406
//           expand_root_node         async_mcts.rs:71-196
//           select_promising_node,
//           find_best_child, puct    alpha_zero/mcts/mcts.rs:306-420
//           expand_node              mcts.rs:23-74
//           backpropagate            mcts.rs:250-280
//           select_action            mcts.rs:185-248
//   nodes   AzNode, value_for_player alpha_zero/mcts/node.rs:31-62, 209-380
//   floats  softmax_inplace          alpha_zero/utils/float_vec_utils.rs:3-17 (exp, sequential sum, divide)
//           RotArr                   alpha_zero/utils/rot_arr.rs (kept here as absolute-player arrays:
//                                    every RotArr read/write goes through get_for_i / index_for_i)
// The network is a callback (the batch processor's `process`): it returns the
// value vector from the evaluated state's current player's point of view and
// 39 policy logits.  The Dirichlet noise of the root is drawn from the search's
// SmallRng as the reference draws it (Dirichlet::new([alpha; 39]).sample(rng),
// async_mcts.rs:111-113, rand_distr 0.5.1: rand_distr05.hpp, parity unpinned), after
// the root's network call and before every other draw of the search: random_bool(1/5000)
// at the end (async_mcts.rs:347), then the temperature pick (mcts.rs:235).  A caller may
// pass the noise instead (the search then draws none).
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <vector>

#include "full_doko.hpp"
#include "rand09.hpp"
#include "rand_distr05.hpp"

namespace oracle {
namespace az {

static constexpr uint64_t ANN_BITS = (1ULL << fdo::A_AnnouncementReContra) | (1ULL << fdo::A_AnnouncementNo90) |
                                     (1ULL << fdo::A_AnnouncementNo60) | (1ULL << fdo::A_AnnouncementNo30) |
                                     (1ULL << fdo::A_AnnouncementBlack);
static constexpr int MIN_EPOCH = 10;   // full_doko.rs:23

// FdoAzEnvState (full_doko.rs:15-172)
struct Env {
    fdo::State doko;
    int current_player() const { return doko.current_player < 0 ? 0 : doko.current_player; }   // :46-48
    bool is_terminal() const { return doko.phase == fdo::Finished; }                           // :50-52
    bool rewards(float out[4]) const {                                                         // :54-71
        if (!doko.has_stats) return false;
        for (int p = 0; p < 4; ++p) out[p] = (float)doko.stats.player_points[p] / 8.0f;
        return true;
    }
    uint64_t allowed(bool is_secondary, int epoch) const {                                     // :80-101
        uint64_t a = fdo::observation_allowed_actions(doko);
        if (is_secondary || epoch < MIN_EPOCH) a &= ~ANN_BITS;
        return a;
    }
    Env take_action(int action, bool skip_single) const {                                      // :121-157
        Env e = *this;
        fdo::play_action(e.doko, action);
        if (skip_single) {
            for (;;) {
                if (e.doko.phase == fdo::Finished) break;
                const uint64_t a = fdo::observation_allowed_actions(e.doko) & ~ANN_BITS;
                if (__builtin_popcountll(a) == 1) fdo::play_action(e.doko, __builtin_ctzll(a));
                else break;
            }
        }
        return e;
    }
};

// value from the evaluated state's current player's POV, logits over the 39 actions
using Evaluator = std::function<void(const Env&, float value_pov[4], float logits[39])>;

struct Node {
    int state = -1;            // index into the state arena (-1 after the leaf's evaluation frees it)
    bool is_terminal = false;
    int current_player = 0;
    int last_action = -1;
    float prior = 0.0f;
    uint32_t visits = 0;
    float win[4] = {0, 0, 0, 0};   // RotArr win_score, by absolute player
    int children[39];
    bool has_children = false;
    int parent = -1;
    Node() { for (int& c : children) c = -1; }
};

struct Options {
    float c = 1.0f;                 // puct_exploration_constant
    float dirichlet_epsilon = 0.25f;
    float dirichlet_alpha = 0.8f;   // used when the caller passes no noise
    int epoch = MIN_EPOCH;          // >= MIN_EPOCH: announcements offered at the root
    bool has_temperature = false;   // None -> greedy (max_by_key visits)
    float temperature = 1.0f;       // +inf -> uniform choose
};

// softmax_inplace (float_vec_utils.rs:3-17)
inline void softmax(float* d, int n) {
    for (int i = 0; i < n; ++i) d[i] = std::exp(d[i]);
    float sum = 0.0f;
    for (int i = 0; i < n; ++i) sum += d[i];
    for (int i = 0; i < n; ++i) d[i] /= sum;
}

struct Search {
    std::vector<Node> nodes;
    std::vector<Env> states;

    int new_node(const Env& st, float prior, int parent, int last_action) {   // node.rs:209-307
        Node n;
        n.is_terminal = st.is_terminal();
        n.current_player = st.current_player();
        n.last_action = last_action;
        n.prior = prior;
        n.parent = parent;
        n.state = (int)states.size();
        states.push_back(st);
        nodes.push_back(n);
        return (int)nodes.size() - 1;
    }

    // value_for_player (node.rs:361-380), virtual loss 0 in this search
    float value_for_player(const Node& n, int player) const {
        if (n.visits == 0) return 0.0f;
        return (n.win[player] + 0.0f) / (float)n.visits;
    }
    // puct_for_child (mcts.rs:382-420)
    float puct(const Node& parent, const Node& child, float c) const {
        const float value = value_for_player(child, parent.current_player);
        const float child_visits = (float)child.visits + 0.0f;
        const float parent_visits = (float)parent.visits + 0.0f;
        const float exploration = child.prior * std::sqrt(parent_visits) / (1.0f + child_visits);
        return value + c * exploration;
    }
    // find_best_child (mcts.rs:343-380): first strict maximum, children in action order
    int find_best_child(int idx, float c) const {
        float best = -3.40282347e+38f;   // f32::MIN
        int best_child = -1;
        for (int a = 0; a < 39; ++a) {
            const int ch = nodes[idx].children[a];
            if (ch < 0) continue;
            const float s = puct(nodes[idx], nodes[ch], c);
            if (s > best) { best = s; best_child = ch; }
        }
        return best_child;
    }
    // expand_node (mcts.rs:23-74)
    void expand_node(int idx, int epoch) {
        const uint64_t allowed = states[nodes[idx].state].allowed(true, epoch);
        for (int a = 0; a < 39; ++a) {
            if (!(allowed >> a & 1)) continue;
            const Env child = states[nodes[idx].state].take_action(a, true);
            const int ch = new_node(child, 0.0f, idx, a);
            nodes[idx].children[a] = ch;
            nodes[idx].has_children = true;
        }
    }
    void backpropagate(int idx, const float r[4]) {   // mcts.rs:250-280
        for (int t = idx; t >= 0; t = nodes[t].parent) {
            nodes[t].visits += 1;
            for (int p = 0; p < 4; ++p) nodes[t].win[p] = nodes[t].win[p] + r[p];
        }
    }

    // mcts_search (async_mcts.rs:224-406) -> (chosen action, visits by action)
    int search(const Env& root_state, const Evaluator& eval, const float noise[39], uint32_t iterations,
               const Options& o, SmallRng& rng, uint32_t visits_out[39], float* root_priors_out = nullptr) {
        nodes.clear(); states.clear();
        nodes.reserve(iterations * 12 + 64); states.reserve(iterations * 12 + 64);
        const int root = new_node(root_state, 0.0f, -1, -1);
        // expand_root_node (async_mcts.rs:71-196)
        {
            const uint64_t allowed = root_state.allowed(false, o.epoch);
            float value[4], probs[39];
            eval(root_state, value, probs);
            softmax(probs, 39);
            float drawn[39];
            if (!noise) {   // Dirichlet::new([dirichlet_alpha; 39]).unwrap().sample(rng)
                float al[39];
                for (float& a : al) a = o.dirichlet_alpha;
                if (!rdist::dirichlet(al, 39, rng, drawn)) return -2;   // (the reference's unwrap panics)
                noise = drawn;
            }
            float nz[39];
            for (int i = 0; i < 39; ++i) probs[i] *= (1.0f - o.dirichlet_epsilon);
            for (int i = 0; i < 39; ++i) nz[i] = noise[i] * o.dirichlet_epsilon;
            for (int i = 0; i < 39; ++i) probs[i] += nz[i];
            float sel[39]; int n = 0;
            for (int a = 0; a < 39; ++a) if (allowed >> a & 1) sel[n++] = probs[a];
            float x = 0.0f;
            for (int i = 0; i < n; ++i) x += sel[i];
            for (int i = 0; i < n; ++i) sel[i] /= x;
            int i = 0;
            for (int a = 0; a < 39; ++a) {
                if (!(allowed >> a & 1)) continue;
                if (root_priors_out) root_priors_out[a] = sel[i];
                const int ch = new_node(root_state.take_action(a, true), sel[i++], root, a);
                nodes[root].children[a] = ch;
                nodes[root].has_children = true;
            }
            nodes[root].visits = 1;
            const int cp = root_state.current_player();
            for (int p = 0; p < 4; ++p) nodes[root].win[p] = value[(p - cp + 4) % 4];   // RotArr::new_from_pov
        }
        for (uint32_t it = 0; it < iterations; ++it) {
            int node = root;   // select_promising_node (mcts.rs:306-350)
            while (nodes[node].has_children) {
                const int nx = find_best_child(node, o.c);
                if (nx < 0) break;
                node = nx;
            }
            if (!nodes[node].is_terminal) expand_node(node, o.epoch);
            float r[4];
            if (nodes[node].is_terminal) {
                states[nodes[node].state].rewards(r);   // RotArr::new_from_0: absolute order
            } else {
                const Env& st = states[nodes[node].state];
                const uint64_t allowed = st.allowed(true, o.epoch);
                float value[4], logits[39];
                eval(st, value, logits);
                float pr[39]; int n = 0;
                for (int a = 0; a < 39; ++a) if (allowed >> a & 1) pr[n++] = logits[a];
                softmax(pr, n);
                int i = 0;
                for (int a = 0; a < 39; ++a) {
                    const int ch = nodes[node].children[a];
                    if (ch < 0) continue;
                    nodes[ch].prior = pr[i++];
                }
                const int cp = nodes[node].current_player;
                for (int p = 0; p < 4; ++p) r[p] = value[(p - cp + 4) % 4];   // RotArr::new_from_pov
            }
            backpropagate(node, r);
        }
        (void)rng.random_bool(1.0 / 5000.0);   // async_mcts.rs:347
        for (int a = 0; a < 39; ++a) {
            const int ch = nodes[root].children[a];
            visits_out[a] = ch < 0 ? 0u : nodes[ch].visits;
        }
        return select_action(root, o, rng);
    }

    // select_action (mcts.rs:185-248)
    int select_action(int root, const Options& o, SmallRng& rng) const {
        int idx[39]; uint32_t cnt[39]; int n = 0;
        for (int a = 0; a < 39; ++a) {
            const int ch = nodes[root].children[a];
            if (ch < 0) continue;
            idx[n] = a; cnt[n] = nodes[ch].visits; n++;
        }
        if (n == 0) return -1;
        if (!o.has_temperature) {   // max_by_key: the LAST maximum
            int best = 0;
            for (int i = 1; i < n; ++i) if (cnt[i] >= cnt[best]) best = i;
            return idx[best];
        }
        if (std::isinf(o.temperature)) return idx[rng.random_range_usize(0, (size_t)n)];   // IndexedRandom::choose
        // WeightedIndex over visits^(1/T) (rand 0.9 distr/weighted/weighted_index.rs), sampled
        // through UniformFloat<f32>::new(0, total) (distr/uniform_float.rs); parity unpinned.
        float w[39];
        for (int i = 0; i < n; ++i) w[i] = std::pow((float)cnt[i], 1.0f / o.temperature);
        float cum[39]; float total = w[0];
        for (int i = 1; i < n; ++i) { cum[i - 1] = total; total += w[i]; }
        const float max_rand = 1.0f - 1.1920929e-07f;
        float scale = total - 0.0f;
        while (scale * max_rand + 0.0f >= total) scale = std::nextafter(scale, 0.0f);
        const uint32_t bits = (rng.next_u32() >> 9) | 0x3F800000u;
        float v12; std::memcpy(&v12, &bits, 4);
        const float chosen = (v12 - 1.0f) * scale + 0.0f;
        int k = 0;
        while (k < n - 1 && cum[k] <= chosen) ++k;   // partition_point(|w| w <= chosen)
        return idx[k];
    }
};

}  // namespace az
}  // namespace oracle
