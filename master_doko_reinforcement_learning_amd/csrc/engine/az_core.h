// AlphaZero PUCT search over the full-doko AZ env, batched over games: one
// lane per game tree, the network evaluated between launches.
// Reference: rs-doko-alpha-zero/src/alpha_zero/mcts/async_mcts.rs:71-406
// (expand_root_node, mcts_search), mcts/mcts.rs:23-420 (expand_node,
// select_action, backpropagate, select_promising_node, find_best_child,
// puct_for_child), mcts/node.rs:209-380, env/envs/full_doko/full_doko.rs:15-172,
// utils/float_vec_utils.rs:3-17 (softmax), utils/rot_arr.rs.
//
// The reference's mcts_search is sequential per game and awaits the network
// for every leaf; its batch processor gathers leaves of many concurrent games.
// Here that batch is explicit: one iteration of G games is
//     select  (this file, one lane per game) -> leaf states, packed
//     network (PyTorch on the same stream)   -> value[G][4], logits[G][39]
//     backup  (this file)                    -> priors of the leaf's children, value backed up
// The trees are exact: which nodes exist, every f32 operation on the
// statistics, and the order of the RNG draws are the reference's.  One layout
// change: a child's state is computed when the child first becomes the leaf
// (from its parent's state and its action), not when its parent is expanded.
// take_action is deterministic and a child's state is read only once it is a
// leaf, so this changes no value, and it saves up to eleven state transitions
// per expansion.
//
// Node records (48 B) of one game form a contiguous region; the children of a
// node are one block in ascending action order (the reference's
// children[action] array order).  win[] is the RotArr win_score by absolute
// player (every RotArr access is get_for_i/index_for_i, so the rotation is
// only a storage convention).  States are kept as dk_az_state records (the
// packed state, card history included, plus the announcement occurrence list):
// they are the network's input (encode_pi.h).
#pragma once
#include <math.h>
#include "fdo_engine.h"
#include "rng.h"

namespace dk {
namespace az {

static constexpr uint64_t ANN_BITS = 0x1FULL << 33;   // AnnouncementReContra .. AnnouncementBlack
static constexpr int MIN_EPOCH = 10;                  // full_doko.rs:23
static constexpr uint32_t NO_NODE = 0xFFFFFFFFu;
static constexpr float F32_MIN = -3.40282347e+38f;

enum : uint32_t { NF_TERMINAL = 1u, NF_STATE = 2u };

struct alignas(16) Node {
    float win[4];          // win_score by absolute player
    uint32_t visits;
    float prior;
    uint32_t child_base;   // first child slot (nchild > 0)
    uint32_t parent;       // NO_NODE for the root
    uint32_t state;        // state slot (flags & NF_STATE)
    uint8_t nchild, action, player, flags;
    uint32_t pad[2];
};

// Per-game search record.
struct Game {
    uint64_t rng[4];
    uint32_t leaf;         // the leaf selected in the current iteration
    uint32_t next_slot;
    uint32_t next_state;
    uint32_t need_eval;    // 1: the leaf's network output is consumed by the backup
    uint32_t status;       // 0 ok, 1 capacity
    uint32_t pad[3];
};

// exp for the softmax.  Rust's f32::exp is libm expf; (float)exp((double)x)
// rounds the (sub-ulp accurate) double result once, and agrees with glibc's
// expf wherever the tests check it.
DK_HD float exp_f32(float x) { return (float)exp((double)x); }

// observation.allowed_actions_current_player, announcements removed for the
// secondary (non-root) expansions or early epochs (full_doko.rs:80-101)
DK_HD uint64_t allowed(const dk_fdo_state& s, bool secondary, int epoch) {
    fdo::Work w; fdo::unpack(s, w);
    uint64_t a = fdo::legal_actions(w);
    if (secondary || epoch < MIN_EPOCH) a &= ~ANN_BITS;
    return a;
}
DK_HD bool terminal(const dk_fdo_state& s) { return s.phase == fdo::PH_FINISHED; }
DK_HD int current_player(const dk_fdo_state& s) { return s.current_player == DK_NONE ? 0 : (int)s.current_player; }

// FdoState::play_action on a record: an announcement action also appends its
// occurrence (internal_play_announcement, announcement.rs:178-215).
DK_HD void step_record(dk_az_state& r, int a) {
    dk_fdo_state& s = r.state.fdo;
    if (a >= 33 && a <= 37 && r.ann_n < 12) {
        r.ann_card[r.ann_n] = s.card_index;
        r.ann_code[r.ann_n] = (uint8_t)((s.current_player << 4) | (uint32_t)(a - 33));
        r.ann_n += 1;
    }
    fdo::step_packed(s, a);
}

// take_action_by_action_index(action, skip_single = true) (full_doko.rs:121-157):
// after the action, forced plies (one legal action once announcements are
// removed) are played too.
DK_HD void take_action(dk_az_state& r, int a) {
    dk_fdo_state& s = r.state.fdo;
    step_record(r, a);
    for (int guard = 0; guard < 256; ++guard) {
        if (s.phase == fdo::PH_FINISHED) break;
        fdo::Work w; fdo::unpack(s, w);
        const uint64_t al = fdo::legal_actions(w) & ~ANN_BITS;
        if (popc64(al) != 1) break;
        step_record(r, ctz64(al));
    }
}

// rewards_or_none: player_points / 8 (full_doko.rs:54-71), absolute order
DK_HD void rewards(const dk_fdo_state& s, float r[4]) {
    fdo::Work w; fdo::unpack(s, w);
    int pts[4];
    fdo::score(w, pts);
    for (int p = 0; p < 4; ++p) r[p] = (float)pts[p] / 8.0f;
}

// softmax_inplace (float_vec_utils.rs:3-17): exp, sequential sum, divide
DK_HD void softmax(float* d, int n) {
    float sum = 0.0f;
    for (int i = 0; i < n; ++i) d[i] = exp_f32(d[i]);
    for (int i = 0; i < n; ++i) sum += d[i];
    for (int i = 0; i < n; ++i) d[i] /= sum;
}

// Memory of one game: node region, state region.
struct Mem {
    Node* nodes;
    dk_az_state* states;
    uint32_t cap_nodes, cap_states;
};

// new_root_node (node.rs:209-244): state 0, no children yet.
DK_HD void init(const dk_az_state& root, Game& g, Mem& m, uint64_t seed) {
    const Rng r = Rng::seed_from_u64(seed);
    g.rng[0] = r.s0; g.rng[1] = r.s1; g.rng[2] = r.s2; g.rng[3] = r.s3;
    Node n;
    for (int p = 0; p < 4; ++p) n.win[p] = 0.0f;
    n.visits = 0; n.prior = 0.0f; n.child_base = 0; n.parent = NO_NODE; n.state = 0; n.nchild = 0;
    n.action = 0xFF; n.player = (uint8_t)current_player(root.state.fdo);
    n.flags = (uint8_t)(NF_STATE | (terminal(root.state.fdo) ? NF_TERMINAL : 0u));
    n.pad[0] = n.pad[1] = 0;
    m.nodes[0] = n;
    m.states[0] = root;
    g.leaf = 0; g.next_slot = 1; g.next_state = 1; g.need_eval = 1; g.status = 0;
}

// Children of node `idx` for the actions of `mask` (ascending), priors given.
DK_HD bool add_children(Game& g, Mem& m, uint32_t idx, uint64_t mask, const float* priors) {
    const uint32_t k = (uint32_t)popc64(mask);
    if (g.next_slot + k > m.cap_nodes) { g.status = 1; return false; }
    const uint32_t base = g.next_slot;
    g.next_slot += k;
    uint32_t i = 0;
    while (mask) {
        const int a = ctz64(mask);
        mask &= mask - 1;
        Node c;
        for (int p = 0; p < 4; ++p) c.win[p] = 0.0f;
        c.visits = 0; c.prior = priors ? priors[i] : 0.0f; c.child_base = 0; c.parent = idx; c.state = 0;
        c.nchild = 0; c.action = (uint8_t)a; c.player = 0; c.flags = 0; c.pad[0] = c.pad[1] = 0;
        m.nodes[base + i] = c;
        ++i;
    }
    m.nodes[idx].child_base = base;
    m.nodes[idx].nchild = (uint8_t)k;
    return true;
}

// expand_root_node (async_mcts.rs:71-196) with the root's network output.
// value is from the root player's POV (RotArr::new_from_pov); noise = the
// Dirichlet sample (an input: see the oracle's note).
DK_HD void root_expand(Game& g, Mem& m, const float value[4], const float logits[39], const float noise[39], float eps,
                       int epoch) {
    const dk_fdo_state& s = m.states[0].state.fdo;
    const uint64_t al = allowed(s, false, epoch);
    float probs[39];
    for (int i = 0; i < 39; ++i) probs[i] = logits[i];
    softmax(probs, 39);
    for (int i = 0; i < 39; ++i) probs[i] *= (1.0f - eps);
    for (int i = 0; i < 39; ++i) probs[i] += noise[i] * eps;
    float sel[39];
    int n = 0;
    for (int a = 0; a < 39; ++a) if ((al >> a) & 1) sel[n++] = probs[a];
    float x = 0.0f;
    for (int i = 0; i < n; ++i) x += sel[i];
    for (int i = 0; i < n; ++i) sel[i] /= x;
    add_children(g, m, 0, al, sel);
    Node& r = m.nodes[0];
    r.visits = 1;
    const int cp = r.player;
    for (int p = 0; p < 4; ++p) r.win[p] = value[(p - cp + 4) & 3];
}

// puct_for_child (mcts.rs:382-420) with value_for_player (node.rs:361-380);
// the virtual loss and virtual visits are zero in this search.
DK_HD float puct(const Node& c, int parent_player, float sqrt_pv, float cexp) {
    const float value = c.visits == 0 ? 0.0f : (c.win[parent_player] + 0.0f) / (float)c.visits;
    const float cv = (float)c.visits + 0.0f;
    const float exploration = c.prior * sqrt_pv / (1.0f + cv);
    return value + cexp * exploration;
}

// One iteration's selection (select_promising_node, mcts.rs:306-380) and the
// expansion of the leaf (expand_node, mcts.rs:23-74).  Returns true when the
// leaf needs the network (non-terminal); the leaf's packed state goes to *eval.
DK_HD bool select(Game& g, Mem& m, float cexp, int epoch, dk_az_state* eval) {
    uint32_t idx = 0;
    for (int guard = 0; guard < 4096; ++guard) {
        const Node nd = m.nodes[idx];
        if (nd.nchild == 0) break;
        const float sqrt_pv = sqrtf((float)nd.visits + 0.0f);
        float best = F32_MIN;
        uint32_t best_child = NO_NODE;
        for (uint32_t j = 0; j < nd.nchild; ++j) {
            const float sc = puct(m.nodes[nd.child_base + j], nd.player, sqrt_pv, cexp);
            if (sc > best) { best = sc; best_child = nd.child_base + j; }
        }
        if (best_child == NO_NODE) break;
        idx = best_child;
    }
    Node& L = m.nodes[idx];
    if (!(L.flags & NF_STATE)) {
        if (g.next_state >= m.cap_states) { g.status = 1; g.need_eval = 0; return false; }
        dk_az_state st = m.states[m.nodes[L.parent].state];
        take_action(st, L.action);
        L.state = g.next_state++;
        m.states[L.state] = st;
        L.player = (uint8_t)current_player(st.state.fdo);
        L.flags = (uint8_t)(NF_STATE | (terminal(st.state.fdo) ? NF_TERMINAL : 0u));
    }
    g.leaf = idx;
    const dk_az_state& ls = m.states[L.state];
    if (L.flags & NF_TERMINAL) { g.need_eval = 0; return false; }
    if (!add_children(g, m, idx, allowed(ls.state.fdo, true, epoch), nullptr)) { g.need_eval = 0; return false; }
    if (eval) *eval = ls;
    g.need_eval = 1;
    return true;
}

// The leaf's network output -> priors of its children (softmax over the
// allowed actions' logits, async_mcts.rs:307-331), then backpropagate
// (mcts.rs:250-280): visits += 1 and win += rewards on the leaf..root path.
DK_HD void backup(Game& g, Mem& m, const float value[4], const float logits[39]) {
    if (g.status) return;
    Node& L = m.nodes[g.leaf];
    float r[4];
    if (g.need_eval) {
        float pr[39];
        const uint32_t n = L.nchild;
        for (uint32_t j = 0; j < n; ++j) pr[j] = logits[m.nodes[L.child_base + j].action];
        softmax(pr, (int)n);
        for (uint32_t j = 0; j < n; ++j) m.nodes[L.child_base + j].prior = pr[j];
        const int cp = L.player;
        for (int p = 0; p < 4; ++p) r[p] = value[(p - cp + 4) & 3];
    } else {
        rewards(m.states[L.state].state.fdo, r);
    }
    for (uint32_t t = g.leaf; t != NO_NODE; t = m.nodes[t].parent) {
        Node& n = m.nodes[t];
        n.visits += 1;
        for (int p = 0; p < 4; ++p) n.win[p] = n.win[p] + r[p];
    }
}

// End of mcts_search: random_bool(1/5000) (async_mcts.rs:347), then
// select_action (mcts.rs:185-248).  temp_mode 0 = None (greedy, last maximum
// of max_by_key), 1 = infinite (uniform choose), 2 = finite temperature
// (WeightedIndex over visits^(1/T), UniformFloat<f32>; parity unpinned).
DK_HD int finish(Game& g, Mem& m, int temp_mode, float temperature, uint32_t visits39[39]) {
    Rng rng; rng.s0 = g.rng[0]; rng.s1 = g.rng[1]; rng.s2 = g.rng[2]; rng.s3 = g.rng[3];
    (void)rng.next_u64();
    for (int a = 0; a < 39; ++a) visits39[a] = 0;
    const Node r = m.nodes[0];
    int action = -1;
    const uint32_t n = r.nchild;
    if (n > 0) {
        for (uint32_t j = 0; j < n; ++j) {
            const Node c = m.nodes[r.child_base + j];
            visits39[c.action] = c.visits;
        }
        if (temp_mode == 0) {
            uint32_t best = 0;
            for (uint32_t j = 1; j < n; ++j) if (m.nodes[r.child_base + j].visits >= m.nodes[r.child_base + best].visits) best = j;
            action = m.nodes[r.child_base + best].action;
        } else if (temp_mode == 1) {
            action = m.nodes[r.child_base + (n >= 1 ? rng.range_u32(n) : 0)].action;
        } else {
            float cum[39];
            float total = powf((float)m.nodes[r.child_base].visits, 1.0f / temperature);
            for (uint32_t j = 1; j < n; ++j) {
                cum[j - 1] = total;
                total += powf((float)m.nodes[r.child_base + j].visits, 1.0f / temperature);
            }
            const float max_rand = 1.0f - 1.1920929e-07f;
            float scale = total;
            for (int guard = 0; guard < 64 && scale * max_rand >= total; ++guard)
                scale = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, scale) - 1u);
            const float v12 = __builtin_bit_cast(float, (rng.next_u32() >> 9) | 0x3F800000u);
            const float chosen = (v12 - 1.0f) * scale + 0.0f;
            uint32_t k = 0;
            while (k + 1 < n && cum[k] <= chosen) ++k;
            action = m.nodes[r.child_base + k].action;
        }
    }
    g.rng[0] = rng.s0; g.rng[1] = rng.s1; g.rng[2] = rng.s2; g.rng[3] = rng.s3;
    return action;
}

}  // namespace az
}  // namespace dk
