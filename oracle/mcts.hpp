// ORACLE — test infrastructure only. Never linked into the product library.
//
// Faithful restatement of the rs-doko-mcts UCT search
// (rs-doko-mcts/src/mcts/mcts.rs:45-321, mcts/node.rs:138-277), generic over
// the env adapters of full_doko.hpp / doko.hpp / ttt.hpp.  Like the reference it
// keeps one full state per node (state arena), recomputes the sibling
// min/max-normalised Q for every child (O(B^2) per level) and consumes the
// SmallRng in the reference's order:
//     per iteration: [expansion pick] -> [one draw per rollout ply]
//     after the last iteration: random_bool(1/1000)  (mcts.rs:231)
// The counters (children scanned, path depth, child-slot demand) feed the
// algorithmic-bytes model in DESIGN.md.
#pragma once
#include <cmath>
#include <cstdint>
#include <vector>
#include "rand09.hpp"

namespace oracle {

struct SearchCounters {
    uint64_t iterations = 0;
    uint64_t children_scanned = 0;   // sum over iterations of children examined by find_best_child
    uint64_t path_nodes = 0;         // sum over iterations of nodes on the backprop path
    uint64_t max_depth = 0;
    uint64_t nodes = 0;              // nodes allocated (incl. root)
    uint64_t child_slots = 0;        // sum of popcount(allowed) over nodes that got >=1 child (+1 root)
    uint64_t rollout_plies = 0;
    // deepest selection path of the device kernel's path stack (search_core.h): a forced
    // chain (single-action nodes) below its head costs one entry, like the skip pointer
    uint64_t max_path_entries = 0;
    // optional: per iteration, the child count of every branching pick (>= 2 children),
    // then a 0 (design data for the device kernel's pick width; tools/pick_width.py)
    std::vector<uint8_t>* pick_trace = nullptr;
};

struct MoveOut { int action; uint64_t visits; double value; };

template <class Env>
struct Mcts {
    struct Node {
        int state;                 // index into the state arena
        bool is_terminal;
        int current_player;
        int last_action;
        uint64_t visits = 0;
        double win_score = 0.0;
        uint64_t unexpanded;
        int n_actions;             // popcount of the allowed actions at creation (for the counters)
        std::vector<int> children;
        int parent;
    };
    std::vector<Node> nodes;
    std::vector<Env> states;

    // node.rs:202-235
    double min_max_normalized_q(const Node& self, int child) const {
        if (self.children.empty()) return 1.0;
        double min_q = INFINITY, max_q = -INFINITY;
        for (int c : self.children) {
            const Node& n = nodes[c];
            const double q = n.visits > 0 ? n.win_score / (double)n.visits : 0.0;
            if (q < min_q) min_q = q;
            if (q > max_q) max_q = q;
        }
        if (std::fabs(max_q - min_q) < 2.220446049250313e-16) return 1.0;
        const Node& ch = nodes[child];
        const double q = ch.visits > 0 ? ch.win_score / (double)ch.visits : 0.0;
        return 2.0 * (q - min_q) / (max_q - min_q) - 1.0;
    }
    // node.rs:238-254
    double uct(int idx, uint64_t total_visits, double c) const {
        const Node& n = nodes[idx];
        if (n.parent < 0) return 0.0;
        if (n.visits == 0) return INFINITY;
        const double norm_q = min_max_normalized_q(nodes[n.parent], idx);
        return norm_q + c * std::sqrt(std::log((double)total_visits) / (double)n.visits);
    }
    // node.rs:258-277
    int find_best_child(int idx, double c, SearchCounters* ctr) const {
        double best = -INFINITY; int best_child = -1;
        const Node& self = nodes[idx];
        for (int ch : self.children) {
            if (ctr) ctr->children_scanned++;
            const double u = uct(ch, self.visits, c);
            if (u > best) { best = u; best_child = ch; }
        }
        return best_child;
    }
    // node.rs:138-200
    int new_node(const Env& st, int parent, bool first) {
        Node n;
        n.is_terminal = st.is_terminal();
        n.current_player = st.current_player();
        n.last_action = st.last_action;
        n.state = (int)states.size();
        states.push_back(st);
        n.unexpanded = states.back().allowed_actions(first);
        n.n_actions = __builtin_popcountll(n.unexpanded);
        n.parent = parent;
        nodes.push_back(n);
        return (int)nodes.size() - 1;
    }

    static uint64_t random_single(uint64_t mask, SmallRng& rng) {
        const uint32_t n = (uint32_t)__builtin_popcountll(mask);
        const uint32_t index = rng.random_range_u32(0, n);
        uint64_t r = index;
        for (int b = 63; b >= 0; --b) if (mask >> b & 1) { if (r == 0) return 1ULL << b; --r; }
        return 0;
    }

    // mcts.rs:172-249
    std::vector<MoveOut> search(const Env& root_state, double c, uint64_t iterations, SmallRng& rng, SearchCounters* ctr) {
        nodes.clear(); states.clear();
        nodes.reserve(iterations + 1); states.reserve(iterations + 1);
        const int root = new_node(root_state, -1, true);
        if (ctr) { ctr->nodes = 1; ctr->child_slots = 1; }
        for (uint64_t it = 0; it < iterations; ++it) {
            // select_promising_node (mcts.rs:45-61)
            int node = root; uint64_t depth = 0, entries = 0;
            while (!nodes[node].children.empty()) {
                if (nodes[node].unexpanded != 0) break;
                const Node& nd = nodes[node];
                const bool forced = nd.n_actions == 1;
                const bool head = nd.parent == root || (nd.parent >= 0 && nodes[nd.parent].n_actions >= 2);
                if (!(node != root && forced && !head)) entries++;
                if (ctr && ctr->pick_trace && nd.children.size() >= 2) ctr->pick_trace->push_back((uint8_t)nd.children.size());
                node = find_best_child(node, c, ctr);
                depth++;
            }
            int explore = node;
            if (nodes[node].unexpanded != 0) {
                // expand_single (mcts.rs:63-102)
                const uint64_t bit = random_single(nodes[node].unexpanded, rng);
                if (ctr && nodes[node].children.empty()) ctr->child_slots += (uint64_t)__builtin_popcountll(nodes[node].unexpanded);
                nodes[node].unexpanded &= ~bit;
                const Env child_state = states[nodes[node].state].by_action(__builtin_ctzll(bit));
                const int child = new_node(child_state, node, false);
                nodes[node].children.push_back(child);
                explore = child;
                depth++;
                entries++;
                if (ctr) ctr->nodes++;
            }
            double result[4];
            states[nodes[explore].state].random_rollout(rng, result);
            // backpropagate (mcts.rs:142-166)
            int t = explore; uint64_t path = 0;
            for (;;) {
                const int p = nodes[t].parent;
                nodes[t].visits += 1;
                path++;
                if (p < 0) break;
                nodes[t].win_score += result[nodes[p].current_player];
                t = p;
            }
            if (ctr && ctr->pick_trace) ctr->pick_trace->push_back(0);
            if (ctr) { ctr->iterations++; ctr->path_nodes += path; if (depth > ctr->max_depth) ctr->max_depth = depth;
                       if (entries > ctr->max_path_entries) ctr->max_path_entries = entries; }
            if (it == iterations - 1) (void)rng.random_bool((double)(1.0f / 1000.0f));
        }
        std::vector<MoveOut> moves;
        for (int ch : nodes[root].children)
            moves.push_back(MoveOut{nodes[ch].last_action, nodes[ch].visits, nodes[ch].win_score / (double)nodes[ch].visits});
        return moves;
    }
};

// rs-doko-evaluator/src/full_doko/policy/mcts_policy.rs:95-111: visits/values
// by action index, best = max_by_key(visits) (the LAST maximum on ties).
inline int moves_to_arrays(const std::vector<MoveOut>& moves, uint32_t* visits, double* values, int n_actions) {
    for (int i = 0; i < n_actions; ++i) { visits[i] = 0; values[i] = 0.0; }
    int best = -1; uint64_t bv = 0;
    for (const MoveOut& m : moves) {
        visits[m.action] = (uint32_t)m.visits;
        values[m.action] = m.value;
        if (best < 0 || m.visits >= bv) { best = m.action; bv = m.visits; }
    }
    return best;
}

}  // namespace oracle
