// One UCT search per root with the reference's sequential semantics
// (rs-doko-mcts/src/mcts/mcts.rs:45-249, node.rs:138-277):
//   select  : descend while the node has children and no unexpanded action;
//             child = first strict maximum of  nq + c*sqrt(ln(N)/n)  where
//             nq is the sibling min/max-normalised mean (1.0 if the spread < eps)
//   expand  : one uniformly drawn unexpanded action (Bitflag::random_single)
//   rollout : random playout of the env adapter
//   backup  : visits += 1 on every path node; win_score += r[parent.player]
//   end     : one random_bool(1/1000) draw (mcts.rs:231)
//
// MI355X layout (not the reference's pointer tree): every node owns a
// contiguous child block reserved at its first expansion (size = number of
// actions it allows), so a level's children are scanned with independent
// 8-byte loads; visits and the integer-exact win_score share one u64
// (visits low, win_score high) updated by a single fire-and-forget atomic add;
// node states live in a per-root pool (the reference's state arena).  The
// select path (slot + parent player) is kept in LDS.  Sibling min/max is
// computed once per level (identical values to the reference's per-child
// recomputation).  ln(N) comes from a host-built table of glibc `log`
// values, which is what Rust's f64::ln calls, so UCT values are bit-exact.
#pragma once
#include <math.h>
#include "common.h"
#include "rng.h"

namespace dk {

struct NodeMeta {
    uint64_t unexpanded;   // actions not yet expanded
    uint32_t child_base;   // first slot of the child block (0 = none yet)
    uint32_t state_idx;    // index into the state pool
    uint32_t parent;       // parent slot (0xFFFFFFFF for the root)
    uint8_t nchild;        // children expanded so far (block prefix)
    uint8_t action;        // action that led here
    uint8_t player;        // current_player of this node's state
    uint8_t flags;         // bit0 terminal
    uint64_t pad;
};

DK_HD int sel4i(const int r[4], int p) { return p == 0 ? r[0] : (p == 1 ? r[1] : (p == 2 ? r[2] : r[3])); }

static constexpr double DK_F64_EPSILON = 2.220446049250313e-16;

// Outcome codes of search_root
enum { SR_OK = 0, SR_CAPACITY = 1 };

template <class E, class Mem>
DK_HD int search_root(const typename E::Work& root, Rng& rng, uint32_t iters, double c, const double* ln_table,
                      Mem& mem, uint32_t* visits39, double* values39, uint8_t* best_out, uint64_t* ctr_scanned) {
    using Work = typename E::Work;
    NodeMeta rm;
    rm.unexpanded = E::allowed(root, true);
    rm.child_base = 0; rm.state_idx = 0; rm.parent = 0xFFFFFFFFu; rm.nchild = 0; rm.action = 0xFF;
    rm.player = (uint8_t)E::current_player(root); rm.flags = E::terminal(root) ? 1 : 0; rm.pad = 0;
    mem.store_meta(0, rm);
    mem.store_stats(0, 0ULL);
    mem.store_state(0, root);
    uint32_t next_slot = 1, next_state = 1;
    int status = SR_OK;
    uint64_t scanned = 0;

    for (uint32_t it = 0; it < iters; ++it) {
        // ---------------- selection
        uint32_t slot = 0;
        NodeMeta x = mem.load_meta(0);
        uint32_t x_visits = it;   // root visits == completed iterations
        int depth = 0;
        mem.path_set(0, 0u);
        while (x.nchild > 0 && x.unexpanded == 0) {
            uint32_t pick = 0;
            uint32_t pick_visits;
            if (x.nchild == 1) {
                pick_visits = (uint32_t)mem.load_stats(x.child_base);
                scanned += 1;
            } else {
                const double lnN = ln_table[x_visits];
                double min_q = INFINITY, max_q = -INFINITY;
                // pass 1: sibling min/max of the mean value (node.rs:202-235)
                for (int j = 0; j < x.nchild; ++j) {
                    const uint64_t st = mem.load_stats(x.child_base + j);
                    const uint32_t v = (uint32_t)st;
                    const double q = v > 0 ? (double)(int32_t)(st >> 32) / (double)v : 0.0;
                    min_q = q < min_q ? q : min_q;
                    max_q = q > max_q ? q : max_q;
                }
                const bool flat = fabs(max_q - min_q) < DK_F64_EPSILON;
                // pass 2: UCT, first strict maximum (node.rs:238-277)
                double best = -INFINITY;
                pick_visits = 0;
                for (int j = 0; j < x.nchild; ++j) {
                    const uint64_t st = mem.load_stats(x.child_base + j);
                    const uint32_t v = (uint32_t)st;
                    double u;
                    if (v == 0) {
                        u = INFINITY;
                    } else {
                        const double q = (double)(int32_t)(st >> 32) / (double)v;
                        const double nq = flat ? 1.0 : 2.0 * (q - min_q) / (max_q - min_q) - 1.0;
                        u = nq + c * sqrt(lnN / (double)v);
                    }
                    if (u > best) { best = u; pick = (uint32_t)j; pick_visits = v; }
                }
                scanned += x.nchild;
            }
            const uint32_t child = x.child_base + pick;
            depth += 1;
            if (depth < (int)mem.max_path) mem.path_set(depth, child | ((uint32_t)x.player << 30));
            slot = child;
            x = mem.load_meta(child);
            x_visits = pick_visits;
        }
        // ---------------- expansion
        Work w;
        if (x.unexpanded != 0) {
            const uint64_t bit = random_single(x.unexpanded, rng);
            const int a = ctz64(bit);
            if (x.nchild == 0) {
                const uint32_t block = (uint32_t)popc64(x.unexpanded);
                if (next_slot + block > mem.cap_slots || next_state >= mem.cap_states) { status = SR_CAPACITY; break; }
                x.child_base = next_slot;
                next_slot += block;
            }
            x.unexpanded &= ~bit;
            const uint32_t child = x.child_base + x.nchild;
            x.nchild += 1;
            mem.store_meta_expand(slot, x.unexpanded, x.child_base, x.nchild);
            w = mem.load_state(x.state_idx);
            E::step(w, a);
            NodeMeta cm;
            cm.unexpanded = E::allowed(w, false);
            cm.child_base = 0; cm.state_idx = next_state; cm.parent = slot; cm.nchild = 0; cm.action = (uint8_t)a;
            cm.player = (uint8_t)E::current_player(w); cm.flags = E::terminal(w) ? 1 : 0; cm.pad = 0;
            mem.store_meta(child, cm);
            mem.store_stats(child, 0ULL);
            mem.store_state(next_state, w);
            next_state += 1;
            depth += 1;
            if (depth < (int)mem.max_path) mem.path_set(depth, child | ((uint32_t)x.player << 30));
            slot = child;
        } else {
            w = mem.load_state(x.state_idx);
        }
        // ---------------- rollout
        int r[4];
        E::rollout(w, rng, r);
        // ---------------- backup (leaf -> root); deep tails beyond the LDS path use parent links
        int k = depth;
        uint32_t s = slot;
        while (k >= (int)mem.max_path) {
            const NodeMeta nm = mem.load_meta(s);
            const NodeMeta pm = mem.load_meta(nm.parent);
            mem.add_stats(s, ((uint64_t)(uint32_t)sel4i(r, pm.player) << 32) | 1ULL);
            s = nm.parent;
            k -= 1;
        }
        for (; k >= 1; --k) {
            const uint32_t e = mem.path_get(k);
            mem.add_stats(e & 0x3FFFFFFFu, ((uint64_t)(uint32_t)sel4i(r, (int)(e >> 30)) << 32) | 1ULL);
        }
        mem.add_stats(0, 1ULL);
        if (it + 1 == iters) (void)rng.next_u64();  // random_bool((1f32/1000f32) as f64)
    }
    if (ctr_scanned) *ctr_scanned = scanned;

    // ---------------- result: root children in expansion order
    for (int a = 0; a < 39; ++a) { visits39[a] = 0; values39[a] = 0.0; }
    const NodeMeta r0 = mem.load_meta(0);
    int best = -1; uint32_t bv = 0;
    for (int j = 0; j < r0.nchild; ++j) {
        const uint64_t st = mem.load_stats(r0.child_base + j);
        const NodeMeta cm = mem.load_meta(r0.child_base + j);
        const uint32_t v = (uint32_t)st;
        visits39[cm.action] = v;
        values39[cm.action] = (double)(int32_t)(st >> 32) / (double)v;
        if (best < 0 || v >= bv) { best = cm.action; bv = v; }   // max_by_key: last maximum
    }
    *best_out = best < 0 ? (uint8_t)0xFF : (uint8_t)best;
    return status;
}

}  // namespace dk
