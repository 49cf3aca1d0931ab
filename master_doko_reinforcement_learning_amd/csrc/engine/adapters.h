// Engine adapters: the McEnvState surface (rs-doko-mcts/src/env/env_state.rs:7-28)
// of each game as static functions for search_core.h and the env kernels.
#pragma once
#include "do_engine.h"
#include "fdo_engine.h"

namespace dk {

struct FdoE {
    using Work = fdo::Work;
    using Node = fdo::Node;   // a node's state in the search pools (64 B)
    using Packed = dk_fdo_state;
    static constexpr int GAME = DK_GAME_FULL_DOKO;
    // search queue in root-index order: longest-first ordering measured 5 % slower on C3
    // (heavy groups started together contend for the caches)
    static constexpr bool ORDER_GROUPS = false;
    DK_HD static void load(const dk_state& s, Work& w) { fdo::unpack(s.fdo, w); }
    DK_HD static uint64_t allowed(const Work& w, bool first) { return fdo::env_allowed(w, first); }
    DK_HD static int current_player(const Work& w) { return fdo::env_current_player(w); }
    DK_HD static bool terminal(const Work& w) { return fdo::is_terminal(w); }
    DK_HD static void step(Work& w, int a) {
        fdo::play_action(w, a);
        w.pad0 = 0;   // padding is don't-care: constant stores instead of carrying the loaded bytes
        w.pad1 = 0;
    }
    DK_HD static int rollout(const Work& w, Rng& rng, int r[4]) { return fdo::rollout(w, rng, r); }
    DK_HD static void rewards(const Work& w, int r[4]) { fdo::score(w, r); }
    DK_HD static void step_packed(dk_state& s, int a) { fdo::step_packed(s.fdo, a); }
    DK_HD static Node pack_node(const Work& w) { return fdo::pack_node(w); }
    DK_HD static Work unpack_node(const Node& n) { return fdo::unpack_node(n); }
    DK_HD static bool node_ok(const Work& w) { return fdo::node_ok(w); }
};

struct DoE {
    using Work = dko::Work;
    using Node = dko::Node;
    using Packed = dk_do_state;
    static constexpr int GAME = DK_GAME_DOKO;
    // search queue longest-first (group_order_kernel): 4 % faster on C2d
    static constexpr bool ORDER_GROUPS = true;
    DK_HD static void load(const dk_state& s, Work& w) { dko::unpack(s.dk, w); }
    DK_HD static uint64_t allowed(const Work& w, bool first) { return dko::env_allowed(w, first); }
    DK_HD static int current_player(const Work& w) { return dko::env_current_player(w); }
    DK_HD static bool terminal(const Work& w) { return dko::is_terminal(w); }
    DK_HD static void step(Work& w, int a) { dko::play_action(w, a); }
    DK_HD static int rollout(const Work& w, Rng& rng, int r[4]) { return dko::rollout(w, rng, r); }
    DK_HD static void rewards(const Work& w, int r[4]) { dko::score(w, r); }
    DK_HD static void step_packed(dk_state& s, int a) { dko::step_packed(s.dk, a); }
    DK_HD static Node pack_node(const Work& w) { return dko::pack_node(w); }
    DK_HD static Work unpack_node(const Node& n) { return dko::unpack_node(n); }
    DK_HD static bool node_ok(const Work& w) { return dko::node_ok(w); }
};

struct TttE {
    using Work = ttt::Work;
    using Node = ttt::Work;
    using Packed = dk_ttt_state;
    static constexpr int GAME = DK_GAME_TTT;
    static constexpr bool ORDER_GROUPS = false;
    DK_HD static void load(const dk_state& s, Work& w) { ttt::unpack(s.ttt, w); }
    DK_HD static uint64_t allowed(const Work& w, bool first) { return ttt::env_allowed(w, first); }
    DK_HD static int current_player(const Work& w) { return ttt::env_current_player(w); }
    DK_HD static bool terminal(const Work& w) { return ttt::is_terminal(w); }
    DK_HD static void step(Work& w, int a) { ttt::play_action(w, a); }
    DK_HD static int rollout(const Work& w, Rng& rng, int r[4]) { return ttt::rollout(w, rng, r); }
    DK_HD static void rewards(const Work& w, int r[4]) { ttt::score(w, r); }
    DK_HD static void step_packed(dk_state& s, int a) { ttt::step_packed(s.ttt, a); }
    DK_HD static Node pack_node(const Work& w) { return w; }
    DK_HD static Work unpack_node(const Node& n) { return n; }
    DK_HD static bool node_ok(const Work&) { return true; }
};

}  // namespace dk
