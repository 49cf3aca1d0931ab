// TEST INFRASTRUCTURE: host-side node pool for search_core.h (same interface as
// the GPU's GpuMem in doko_amd.hip).
#pragma once
#include <vector>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/search_core.h"

template <class W>
struct HostMem {
    using Hot = dk::NodeHot;   // the host build's layout (DK_HOT16)
    uint32_t cap_slots, cap_states, max_path;
    std::vector<dk::NodeHot> hot;
    std::vector<dk::NodeCold> cold;
    std::vector<W> states;
    std::vector<uint32_t> path;
    std::vector<uint64_t> path_st;
    const double* ln_table = nullptr;
    double ln(uint32_t v) const { return ln_table[v]; }
    // `mp` = entries of the fast (LDS) part of the path on the GPU; the host keeps
    // the overflow in the same vector, so `mp` only matters to the GPU layout.
    HostMem(uint32_t slots, uint32_t nstates, uint32_t mp)
        : cap_slots(slots), cap_states(nstates), max_path(mp), hot(slots), cold(slots), states(nstates),
          path(dk::MAX_DEPTH), path_st(dk::MAX_DEPTH) {}
    dk::NodeHot load_hot(uint32_t s) { return hot[s]; }
    void store_hot(uint32_t s, const dk::NodeHot& h) { hot[s] = h; }
    void store_stats(uint32_t s, uint64_t v) { hot[s].stats = v; }
    void store_backup(uint32_t s, uint64_t v, double q, float isv) {
        dk::hot_backup(hot[s], v, q, isv);
    }
    void store_child_base(uint32_t s, uint32_t cb) { hot[s].child_base = cb; }
    void store_node_tail(uint32_t s, uint32_t cb, uint32_t info) { hot[s].child_base = cb; hot[s].info = info; }
    dk::NodeCold load_cold(uint32_t s) { return cold[s]; }
    void store_cold(uint32_t s, const dk::NodeCold& c) { cold[s] = c; }
    void store_unexpanded(uint32_t s, uint64_t u) { cold[s].unexpanded = u; }
    W load_state(uint32_t i) { return states[i]; }
    void store_state(uint32_t i, const W& w) { states[i] = w; }
    int lds_entries() const { return (int)max_path; }
    uint32_t path_get_lds(int k, uint64_t* st) { *st = path_st[k]; return path[k]; }
    uint32_t path_get_ovf(int k, uint64_t* st) { *st = path_st[k]; return path[k]; }
    void path_set(int k, uint32_t v, uint64_t st) { path[k] = v; path_st[k] = st; }
};
