// TEST INFRASTRUCTURE: host-side node pool for search_core.h (same interface as
// the GPU's GpuMem in doko_amd.hip).
#pragma once
#include <cstring>
#include <vector>

#include "../../master_doko_reinforcement_learning_amd/csrc/engine/search_core.h"

template <class W, class R>
struct HostMemBase {
    using Rec = R;               // the stored layout
    uint32_t cap_slots, cap_states, max_path;
    uint32_t balign = 1;         // child-block alignment in slots (GpuMem::balign)
    std::vector<R> hot;
    std::vector<dk::NodeCold> cold;
    std::vector<W> states;
    std::vector<uint32_t> path;
    std::vector<uint64_t> path_st;
    const double* ln_table = nullptr;
    double ln(uint32_t v) const { return ln_table[v]; }
    // `mp` = entries of the fast (LDS) part of the path on the GPU; the host keeps
    // the overflow in the same vector, so `mp` only matters to the GPU layout.
    HostMemBase(uint32_t slots, uint32_t nstates, uint32_t mp)
        : cap_slots(slots), cap_states(nstates), max_path(mp), hot(slots), cold(slots), states(nstates),
          path(dk::MAX_DEPTH), path_st(dk::MAX_DEPTH) {}
    dk::NodeCold load_cold(uint32_t s) { return cold[s]; }
    void store_cold(uint32_t s, const dk::NodeCold& c) { cold[s] = c; }
    void store_unexpanded(uint32_t s, uint64_t u) { cold[s].unexpanded = u; }
    W load_state(uint32_t i) { return states[i]; }
    void store_state(uint32_t i, const W& w) { states[i] = w; }
    int lds_entries() const { return (int)max_path; }
    uint32_t path_get_lds(int k, uint64_t* st) { *st = path_st[k]; return path[k]; }
    uint32_t path_get_ovf(int k, uint64_t* st) { *st = path_st[k]; return path[k]; }
    void path_set(int k, uint32_t v, uint64_t st) { path[k] = v; path_st[k] = st; }
    void touch_next(uint32_t, uint32_t, uint32_t) {}   // (the GPU's L2 prefetch)
};

// the 16-B / 32-B layouts store the in-register form itself (the host build's DK_HOT16)
template <class W>
struct HostMem : HostMemBase<W, dk::NodeHot> {
    using Hot = dk::NodeHot;
    using HostMemBase<W, dk::NodeHot>::HostMemBase;
    dk::NodeHot load_hot(uint32_t s) { return this->hot[s]; }
    void store_hot(uint32_t s, const dk::NodeHot& h) { this->hot[s] = h; }
    void store_stats(uint32_t s, uint64_t v) { this->hot[s].stats = v; }
    void store_backup(uint32_t s, uint64_t v, double q, float isv) { dk::hot_backup(this->hot[s], v, q, isv); }
    void store_child_base(uint32_t s, uint32_t cb, uint32_t) { this->hot[s].child_base = cb; }
    void store_node_tail(uint32_t s, uint32_t cb, uint32_t info) { this->hot[s].child_base = cb; this->hot[s].info = info; }
    void store_rec8(uint32_t, uint32_t, uint32_t) {}
};

// 8-B records (search_core.h NodeHot8): encoded on store, decoded on load
template <class W>
struct HostMem8 : HostMemBase<W, dk::NodeHot8> {
    using Hot = dk::NodeHot16;   // in-register form
    using HostMemBase<W, dk::NodeHot8>::HostMemBase;
    dk::NodeHot16 load_hot(uint32_t s) {
        const dk::NodeHot8 r = this->hot[s];
        dk::NodeHot16 h;
        h.stats = dk::p8_stats(r.w0); h.child_base = dk::p8_cb(r.w1); h.info = dk::p8_info(r.w1);
        return h;
    }
    dk::U4 load_pair(uint32_t i) {
        dk::U4 q;
        memcpy(&q, &this->hot[2 * i], 16);
        return q;
    }
    void store_hot(uint32_t s, const dk::NodeHot16& h) { this->hot[s].w0 = dk::p8_w0(h.stats); this->hot[s].w1 = dk::p8_w1(h.child_base, h.info); }
    void store_rec8(uint32_t s, uint32_t w0, uint32_t w1) { this->hot[s].w0 = w0; this->hot[s].w1 = w1; }
    void store_stats(uint32_t s, uint64_t v) { this->hot[s].w0 = dk::p8_w0(v); }
    void store_backup(uint32_t s, uint64_t v, double, float) { this->hot[s].w0 = dk::p8_w0(v); }
    void store_child_base(uint32_t s, uint32_t cb, uint32_t info) { this->hot[s].w1 = dk::p8_w1(cb, info); }
    void store_node_tail(uint32_t s, uint32_t cb, uint32_t info) { this->hot[s].w1 = dk::p8_w1(cb, info); }
};
