// libdoko_amd.so — HIP kernels for gfx950 and the C-ABI of include/doko_amd.h.
//
// One lane = one determinized root (or one env state).  The UCT search keeps
// the reference's sequential per-root semantics; all parallelism is across
// roots.  Node pools are interleaved across roots ([slot][root]) so that the
// lanes of a wave — which hold roots of the same infostate in the determinized
// workload — touch the same slot indices (root children) with coalesced loads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/doko_amd.h"
#include "engine/adapters.h"
#include "engine/assign_engine.h"
#include "engine/ar_engine.h"
#include "engine/az_core.h"
#include "engine/rand_distr.h"
#include "engine/encode_pi.h"
#include "az_net_kernels.h"
#include "az_net_f32_kernels.h"
#include "engine/cap_engine.h"
#include "engine/search_core.h"
#include "state_fields.h"

namespace {

constexpr int WAVE = 64;
// register budget of the search kernel: per hot-record layout (NodeHot16::MIN_WAVES = 3 waves
// per SIMD, 167 VGPRs with a 24-B spill; NodeHot32: the compiler's choice, two waves).
// Resident single-wave workgroups per CU at that budget (sizes the node pools):
#ifndef DK_RESIDENT_WG
#define DK_RESIDENT_WG 12
#endif
constexpr uint32_t RESIDENT_WG_PER_CU = DK_RESIDENT_WG;
constexpr int MAX_PATH = 64;   // LDS path entries per lane (deeper paths spill to a global overflow)

#define DK_HIP(call)                                              \
    do {                                                          \
        hipError_t e_ = (call);                                   \
        if (e_ != hipSuccess) {                                   \
            fprintf(stderr, "doko_amd: %s failed: %s (%s:%d)\n", #call, hipGetErrorString(e_), __FILE__, __LINE__); \
            return DK_E_LAUNCH;                                   \
        }                                                         \
    } while (0)

// Dynamic LDS of the search kernel: [ln table (optional)][path stats][path slots]
extern __shared__ uint64_t dk_lds[];
// destination of the prefetch loads (GpuMem::touch_next): one dword per lane, never read.
// Off by default: alternated contexts (profiles/r04/ab_touch.log) put it at -1.9 % on C2, +4 % on
// the 512-infostate batch and neutral to +1 % on C3; -DDK_TOUCH=1 builds it.
#ifndef DK_TOUCH
#define DK_TOUCH 0
#endif
__shared__ uint32_t dk_touch_lds[64];
typedef __attribute__((address_space(3))) void dk_lds_void;
__device__ __forceinline__ void touch(const void* g) {
    __builtin_amdgcn_global_load_lds(g, (dk_lds_void*)dk_touch_lds, 4, 0, 0);
}
constexpr uint32_t LN_LDS_MAX = 2048;   // ln(N) entries staged in LDS (16 KB)

// ---------------------------------------------------------------- node pool access
// Node pool of one root, root-major: [root][slot] so that a node's child block
// is one contiguous run of 16- or 32-byte hot records (one or a few cache lines).
// Only the owning lane ever touches a root's tree, so plain loads and stores
// (L1-cacheable, program-ordered within the lane) are sufficient.
template <class W, bool LN_LDS, class H>
struct GpuMem {
    static constexpr bool P8 = dk::is_p8<H>::value;
    using Rec = H;                                                  // the stored layout
    using Hot = typename std::conditional<P8, dk::NodeHot16, H>::type;   // the in-register form
    // Wave-uniform region bases (SGPRs) and this lane's 32-bit element offsets: every
    // access is base + 32-bit byte offset (saddr + voffset), no per-lane 64-bit pointers.
    // A lane's region is lane * capacity elements past the wave's base (root-major).
    H* hot;
    dk::NodeCold* cold;
    W* states;
    uint32_t lslot, lstate, lovf;   // lane * cap_slots, lane * cap_states, lane * MAX_DEPTH
    template <class T> __device__ static T& at(T* base, uint32_t idx) {
        if constexpr (H::WIDE) return base[idx];   // 64-bit byte offsets (regions >= 4 GiB)
        else return *reinterpret_cast<T*>(reinterpret_cast<char*>(base) + (uint32_t)(idx * (uint32_t)sizeof(T)));
    }
    __device__ H& hr(uint32_t s) const { return at(hot, lslot + s); }
    __device__ dk::NodeCold& cr(uint32_t s) const { return at(cold, lslot + s); }
    __device__ W& sr(uint32_t i) const { return at(states, lstate + i); }
    // LDS regions are addressed as offsets into dk_lds (u64 words) so that the
    // compiler keeps the LDS address space (ds_* instructions, not flat_*)
    uint32_t path_st_off; // path stats: dk_lds[path_st_off + k*stride] (8-B records: their stats
                          // word, ((uint32_t*)dk_lds)[path_st_off + k*stride])
    uint32_t path_off;    // path slots: ((uint32_t*)dk_lds)[path_off + k*stride]
    uint32_t* ovf;        // global overflow of the path (entries >= lds_n)
    uint64_t* ovf_st;
    uint32_t path_stride;
    uint32_t half;        // lane pairs (NodeHot16P): 0 = the lower lane of the pair, 1 = its partner
    int lds_n;            // path entries held in LDS
    const double* ln_glob;
    uint32_t cap_slots, cap_states;
    uint32_t balign;      // child blocks start at multiples of this many slots (a power of two)
#ifdef DK_PHASE_PROF
    uint64_t* prof;
#endif

    __device__ double ln(uint32_t v) const {
        // one address space per instantiation: a runtime choice would make the compiler
        // select between pointers and emit flat loads
        if constexpr (LN_LDS) return __longlong_as_double((long long)dk_lds[v]);
        else return ln_glob[v];
    }
    __device__ Hot load_hot(uint32_t s) const {
        if constexpr (P8) {
            const dk::NodeHot8 r = hr(s);
            Hot h;
            h.stats = dk::p8_stats(r.w0); h.child_base = dk::p8_cb(r.w1); h.info = dk::p8_info(r.w1);
            return h;
        } else {
            return hr(s);
        }
    }
    // a whole 8-B record from its two words
    __device__ void store_rec8(uint32_t s, uint32_t w0, uint32_t w1) const {
        if constexpr (P8) { dk::NodeHot8 r; r.w0 = w0; r.w1 = w1; hr(s) = r; }
    }
    // two 8-B records (the pair starting at slot 2i)
    __device__ dk::U4 load_pair(uint32_t i) const { return at(reinterpret_cast<dk::U4*>(hot), (lslot >> 1) + i); }
    __device__ void store_hot(uint32_t s, const Hot& h) const {
        if constexpr (P8) {
            dk::NodeHot8 r;
            r.w0 = dk::p8_w0(h.stats); r.w1 = dk::p8_w1(h.child_base, h.info);
            hr(s) = r;
        } else {
            hr(s) = h;
        }
    }
    __device__ void store_stats(uint32_t s, uint64_t v) const {
        if constexpr (P8) hr(s).w0 = dk::p8_w0(v);
        else hr(s).stats = v;
    }
    __device__ void store_backup(uint32_t s, uint64_t v, double q, float isv) const {
        if constexpr (P8) hr(s).w0 = dk::p8_w0(v);
        else dk::hot_backup(hr(s), v, q, isv);
    }
    // the chain head's skip pointer (8-B records rewrite the structure word: `info` is the head's)
    __device__ void store_child_base(uint32_t s, uint32_t child_base, uint32_t info) const {
        if constexpr (P8) hr(s).w1 = dk::p8_w1(child_base, info);
        else hr(s).child_base = child_base;
    }
    __device__ void store_node_tail(uint32_t s, uint32_t child_base, uint32_t info) const {
        if constexpr (P8) {
            hr(s).w1 = dk::p8_w1(child_base, info);
        } else {
            hr(s).child_base = child_base;
            hr(s).info = info;
        }
    }
    __device__ dk::NodeCold load_cold(uint32_t s) const { return cr(s); }
    __device__ void store_cold(uint32_t s, const dk::NodeCold& c) const { cr(s) = c; }
    __device__ void store_unexpanded(uint32_t s, uint64_t u) const { cr(s).unexpanded = u; }
    __device__ W load_state(uint32_t i) const { return sr(i); }
    __device__ void store_state(uint32_t i, const W& w) const { sr(i) = w; }
    __device__ int lds_entries() const { return lds_n; }
    __device__ uint32_t path_get_lds(int k, uint64_t* st) const {
        if constexpr (P8) *st = dk::p8_stats(reinterpret_cast<const uint32_t*>(dk_lds)[path_st_off + k * path_stride]);
        else *st = dk_lds[path_st_off + k * path_stride];
        return reinterpret_cast<const uint32_t*>(dk_lds)[path_off + k * path_stride];
    }
    __device__ uint32_t path_get_ovf(int k, uint64_t* st) const {
        *st = at(ovf_st, lovf + (uint32_t)(k - lds_n));
        return at(ovf, lovf + (uint32_t)(k - lds_n));
    }
    __device__ void path_set(int k, uint32_t v, uint64_t st) const {
        if (k < lds_n) {
            reinterpret_cast<uint32_t*>(dk_lds)[path_off + k * path_stride] = v;
            if constexpr (P8) reinterpret_cast<uint32_t*>(dk_lds)[path_st_off + k * path_stride] = dk::p8_w0(st);
            else dk_lds[path_st_off + k * path_stride] = st;
        } else {
            at(ovf, lovf + (uint32_t)(k - lds_n)) = v;
            at(ovf_st, lovf + (uint32_t)(k - lds_n)) = st;
        }
    }
    // Prefetch for the pick's leading candidate (pick_child_x / pick_child_pair): the record the
    // next step will load -- its state and cold record if it is open (the expansion), the head of
    // its child block if it branches -- is requested now, while the pick finishes, and the real
    // load later finds it on its way into the caches.  A 4-byte global_load_lds per lane (no
    // destination register; the LDS bytes are never read).  Forced chain heads are loaded by the
    // pick itself (the chain-end prefetch).
    __device__ void touch_next(uint32_t slot, uint32_t cb, uint32_t info) const {
#if DK_TOUCH
        const uint32_t nch = dk::ni_nchild(info);
        if (dk::ni_open(info)) {
            touch(&sr(dk::ni_state(info)));
            if (nch) touch(&cr(slot));
        } else if (nch >= 2 || (P8 && dk::ni_resolved(info))) {
            touch(&hr(cb));
        }
#else
        (void)slot; (void)cb; (void)info;
#endif
    }
    // the same request, made before the pick for a lane-pair half's most visited child
    // (pick_child_pair, -DDK_TOUCH_EARLY=1)
    __device__ void touch_early(uint32_t slot, uint32_t cb, uint32_t info) const {
        const uint32_t nch = dk::ni_nchild(info);
        if (dk::ni_open(info)) {
            touch(&sr(dk::ni_state(info)));
            if (nch) touch(&cr(slot));
        } else if (nch >= 2) {
            touch(&hr(cb));
        }
    }
#ifdef DK_PHASE_PROF
    __device__ void prof_add(int k, uint64_t v) const { prof[k] += v; }
#endif
};

// ---------------------------------------------------------------- kernels
// One lane per root, `rpw` roots per 64-lane wave (lanes >= rpw idle).  The grid is
// persistent: each single-wave workgroup owns one pool region of `rpw` roots (node
// records, states, path overflow) and pulls root groups g = [g*rpw, (g+1)*rpw) from a
// queue counter until the batch is drained, so a wave that finishes early takes the
// next group instead of idling until the slowest wave of the launch ends, and the pools
// are sized for the resident waves, not for the batch.  The LDS holds each lane's
// selection path: lds_n x (u32 slot|player, u64 stats).
template <class E, bool LN_LDS, class H>
__global__ void __launch_bounds__(WAVE, H::MIN_WAVES) search_kernel(const dk_state* __restrict__ roots,
                                                      const uint64_t* __restrict__ seeds, uint32_t n,
                                                      uint32_t iters, double c, const double* __restrict__ ln_table,
                                                      void* hot_pool, dk::NodeCold* cold, typename E::Node* states,
                                                      uint32_t* ovf, uint64_t* ovf_st,
                                                      uint32_t cap_slots, uint32_t st_stride, uint32_t balign,
                                                      uint32_t rpw, int lds_n,
                                                      uint32_t* visits, double* values,
                                                      uint8_t* best, int* err, uint32_t* queue, uint64_t* prof,
                                                      const uint32_t* __restrict__ order, uint32_t* retry,
                                                      const uint32_t* __restrict__ list, uint32_t* high_water,
                                                      const uint32_t* __restrict__ perm, uint32_t lane_base,
                                                      uint64_t* wave_clock, uint64_t* rng_io) {
    const uint32_t lane = threadIdx.x;
    // lane pairs (NodeHot16P, rpw <= 32): lanes l and l + 32 search the same root
    constexpr bool PAIR = H::PAIR;
    const uint32_t rl = PAIR ? (lane & 31u) : lane;                    // the root's lane in the group
    const bool lead = !PAIR || lane < 32u;                              // one lane per root for atomics
    const uint32_t pw = PAIR ? (uint32_t)WAVE : rpw;                    // LDS path width (lanes)
    // per-wave start / end of the realtime counter (100 MHz), indexed by the wave's first pool
    // lane (dk_last_search_waves): how long each wave had work before the group queue drained
    const uint32_t clock_idx = lane_base + blockIdx.x * rpw;
    // (and the shader-clock counter, s_memtime, beside it: cycles per real time = the launch's clock)
    if (wave_clock && lane == 0) {
        wave_clock[4 * clock_idx] = __builtin_amdgcn_s_memrealtime();
        wave_clock[4 * clock_idx + 2] = __builtin_amdgcn_s_memtime();
    }
    const uint32_t T = iters + 1;
    const uint32_t n_ln = LN_LDS ? T : 0u;
    for (uint32_t i = lane; i < n_ln; i += WAVE) dk_lds[i] = (uint64_t)__double_as_longlong(ln_table[i]);
    if (E::GAME != DK_GAME_TTT) dk::fdo::card_table_init();   // ends with a barrier
    __syncthreads();
    const uint32_t n_ln16 = (n_ln + 1u) & ~1u;                           // keep the next region 16-B aligned
    // path stats: u64 words (8-B records: u32 words), then the u32 slots
    constexpr bool P8 = dk::is_p8<H>::value;
    const uint32_t path_st_base = P8 ? 2u * n_ln16 : n_ln16;
    const uint32_t path_base32 = P8 ? path_st_base + (uint32_t)lds_n * pw : 2u * (path_st_base + (uint32_t)lds_n * pw);
    // fallback pass (list != nullptr): the roots the main pass could not fit, list[0] of them
    // at list[1..], searched again in a pool with the proven capacity
    if (list) n = list[0];
    const uint32_t groups = (n + rpw - 1) / rpw;
    uint32_t hw = 0;                                                    // slot high-water of this lane's roots
    for (;;) {
        uint32_t g = 0;
        if (lane == 0) g = atomicAdd(queue, 1u);
        g = __shfl(g, 0);
        if (g >= groups) break;                                         // every wave reaches this
        if (order) g = order[g];                                        // longest groups first
        const uint32_t idx = g * rpw + rl;
        if (rl >= rpw || idx >= n) continue;
        const uint32_t root = list ? list[1 + idx] : perm ? perm[idx] : idx;   // perm: depth-sorted order
        typename E::Work w;
        E::load(roots[root], w);
        // rng_io: the caller's SmallRng states, continued (dk_search_batch_rng_async); else seeded
        dk::Rng rng = rng_io ? dk::Rng{rng_io[4 * (size_t)root], rng_io[4 * (size_t)root + 1], rng_io[4 * (size_t)root + 2],
                                       rng_io[4 * (size_t)root + 3]}
                             : dk::Rng::seed_from_u64(seeds[root]);
        GpuMem<typename E::Node, LN_LDS, H> mem;
        // wave bases (uniform) + lane offsets: pool lane = lane_base + blockIdx.x * rpw + lane (a launch
        // owns the lanes [lane_base, lane_base + grid * rpw) of the pools, dk_ctx::Slot)
        const size_t wr = (size_t)lane_base + (size_t)blockIdx.x * rpw;
        mem.hot = reinterpret_cast<H*>(hot_pool) + wr * cap_slots;
        mem.cold = cold + wr * cap_slots;
        mem.states = states + wr * st_stride;
        mem.lslot = rl * cap_slots; mem.lstate = rl * st_stride; mem.lovf = rl * (uint32_t)dk::MAX_DEPTH;
        mem.path_st_off = path_st_base + lane;
        mem.path_off = path_base32 + lane;
        mem.ln_glob = ln_table;
        mem.lds_n = lds_n;
        mem.path_stride = pw;
        mem.half = PAIR ? lane >> 5 : 0u;
        mem.ovf = ovf + wr * dk::MAX_DEPTH;
        mem.ovf_st = ovf_st + wr * dk::MAX_DEPTH;
        mem.cap_slots = cap_slots; mem.cap_states = T; mem.balign = balign;
#ifdef DK_PHASE_PROF
        mem.prof = prof + (size_t)root * dk::PROF_SLOTS;
#else
        (void)prof;
#endif
        uint8_t b;
        uint32_t used[2];
        const int st = dk::search_root<E>(w, rng, iters, c, mem, visits + (size_t)root * 39,
                                          values + (size_t)root * 39, &b, nullptr, used);
        if (st == dk::SR_STATE) {
            atomicOr(err, 2);                                           // malformed root (DK_E_STATE)
        } else if (st != dk::SR_OK) {
            if (retry) {                                                // searched again by the fallback pass
                if (lead) {
                    retry[1 + atomicAdd(retry, 1u)] = root;
                    atomicAdd(high_water + 1, 1u);
                }
            } else {
                atomicOr(err, 1);
            }
        } else {
            hw = used[0] > hw ? used[0] : hw;
            // the advanced stream goes back only for a completed search: a root that ran out
            // of slots is searched again by the fallback pass from the caller's state
            if (rng_io) {
                rng_io[4 * (size_t)root] = rng.s0; rng_io[4 * (size_t)root + 1] = rng.s1;
                rng_io[4 * (size_t)root + 2] = rng.s2; rng_io[4 * (size_t)root + 3] = rng.s3;
            }
        }
        best[root] = b;
    }
    if (hw) atomicMax(high_water, hw);
    if (wave_clock && lane == 0) {
        wave_clock[4 * clock_idx + 3] = __builtin_amdgcn_s_memtime();
        wave_clock[4 * clock_idx + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// is_consistent (rs-full-doko/src/matching/is_consistent.rs:38-305) of assumed hands and
// reservations for an infostate record, one lane per check: the IMPI lanes' facts (init)
// with the given assumption, then the same consistency pass the sampler ends with.
__global__ void is_consistent_kernel(const dk_az_state* info, const uint64_t* hands, const uint8_t* res, uint32_t n,
                                     uint8_t* reasons) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const dk_az_state r = info[i];
    dk::ar::Lane L;
    (void)dk::ar::init(r, 0, L);
    for (int p = 0; p < 4; ++p) { L.hands[p] = hands[4 * (size_t)i + p]; L.res[p] = res[4 * (size_t)i + p]; }
    reasons[i] = L.status == dk::ar::PANIC ? (uint8_t)0xFE : dk::ar::consistency(r, L);
}

__device__ void new_game_packed(int game, uint64_t seed, dk_state& out) {
    dk::Rng rng = dk::Rng::seed_from_u64(seed);
    const uint32_t start = rng.range_u32(4);  // FdoPlayer::from_rng / gen_range(0..4)
    uint8_t deck[48];
    for (int i = 0; i < 24; ++i) { deck[2 * i] = (uint8_t)i; deck[2 * i + 1] = (uint8_t)i; }
    dk::shuffle48(deck, rng);
    for (int i = 0; i < DK_STATE_BYTES; ++i) out.raw[i] = 0;
    uint64_t hands[4] = {0, 0, 0, 0};
    for (int p = 0; p < 4; ++p)
        for (int j = 0; j < 12; ++j) hands[p] = dk::cap::h_add(hands[p], deck[p * 12 + j]);
    if (game == DK_GAME_FULL_DOKO) {
        dk_fdo_state& s = out.fdo;
        for (int p = 0; p < 4; ++p) s.hands[p] = hands[p];
        for (int i = 0; i < 48; ++i) s.cards[i] = DK_NONE;
        for (int i = 0; i < 4; ++i) s.res[i] = DK_NONE;
        s.res_start = (uint8_t)start; s.current_player = (uint8_t)start;
        s.game_type = DK_NONE; s.rr_kind = DK_NONE; s.game = DK_GAME_FULL_DOKO;
    } else {
        dk_do_state& s = out.dk;
        for (int p = 0; p < 4; ++p) s.hands[p] = hands[p];
        for (int i = 0; i < 48; ++i) s.cards[i] = DK_NONE;
        for (int i = 0; i < 4; ++i) s.res[i] = DK_NONE;
        s.res_start = (uint8_t)start; s.current_player = (uint8_t)start;
        s.rr_kind = DK_NONE; s.game = DK_GAME_DOKO;
    }
}

__global__ void new_game_kernel(int game, const uint64_t* seeds, uint32_t n, dk_state* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dk_state s;
    new_game_packed(game, seeds[i], s);
    out[i] = s;
}

__device__ uint64_t legal_of(const dk_state& s) {
    switch (s.raw[127]) {
        case DK_GAME_FULL_DOKO: { dk::fdo::Work w; dk::fdo::unpack(s.fdo, w); return dk::fdo::legal_actions(w); }
        case DK_GAME_DOKO: { dk::dko::Work w; dk::dko::unpack(s.dk, w); return dk::dko::legal_actions(w); }
        case DK_GAME_TTT: { dk::ttt::Work w; dk::ttt::unpack(s.ttt, w); return dk::ttt::env_allowed(w, true); }
    }
    return 0;
}

__global__ void env_allowed_kernel(const dk_state* states, uint32_t n, int first, uint64_t* masks, int* err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const dk_state s = states[i];
    uint64_t m = 0;
    switch (s.raw[127]) {
        case DK_GAME_FULL_DOKO: { dk::fdo::Work w; dk::fdo::unpack(s.fdo, w); m = dk::fdo::env_allowed(w, first != 0); break; }
        case DK_GAME_DOKO: { dk::dko::Work w; dk::dko::unpack(s.dk, w); m = dk::dko::env_allowed(w, first != 0); break; }
        case DK_GAME_TTT: { dk::ttt::Work w; dk::ttt::unpack(s.ttt, w); m = dk::ttt::env_allowed(w, first != 0); break; }
        default: atomicOr(err, 2);
    }
    masks[i] = m;
}

__global__ void legal_kernel(const dk_state* states, uint32_t n, uint64_t* masks) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    masks[i] = legal_of(states[i]);
}

__global__ void env_step_kernel(dk_state* states, const uint64_t* actions, uint32_t n, int* err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dk_state s = states[i];
    const uint64_t a = actions[i];
    if (__builtin_popcountll(a) != 1 || !(legal_of(s) & a)) { atomicOr(err, 2); return; }
    const int ai = __builtin_ctzll(a);
    switch (s.raw[127]) {
        case DK_GAME_FULL_DOKO: dk::FdoE::step_packed(s, ai); break;
        case DK_GAME_DOKO: dk::DoE::step_packed(s, ai); break;
        case DK_GAME_TTT: dk::TttE::step_packed(s, ai); break;
    }
    states[i] = s;
}

__global__ void env_rewards_kernel(const dk_state* states, uint32_t n, int32_t* has, double* rewards) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const dk_state s = states[i];
    int r[4] = {0, 0, 0, 0};
    bool fin = false;
    switch (s.raw[127]) {
        case DK_GAME_FULL_DOKO: { dk::fdo::Work w; dk::fdo::unpack(s.fdo, w); fin = dk::fdo::is_terminal(w); if (fin) dk::fdo::score(w, r); break; }
        case DK_GAME_DOKO: { dk::dko::Work w; dk::dko::unpack(s.dk, w); fin = dk::dko::is_terminal(w); if (fin) dk::dko::score(w, r); break; }
        case DK_GAME_TTT: { dk::ttt::Work w; dk::ttt::unpack(s.ttt, w); fin = dk::ttt::is_terminal(w); if (fin) dk::ttt::score(w, r); break; }
    }
    has[i] = fin ? 1 : 0;
    for (int p = 0; p < 4; ++p) rewards[4 * (size_t)i + p] = fin ? (double)r[p] : 0.0;
}

template <class E>
__device__ void rollout_one(const dk_state& s, dk::Rng& rng, double* out) {
    typename E::Work w;
    E::load(s, w);
    int r[4];
    E::rollout(w, rng, r);
    for (int p = 0; p < 4; ++p) out[p] = (double)r[p];
}

__global__ void __launch_bounds__(WAVE) env_rollout_kernel(const dk_state* states, uint64_t* rng_states, uint32_t n,
                                                           double* rewards) {
    dk::fdo::card_table_init();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const dk_state s = states[i];
    dk::Rng rng{rng_states[4 * (size_t)i], rng_states[4 * (size_t)i + 1], rng_states[4 * (size_t)i + 2], rng_states[4 * (size_t)i + 3]};
    double out[4] = {0, 0, 0, 0};
    switch (s.raw[127]) {
        case DK_GAME_FULL_DOKO: rollout_one<dk::FdoE>(s, rng, out); break;
        case DK_GAME_DOKO: rollout_one<dk::DoE>(s, rng, out); break;
        case DK_GAME_TTT: rollout_one<dk::TttE>(s, rng, out); break;
    }
    for (int p = 0; p < 4; ++p) rewards[4 * (size_t)i + p] = out[p];
    rng_states[4 * (size_t)i] = rng.s0; rng_states[4 * (size_t)i + 1] = rng.s1;
    rng_states[4 * (size_t)i + 2] = rng.s2; rng_states[4 * (size_t)i + 3] = rng.s3;
}

// random_action_for_current_player_no_announcement (full doko) /
// random_action_for_current_player (rs-doko, tic-tac-toe), k times, on the wire format.
__global__ void random_plies_kernel(dk_state* states, uint64_t* rng_states, const uint32_t* plies, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dk_state s = states[i];
    dk::Rng rng{rng_states[4 * (size_t)i], rng_states[4 * (size_t)i + 1], rng_states[4 * (size_t)i + 2], rng_states[4 * (size_t)i + 3]};
    for (uint32_t k = 0; k < plies[i]; ++k) {
        uint64_t a = legal_of(s);
        if (s.raw[127] == DK_GAME_FULL_DOKO) {
            if (s.fdo.phase == dk::fdo::PH_FINISHED) break;
            a &= ~dk::fdo::ANN_ACTIONS;
        } else if (s.raw[127] == DK_GAME_DOKO) {
            if (s.dk.phase == dk::dko::PH_FINISHED) break;
        }
        if (a == 0) break;
        const int ai = dk::ctz64(dk::random_single(a, rng));
        switch (s.raw[127]) {
            case DK_GAME_FULL_DOKO: dk::FdoE::step_packed(s, ai); break;
            case DK_GAME_DOKO: dk::DoE::step_packed(s, ai); break;
            default: dk::TttE::step_packed(s, ai); break;
        }
    }
    states[i] = s;
    rng_states[4 * (size_t)i] = rng.s0; rng_states[4 * (size_t)i + 1] = rng.s1;
    rng_states[4 * (size_t)i + 2] = rng.s2; rng_states[4 * (size_t)i + 3] = rng.s3;
}

__global__ void __launch_bounds__(WAVE) determinize_kernel(const dk_state* info, uint32_t n_info, uint32_t samples,
                                                           const uint64_t* seeds, dk_state* out, int* err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_info * samples) return;
    const dk_state& s = info[i / samples];
    dk_state o;
    dk::Rng rng = dk::Rng::seed_from_u64(seeds[i]);
    if (s.raw[127] == DK_GAME_FULL_DOKO && s.fdo.current_player != DK_NONE) {
        dk::cap::card_matching_full(s.fdo, rng, o.fdo);          // CAPSampling (rs-full-doko)
    } else if (s.raw[127] == DK_GAME_DOKO) {
        if (dk::asg::sample_assignment_full(s.dk, rng, o.dk))    // rule-based sampler (rs-doko)
            atomicOr(err, 2);
    } else {
        atomicOr(err, 2);
        o = s;
    }
    out[i] = o;
}

// ---------------------------------------------------------------- AlphaZero PUCT (az_core.h)
// One lane per game; game g owns nodes [g*cap_nodes, (g+1)*cap_nodes) and states
// [g*cap_states, ...).  The network runs between the launches on the same stream.
__device__ inline dk::az::Mem az_mem(dk::az::Node* nodes, dk_az_state* states, uint32_t g, uint32_t cap_nodes,
                                     uint32_t cap_states) {
    dk::az::Mem m;
    m.nodes = nodes + (size_t)g * cap_nodes;
    m.states = states + (size_t)g * cap_states;
    m.cap_nodes = cap_nodes; m.cap_states = cap_states;
    return m;
}

__global__ void az_init_kernel(const dk_az_state* roots, const uint64_t* seeds, uint32_t n, dk::az::Node* nodes,
                               dk_az_state* states, dk::az::Game* games, uint32_t cap_nodes, uint32_t cap_states,
                               dk_az_state* eval, int* err) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    const dk_az_state r = roots[g];
    if (r.state.raw[127] != DK_GAME_FULL_DOKO) { atomicOr(err, 2); return; }
    dk::az::Mem m = az_mem(nodes, states, g, cap_nodes, cap_states);
    dk::az::Game gm;
    dk::az::init(r, gm, m, seeds[g]);
    games[g] = gm;
    eval[g] = r;
}

// noise == nullptr: the root's Dirichlet([alpha; 39]) noise is drawn from the game's own SmallRng
// (async_mcts.rs:111-113, rand_distr.h) before any other draw of the search.
__global__ void az_root_kernel(const float* value, const float* logits, const float* noise, float alpha, dk::rd::Open01Tab tab,
                               float eps, int epoch, uint32_t n, dk::az::Node* nodes, dk_az_state* states,
                               dk::az::Game* games, uint32_t cap_nodes, uint32_t cap_states, int* err) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    dk::az::Mem m = az_mem(nodes, states, g, cap_nodes, cap_states);
    dk::az::Game gm = games[g];
    float drawn[39];
    const float* nz = noise + 39 * (size_t)g;
    if (!noise) {
        dk::Rng r;
        r.s0 = gm.rng[0]; r.s1 = gm.rng[1]; r.s2 = gm.rng[2]; r.s3 = gm.rng[3];
        dk::rd::dirichlet39(alpha, r, tab, drawn);
        gm.rng[0] = r.s0; gm.rng[1] = r.s1; gm.rng[2] = r.s2; gm.rng[3] = r.s3;
        nz = drawn;
    }
    dk::az::root_expand(gm, m, value + 4 * (size_t)g, logits + 39 * (size_t)g, nz, eps, epoch);
    if (gm.status) atomicOr(err, 1);
    games[g] = gm;
}

__global__ void az_select_kernel(float c, int epoch, uint32_t n, dk::az::Node* nodes, dk_az_state* states,
                                 dk::az::Game* games, uint32_t cap_nodes, uint32_t cap_states, dk_az_state* eval,
                                 uint8_t* need_eval, int* err) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    dk::az::Mem m = az_mem(nodes, states, g, cap_nodes, cap_states);
    dk::az::Game gm = games[g];
    if (gm.status == 0) dk::az::select(gm, m, c, epoch, eval + g);
    if (gm.status) atomicOr(err, 1);
    if (need_eval) need_eval[g] = (uint8_t)gm.need_eval;
    games[g] = gm;
}

__global__ void az_backup_kernel(const float* value, const float* logits, uint32_t n, dk::az::Node* nodes,
                                 dk_az_state* states, dk::az::Game* games, uint32_t cap_nodes, uint32_t cap_states) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    dk::az::Mem m = az_mem(nodes, states, g, cap_nodes, cap_states);
    dk::az::Game gm = games[g];
    dk::az::backup(gm, m, value + 4 * (size_t)g, logits + 39 * (size_t)g);
    games[g] = gm;
}

__global__ void az_finish_kernel(int temp_mode, float temperature, uint32_t n, dk::az::Node* nodes, dk_az_state* states,
                                 dk::az::Game* games, uint32_t cap_nodes, uint32_t cap_states, uint32_t* visits,
                                 uint8_t* action) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    dk::az::Mem m = az_mem(nodes, states, g, cap_nodes, cap_states);
    dk::az::Game gm = games[g];
    uint32_t v[39];
    const int a = dk::az::finish(gm, m, temp_mode, temperature, v);
    for (int k = 0; k < 39; ++k) visits[39 * (size_t)g + k] = v[k];
    action[g] = a < 0 ? (uint8_t)DK_NONE : (uint8_t)a;
    games[g] = gm;
}

// the games' SmallRng states: dir 0 reads them into rng[g][4], dir 1 sets them (a caller's
// &mut SmallRng carried across searches, async_mcts.rs:224-406 takes `rng: &mut SmallRng`)
__global__ void az_rng_kernel(dk::az::Game* games, uint32_t n, uint64_t* rng, int dir) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n) return;
    for (int i = 0; i < 4; ++i) {
        if (dir) games[g].rng[i] = rng[4 * (size_t)g + i];
        else rng[4 * (size_t)g + i] = games[g].rng[i];
    }
}

// records of packed states that have no announcements yet
__global__ void az_records_kernel(const dk_state* states, uint32_t n, dk_az_state* out, int* err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dk_az_state r;
    r.state = states[i];
    for (int k = 0; k < 12; ++k) { r.ann_card[k] = 0; r.ann_code[k] = 0; }
    r.ann_n = 0;
    for (int k = 0; k < 7; ++k) r.reserved[k] = 0;
    if (r.state.raw[127] != DK_GAME_FULL_DOKO || r.state.fdo.ann_count != 0) atomicOr(err, 2);
    out[i] = r;
}

// take_action_by_action_index(a, skip_single = true) on game records (self-play moves);
// DK_NONE leaves a record unchanged
__global__ void az_step_kernel(dk_az_state* records, const uint8_t* actions, uint32_t n, int* err) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t a = actions[i];
    if (a == DK_NONE) return;
    dk_az_state r = records[i];
    dk::fdo::Work w; dk::fdo::unpack(r.state.fdo, w);
    if (a >= 39 || !((dk::fdo::legal_actions(w) >> a) & 1)) { atomicOr(err, 2); return; }
    dk::az::take_action(r, a);
    records[i] = r;
}

// encode_state_pi: one lane per record, 311 int32 tokens
__global__ void az_encode_kernel(const dk_az_state* records, uint32_t n, int32_t* tokens) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int32_t* o = tokens + 311 * (size_t)i;
    auto put = [o](uint32_t k, uint32_t v) { o[k] = (int32_t)v; };
    dk::enc::encode_state_pi(records[i], put);
}

// IMPI autoregressive determinization (engine/ar_engine.h), one thread per lane
__global__ void ar_begin_kernel(const dk_az_state* info, uint32_t samples, const uint64_t* seeds, uint32_t n,
                                dk::ar::Lane* lanes, uint32_t* rounds) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dk::ar::Lane L;
    const uint32_t g = dk::ar::init(info[i / samples], seeds[i], L);
    lanes[i] = L;
    atomicMax(rounds, g);
}

__global__ void ar_guesses_kernel(const dk_az_state* info, uint32_t n, uint32_t* counts) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dk::ar::Lane L;
    counts[i] = dk::ar::init(info[i], 0, L);
}

__global__ void ar_prepare_kernel(const dk_az_state* info, uint32_t samples, uint32_t n, dk::ar::Lane* lanes,
                                  float log_chance, int32_t* tokens) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dk::ar::Lane L = lanes[i];
    if (L.status != dk::ar::RUNNING) return;
    int32_t* o = tokens + (size_t)dk::ar::TOKENS * i;
    auto put = [o](uint32_t k, uint32_t v) { o[k] = (int32_t)v; };
    dk::ar::prepare(info[i / samples], L, log_chance, put);
    lanes[i] = L;
}

__global__ void ar_choose_kernel(uint32_t n, dk::ar::Lane* lanes, const float* logits, float temperature) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dk::ar::Lane L = lanes[i];
    if (L.status != dk::ar::RUNNING || L.guess == DK_NONE) return;
    dk::ar::choose(L, logits + (size_t)dk::ar::OUT * i, temperature);
    lanes[i] = L;
}

// DefaultImpiPolicy::execute without one consistent sample (compare_impi.rs:355-370):
// a random legal action other than the five announcements (FdoAllowedActions::random).
__global__ void ar_fallback_kernel(uint32_t n_info, uint32_t samples, const uint8_t* status, const uint64_t* allowed,
                                   const uint64_t* seeds, uint8_t* action, uint32_t* successes) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_info) return;
    uint32_t ok = 0;
    for (uint32_t s = 0; s < samples; ++s) ok += status[(size_t)i * samples + s] == 0 ? 1u : 0u;
    successes[i] = ok;
    if (ok) return;
    const uint64_t m = allowed[i] & ~dk::fdo::ANN_ACTIONS;
    if (m == 0) { action[i] = DK_NONE; return; }
    dk::Rng rng = dk::Rng::seed_from_u64(seeds[i]);
    action[i] = (uint8_t)dk::ctz64(dk::random_single(m, rng));
}

__global__ void ar_output_kernel(const dk_az_state* info, uint32_t samples, uint32_t n, const dk::ar::Lane* lanes,
                                 dk_state* out, uint8_t* status, uint8_t* reason) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const dk::ar::Lane L = lanes[i];
    dk::ar::output(info[i / samples], L, out[i].fdo);
    // lane status -> ABI status: 0 consistent, 1 not consistent, 2 reference panic, 3 unfinished
    status[i] = L.status == dk::ar::CONSISTENT ? 0 : L.status == dk::ar::NOT_CONSISTENT ? 1 : L.status == dk::ar::PANIC ? 2 : 3;
    reason[i] = L.reason;
}

// PolicyFusionMaxN / PolicyFusionAverageStrategy accumulators (policy_fusion.rs:23-123).
// One thread per (infostate, action).
// Queue order of the search's root groups: descending cards left to play (the group's first
// root), so the longest trees start first and the persistent grid's tail is made of short
// groups (longest-processing-time-first).  Roots are independent, so the order changes no
// result.  One workgroup: a 64-bin counting sort (order within a bin is arbitrary).
__global__ void __launch_bounds__(1024) group_order_kernel(const dk_state* roots, uint32_t n, uint32_t rpw,
                                                           uint32_t groups, uint32_t* order, const uint32_t* perm) {
    __shared__ uint32_t hist[64];
    if (threadIdx.x < 64) hist[threadIdx.x] = 0;
    __syncthreads();
    auto key = [&](uint32_t g) {
        const uint32_t ci = roots[perm ? perm[(size_t)g * rpw] : (size_t)g * rpw].fdo.card_index;
        return 63u - (ci < 48u ? 48u - ci : 0u);   // ascending key = descending cards left
    };
    for (uint32_t g = threadIdx.x; g < groups; g += blockDim.x) atomicAdd(&hist[key(g)], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t sum = 0;
        for (int b = 0; b < 64; ++b) { const uint32_t c = hist[b]; hist[b] = sum; sum += c; }
    }
    __syncthreads();
    for (uint32_t g = threadIdx.x; g < groups; g += blockDim.x) order[atomicAdd(&hist[key(g)], 1u)] = g;
    (void)n;
}

// Depth-homogeneous waves.  A wave pays for the union of its lanes' instruction streams:
// roots of different depths (cards left) in one wave pay the selection of the deep ones
// AND the rollouts of the shallow ones.  A batch whose 64-root groups mix depths (the
// samples of several infostates per group, e.g. one rank's share of a sample-split batch)
// is therefore searched through a permutation: within each window of W consecutive roots,
// a STABLE counting sort by cards left (most first).  Root i of the launch order is
// perm[i]; results stay indexed by root, so the order changes no value.  One 256-thread
// workgroup per window; stable ranks per 64-root chunk from wave ballots.
constexpr uint32_t ROOT_SORT_MAX_WINDOW = 4096;
constexpr uint32_t ROOT_SORT_BINS = 49;   // card_index 0..48 (48 = finished)
__global__ void __launch_bounds__(256) root_sort_kernel(const dk_state* roots, uint32_t n, uint32_t window,
                                                        uint32_t* perm) {
    __shared__ uint32_t cnt[ROOT_SORT_MAX_WINDOW / 64][ROOT_SORT_BINS];   // per-chunk counts -> chunk prefixes
    __shared__ uint32_t base[ROOT_SORT_BINS];
    const uint32_t start = blockIdx.x * window;
    const uint32_t len = n - start < window ? n - start : window;
    const uint32_t chunks = (len + 63) / 64;
    const uint32_t wv = threadIdx.x / 64, lane = threadIdx.x % 64;
    for (uint32_t t = threadIdx.x; t < chunks * ROOT_SORT_BINS; t += blockDim.x) cnt[t / ROOT_SORT_BINS][t % ROOT_SORT_BINS] = 0;
    __syncthreads();
    auto key_of = [&](uint32_t i) {
        const uint32_t ci = roots[start + i].fdo.card_index;
        return ci < 48u ? ci : 48u;
    };
    for (uint32_t c = wv; c < chunks; c += blockDim.x / 64) {
        const uint32_t i = c * 64 + lane;
        if (i < len) atomicAdd(&cnt[c][key_of(i)], 1u);
    }
    __syncthreads();
    if (threadIdx.x < ROOT_SORT_BINS) {   // exclusive prefix over the chunks, per bin
        uint32_t s = 0;
        for (uint32_t c = 0; c < chunks; ++c) { const uint32_t v = cnt[c][threadIdx.x]; cnt[c][threadIdx.x] = s; s += v; }
        base[threadIdx.x] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {               // exclusive prefix over the bins (ascending card_index = most cards left first)
        uint32_t s = 0;
        for (uint32_t b = 0; b < ROOT_SORT_BINS; ++b) { const uint32_t v = base[b]; base[b] = s; s += v; }
    }
    __syncthreads();
    for (uint32_t c = wv; c < chunks; c += blockDim.x / 64) {
        const uint32_t i = c * 64 + lane;
        const bool live = i < len;
        const uint32_t k = live ? key_of(i) : 0xFFFFFFFFu;
        const uint64_t lt = lane ? (~0ULL >> (64 - lane)) : 0ULL;
        uint32_t rank = 0;
        uint64_t todo = __ballot(live);
        while (todo) {                    // one ballot per distinct key in the chunk
            const uint32_t src = (uint32_t)__builtin_ctzll(todo);
            const uint32_t kk = (uint32_t)__shfl((int)k, (int)src);
            const uint64_t m = __ballot(live && k == kk);
            if (live && k == kk) rank = (uint32_t)__builtin_popcountll(m & lt);
            todo &= ~m;
        }
        if (live) perm[start + base[k] + cnt[c][k] + rank] = start + i;
    }
}

// `valid` (nullable): per-sample flags; samples with valid == 0 (failed determinizations,
// compare_impi.rs:276-288) take no part in the fusion.
__global__ void fuse_accumulate_kernel(const uint32_t* visits, uint32_t n_info, uint32_t samples, const uint8_t* valid,
                                       const uint64_t* allowed, int mode, uint32_t* acc_u32, float* acc_f32) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_info * 39) return;
    const uint32_t info = t / 39, a = t % 39;
    const uint64_t al = allowed[info];
    if (mode == DK_FUSE_MAXN) {
        if (!((al >> a) & 1)) { acc_u32[t] = 0u; return; }   // masked to UINT32_MAX in select (summable across ranks)
        uint32_t cum = 0;
        for (uint32_t s = 0; s < samples; ++s) {
            if (valid && !valid[(size_t)info * samples + s]) continue;
            const uint32_t* row = visits + ((size_t)info * samples + s) * 39;
            const uint32_t va = row[a];
            uint32_t rank = 1;
            for (uint32_t b = 0; b < 39; ++b) {
                if (!((al >> b) & 1)) continue;
                const uint32_t vb = row[b];
                rank += (vb > va || (vb == va && b < a)) ? 1u : 0u;   // stable sort by Reverse(visits)
            }
            cum += rank;
        }
        acc_u32[t] = cum;
    } else {
        float sum = 0.0f;
        for (uint32_t s = 0; s < samples; ++s) {
            if (valid && !valid[(size_t)info * samples + s]) continue;
            const uint32_t* row = visits + ((size_t)info * samples + s) * 39;
            uint64_t total = 0;
            for (uint32_t b = 0; b < 39; ++b) total += row[b];
            sum += (float)row[a] / (float)total;
        }
        acc_f32[t] = sum;
    }
}

__global__ void fuse_select_kernel(uint32_t n_info, int mode, const uint64_t* allowed, const uint32_t* acc_u32,
                                   const float* acc_f32, uint8_t* action) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_info) return;
    int best = 0;
    if (mode == DK_FUSE_MAXN) {
        const uint32_t* r = acc_u32 + (size_t)i * 39;
        const uint64_t al = allowed[i];
        uint32_t bk = (al & 1) ? r[0] : 0xFFFFFFFFu;   // disallowed actions rank u32::MAX (policy_fusion.rs:33-39)
        for (int a = 1; a < 39; ++a) {
            const uint32_t k = ((al >> a) & 1) ? r[a] : 0xFFFFFFFFu;
            if (k < bk) { bk = k; best = a; }                          // min_by_key: first minimum
        }
    } else {
        const float* p = acc_f32 + (size_t)i * 39;
        for (int a = 1; a < 39; ++a) if (!(p[best] > p[a])) best = a;     // max_by: last maximum
    }
    action[i] = (uint8_t)best;
}

}  // namespace

// ==================================================================== host side
struct dk_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    uint32_t max_roots = 0, max_iters = 0, cap_slots = 0;
    uint32_t state_stride = 0;      // node-state records per lane region (>= max_iters + 1)
    uint32_t pool_roots = 0;        // roots the node pools hold at once (min(max_roots, DK_POOL_ROOTS or
                                    // the resident capacity: CUs x 12 single-wave workgroups x 64 lanes))
    int cu_count = 0;
    // In-flight search launches.  dk_search_batch_async may be called on several streams at
    // once (independent decision batches in flight, as the reference's evaluator runs many
    // games at a time).  Each launch takes a Slot -- its own group-queue counters, retry list,
    // root orders, error flag and events -- and a range of pool lanes [lane_base, lane_base +
    // lanes), allocated round-robin over the pools.  Before it starts, the launch waits
    // (hipStreamWaitEvent, on the GPU) for the previous user of its slot and for every earlier
    // launch whose lanes overlap its own, so launches whose lane ranges are disjoint (batches
    // smaller than the resident grid) run concurrently and larger ones serialise.  The fallback
    // pool is shared: fallback passes wait for the previous one.
    struct Slot {
        uint32_t* queue = nullptr;      // root-group counter of the persistent search grid
        uint32_t* queue_fb = nullptr;   // the fallback pass's counter
        uint32_t* retry = nullptr;      // [0] = count, then the roots the main pools could not hold
        uint32_t* order = nullptr;      // queue order of the root groups (group_order_kernel)
        uint32_t* perm = nullptr;       // depth-sorted root order (root_sort_kernel)
        hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
        uint32_t lane_base = 0, lanes = 0;
        bool used = false;              // `done` has been recorded
        bool pending = false;           // err[slot] not yet collected by dk_sync on `stream`
        uint32_t clock_first = 0, clock_n = 0, clock_stride = 1;   // its waves' entries in wave_clock
        hipStream_t stream = nullptr;
    };
    static constexpr int MAX_INFLIGHT = 8;
    std::vector<Slot> slots;
    // The latest launch on each fixed region of REGION_LANES pool lanes (a slot index, -1 =
    // none).  A launch waits for every region it covers, so an earlier launch that still runs
    // on those lanes is waited for even after its slot has been reused for other lanes: a
    // slot's latest launch is ordered after all of its earlier ones (same stream, or the
    // reuse waited for them), so waiting on its `done` covers them.
    static constexpr uint32_t REGION_LANES = 1024;
    std::vector<int> region_slot;
    // Errors of search launches folded in when their slot was reused before dk_sync collected
    // them (more than MAX_INFLIGHT launches in flight), per stream; dk_sync(stream) reports them.
    std::vector<std::pair<hipStream_t, int>> stream_err;
    int* slot_err = nullptr;        // [MAX_INFLIGHT] error flags of the search launches
    uint32_t next_slot = 0, lane_cursor = 0;
    int last_slot = -1;             // the latest launch (dk_last_search_ms)
    hipEvent_t fb_done = nullptr;   // the latest fallback pass
    bool fb_used = false;
    // Slot-capacity fallback: pools are sized from the measured demand (default 64 + 8 x
    // iterations slots per root, against the proven 42 + 12 x iterations); a root that runs out
    // is appended to its launch's `retry` list ([0] = count) and searched again, from its seed,
    // by a second launch over a small pool with the proven capacity (fb_*).  Results do not change.
    uint32_t* high_water = nullptr; // [0] largest slot demand of a root completed in the main pools, [1] roots
                                    // that overflowed them, [2] largest demand of a root the fallback pass
                                    // completed (cumulative since dk_create; dk_pool_high_water)
    void* fb_hot = nullptr;
    dk::NodeCold* fb_cold = nullptr;
    uint32_t* fb_ovf = nullptr;
    uint64_t* fb_ovf_st = nullptr;
    void* fb_states = nullptr;
    uint32_t fb_slots = 0, fb_roots = 0;
    uint64_t fb_bytes = 0;
    uint32_t root_window = 1024;    // roots per depth-sort window (DK_ROOT_WINDOW; 0 = launch order = root order):
                                    // one rank's share of C4 at N = 8 (8 samples per infostate) 410 -> 389 ms,
                                    // C3 at N = 1 unchanged (381 / 382 ms); 4096 reorders C3's groups (+2.4 %)
    int group_order = -1;           // DK_GROUP_ORDER=0 / 1 forces index order / longest-first; -1: per engine
    void* hot = nullptr;            // hot records, 32 B per slot (NodeHot16 launches use half)
    dk::NodeCold* cold = nullptr;
    uint32_t* ovf = nullptr;
    uint64_t* ovf_st = nullptr;
    void* states = nullptr;
    double* ln_table = nullptr;
    int* err = nullptr;
    int last_error = DK_OK;
    uint64_t pool_bytes = 0;
    uint32_t roots_per_wave = 64;   // pool region width; DK_ROOTS_PER_WAVE fixes the launch width too
    bool rpw_fixed = false;
    int hot_layout = 0;             // DK_HOT_RECORD=8|16|32 fixes the hot-record layout; 0 = per launch
    int pair = -1;                  // DK_PAIR=0 / 1: lane pairs off / on for launches of <= 32 roots per wave
    bool p8_ok = false;             // the pools' slot capacities suit the 8-B records (even-aligned blocks)
    bool wide = false;              // a wave's pool region reaches 4 GiB: NodeHot32W (64-bit offsets) only
    size_t hot_rec = 16;            // bytes per hot-record slot in the pools (16, or 32: forced / wide)
    uint32_t block_align = 1;       // DK_BLOCK_ALIGN: child blocks of the main pass start at multiples of
                                    // this many slots (8-B records: at least 2); the fallback pass packs
    bool ln_in_lds = false;         // DK_LN_LDS=1: ln(N) table copied into every workgroup's LDS (8 KB at
                                    // 1000 iterations); by default it is read through the L1/L2 caches
    int lds_path = 16;              // path entries kept in LDS (deeper ones spill to global): at most
                                    // 16, shortened per launch while it costs residency (launch_search_t)
    bool lds_path_fixed = false;    // DK_LDS_PATH (1..MAX_PATH) fixes it
    bool verbose = false;           // DK_VERBOSE=1: one stderr line per search launch (shape, residency)
    uint64_t* prof = nullptr;       // phase timers (DK_PHASE_PROF builds only)
    uint64_t* wave_clock = nullptr; // [pool_roots][4] realtime start / end, shader-clock start / end of the search waves (by first lane)
    // AlphaZero PUCT search (dk_az_*): per-game node / state regions, allocated on first use
    dk::az::Node* az_nodes = nullptr;
    dk_az_state* az_states = nullptr;
    dk::az::Game* az_games = nullptr;
    size_t az_bytes = 0;
    uint32_t az_n = 0, az_iters = 0, az_cap_nodes = 0, az_cap_states = 0, az_done = 0;
    // IMPI autoregressive determinization (dk_ar_*): one lane per (infostate, sample)
    dk::ar::Lane* ar_lanes = nullptr;
    const dk_az_state* ar_info = nullptr;
    uint32_t ar_cap = 0, ar_n = 0, ar_samples = 0;
    float ar_log_chance = 0.0f;
    int az_epoch = 0;
    bool az_root_done = false;
    // glibc logf / powf(., 1 / shape) of the 2^23 Open01<f32> values (rand_distr.h), built on first use
    float* rd_ln = nullptr;
    // powf(u, 1/alpha) tables per shape (alpha < 1), most recently built first: a few alphas in use
    // on one context (e.g. 0.5 for evaluation, 0.8 for training) each keep their table
    static constexpr int RD_PW_CACHE = 4;
    float* rd_pw[RD_PW_CACHE] = {};
    float rd_inv_shape[RD_PW_CACHE] = {};
    std::vector<void*> scratch;
    std::vector<size_t> scratch_size;
    // results of the synchronous (host-pointer) entry points: DMA into this page-locked buffer,
    // copied into the caller's memory by the CPU once the stream is drained (copy_out / finish)
    char* pinned = nullptr;
    size_t pinned_size = 0, pinned_used = 0;
    struct OutCopy { void* dst; size_t off, bytes; };
    std::vector<OutCopy> outs;
    std::mutex mu;                  // host-pointer calls (scratch buffers, ctx->stream)
    std::mutex slot_mu;             // search slots and lane ranges
};

namespace {

constexpr size_t FALLBACK_ROOTS = 64 * 64;   // roots the fallback pool holds at once
constexpr size_t FALLBACK_BYTES = 16ull << 30; // ... within this many bytes (at least one 64-root region)

// node-state records (adapters.h Node: 64 B for both card games)
constexpr size_t STATE_SLOT_BYTES =
    sizeof(dk::fdo::Node) > sizeof(dk::dko::Node) ? sizeof(dk::fdo::Node) : sizeof(dk::dko::Node);
static_assert(STATE_SLOT_BYTES == 64 && sizeof(dk::ttt::Work) <= STATE_SLOT_BYTES, "node-state records");

unsigned grid_for(size_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

hipStream_t pick(dk_ctx* ctx, void* s) { return s ? (hipStream_t)s : ctx->stream; }

// scratch buffer k of at least `bytes` (host-pointer convenience API only)
void* scratch(dk_ctx* ctx, int k, size_t bytes) {
    if ((int)ctx->scratch.size() <= k) { ctx->scratch.resize(k + 1, nullptr); ctx->scratch_size.resize(k + 1, 0); }
    if (ctx->scratch_size[k] < bytes) {
        if (ctx->scratch[k]) (void)hipFree(ctx->scratch[k]);
        ctx->scratch[k] = nullptr;
        if (hipMalloc(&ctx->scratch[k], bytes) != hipSuccess) { ctx->scratch_size[k] = 0; return nullptr; }
        ctx->scratch_size[k] = bytes;
    }
    return ctx->scratch[k];
}

// The queued result copies of a synchronous entry point, after its stream is drained.
void flush_outs(dk_ctx* ctx) {
    for (const dk_ctx::OutCopy& o : ctx->outs) memcpy(o.dst, ctx->pinned + o.off, o.bytes);
    ctx->outs.clear();
    ctx->pinned_used = 0;
}

// A device-to-host result copy of a synchronous entry point (round 4, the review's pageable-copy
// concern): the DMA lands in the context's page-locked staging buffer on ctx->stream, and
// finish() copies it into the caller's (possibly pageable) buffer with the CPU after the stream
// is drained, so nothing depends on how the runtime stages a copy into pageable memory.
hipError_t copy_out(dk_ctx* ctx, void* dst, const void* src, size_t bytes) {
    hipError_t e = hipSuccess;
    const size_t off = (ctx->pinned_used + 255) & ~(size_t)255;
    if (off + bytes > ctx->pinned_size) {
        // drain what is queued, then grow to hold everything this call has queued so far (the
        // next call with the same sizes then fits without a mid-call drain)
        const size_t want = off + bytes;
        if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) { ctx->outs.clear(); ctx->pinned_used = 0; return e; }
        flush_outs(ctx);
        if (want > ctx->pinned_size) {
            if (ctx->pinned) (void)hipHostFree(ctx->pinned);
            const size_t grown = 2 * ctx->pinned_size > want ? 2 * ctx->pinned_size : want;
            ctx->pinned = nullptr;
            ctx->pinned_size = 0;
            const size_t sz = grown < ((size_t)1 << 20) ? ((size_t)1 << 20) : grown;
            if ((e = hipHostMalloc((void**)&ctx->pinned, sz, hipHostMallocDefault)) != hipSuccess) { ctx->pinned = nullptr; return e; }
            ctx->pinned_size = sz;
        }
        return copy_out(ctx, dst, src, bytes);
    }
    if ((e = hipMemcpyAsync(ctx->pinned + off, src, bytes, hipMemcpyDeviceToHost, ctx->stream)) != hipSuccess) {
        ctx->outs.clear();
        ctx->pinned_used = 0;
        return e;
    }
    ctx->outs.push_back({dst, off, bytes});
    ctx->pinned_used = off + bytes;
    return hipSuccess;
}

// Wait for stream `st`, then collect the error flags: the context's (env, sampler, AlphaZero
// kernels) and those of the search launches issued on `st` since its last sync.  host_copies:
// the caller is a synchronous host-pointer entry point holding ctx->mu, whose queued result
// copies (ctx->outs, the staging buffer) are flushed here.  dk_sync passes false: it never
// touches another thread's staging state (a dk_sync racing a host-pointer call).
int finish(dk_ctx* ctx, hipStream_t st, bool host_copies = true) {
    if (hipStreamSynchronize(st) != hipSuccess) {
        if (host_copies) { ctx->outs.clear(); ctx->pinned_used = 0; }
        return ctx->last_error = DK_E_LAUNCH;
    }
    if (host_copies && st == ctx->stream) flush_outs(ctx);
    int flag = 0;
    if (hipMemcpy(&flag, ctx->err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return ctx->last_error = DK_E_LAUNCH;
    (void)hipMemset(ctx->err, 0, sizeof(int));
    {
        std::lock_guard<std::mutex> g(ctx->slot_mu);
        for (size_t i = 0; i < ctx->stream_err.size();) {
            if (ctx->stream_err[i].first == st) {
                flag |= ctx->stream_err[i].second;
                ctx->stream_err.erase(ctx->stream_err.begin() + (long)i);
            } else {
                ++i;
            }
        }
        int se[dk_ctx::MAX_INFLIGHT];
        bool any = false;
        for (const dk_ctx::Slot& sl : ctx->slots) any |= sl.pending && sl.stream == st;
        if (any) {
            if (hipMemcpy(se, ctx->slot_err, sizeof(se), hipMemcpyDeviceToHost) != hipSuccess) return ctx->last_error = DK_E_LAUNCH;
            for (int k = 0; k < (int)ctx->slots.size(); ++k) {
                dk_ctx::Slot& sl = ctx->slots[k];
                if (!sl.pending || sl.stream != st) continue;
                flag |= se[k];
                sl.pending = false;
            }
        }
    }
    if (flag & 1) return ctx->last_error = DK_E_CAPACITY;
    if (flag & 2) return ctx->last_error = DK_E_STATE;
    return ctx->last_error = DK_OK;
}

// Roots per wave of one launch.  A wave64 instruction costs the same whatever its
// exec mask, so full 64-root waves do the most work per instruction; but a batch
// too small to give every SIMD a wave leaves SIMDs idle.  Take the widest wave
// (a multiple of 16) that still puts one wave on every SIMD: 32,768 roots on 256
// CUs run as 1,024 waves of 32 (756 M/s for C2, against 679 M/s as 512 waves of
// 64 and 646 M/s as 2,048 waves of 16).  Results do not depend on the width.
uint32_t launch_rpw(const dk_ctx* ctx, uint32_t n) {
    if (ctx->rpw_fixed) return ctx->roots_per_wave;
    const uint32_t simds = 4u * (uint32_t)ctx->cu_count;
    uint32_t r = (n + simds - 1) / simds;
    r = (r + 15u) & ~15u;
    return r < 16u ? 16u : (r > ctx->roots_per_wave ? ctx->roots_per_wave : r);
}

template <class E, bool LN, class H>
hipError_t launch_search_t(dk_ctx* ctx, const dk_state* roots, const uint64_t* seeds, uint32_t n, uint32_t iters,
                           double c, uint32_t* visits, double* values, uint8_t* best, hipStream_t st,
                           size_t ln_bytes, uint32_t rpw, dk_ctx::Slot& sl, int* err, uint64_t* rng_io) {
    const auto kern = search_kernel<E, LN, H>;
    // LDS per path entry and lane: slot word + stats (8-B records: their 32-bit stats word)
    constexpr size_t PATH_ENTRY_BYTES = dk::is_p8<H>::value ? 8 : 12;
    const size_t pw = H::PAIR ? (size_t)WAVE : rpw;   // lanes with a path (lane pairs: both lanes)
    auto occupancy = [&](int lp) {
        int b = 0;
        const size_t bytes = ln_bytes + (size_t)lp * pw * PATH_ENTRY_BYTES;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, kern, WAVE, bytes) == hipSuccess ? b : 0;
    };
    // LDS path length: DK_LDS_PATH, or else the longest (<= 16) that keeps the residency
    // the registers allow with one entry of headroom.  At 64 roots per wave a 16-entry
    // path (12 KB + the card table) fits 11 workgroups per CU; the calculator admits 12
    // at 15 entries, but 15 measured no faster than 16 (the hardware's LDS allocation
    // granularity), while 14 (12 workgroups per CU) is 12 % faster on C3 than 16: medians of 5
    // interleaved runs, 1,885 against 1,685 M rollouts/s (tools/ab_ldspath.sh).
    // Paths deeper than 14 are rare and spill to the global overflow.
    int lp = ctx->lds_path;
    if (!ctx->lds_path_fixed) {
        const int best = occupancy(1);
        while (lp > 1 && occupancy(lp + 1) < best) --lp;
    }
    const size_t lds_bytes = ln_bytes + (size_t)lp * pw * PATH_ENTRY_BYTES;
    int per_cu = occupancy(lp);
    if (per_cu < 1) per_cu = 1;
    const uint32_t groups = grid_for(n, rpw);
    const uint32_t resident = (uint32_t)per_cu * (uint32_t)ctx->cu_count;
    const uint32_t regions = ctx->pool_roots / rpw;
    uint32_t grid = groups < resident ? groups : resident;
    grid = grid < regions ? grid : regions;
    if (grid == 0) return hipErrorInvalidValue;
    // this launch's pool lanes, round-robin over the pools; wait for the earlier launches on them
    const uint32_t lanes = grid * rpw;
    if (ctx->lane_cursor + lanes > ctx->pool_roots) ctx->lane_cursor = 0;
    const uint32_t base = ctx->lane_cursor;
    ctx->lane_cursor += lanes;
    hipError_t e = hipSuccess;
    const int self = (int)(&sl - ctx->slots.data());
    const uint32_t r0 = base / dk_ctx::REGION_LANES, r1 = (base + lanes - 1) / dk_ctx::REGION_LANES;
    uint32_t waited = 0;   // slots already waited for
    for (uint32_t r = r0; r <= r1; ++r) {
        const int k = ctx->region_slot[r];
        if (k < 0 || k == self || ((waited >> k) & 1u)) continue;
        const dk_ctx::Slot& o = ctx->slots[k];
        waited |= 1u << k;
        if (o.used && o.stream != st && (e = hipStreamWaitEvent(st, o.done, 0)) != hipSuccess) return e;
    }
    for (uint32_t r = r0; r <= r1; ++r) ctx->region_slot[r] = self;
    sl.lane_base = base;
    sl.lanes = lanes;
    if (ctx->verbose)
        fprintf(stderr, "doko_amd: search n=%u rpw=%u hot=%dB lds_path=%d lds=%zuB resident/CU=%d grid=%u root_window=%u "
                "wide=%d lanes=%u+%u pair=%d long=%d\n", n, rpw, (int)sizeof(H), lp, lds_bytes, per_cu, grid, ctx->root_window,
                (int)H::WIDE, base, lanes, (int)H::PAIR, (int)H::LONG);
    e = hipMemsetAsync(sl.queue, 0, sizeof(uint32_t), st);
    if (e != hipSuccess) return e;
    // group order only matters when waves take several groups each
    const bool want = ctx->group_order < 0 ? E::ORDER_GROUPS : ctx->group_order == 1;
    // depth-homogeneous waves (root_sort_kernel) when the batch has several groups
    const uint32_t W = ctx->root_window;
    const bool sorted = W && E::GAME != DK_GAME_TTT && groups > 1;
    if (sorted) {
        hipLaunchKernelGGL(root_sort_kernel, dim3(grid_for(n, W)), dim3(256), 0, st, roots, n, W, sl.perm);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const uint32_t* perm = sorted ? (const uint32_t*)sl.perm : (const uint32_t*)nullptr;
    const bool ordered = want && E::GAME != DK_GAME_TTT && groups > grid;
    if (ordered) {
        hipLaunchKernelGGL(group_order_kernel, dim3(1), dim3(1024), 0, st, roots, n, rpw, groups, sl.order, perm);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const bool fallback = ctx->fb_hot != nullptr;
    if (fallback) {
        e = hipMemsetAsync(sl.retry, 0, sizeof(uint32_t), st);
        if (e == hipSuccess) e = hipMemsetAsync(sl.queue_fb, 0, sizeof(uint32_t), st);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, dim3(grid), dim3(WAVE), lds_bytes, st, roots, seeds, n, iters, c, ctx->ln_table,
                       ctx->hot, ctx->cold, (typename E::Node*)ctx->states, ctx->ovf, ctx->ovf_st, ctx->cap_slots,
                       ctx->state_stride,
                       ctx->block_align == dk::BALIGN_LINE ? dk::BALIGN_LINE | (uint32_t)(128 / sizeof(H)) : ctx->block_align,
                       rpw, lp, visits, values, best, err, sl.queue, ctx->prof,
                       ordered ? (const uint32_t*)sl.order : (const uint32_t*)nullptr,
                       fallback ? sl.retry : (uint32_t*)nullptr, (const uint32_t*)nullptr, ctx->high_water, perm, base,
                       ctx->wave_clock, rng_io);
    sl.clock_first = base;
    sl.clock_n = grid;
    sl.clock_stride = rpw;
    e = hipGetLastError();
    if (e != hipSuccess || !fallback) return e;
    // the fallback pool is shared by all launches: one fallback pass at a time
    if (ctx->fb_used && (e = hipStreamWaitEvent(st, ctx->fb_done, 0)) != hipSuccess) return e;
    // Second pass over the roots the main pool could not hold (retry[0] of them; the grid
    // drains at once when there are none): same kernel, proven-capacity pool, no retry list,
    // so running out there is DK_E_CAPACITY.
    const uint32_t fb_grid = ctx->fb_roots / rpw;
    hipLaunchKernelGGL(kern, dim3(fb_grid), dim3(WAVE), lds_bytes, st, roots, seeds, n, iters, c, ctx->ln_table,
                       ctx->fb_hot, ctx->fb_cold, (typename E::Node*)ctx->fb_states, ctx->fb_ovf, ctx->fb_ovf_st,
                       ctx->fb_slots, ctx->state_stride, 1u, rpw, lp, visits, values, best, err, sl.queue_fb, ctx->prof,
                       (const uint32_t*)nullptr, (uint32_t*)nullptr, (const uint32_t*)sl.retry, ctx->high_water + 2,
                       (const uint32_t*)nullptr, 0u, (uint64_t*)nullptr, rng_io);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipEventRecord(ctx->fb_done, st)) != hipSuccess) return e;
    ctx->fb_used = true;
    return hipSuccess;
}

template <class E>
hipError_t launch_search(dk_ctx* ctx, const dk_state* roots, const uint64_t* seeds, uint32_t n, uint32_t iters,
                         double c, uint32_t* visits, double* values, uint8_t* best, hipStream_t st, dk_ctx::Slot& sl,
                         int* err, uint64_t* rng_io) {
    const bool ln = iters + 1 <= LN_LDS_MAX && ctx->ln_in_lds;
    const uint32_t rpw = launch_rpw(ctx, n);
    const size_t ln_bytes = ln ? (size_t)((iters + 2) & ~1u) * 8 : 0;
    // hot-record layout (search_core.h): 8 B once the batch gives every SIMD two waves, 16 B
    // when a single wave per SIMD leaves the pick's latency exposed (round 4, alternated
    // contexts: C2 33.0 ms against 33.8 ms for the 32-B records and 35.3 ms for 8 B, the
    // 512-infostate batch 41.6 / 42.8 / 43.6 ms; profiles/r04/layout_single_wave.log), 32 B
    // (cached exact means) beyond the 16-B records' 24-bit cross products (P24_MAX_ITERS)
    // beyond P24_MAX_ITERS the 16-B records compare by 64-bit cross products (NodeHot16L /
    // NodeHot16PL, round 5); the 32-B records remain for DK_HOT_RECORD=32 and the wide pools
    const uint32_t simds = 4u * (uint32_t)ctx->cu_count;
    const bool multi = grid_for(n, rpw) >= 2u * simds;
    const bool lng = iters > dk::P24_MAX_ITERS;
    const bool h16 = ctx->hot_layout ? ctx->hot_layout <= 16 : true;
    // 8-B records where their fields hold the search (visits, state index, slots: P8_MAX_ITERS)
    // (with child blocks placed beyond even slots -- DK_BLOCK_ALIGN > 2 or "line" -- only while the main
    // pool's capacity keeps every slot index within the 13-bit child_base / 2 field: the capacity
    // check then bounds the padded blocks; the fallback pass packs, P8_SLOT_BOUND)
    const bool h8 = h16 && iters <= dk::P8_MAX_ITERS && ctx->hot_layout != 16 && ctx->p8_ok &&
                    (ctx->block_align <= 2u || ctx->cap_slots <= (1u << 14)) && (ctx->hot_layout == 8 || multi);
    if (ctx->wide)   // per-wave pool regions of >= 4 GiB: 64-bit offsets (never with ln in LDS: iterations > 2047)
        return launch_search_t<E, false, dk::NodeHot32W>(ctx, roots, seeds, n, iters, c, visits, values, best, st, 0, rpw, sl, err, rng_io);
    // lane pairs where a single wave per SIMD holds at most 32 roots (DK_PAIR=0 / 1 forces)
    const bool pair = h16 && !h8 && rpw <= 32u && (ctx->pair < 0 ? !multi : ctx->pair == 1);
    if (pair && lng)   // (iterations > 4095: never the LDS ln table)
        return launch_search_t<E, false, dk::NodeHot16PL>(ctx, roots, seeds, n, iters, c, visits, values, best, st, 0, rpw, sl, err, rng_io);
    if (pair)
        return ln ? launch_search_t<E, true, dk::NodeHot16P>(ctx, roots, seeds, n, iters, c, visits, values, best, st, ln_bytes, rpw, sl, err, rng_io)
                  : launch_search_t<E, false, dk::NodeHot16P>(ctx, roots, seeds, n, iters, c, visits, values, best, st, ln_bytes, rpw, sl, err, rng_io);
    if (h16 && lng)
        return launch_search_t<E, false, dk::NodeHot16L>(ctx, roots, seeds, n, iters, c, visits, values, best, st, 0, rpw, sl, err, rng_io);
    if (h8)
        return ln ? launch_search_t<E, true, dk::NodeHot8>(ctx, roots, seeds, n, iters, c, visits, values, best, st, ln_bytes, rpw, sl, err, rng_io)
                  : launch_search_t<E, false, dk::NodeHot8>(ctx, roots, seeds, n, iters, c, visits, values, best, st, ln_bytes, rpw, sl, err, rng_io);
    if (h16)
        return ln ? launch_search_t<E, true, dk::NodeHot16>(ctx, roots, seeds, n, iters, c, visits, values, best, st, ln_bytes, rpw, sl, err, rng_io)
                  : launch_search_t<E, false, dk::NodeHot16>(ctx, roots, seeds, n, iters, c, visits, values, best, st, ln_bytes, rpw, sl, err, rng_io);
    return ln ? launch_search_t<E, true, dk::NodeHot32>(ctx, roots, seeds, n, iters, c, visits, values, best, st, ln_bytes, rpw, sl, err, rng_io)
              : launch_search_t<E, false, dk::NodeHot32>(ctx, roots, seeds, n, iters, c, visits, values, best, st, ln_bytes, rpw, sl, err, rng_io);
}

}  // namespace

extern "C" {

int dk_abi_version(void) { return DK_ABI_VERSION; }

const char* dk_status_string(int s) {
    switch (s) {
        case DK_OK: return "ok";
        case DK_E_INVALID: return "invalid argument";
        case DK_E_CAPACITY: return "capacity exceeded";
        case DK_E_STATE: return "illegal action or malformed state";
        case DK_E_NO_DEVICE: return "no usable gfx950 device";
        case DK_E_LAUNCH: return "kernel launch failure";
    }
    return "unknown";
}

dk_ctx* dk_create(const dk_config* cfg) {
    if (!cfg || cfg->max_roots == 0 || cfg->max_iterations == 0) return nullptr;
    if (cfg->max_iterations >= dk::NI_MAX_STATES) return nullptr;  // node state index is 22 bits
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || cfg->device < 0 || cfg->device >= count) return nullptr;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cfg->device) != hipSuccess) return nullptr;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        fprintf(stderr, "doko_amd: device %d is %s, this library is built for gfx950 only\n", cfg->device, prop.gcnArchName);
        return nullptr;
    }
    if (hipSetDevice(cfg->device) != hipSuccess) return nullptr;
    dk_ctx* ctx = new dk_ctx();
    ctx->device = cfg->device;
    ctx->max_roots = cfg->max_roots;
    ctx->max_iters = cfg->max_iterations;
    // Proven bound: the root block (<= 39) plus one block of <= 12 children per
    // iteration (non-root nodes offer at most 12 cards / 9 reservations / 1 pass).
    // The measured demand is far lower (largest over the C3 bench roots: 3,546 slots at
    // 1,000 iterations), so by default the main pools hold 64 + 8 x iterations
    // slots per root (8,192 at 1,000: 43 % high water, where 4,096 was 87 %; the same speed,
    // profiles/r03/cap_ab_4096_8192.log) and the rare root that needs more is
    // searched again in the fallback pool, which has the proven bound.  The default halves
    // (down to 64 + 4 x iterations) while the main pools would take more than half of the free
    // device memory.  cfg->slot_capacity (or env DK_SLOT_CAPACITY) sets the main pools'
    // capacity; at or above the proven bound there is no fallback pool.
    // The capacity is also the stride between the lanes' pool regions, and it is rounded up
    // to a multiple of 256 slots (4 KB of 16-B records): strides 512 B off a multiple of
    // 64 KB (4,064 or 4,128 slots) ran the C3 search 1.6x slower than 4,096 or 12,040
    // (tools/cap_sweep.py; the lanes' accesses fall into the same memory channels).
    // (+2 for the 8-B records' even-aligned blocks: search_core.h P8_SLOT_BOUND)
    const uint32_t proven = dk::P8_SLOT_BOUND(cfg->max_iterations);
    bool cap_default = cfg->slot_capacity == 0;
    uint32_t cap = cfg->slot_capacity ? cfg->slot_capacity : 64u + 8u * cfg->max_iterations;
    if (const char* e = getenv("DK_SLOT_CAPACITY")) {
        const long v = atol(e);
        if (v >= 1) { cap = (uint32_t)v; cap_default = false; }
    }
    cap = cap < proven ? (cap + 255u) & ~255u : proven;
    ctx->cap_slots = cap < proven ? cap : proven;
    ctx->cu_count = prop.multiProcessorCount;
    if (const char* e = getenv("DK_ROOTS_PER_WAVE")) {
        const int v = atoi(e);
        if (v >= 1 && v <= WAVE) { ctx->roots_per_wave = (uint32_t)v; ctx->rpw_fixed = true; }
    }
    if (const char* e = getenv("DK_GROUP_ORDER")) ctx->group_order = atoi(e) != 0 ? 1 : 0;
    if (const char* e = getenv("DK_ROOT_WINDOW")) {
        const long v = atol(e);
        if (v >= 0 && v <= (long)ROOT_SORT_MAX_WINDOW) ctx->root_window = (uint32_t)v;
    }
    if (const char* e = getenv("DK_HOT_RECORD")) {
        const int v = atoi(e);
        if (v == 8 || v == 16 || v == 32) ctx->hot_layout = v;
    }
    if (const char* e = getenv("DK_VERBOSE")) ctx->verbose = atoi(e) != 0;
    if (const char* e = getenv("DK_BLOCK_ALIGN")) {
        // a power of two 1..64: blocks start at multiples of it; "line": blocks kept within one
        // 128-B line (search_core.h block_base; the launch passes the line's slots per layout)
        const int v = atoi(e);
        if (v >= 1 && v <= 64 && (v & (v - 1)) == 0) ctx->block_align = (uint32_t)v;
        else if (strcmp(e, "line") == 0) ctx->block_align = dk::BALIGN_LINE;
    }
    if (const char* e = getenv("DK_PAIR")) ctx->pair = atoi(e) != 0 ? 1 : 0;
    if (const char* e = getenv("DK_LN_LDS")) ctx->ln_in_lds = atoi(e) != 0;
    if (const char* e = getenv("DK_LDS_PATH")) {
        const int v = atoi(e);
        if (v >= 1 && v <= MAX_PATH) { ctx->lds_path = v; ctx->lds_path_fixed = true; }
    }
    // The search grid is persistent (search_kernel): the pools hold the resident waves'
    // roots, and a larger batch streams through them.
    uint64_t pool = (uint64_t)prop.multiProcessorCount * RESIDENT_WG_PER_CU * WAVE;
    if (const char* e = getenv("DK_POOL_ROOTS")) {
        const long long v = atoll(e);
        if (v >= 1) pool = (uint64_t)v;
    }
    if (pool > cfg->max_roots) pool = cfg->max_roots;
    const uint32_t rpw = ctx->roots_per_wave;
    ctx->pool_roots = (uint32_t)((pool + rpw - 1) / rpw * rpw);   // whole regions of rpw roots
    const size_t T = (size_t)cfg->max_iterations + 1;
    // node states per lane region (>= T): DK_STATE_STRIDE, else T
    size_t ST = T;
    if (const char* e = getenv("DK_STATE_STRIDE")) {
        const long long v = atoll(e);
        if (v >= (long long)T) ST = (size_t)v;
    }
    ctx->state_stride = (uint32_t)ST;
    // Hot records per slot for a capacity of S slots: 16 B (the 8-B, 16-B and long 16-B layouts all
    // fit; rounds 1-4 always allocated 32 B), 32 B only when DK_HOT_RECORD=32 forces the cached-mean
    // layout or a wave's regions reach 4 GiB (NodeHot32W, 64-bit offsets).  32-bit pool offsets
    // (GpuMem::at) cover a wave's region only below 4 GiB: 64 lanes x the capacity x the record, in
    // the main and the fallback pools, and the node states.  The default sizing below prices a slot
    // with the record this rule then picks.
    auto hot_rec_for = [&](uint64_t S_, bool* wide) {
        const uint64_t lim = 1ULL << 32, lanes = WAVE;
        const uint64_t slots = S_ < proven ? std::max<uint64_t>(S_, proven) : S_;
        auto wide_at = [&](uint64_t rec) {
            return lanes * slots * rec >= lim || lanes * slots * sizeof(dk::NodeCold) >= lim ||
                   lanes * ST * STATE_SLOT_BYTES >= lim;
        };
        size_t rec = ctx->hot_layout == 32 ? sizeof(dk::NodeHot32) : sizeof(dk::NodeHot16);
        *wide = wide_at(rec);
        return *wide ? sizeof(dk::NodeHot32) : rec;
    };
    if (cap_default) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
            const uint32_t floor_cap = ((64u + 4u * cfg->max_iterations) + 255u) & ~255u;
            auto per_slot = [&](uint32_t S_) { bool w; return hot_rec_for(S_, &w) + sizeof(dk::NodeCold); };
            while (ctx->cap_slots > floor_cap && (size_t)ctx->pool_roots * ctx->cap_slots * per_slot(ctx->cap_slots) > free_b / 2)
                ctx->cap_slots = (ctx->cap_slots / 2 + 255u) & ~255u;
            if (ctx->cap_slots < floor_cap) ctx->cap_slots = floor_cap < proven ? floor_cap : proven;
        }
    }
    const bool with_fallback = ctx->cap_slots < proven;
    const size_t R = ctx->pool_roots, S = ctx->cap_slots;
    {
        bool wide = false;
        ctx->hot_rec = hot_rec_for(S, &wide);
        ctx->wide = wide;
    }
    const size_t HR = ctx->hot_rec;
    bool ok = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMalloc(&ctx->hot, R * S * HR) == hipSuccess;
    ok = ok && hipMalloc(&ctx->cold, R * S * sizeof(dk::NodeCold)) == hipSuccess;
    ok = ok && hipMalloc(&ctx->ovf, R * dk::MAX_DEPTH * sizeof(uint32_t)) == hipSuccess;
    ok = ok && hipMalloc(&ctx->ovf_st, R * dk::MAX_DEPTH * sizeof(uint64_t)) == hipSuccess;
    ok = ok && hipMalloc(&ctx->states, R * ST * STATE_SLOT_BYTES) == hipSuccess;
    ok = ok && hipMalloc(&ctx->ln_table, (T + 1) * sizeof(double)) == hipSuccess;
    ok = ok && hipMalloc(&ctx->err, sizeof(int)) == hipSuccess;
    ok = ok && hipMalloc(&ctx->high_water, 4 * sizeof(uint32_t)) == hipSuccess;
    ok = ok && hipMemset(ctx->high_water, 0, 4 * sizeof(uint32_t)) == hipSuccess;
    ok = ok && hipMalloc(&ctx->wave_clock, (R + 1) * 4 * sizeof(uint64_t)) == hipSuccess;
    ctx->region_slot.assign((R + dk_ctx::REGION_LANES - 1) / dk_ctx::REGION_LANES, -1);
    if (ok && with_fallback) {
        // 64 waves of 64 roots (fewer when the context is smaller): overflow is rare, and the
        // pass only has to finish the few roots that need it
        // (long searches: at most FALLBACK_BYTES, in whole 64-root regions; 64 roots at 200,000
        // iterations are 8 GB)
        const size_t FS = proven, per_root = FS * (HR + sizeof(dk::NodeCold)) + ST * STATE_SLOT_BYTES;
        size_t FR = R < FALLBACK_ROOTS ? R : FALLBACK_ROOTS;
        const size_t by_bytes = std::max<size_t>(64, FALLBACK_BYTES / per_root / 64 * 64);
        FR = FR < by_bytes ? FR : by_bytes;
        ctx->fb_roots = (uint32_t)FR;
        ctx->fb_slots = proven;
        ok = hipMalloc(&ctx->fb_hot, FR * FS * HR) == hipSuccess;
        ok = ok && hipMalloc(&ctx->fb_cold, FR * FS * sizeof(dk::NodeCold)) == hipSuccess;
        ok = ok && hipMalloc(&ctx->fb_ovf, FR * dk::MAX_DEPTH * sizeof(uint32_t)) == hipSuccess;
        ok = ok && hipMalloc(&ctx->fb_ovf_st, FR * dk::MAX_DEPTH * sizeof(uint64_t)) == hipSuccess;
        ok = ok && hipMalloc(&ctx->fb_states, FR * ST * STATE_SLOT_BYTES) == hipSuccess;
        ctx->fb_bytes = FR * FS * (HR + sizeof(dk::NodeCold)) + FR * ST * STATE_SLOT_BYTES;
    }
    // search slots (in-flight launches); the slot's lists are sized for max_roots
    ctx->slots.resize(dk_ctx::MAX_INFLIGHT);
    for (dk_ctx::Slot& sl : ctx->slots) {
        const size_t list = ((size_t)cfg->max_roots + 1) * sizeof(uint32_t);
        ok = ok && hipMalloc(&sl.queue, 2 * sizeof(uint32_t)) == hipSuccess;
        if (ok) sl.queue_fb = sl.queue + 1;
        ok = ok && hipMalloc(&sl.order, list) == hipSuccess && hipMalloc(&sl.perm, list) == hipSuccess;
        ok = ok && (!with_fallback || hipMalloc(&sl.retry, list) == hipSuccess);
        ok = ok && hipEventCreate(&sl.ev0) == hipSuccess && hipEventCreate(&sl.ev1) == hipSuccess &&
             hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) == hipSuccess;
    }
    ok = ok && hipMalloc(&ctx->slot_err, dk_ctx::MAX_INFLIGHT * sizeof(int)) == hipSuccess &&
         hipMemset(ctx->slot_err, 0, dk_ctx::MAX_INFLIGHT * sizeof(int)) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&ctx->fb_done, hipEventDisableTiming) == hipSuccess;
#ifdef DK_PHASE_PROF
    ok = ok && hipMalloc(&ctx->prof, (size_t)cfg->max_roots * dk::PROF_SLOTS * sizeof(uint64_t)) == hipSuccess;
    ok = ok && hipMemset(ctx->prof, 0, (size_t)cfg->max_roots * dk::PROF_SLOTS * sizeof(uint64_t)) == hipSuccess;
#endif
    if (ok) {
        // ln(N) exactly as glibc `log` computes it — what Rust's f64::ln calls (node.rs:253).
        std::vector<double> ln(T + 1);
        for (size_t i = 0; i < ln.size(); ++i) ln[i] = std::log((double)i);
        ok = hipMemcpy(ctx->ln_table, ln.data(), ln.size() * sizeof(double), hipMemcpyHostToDevice) == hipSuccess;
        ok = ok && hipMemset(ctx->err, 0, sizeof(int)) == hipSuccess;
    }
    // A launch of <= P8_MAX_ITERS iterations uses at most P8_SLOT_BOUND(iterations) < 2^14 slots per
    // root, whatever the pools' capacity (sized for max_iterations), so the 8-B records' 13-bit
    // child_base/2 field always holds its slots: only the even block alignment is a condition.
    ctx->p8_ok = ctx->cap_slots % 2 == 0 && ctx->fb_slots % 2 == 0;
    ctx->pool_bytes = R * S * (HR + sizeof(dk::NodeCold)) + R * ST * STATE_SLOT_BYTES + ctx->fb_bytes;
    if (!ok) { dk_destroy(ctx); return nullptr; }
    return ctx;
}

void dk_destroy(dk_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (void* p : ctx->scratch) if (p) (void)hipFree(p);
    if (ctx->pinned) (void)hipHostFree(ctx->pinned);
    if (ctx->hot) (void)hipFree(ctx->hot);
    if (ctx->cold) (void)hipFree(ctx->cold);
    if (ctx->ovf) (void)hipFree(ctx->ovf);
    if (ctx->ovf_st) (void)hipFree(ctx->ovf_st);
    if (ctx->states) (void)hipFree(ctx->states);
    if (ctx->ln_table) (void)hipFree(ctx->ln_table);
    if (ctx->err) (void)hipFree(ctx->err);
    for (dk_ctx::Slot& sl : ctx->slots) {
        if (sl.stream) (void)hipStreamSynchronize(sl.stream);
        for (void* p : {(void*)sl.queue, (void*)sl.order, (void*)sl.perm, (void*)sl.retry})
            if (p) (void)hipFree(p);
        for (hipEvent_t ev : {sl.ev0, sl.ev1, sl.done})
            if (ev) (void)hipEventDestroy(ev);
    }
    if (ctx->slot_err) (void)hipFree(ctx->slot_err);
    if (ctx->fb_done) (void)hipEventDestroy(ctx->fb_done);
    for (void* p : {(void*)ctx->high_water, (void*)ctx->wave_clock, ctx->fb_hot, (void*)ctx->fb_cold,
                    (void*)ctx->fb_ovf, (void*)ctx->fb_ovf_st, ctx->fb_states})
        if (p) (void)hipFree(p);
    if (ctx->prof) (void)hipFree(ctx->prof);
    if (ctx->az_nodes) (void)hipFree(ctx->az_nodes);
    if (ctx->ar_lanes) (void)hipFree(ctx->ar_lanes);
    if (ctx->az_states) (void)hipFree(ctx->az_states);
    if (ctx->az_games) (void)hipFree(ctx->az_games);
    if (ctx->rd_ln) (void)hipFree(ctx->rd_ln);
    for (float* p : ctx->rd_pw)
        if (p) (void)hipFree(p);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int dk_last_error(const dk_ctx* ctx) { return ctx ? ctx->last_error : DK_E_INVALID; }

#ifdef DK_PHASE_PROF
// profiling builds only (not part of the ABI): per-root phase cycle totals
int dk_phase_profile(dk_ctx* ctx, uint64_t* out, uint32_t n) {
    if (!ctx || !ctx->prof || n > ctx->max_roots) return DK_E_INVALID;
    DK_HIP(hipDeviceSynchronize());
    DK_HIP(hipMemcpy(out, ctx->prof, (size_t)n * dk::PROF_SLOTS * sizeof(uint64_t), hipMemcpyDeviceToHost));
    DK_HIP(hipMemset(ctx->prof, 0, (size_t)ctx->max_roots * dk::PROF_SLOTS * sizeof(uint64_t)));
    return DK_OK;
}
#endif
uint64_t dk_pool_bytes(const dk_ctx* ctx) { return ctx ? ctx->pool_bytes : 0; }

int dk_pool_high_water(dk_ctx* ctx, void* stream, uint32_t* slots, uint32_t* capacity, uint32_t* overflowed) {
    if (!ctx || !slots || !capacity || !overflowed) return DK_E_INVALID;
    uint32_t h[4];
    DK_HIP(hipStreamSynchronize(pick(ctx, stream)));
    DK_HIP(hipMemcpy(h, ctx->high_water, sizeof(h), hipMemcpyDeviceToHost));
    *slots = h[0] > h[2] ? h[0] : h[2];
    *capacity = ctx->cap_slots;
    *overflowed = h[1];
    return DK_OK;
}

// the per-wave stamps of the last search launch: [wave][rt0, rt1, clk0, clk1]
static int last_wave_stamps(dk_ctx* ctx, std::vector<uint64_t>& t, uint32_t* nw_out) {
    uint32_t first, nw, stride;
    hipEvent_t e1;
    {
        std::lock_guard<std::mutex> g(ctx->slot_mu);
        if (ctx->last_slot < 0) return DK_E_INVALID;
        const dk_ctx::Slot& sl = ctx->slots[ctx->last_slot];
        first = sl.clock_first; nw = sl.clock_n; stride = sl.clock_stride; e1 = sl.ev1;
    }
    if (nw == 0) return DK_E_INVALID;
    DK_HIP(hipEventSynchronize(e1));
    std::vector<uint64_t> raw((size_t)nw * stride * 4);
    DK_HIP(hipMemcpy(raw.data(), ctx->wave_clock + 4 * (size_t)first, raw.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    t.resize((size_t)nw * 4);
    for (uint32_t w = 0; w < nw; ++w)
        for (int k = 0; k < 4; ++k) t[4 * (size_t)w + k] = raw[4 * (size_t)w * stride + k];
    *nw_out = nw;
    return DK_OK;
}

int dk_last_search_waves(dk_ctx* ctx, double* out) {
    if (!ctx || !out) return DK_E_INVALID;
    std::vector<uint64_t> t;
    uint32_t nw = 0;
    const int rc = last_wave_stamps(ctx, t, &nw);
    if (rc != DK_OK) return rc;
    uint64_t t0 = ~0ull, t1 = 0, e_min = ~0ull;
    std::vector<uint64_t> ends(nw);
    double busy = 0.0;
    for (uint32_t w = 0; w < nw; ++w) {
        const uint64_t a = t[4 * (size_t)w], b = t[4 * (size_t)w + 1];
        t0 = a < t0 ? a : t0; t1 = b > t1 ? b : t1; e_min = b < e_min ? b : e_min;
        busy += (double)(b - a);
        ends[w] = b;
    }
    std::sort(ends.begin(), ends.end());
    const double span = (double)(t1 - t0);
    out[0] = span / 1e5;                                   // first start -> last end (ms, 100 MHz counter)
    out[1] = span > 0 ? busy / ((double)nw * span) : 1.0;  // mean fraction of the span a wave had work
    out[2] = (double)(e_min - t0) / 1e5;                   // first wave out of work (ms)
    out[3] = (double)(ends[nw / 2] - t0) / 1e5;            // median wave end (ms)
    out[4] = (double)nw;
    return DK_OK;
}

int dk_last_search_clocks(dk_ctx* ctx, double* out) {
    if (!ctx || !out) return DK_E_INVALID;
    std::vector<uint64_t> t;
    uint32_t nw = 0;
    const int rc = last_wave_stamps(ctx, t, &nw);
    if (rc != DK_OK) return rc;
    double rt = 0.0, clk = 0.0, lo = 1e30, hi = 0.0;
    for (uint32_t w = 0; w < nw; ++w) {
        const double r = (double)(t[4 * (size_t)w + 1] - t[4 * (size_t)w]);
        const double c = (double)(t[4 * (size_t)w + 3] - t[4 * (size_t)w + 2]);
        rt += r; clk += c;
        if (r > 0) { const double f = c / r * 100.0; lo = f < lo ? f : lo; hi = f > hi ? f : hi; }
    }
    out[0] = rt > 0 ? clk / rt * 100.0 : 0.0;   // shader clock (MHz): cycles per 100 MHz tick x 100
    out[1] = lo < 1e30 ? lo : 0.0;             // slowest / fastest wave's clock (MHz)
    out[2] = hi;
    out[3] = clk / (double)nw;                 // mean shader cycles a wave was busy
    return DK_OK;
}

int dk_sync(dk_ctx* ctx, void* stream) {
    if (!ctx) return DK_E_INVALID;
    return finish(ctx, pick(ctx, stream), false);
}

int dk_last_search_ms(dk_ctx* ctx, float* ms) {
    if (!ctx || !ms) return DK_E_INVALID;
    hipEvent_t e0, e1;
    {
        std::lock_guard<std::mutex> g(ctx->slot_mu);
        if (ctx->last_slot < 0) return DK_E_INVALID;
        e0 = ctx->slots[ctx->last_slot].ev0;
        e1 = ctx->slots[ctx->last_slot].ev1;
    }
    DK_HIP(hipEventSynchronize(e1));
    DK_HIP(hipEventElapsedTime(ms, e0, e1));
    return DK_OK;
}

// ---------------------------------------------------------------- new games
int dk_new_game_batch_async(dk_ctx* ctx, int game, const uint64_t* d_seeds, uint32_t n, dk_state* d_out, void* stream) {
    if (!ctx || (game != DK_GAME_FULL_DOKO && game != DK_GAME_DOKO)) return DK_E_INVALID;
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(new_game_kernel, dim3(grid_for(n, 64)), dim3(64), 0, pick(ctx, stream), game, d_seeds, n, d_out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_new_game_batch(dk_ctx* ctx, int game, const uint64_t* seeds, uint32_t n, dk_state* out) {
    if (!ctx || !seeds || !out) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n == 0) return DK_OK;
    uint64_t* d_seeds = (uint64_t*)scratch(ctx, 0, n * sizeof(uint64_t));
    dk_state* d_out = (dk_state*)scratch(ctx, 1, n * sizeof(dk_state));
    if (!d_seeds || !d_out) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_seeds, seeds, n * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
    int rc = dk_new_game_batch_async(ctx, game, d_seeds, n, d_out, ctx->stream);
    if (rc) return rc;
    DK_HIP(copy_out(ctx, out, d_out, n * sizeof(dk_state)));
    return finish(ctx, ctx->stream);
}

// ---------------------------------------------------------------- env
int dk_env_allowed_batch(dk_ctx* ctx, const dk_state* states, uint32_t n, int first_expansion, uint64_t* masks) {
    if (!ctx || !states || !masks) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n == 0) return DK_OK;
    dk_state* d_s = (dk_state*)scratch(ctx, 0, n * sizeof(dk_state));
    uint64_t* d_m = (uint64_t*)scratch(ctx, 1, n * sizeof(uint64_t));
    if (!d_s || !d_m) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_s, states, n * sizeof(dk_state), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(env_allowed_kernel, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, d_s, n, first_expansion, d_m, ctx->err);
    DK_HIP(hipGetLastError());
    DK_HIP(copy_out(ctx, masks, d_m, n * sizeof(uint64_t)));
    return finish(ctx, ctx->stream);
}

int dk_env_step_batch(dk_ctx* ctx, dk_state* states, const uint64_t* action_bits, uint32_t n) {
    if (!ctx || !states || !action_bits) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n == 0) return DK_OK;
    dk_state* d_s = (dk_state*)scratch(ctx, 0, n * sizeof(dk_state));
    uint64_t* d_a = (uint64_t*)scratch(ctx, 1, n * sizeof(uint64_t));
    if (!d_s || !d_a) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_s, states, n * sizeof(dk_state), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_a, action_bits, n * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(env_step_kernel, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, d_s, d_a, n, ctx->err);
    DK_HIP(hipGetLastError());
    DK_HIP(copy_out(ctx, states, d_s, n * sizeof(dk_state)));
    return finish(ctx, ctx->stream);
}

int dk_env_rewards_batch(dk_ctx* ctx, const dk_state* states, uint32_t n, int32_t* has_rewards, double* rewards) {
    if (!ctx || !states || !has_rewards || !rewards) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n == 0) return DK_OK;
    dk_state* d_s = (dk_state*)scratch(ctx, 0, n * sizeof(dk_state));
    int32_t* d_h = (int32_t*)scratch(ctx, 1, n * sizeof(int32_t));
    double* d_r = (double*)scratch(ctx, 2, 4 * n * sizeof(double));
    if (!d_s || !d_h || !d_r) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_s, states, n * sizeof(dk_state), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(env_rewards_kernel, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, d_s, n, d_h, d_r);
    DK_HIP(hipGetLastError());
    DK_HIP(copy_out(ctx, has_rewards, d_h, n * sizeof(int32_t)));
    DK_HIP(copy_out(ctx, rewards, d_r, 4 * n * sizeof(double)));
    return finish(ctx, ctx->stream);
}

int dk_env_rollout_batch_async(dk_ctx* ctx, const dk_state* d_states, uint64_t* d_rng, uint32_t n, double* d_rewards, void* stream) {
    if (!ctx) return DK_E_INVALID;
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(env_rollout_kernel, dim3(grid_for(n, WAVE)), dim3(WAVE), 0, pick(ctx, stream), d_states, d_rng, n, d_rewards);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_env_rollout_batch(dk_ctx* ctx, const dk_state* states, uint64_t* rng_states, uint32_t n, double* rewards) {
    if (!ctx || !states || !rng_states || !rewards) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n == 0) return DK_OK;
    dk_state* d_s = (dk_state*)scratch(ctx, 0, n * sizeof(dk_state));
    uint64_t* d_g = (uint64_t*)scratch(ctx, 1, 4 * n * sizeof(uint64_t));
    double* d_r = (double*)scratch(ctx, 2, 4 * n * sizeof(double));
    if (!d_s || !d_g || !d_r) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_s, states, n * sizeof(dk_state), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_g, rng_states, 4 * n * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
    int rc = dk_env_rollout_batch_async(ctx, d_s, d_g, n, d_r, ctx->stream);
    if (rc) return rc;
    DK_HIP(copy_out(ctx, rewards, d_r, 4 * n * sizeof(double)));
    DK_HIP(copy_out(ctx, rng_states, d_g, 4 * n * sizeof(uint64_t)));
    return finish(ctx, ctx->stream);
}

int dk_env_random_plies_batch(dk_ctx* ctx, dk_state* states, uint64_t* rng_states, const uint32_t* plies, uint32_t n) {
    if (!ctx || !states || !rng_states || !plies) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n == 0) return DK_OK;
    dk_state* d_s = (dk_state*)scratch(ctx, 0, n * sizeof(dk_state));
    uint64_t* d_g = (uint64_t*)scratch(ctx, 1, 4 * n * sizeof(uint64_t));
    uint32_t* d_p = (uint32_t*)scratch(ctx, 2, n * sizeof(uint32_t));
    if (!d_s || !d_g || !d_p) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_s, states, n * sizeof(dk_state), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_g, rng_states, 4 * n * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_p, plies, n * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(random_plies_kernel, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, d_s, d_g, d_p, n);
    DK_HIP(hipGetLastError());
    DK_HIP(copy_out(ctx, states, d_s, n * sizeof(dk_state)));
    DK_HIP(copy_out(ctx, rng_states, d_g, 4 * n * sizeof(uint64_t)));
    return finish(ctx, ctx->stream);
}

// ---------------------------------------------------------------- search
namespace {
// One search launch on `stream` (seeded from d_seeds, or continuing the states d_rng in place).
int search_async(dk_ctx* ctx, int game, const dk_state* d_roots, const uint64_t* d_seeds, uint64_t* d_rng, uint32_t n,
                 uint32_t iterations, double c, uint32_t* d_visits, double* d_values, uint8_t* d_best, void* stream) {
    if (!ctx) return DK_E_INVALID;
    if (n > ctx->max_roots || iterations > ctx->max_iters) return ctx->last_error = DK_E_CAPACITY;
    if (n == 0 || iterations == 0) return DK_E_INVALID;
    if (game != DK_GAME_FULL_DOKO && game != DK_GAME_DOKO && game != DK_GAME_TTT) return DK_E_INVALID;
    hipStream_t st = pick(ctx, stream);
    std::lock_guard<std::mutex> g(ctx->slot_mu);
    // the next slot, round-robin; its previous launch must be done before its lists are reused
    const int k = (int)(ctx->next_slot++ % dk_ctx::MAX_INFLIGHT);
    dk_ctx::Slot& sl = ctx->slots[k];
    int* err = ctx->slot_err + k;
    if (sl.used && sl.pending) {
        // More than MAX_INFLIGHT launches since the previous user's stream was synchronised:
        // wait for that launch and keep its error flag for dk_sync of its stream before the
        // flag is cleared for this launch.
        int f = 0;
        DK_HIP(hipEventSynchronize(sl.done));
        DK_HIP(hipMemcpy(&f, err, sizeof(int), hipMemcpyDeviceToHost));
        if (f) ctx->stream_err.emplace_back(sl.stream, f);
        sl.pending = false;
    }
    if (sl.used && sl.stream != st) DK_HIP(hipStreamWaitEvent(st, sl.done, 0));
    DK_HIP(hipMemsetAsync(err, 0, sizeof(int), st));
    DK_HIP(hipEventRecord(sl.ev0, st));
    hipError_t e;
    switch (game) {
        case DK_GAME_FULL_DOKO: e = launch_search<dk::FdoE>(ctx, d_roots, d_seeds, n, iterations, c, d_visits, d_values, d_best, st, sl, err, d_rng); break;
        case DK_GAME_DOKO: e = launch_search<dk::DoE>(ctx, d_roots, d_seeds, n, iterations, c, d_visits, d_values, d_best, st, sl, err, d_rng); break;
        default: e = launch_search<dk::TttE>(ctx, d_roots, d_seeds, n, iterations, c, d_visits, d_values, d_best, st, sl, err, d_rng); break;
    }
    if (e != hipSuccess) { fprintf(stderr, "doko_amd: search launch: %s\n", hipGetErrorString(e)); return DK_E_LAUNCH; }
    DK_HIP(hipEventRecord(sl.ev1, st));
    DK_HIP(hipEventRecord(sl.done, st));
    sl.used = true;
    sl.pending = true;
    sl.stream = st;
    ctx->last_slot = k;
    return DK_OK;
}

// Host-pointer search: seeds (d_seeds) or caller states (rng_states, copied in and back out).
int search_host(dk_ctx* ctx, int game, const dk_state* roots, const uint64_t* seeds, uint64_t* rng_states, uint32_t n,
                uint32_t iterations, double c, uint32_t* visits, double* values, uint8_t* best) {
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n > ctx->max_roots || iterations > ctx->max_iters) return ctx->last_error = DK_E_CAPACITY;
    const size_t words = rng_states ? 4 : 1;
    dk_state* d_r = (dk_state*)scratch(ctx, 0, n * sizeof(dk_state));
    uint64_t* d_s = (uint64_t*)scratch(ctx, 1, words * n * sizeof(uint64_t));
    uint32_t* d_v = (uint32_t*)scratch(ctx, 2, (size_t)n * 39 * sizeof(uint32_t));
    double* d_val = (double*)scratch(ctx, 3, (size_t)n * 39 * sizeof(double));
    uint8_t* d_b = (uint8_t*)scratch(ctx, 4, n);
    if (!d_r || !d_s || !d_v || !d_val || !d_b) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_r, roots, n * sizeof(dk_state), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_s, rng_states ? (const uint64_t*)rng_states : seeds, words * n * sizeof(uint64_t),
                          hipMemcpyHostToDevice, ctx->stream));
    int rc = search_async(ctx, game, d_r, rng_states ? nullptr : d_s, rng_states ? d_s : nullptr, n, iterations, c, d_v,
                          d_val, d_b, ctx->stream);
    if (rc) return rc;
    DK_HIP(copy_out(ctx, visits, d_v, (size_t)n * 39 * sizeof(uint32_t)));
    DK_HIP(copy_out(ctx, values, d_val, (size_t)n * 39 * sizeof(double)));
    DK_HIP(copy_out(ctx, best, d_b, n));
    if (rng_states)
        DK_HIP(copy_out(ctx, rng_states, d_s, 4 * (size_t)n * sizeof(uint64_t)));
    return finish(ctx, ctx->stream);
}
}  // namespace

int dk_search_batch_async(dk_ctx* ctx, int game, const dk_state* d_roots, const uint64_t* d_seeds, uint32_t n,
                          uint32_t iterations, double c, uint32_t* d_visits, double* d_values, uint8_t* d_best,
                          void* stream) {
    if (!d_seeds) return DK_E_INVALID;
    return search_async(ctx, game, d_roots, d_seeds, nullptr, n, iterations, c, d_visits, d_values, d_best, stream);
}

int dk_search_batch_rng_async(dk_ctx* ctx, int game, const dk_state* d_roots, uint64_t* d_rng_states, uint32_t n,
                              uint32_t iterations, double c, uint32_t* d_visits, double* d_values, uint8_t* d_best,
                              void* stream) {
    if (!d_rng_states) return DK_E_INVALID;
    return search_async(ctx, game, d_roots, nullptr, d_rng_states, n, iterations, c, d_visits, d_values, d_best, stream);
}

int dk_search_batch(dk_ctx* ctx, int game, const dk_state* roots, const uint64_t* seeds, uint32_t n, uint32_t iterations,
                    double c, uint32_t* visits, double* values, uint8_t* best) {
    if (!ctx || !roots || !seeds || !visits || !values || !best) return DK_E_INVALID;
    return search_host(ctx, game, roots, seeds, nullptr, n, iterations, c, visits, values, best);
}

int dk_search_batch_rng(dk_ctx* ctx, int game, const dk_state* roots, uint64_t* rng_states, uint32_t n, uint32_t iterations,
                        double c, uint32_t* visits, double* values, uint8_t* best) {
    if (!ctx || !roots || !rng_states || !visits || !values || !best) return DK_E_INVALID;
    return search_host(ctx, game, roots, nullptr, rng_states, n, iterations, c, visits, values, best);
}

// ---------------------------------------------------------------- determinization
int dk_determinize_batch_async(dk_ctx* ctx, const dk_state* d_info, uint32_t n_info, uint32_t samples,
                               const uint64_t* d_seeds, dk_state* d_out, void* stream) {
    if (!ctx) return DK_E_INVALID;
    const size_t n = (size_t)n_info * samples;
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(determinize_kernel, dim3(grid_for(n, WAVE)), dim3(WAVE), 0, pick(ctx, stream), d_info, n_info,
                       samples, d_seeds, d_out, ctx->err);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_determinize_batch(dk_ctx* ctx, const dk_state* infostates, uint32_t n_info, uint32_t samples,
                         const uint64_t* seeds, dk_state* out) {
    if (!ctx || !infostates || !seeds || !out) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    const size_t n = (size_t)n_info * samples;
    if (n == 0) return DK_OK;
    dk_state* d_i = (dk_state*)scratch(ctx, 0, n_info * sizeof(dk_state));
    uint64_t* d_s = (uint64_t*)scratch(ctx, 1, n * sizeof(uint64_t));
    dk_state* d_o = (dk_state*)scratch(ctx, 2, n * sizeof(dk_state));
    if (!d_i || !d_s || !d_o) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_i, infostates, n_info * sizeof(dk_state), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_s, seeds, n * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
    int rc = dk_determinize_batch_async(ctx, d_i, n_info, samples, d_s, d_o, ctx->stream);
    if (rc) return rc;
    DK_HIP(copy_out(ctx, out, d_o, n * sizeof(dk_state)));
    return finish(ctx, ctx->stream);
}

// ---------------------------------------------------------------- fusion
int dk_fuse_accumulate_async(dk_ctx* ctx, const uint32_t* d_visits, uint32_t n_info, uint32_t samples,
                             const uint64_t* d_allowed, int mode, uint32_t* d_acc_u32, float* d_acc_f32, void* stream) {
    if (!ctx || (mode != DK_FUSE_MAXN && mode != DK_FUSE_AVG)) return DK_E_INVALID;
    if (n_info == 0) return DK_OK;
    hipLaunchKernelGGL(fuse_accumulate_kernel, dim3(grid_for((size_t)n_info * 39, 64)), dim3(64), 0, pick(ctx, stream),
                       d_visits, n_info, samples, (const uint8_t*)nullptr, d_allowed, mode, d_acc_u32, d_acc_f32);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_fuse_accumulate_masked_async(dk_ctx* ctx, const uint32_t* d_visits, uint32_t n_info, uint32_t samples,
                                    const uint8_t* d_valid, const uint64_t* d_allowed, int mode, uint32_t* d_acc_u32,
                                    float* d_acc_f32, void* stream) {
    if (!ctx || !d_valid || (mode != DK_FUSE_MAXN && mode != DK_FUSE_AVG)) return DK_E_INVALID;
    if (n_info == 0) return DK_OK;
    hipLaunchKernelGGL(fuse_accumulate_kernel, dim3(grid_for((size_t)n_info * 39, 64)), dim3(64), 0, pick(ctx, stream),
                       d_visits, n_info, samples, d_valid, d_allowed, mode, d_acc_u32, d_acc_f32);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_fuse_select_async(dk_ctx* ctx, uint32_t n_info, int mode, const uint64_t* d_allowed, const uint32_t* d_acc_u32,
                         const float* d_acc_f32, uint8_t* d_action, void* stream) {
    if (!ctx || (mode != DK_FUSE_MAXN && mode != DK_FUSE_AVG)) return DK_E_INVALID;
    if (n_info == 0) return DK_OK;
    hipLaunchKernelGGL(fuse_select_kernel, dim3(grid_for(n_info, 64)), dim3(64), 0, pick(ctx, stream), n_info, mode,
                       d_allowed, d_acc_u32, d_acc_f32, d_action);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_fuse(dk_ctx* ctx, const uint32_t* visits, uint32_t n_info, uint32_t samples, const uint64_t* allowed, int mode,
            uint8_t* action) {
    if (!ctx || !visits || !allowed || !action) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n_info == 0) return DK_OK;
    const size_t nv = (size_t)n_info * samples * 39;
    uint32_t* d_v = (uint32_t*)scratch(ctx, 0, nv * sizeof(uint32_t));
    uint64_t* d_a = (uint64_t*)scratch(ctx, 1, n_info * sizeof(uint64_t));
    uint32_t* d_u = (uint32_t*)scratch(ctx, 2, (size_t)n_info * 39 * sizeof(uint32_t));
    float* d_f = (float*)scratch(ctx, 3, (size_t)n_info * 39 * sizeof(float));
    uint8_t* d_out = (uint8_t*)scratch(ctx, 4, n_info);
    if (!d_v || !d_a || !d_u || !d_f || !d_out) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_v, visits, nv * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_a, allowed, n_info * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
    int rc = dk_fuse_accumulate_async(ctx, d_v, n_info, samples, d_a, mode, d_u, d_f, ctx->stream);
    if (rc) return rc;
    rc = dk_fuse_select_async(ctx, n_info, mode, d_a, d_u, d_f, d_out, ctx->stream);
    if (rc) return rc;
    DK_HIP(copy_out(ctx, action, d_out, n_info));
    return finish(ctx, ctx->stream);
}

int dk_is_consistent_batch(dk_ctx* ctx, const dk_az_state* infostates, const uint64_t* hands, const uint8_t* reservations,
                           uint32_t n, uint8_t* reasons) {
    if (!ctx || !infostates || !hands || !reservations || !reasons) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    if (n == 0) return DK_OK;
    dk_az_state* d_i = (dk_az_state*)scratch(ctx, 0, n * sizeof(dk_az_state));
    uint64_t* d_h = (uint64_t*)scratch(ctx, 1, 4 * (size_t)n * sizeof(uint64_t));
    uint8_t* d_r = (uint8_t*)scratch(ctx, 2, 4 * (size_t)n);
    uint8_t* d_o = (uint8_t*)scratch(ctx, 3, n);
    if (!d_i || !d_h || !d_r || !d_o) return DK_E_CAPACITY;
    DK_HIP(hipMemcpyAsync(d_i, infostates, n * sizeof(dk_az_state), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_h, hands, 4 * (size_t)n * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_r, reservations, 4 * (size_t)n, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(is_consistent_kernel, dim3(grid_for(n, 64)), dim3(64), 0, ctx->stream, d_i, d_h, d_r, n, d_o);
    DK_HIP(hipGetLastError());
    DK_HIP(copy_out(ctx, reasons, d_o, n));
    return finish(ctx, ctx->stream);
}

int dk_legal_actions_async(dk_ctx* ctx, const dk_state* d_states, uint32_t n, uint64_t* d_masks, void* stream) {
    if (!ctx) return DK_E_INVALID;
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(legal_kernel, dim3(grid_for(n, 64)), dim3(64), 0, pick(ctx, stream), d_states, n, d_masks);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_env_step_batch_async(dk_ctx* ctx, dk_state* d_states, const uint64_t* d_actions, uint32_t n, void* stream) {
    if (!ctx) return DK_E_INVALID;
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(env_step_kernel, dim3(grid_for(n, 64)), dim3(64), 0, pick(ctx, stream), d_states, d_actions, n, ctx->err);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_env_random_plies_batch_async(dk_ctx* ctx, dk_state* d_states, uint64_t* d_rng, const uint32_t* d_plies, uint32_t n,
                                    void* stream) {
    if (!ctx) return DK_E_INVALID;
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(random_plies_kernel, dim3(grid_for(n, 64)), dim3(64), 0, pick(ctx, stream), d_states, d_rng, d_plies, n);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

// ---------------------------------------------------------------- end-to-end decision
int dk_decide_batch(dk_ctx* ctx, const dk_state* infostates, uint32_t n_info, uint32_t samples, const uint64_t* seeds,
                    uint32_t iterations, double c, int fuse_mode, uint8_t* actions, uint32_t* visits) {
    if (!ctx || !infostates || !seeds || !actions) return DK_E_INVALID;
    std::lock_guard<std::mutex> g(ctx->mu);
    const size_t n = (size_t)n_info * samples;
    if (n == 0) return DK_OK;
    if (n > ctx->max_roots || iterations > ctx->max_iters) return ctx->last_error = DK_E_CAPACITY;
    const int game = infostates[0].raw[127];
    if (game != DK_GAME_FULL_DOKO && game != DK_GAME_DOKO) return ctx->last_error = DK_E_INVALID;
    for (uint32_t j = 1; j < n_info; ++j)
        if (infostates[j].raw[127] != game) return ctx->last_error = DK_E_INVALID;
    dk_state* d_i = (dk_state*)scratch(ctx, 0, n_info * sizeof(dk_state));
    uint64_t* d_seeds = (uint64_t*)scratch(ctx, 1, 2 * n * sizeof(uint64_t));
    dk_state* d_roots = (dk_state*)scratch(ctx, 2, n * sizeof(dk_state));
    uint32_t* d_v = (uint32_t*)scratch(ctx, 3, n * 39 * sizeof(uint32_t));
    double* d_val = (double*)scratch(ctx, 4, n * 39 * sizeof(double));
    uint8_t* d_b = (uint8_t*)scratch(ctx, 5, n + n_info);
    uint64_t* d_allowed = (uint64_t*)scratch(ctx, 6, n_info * sizeof(uint64_t));
    uint32_t* d_u = (uint32_t*)scratch(ctx, 7, (size_t)n_info * 39 * sizeof(uint32_t));
    float* d_f = (float*)scratch(ctx, 8, (size_t)n_info * 39 * sizeof(float));
    if (!d_i || !d_seeds || !d_roots || !d_v || !d_val || !d_b || !d_allowed || !d_u || !d_f) return DK_E_CAPACITY;
    // seeds: [n] sampling seeds followed by [n] search seeds
    DK_HIP(hipMemcpyAsync(d_i, infostates, n_info * sizeof(dk_state), hipMemcpyHostToDevice, ctx->stream));
    DK_HIP(hipMemcpyAsync(d_seeds, seeds, 2 * n * sizeof(uint64_t), hipMemcpyHostToDevice, ctx->stream));
    int rc = dk_determinize_batch_async(ctx, d_i, n_info, samples, d_seeds, d_roots, ctx->stream);
    if (rc) return rc;
    rc = dk_search_batch_async(ctx, game, d_roots, d_seeds + n, (uint32_t)n, iterations, c, d_v, d_val, d_b, ctx->stream);
    if (rc) return rc;
    hipLaunchKernelGGL(legal_kernel, dim3(grid_for(n_info, 64)), dim3(64), 0, ctx->stream, d_i, n_info, d_allowed);
    DK_HIP(hipGetLastError());
    rc = dk_fuse_accumulate_async(ctx, d_v, n_info, samples, d_allowed, fuse_mode, d_u, d_f, ctx->stream);
    if (rc) return rc;
    rc = dk_fuse_select_async(ctx, n_info, fuse_mode, d_allowed, d_u, d_f, d_b + n, ctx->stream);
    if (rc) return rc;
    DK_HIP(copy_out(ctx, actions, d_b + n, n_info));
    if (visits) DK_HIP(copy_out(ctx, visits, d_v, n * 39 * sizeof(uint32_t)));
    return finish(ctx, ctx->stream);
}

// ---------------------------------------------------------------- AlphaZero PUCT search
int dk_az_begin_async(dk_ctx* ctx, const dk_az_state* d_roots, const uint64_t* d_seeds, uint32_t n_games,
                      uint32_t iterations, int epoch, dk_az_state* d_eval, void* stream) {
    if (!ctx || !d_roots || !d_seeds || !d_eval || n_games == 0) return DK_E_INVALID;
    if (iterations >= dk::NI_MAX_STATES) return ctx->last_error = DK_E_CAPACITY;
    const uint32_t cap_nodes = 1u + 12u * (iterations + 1u) + 39u, cap_states = iterations + 2u;
    const size_t need = (size_t)n_games * ((size_t)cap_nodes * sizeof(dk::az::Node) + (size_t)cap_states * sizeof(dk_az_state) +
                                           sizeof(dk::az::Game));
    if (need > ctx->az_bytes) {
        hipStream_t st = pick(ctx, stream);
        (void)hipStreamSynchronize(st);
        if (ctx->az_nodes) (void)hipFree(ctx->az_nodes);
        if (ctx->az_states) (void)hipFree(ctx->az_states);
        if (ctx->az_games) (void)hipFree(ctx->az_games);
        ctx->az_nodes = nullptr; ctx->az_states = nullptr; ctx->az_games = nullptr; ctx->az_bytes = 0;
        bool ok = hipMalloc(&ctx->az_nodes, (size_t)n_games * cap_nodes * sizeof(dk::az::Node)) == hipSuccess;
        ok = ok && hipMalloc(&ctx->az_states, (size_t)n_games * cap_states * sizeof(dk_az_state)) == hipSuccess;
        ok = ok && hipMalloc(&ctx->az_games, (size_t)n_games * sizeof(dk::az::Game)) == hipSuccess;
        if (!ok) return ctx->last_error = DK_E_CAPACITY;
        ctx->az_bytes = need;
    }
    ctx->az_n = n_games; ctx->az_iters = iterations; ctx->az_epoch = epoch; ctx->az_done = 0; ctx->az_root_done = false;
    ctx->az_cap_nodes = cap_nodes; ctx->az_cap_states = cap_states;
    hipLaunchKernelGGL(az_init_kernel, dim3(grid_for(n_games, 64)), dim3(64), 0, pick(ctx, stream), d_roots, d_seeds,
                       n_games, ctx->az_nodes, ctx->az_states, ctx->az_games, cap_nodes, cap_states, d_eval, ctx->err);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

// The Open01<f32> tables of rand_distr.h: u_k = (1 + k 2^-23) - (1 - 2^-24), k < 2^23, and glibc's
// logf(u_k) / powf(u_k, inv_shape) -- what Rust's f32::ln / f32::powf call.  Built on the host like
// the ln(N) table of the UCT search (64 MB at most; rebuilt when the shape changes).
// A table is published in the context only once its copy has succeeded (a failed build leaves
// no half-initialised table behind); *pw receives the table of this alpha (nullptr for alpha >= 1).
static int rd_tables(dk_ctx* ctx, float alpha, hipStream_t st, float** pw) {
    constexpr uint32_t K = 1u << 23;
    constexpr int NC = dk_ctx::RD_PW_CACHE;
    const bool small = alpha < 1.0f;
    const float inv_shape = 1.0f / alpha;
    *pw = nullptr;
    int hit = -1;
    for (int i = 0; i < NC && small; ++i)
        if (ctx->rd_pw[i] && ctx->rd_inv_shape[i] == inv_shape) hit = i;
    if (ctx->rd_ln && (!small || hit >= 0)) {
        if (hit > 0) {   // most recently used first
            float* p = ctx->rd_pw[hit]; const float v = ctx->rd_inv_shape[hit];
            for (int i = hit; i > 0; --i) { ctx->rd_pw[i] = ctx->rd_pw[i - 1]; ctx->rd_inv_shape[i] = ctx->rd_inv_shape[i - 1]; }
            ctx->rd_pw[0] = p; ctx->rd_inv_shape[0] = v;
        }
        if (small) *pw = ctx->rd_pw[0];
        return DK_OK;
    }
    std::vector<float> h(K);
    auto u_of = [](uint32_t k) { return __builtin_bit_cast(float, k | 0x3F800000u) - (1.0f - FLT_EPSILON / 2.0f); };
    if (hipStreamSynchronize(st) != hipSuccess) return DK_E_LAUNCH;   // (a running root kernel may read the tables)
    auto build = [&](float** slot, bool log_table) -> int {
        for (uint32_t k = 0; k < K; ++k) h[k] = log_table ? logf(u_of(k)) : powf(u_of(k), inv_shape);
        float* d = nullptr;
        if (hipMalloc(&d, K * sizeof(float)) != hipSuccess) return DK_E_CAPACITY;
        if (hipMemcpy(d, h.data(), K * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d);
            return DK_E_LAUNCH;
        }
        *slot = d;
        return DK_OK;
    };
    if (!ctx->rd_ln) {
        float* d = nullptr;
        const int rc = build(&d, true);
        if (rc != DK_OK) return rc;
        ctx->rd_ln = d;
    }
    if (small) {
        float* d = nullptr;
        const int rc = build(&d, false);
        if (rc != DK_OK) return rc;
        if (ctx->rd_pw[NC - 1]) (void)hipFree(ctx->rd_pw[NC - 1]);   // evict the least recently used shape
        for (int i = NC - 1; i > 0; --i) { ctx->rd_pw[i] = ctx->rd_pw[i - 1]; ctx->rd_inv_shape[i] = ctx->rd_inv_shape[i - 1]; }
        ctx->rd_pw[0] = d; ctx->rd_inv_shape[0] = inv_shape;
        *pw = d;
    }
    return DK_OK;
}

int dk_az_root_async(dk_ctx* ctx, const float* d_value, const float* d_logits, const float* d_noise, float dirichlet_alpha,
                     float dirichlet_epsilon, void* stream) {
    if (!ctx || !ctx->az_n || !d_value || !d_logits) return DK_E_INVALID;
    dk::rd::Open01Tab tab{nullptr, nullptr};
    if (!d_noise && !dk::rd::dirichlet_alpha_ok(dirichlet_alpha)) return DK_E_INVALID;
    if (!d_noise && dk::rd::dirichlet_needs_tables(dirichlet_alpha)) {   // (FromBeta reads none)
        float* pw = nullptr;
        const int rc = rd_tables(ctx, dirichlet_alpha, pick(ctx, stream), &pw);
        if (rc) return ctx->last_error = rc;
        tab.ln = ctx->rd_ln;
        tab.pw = pw;
    }
    hipLaunchKernelGGL(az_root_kernel, dim3(grid_for(ctx->az_n, 64)), dim3(64), 0, pick(ctx, stream), d_value, d_logits,
                       d_noise, dirichlet_alpha, tab, dirichlet_epsilon, ctx->az_epoch, ctx->az_n, ctx->az_nodes,
                       ctx->az_states, ctx->az_games, ctx->az_cap_nodes, ctx->az_cap_states, ctx->err);
    DK_HIP(hipGetLastError());
    ctx->az_root_done = true;
    return DK_OK;
}

__global__ void f32_libm_kernel(int fn, uint32_t first, uint32_t stride, uint64_t n, float* y) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __builtin_bit_cast(float, (uint32_t)(first + (uint32_t)i * stride));
        y[i] = fn ? dk::lm::expf_glibc(x) : dk::lm::logf_glibc(x);
    }
}

int dk_f32_libm_async(int fn, uint32_t first, uint32_t stride, uint64_t n, float* d_y, void* stream) {
    if ((fn != 0 && fn != 1) || (n && !d_y)) return DK_E_INVALID;
    if (!n) return DK_OK;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(f32_libm_kernel, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, fn, first, stride, n, d_y);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_az_rng_async(dk_ctx* ctx, uint64_t* d_rng, int set, void* stream) {
    if (!ctx || !ctx->az_n || !d_rng || (set != 0 && set != 1)) return DK_E_INVALID;
    if (set && ctx->az_root_done) return DK_E_INVALID;   // the root has drawn from the old streams
    hipLaunchKernelGGL(az_rng_kernel, dim3(grid_for(ctx->az_n, 64)), dim3(64), 0, pick(ctx, stream), ctx->az_games,
                       ctx->az_n, d_rng, set);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_az_select_async(dk_ctx* ctx, float c, dk_az_state* d_eval, uint8_t* d_need_eval, void* stream) {
    if (!ctx || !ctx->az_n || !ctx->az_root_done || !d_eval) return DK_E_INVALID;
    if (ctx->az_done >= ctx->az_iters) return DK_E_INVALID;
    hipLaunchKernelGGL(az_select_kernel, dim3(grid_for(ctx->az_n, 64)), dim3(64), 0, pick(ctx, stream), c,
                       ctx->az_epoch, ctx->az_n, ctx->az_nodes, ctx->az_states, ctx->az_games, ctx->az_cap_nodes,
                       ctx->az_cap_states, d_eval, d_need_eval, ctx->err);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_az_backup_async(dk_ctx* ctx, const float* d_value, const float* d_logits, void* stream) {
    if (!ctx || !ctx->az_n || !d_value || !d_logits) return DK_E_INVALID;
    hipLaunchKernelGGL(az_backup_kernel, dim3(grid_for(ctx->az_n, 64)), dim3(64), 0, pick(ctx, stream), d_value,
                       d_logits, ctx->az_n, ctx->az_nodes, ctx->az_states, ctx->az_games, ctx->az_cap_nodes,
                       ctx->az_cap_states);
    DK_HIP(hipGetLastError());
    ctx->az_done += 1;
    return DK_OK;
}

int dk_az_records_async(dk_ctx* ctx, const dk_state* d_states, uint32_t n, dk_az_state* d_out, void* stream) {
    if (!ctx || !d_states || !d_out) return DK_E_INVALID;
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(az_records_kernel, dim3(grid_for(n, 64)), dim3(64), 0, pick(ctx, stream), d_states, n, d_out, ctx->err);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_az_step_async(dk_ctx* ctx, dk_az_state* d_records, const uint8_t* d_actions, uint32_t n, void* stream) {
    if (!ctx || !d_records || !d_actions) return DK_E_INVALID;
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(az_step_kernel, dim3(grid_for(n, 64)), dim3(64), 0, pick(ctx, stream), d_records, d_actions, n, ctx->err);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_az_encode_async(dk_ctx* ctx, const dk_az_state* d_records, uint32_t n, int32_t* d_tokens, void* stream) {
    if (!ctx || !d_records || !d_tokens) return DK_E_INVALID;
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(az_encode_kernel, dim3(grid_for(n, 64)), dim3(64), 0, pick(ctx, stream), d_records, n, d_tokens);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_az_finish_async(dk_ctx* ctx, int temperature_mode, float temperature, uint32_t* d_visits, uint8_t* d_action,
                       void* stream) {
    if (!ctx || !ctx->az_n || !d_visits || !d_action || temperature_mode < 0 || temperature_mode > 2) return DK_E_INVALID;
    if (ctx->az_done != ctx->az_iters) return DK_E_INVALID;
    hipLaunchKernelGGL(az_finish_kernel, dim3(grid_for(ctx->az_n, 64)), dim3(64), 0, pick(ctx, stream), temperature_mode,
                       temperature, ctx->az_n, ctx->az_nodes, ctx->az_states, ctx->az_games, ctx->az_cap_nodes,
                       ctx->az_cap_states, d_visits, d_action);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

// ---------------------------------------------------------------- IMPI autoregressive determinization
int dk_ar_begin_async(dk_ctx* ctx, const dk_az_state* d_infostates, uint32_t n_info, uint32_t samples,
                      const uint64_t* d_seeds, float log_chance, uint32_t* d_rounds, void* stream) {
    if (!ctx || !d_infostates || !d_seeds || !d_rounds || samples == 0) return DK_E_INVALID;
    const uint64_t n64 = (uint64_t)n_info * samples;
    if (n64 > 0xFFFFFFFFull / dk::ar::TOKENS) return DK_E_INVALID;
    const uint32_t n = (uint32_t)n64;
    hipStream_t st = pick(ctx, stream);
    if (n > ctx->ar_cap) {
        (void)hipStreamSynchronize(st);
        if (ctx->ar_lanes) (void)hipFree(ctx->ar_lanes);
        ctx->ar_lanes = nullptr; ctx->ar_cap = 0;
        if (hipMalloc(&ctx->ar_lanes, (size_t)n * sizeof(dk::ar::Lane)) != hipSuccess) return ctx->last_error = DK_E_CAPACITY;
        ctx->ar_cap = n;
    }
    ctx->ar_info = d_infostates; ctx->ar_n = n; ctx->ar_samples = samples; ctx->ar_log_chance = log_chance;
    DK_HIP(hipMemsetAsync(d_rounds, 0, sizeof(uint32_t), st));
    if (n == 0) return DK_OK;
    hipLaunchKernelGGL(ar_begin_kernel, dim3(grid_for(n, 64)), dim3(64), 0, st, d_infostates, samples, d_seeds, n,
                       ctx->ar_lanes, d_rounds);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_ar_guesses_async(dk_ctx* ctx, const dk_az_state* d_infostates, uint32_t n_info, uint32_t* d_counts, void* stream) {
    if (!ctx || !d_infostates || !d_counts) return DK_E_INVALID;
    if (n_info == 0) return DK_OK;
    hipLaunchKernelGGL(ar_guesses_kernel, dim3(grid_for(n_info, 64)), dim3(64), 0, pick(ctx, stream), d_infostates, n_info,
                       d_counts);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_ar_prepare_async(dk_ctx* ctx, int32_t* d_tokens, void* stream) {
    if (!ctx || !ctx->ar_info || !d_tokens) return DK_E_INVALID;
    if (ctx->ar_n == 0) return DK_OK;
    hipLaunchKernelGGL(ar_prepare_kernel, dim3(grid_for(ctx->ar_n, 64)), dim3(64), 0, pick(ctx, stream), ctx->ar_info,
                       ctx->ar_samples, ctx->ar_n, ctx->ar_lanes, ctx->ar_log_chance, d_tokens);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_ar_choose_async(dk_ctx* ctx, const float* d_logits, float temperature, void* stream) {
    if (!ctx || !ctx->ar_info || !d_logits) return DK_E_INVALID;
    if (ctx->ar_n == 0) return DK_OK;
    hipLaunchKernelGGL(ar_choose_kernel, dim3(grid_for(ctx->ar_n, 64)), dim3(64), 0, pick(ctx, stream), ctx->ar_n,
                       ctx->ar_lanes, d_logits, temperature);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_ar_fallback_async(dk_ctx* ctx, uint32_t n_info, uint32_t samples, const uint8_t* d_status, const uint64_t* d_allowed,
                         const uint64_t* d_seeds, uint8_t* d_action, uint32_t* d_successes, void* stream) {
    if (!ctx || !d_status || !d_allowed || !d_seeds || !d_action || !d_successes) return DK_E_INVALID;
    if (n_info == 0) return DK_OK;
    hipLaunchKernelGGL(ar_fallback_kernel, dim3(grid_for(n_info, 64)), dim3(64), 0, pick(ctx, stream), n_info, samples,
                       d_status, d_allowed, d_seeds, d_action, d_successes);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_ar_output_async(dk_ctx* ctx, dk_state* d_out, uint8_t* d_status, uint8_t* d_reason, void* stream) {
    if (!ctx || !ctx->ar_info || !d_out || !d_status || !d_reason) return DK_E_INVALID;
    if (ctx->ar_n == 0) return DK_OK;
    hipLaunchKernelGGL(ar_output_kernel, dim3(grid_for(ctx->ar_n, 64)), dim3(64), 0, pick(ctx, stream), ctx->ar_info,
                       ctx->ar_samples, ctx->ar_n, ctx->ar_lanes, d_out, d_status, d_reason);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

// ---------------------------------------------------------------- AlphaZero network row kernels
namespace {
// bf16 pairs per lane of a 32-lane row group (d even, d <= 512)
int ln_per(uint32_t d) { return (d % 32u == 0u && d >= 32u && d <= 64u * (uint32_t)dk::net::LN_MAX_PER_LANE) ? (int)((d + 63u) / 64u) : 0; }
}  // namespace

#define DK_LN_CASES(M) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8)

int dk_net_embed_ln_bf16_async(const int32_t* d_tokens, uint32_t batch, const void* const* tables, uint32_t d,
                               const void* gamma, const void* beta, float eps, void* x_out, void* h_out, void* stream) {
    const int per = ln_per(d);
    if (!tables || !d_tokens || !x_out || !h_out || !gamma || !beta || per == 0) return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    const uint32_t rows = batch * 62u;
    const dim3 grid((rows + 7u) / 8u), block(256);
    hipStream_t st = (hipStream_t)stream;
    const uint16_t* const* t = (const uint16_t* const*)tables;
    switch (per) {
#define M(P) case P: hipLaunchKernelGGL(dk::net::embed_ln_kernel<P>, grid, block, 0, st, d_tokens, batch, (int)d, t[0], t[1], t[2], \
                                        t[3], t[4], t[5], (const uint16_t*)gamma, (const uint16_t*)beta, eps,            \
                                        (uint16_t*)x_out, (uint16_t*)h_out); break;
        DK_LN_CASES(M)
#undef M
    }
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_fc_gelu_bf16_async(const void* x, const void* w, const void* bias, uint32_t rows, uint32_t k, uint32_t n,
                              void* y, void* stream) {
    if (!x || !w || !bias || !y || (k != 160u && k != 256u) || n == 0 || n % (k == 160u ? 64u : 32u)) return DK_E_INVALID;
    if (rows == 0) return DK_OK;
    const uint32_t wg_rows = k == 160u ? 256u : 128u;   // 4 waves x (2 or 1) row tiles of 32
    const dim3 grid((rows + wg_rows - 1u) / wg_rows), block(256);
    if (k == 160u)
        hipLaunchKernelGGL(dk::net::fc_gelu_kernel<160>, grid, block, 0, (hipStream_t)stream, (const uint16_t*)x,
                           (const uint16_t*)w, (const uint16_t*)bias, (uint16_t*)y, rows, n);
    else
        hipLaunchKernelGGL(dk::net::fc_gelu_kernel<256>, grid, block, 0, (hipStream_t)stream, (const uint16_t*)x,
                           (const uint16_t*)w, (const uint16_t*)bias, (uint16_t*)y, rows, n);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_mlp_ln_bf16_async(const void* h, void* x_io, const void* w1, const void* b1, const void* w2, const void* b2,
                             uint32_t rows, uint32_t d, uint32_t n_hidden, const void* gamma, const void* beta, float eps,
                             void* h_out, void* stream) {
    if (!h || !x_io || !w1 || !b1 || !w2 || !b2 || !gamma || !beta || !h_out || (d != 160u && d != 256u) ||
        n_hidden == 0 || n_hidden > dk::net::MLP_MAX_HIDDEN || n_hidden % (d == 160u ? DK_MLP_NC160 : 32u))
        return DK_E_INVALID;
    if (rows == 0) return DK_OK;
    const uint32_t W = d == 160u ? DK_MLP_WAVES160 : DK_MLP_WAVES256;   // waves per workgroup, 32 rows each
    const dim3 grid((rows + 32u * W - 1u) / (32u * W)), block(64u * W);
    if (d == 160u)
        hipLaunchKernelGGL((dk::net::mlp_ln_kernel<160, DK_MLP_NC160, DK_MLP_WAVES160>), grid, block, 0, (hipStream_t)stream, (const uint16_t*)h,
                           (uint16_t*)x_io, (const uint16_t*)w1, (const uint16_t*)b1, (const uint16_t*)w2, (const uint16_t*)b2,
                           rows, n_hidden, (const uint16_t*)gamma, (const uint16_t*)beta, eps, (uint16_t*)h_out);
    else
        hipLaunchKernelGGL((dk::net::mlp_ln_kernel<256, 32, DK_MLP_WAVES256>), grid, block, 0, (hipStream_t)stream, (const uint16_t*)h,
                           (uint16_t*)x_io, (const uint16_t*)w1, (const uint16_t*)b1, (const uint16_t*)w2, (const uint16_t*)b2,
                           rows, n_hidden, (const uint16_t*)gamma, (const uint16_t*)beta, eps, (uint16_t*)h_out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

// The MLP half at the reference's precision: f32 activations, bf16x3 products (mlp_ln_f32x3_kernel).
int dk_net_mlp_ln_f32x3_async(const float* h, float* x_io, const void* w1_hi, const void* w1_lo, const float* b1,
                              const void* w2_hi, const void* w2_lo, const float* b2, uint32_t rows, uint32_t d,
                              uint32_t n_hidden, const float* gamma, const float* beta, float eps, float* h_out,
                              void* stream) {
    if (!h || !x_io || !w1_hi || !w1_lo || !b1 || !w2_hi || !w2_lo || !b2 || !gamma || !beta || !h_out ||
        (d != 160u && d != 256u) || n_hidden == 0 || n_hidden > dk::net::MLP_MAX_HIDDEN || n_hidden % 32u ||
        (d == 256u && n_hidden % 64u))   // (d = 256: an even number of 32-unit chunks)
        return DK_E_INVALID;
    if (rows == 0) return DK_OK;
    // 4 waves x 32 rows per workgroup, double-buffered weight chunks: two workgroups per CU at
    // d = 160 (80 KiB of LDS each), one at d = 256
    // (DK_MLPF32_WAVES=8: d = 160 as one 8-wave workgroup of 256 rows per CU, half the weight
    // staging per row; measurement switch)
    static const int waves8 = getenv("DK_MLPF32_WAVES") && atoi(getenv("DK_MLPF32_WAVES")) == 8;
    if (d == 160u && waves8) {
        hipLaunchKernelGGL((dk::net::mlp_ln_f32x3_kernel<160, 32, 8>), dim3((rows + 255u) / 256u), dim3(512u), 0,
                           (hipStream_t)stream, h, x_io, (const uint16_t*)w1_hi, (const uint16_t*)w1_lo, b1,
                           (const uint16_t*)w2_hi, (const uint16_t*)w2_lo, b2, rows, n_hidden, gamma, beta, eps, h_out);
        DK_HIP(hipGetLastError());
        return DK_OK;
    }
    const dim3 grid((rows + 127u) / 128u), block(256u);
    if (d == 160u)
        hipLaunchKernelGGL((dk::net::mlp_ln_f32x3_kernel<160, 32, 4>), grid, block, 0, (hipStream_t)stream, h, x_io,
                           (const uint16_t*)w1_hi, (const uint16_t*)w1_lo, b1, (const uint16_t*)w2_hi, (const uint16_t*)w2_lo,
                           b2, rows, n_hidden, gamma, beta, eps, h_out);
    else
        // d = 256: 16 rows per wave, eight waves, two per SIMD (mlp16_ln_f32x3_kernel; W2 in its split layout)
        hipLaunchKernelGGL((dk::net::mlp16_ln_f32x3_kernel<256, 32>), grid, dim3(512u), 0, (hipStream_t)stream, h, x_io,
                           (const uint16_t*)w1_hi, (const uint16_t*)w1_lo, b1, (const uint16_t*)w2_hi, (const uint16_t*)w2_lo,
                           b2, rows, n_hidden, gamma, beta, eps, h_out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

// The attention half at the reference's precision: f32 activations, bf16x3 products
// (qkv_attn_ln_f32x3_kernel; d = 160, four heads of 40).
int dk_net_qkv_attn_ln_f32x3_async(const float* h, float* x_io, const void* wqkv_hi, const void* wqkv_lo, const float* bqkv,
                                   const void* wp_hi, const void* wp_lo, const float* bp, uint32_t batch, uint32_t heads,
                                   uint32_t head_dim, const float* gamma, const float* beta, float eps, float* h_out,
                                   void* stream) {
    if (!h || !x_io || !wqkv_hi || !wqkv_lo || !bqkv || !wp_hi || !wp_lo || !bp || !gamma || !beta || !h_out ||
        h == h_out || heads != 4u || (head_dim != 40u && head_dim != 64u))
        return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    const float scale = 1.0f / sqrtf((float)head_dim);
    if (head_dim == 40u)
        hipLaunchKernelGGL((dk::net::qkv_attn_ln_f32x3_kernel<40>), dim3(batch), dim3(256), 0, (hipStream_t)stream, h, x_io,
                           (const uint16_t*)wqkv_hi, (const uint16_t*)wqkv_lo, bqkv, (const uint16_t*)wp_hi,
                           (const uint16_t*)wp_lo, bp, scale, gamma, beta, eps, h_out);
    else
        hipLaunchKernelGGL((dk::net::qkv_attn_ln_f32x3_kernel<64>), dim3(batch), dim3(256), 0, (hipStream_t)stream, h, x_io,
                           (const uint16_t*)wqkv_hi, (const uint16_t*)wqkv_lo, bqkv, (const uint16_t*)wp_hi,
                           (const uint16_t*)wp_lo, bp, scale, gamma, beta, eps, h_out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

// The halves with the LayerNorm moved to the consumer (d = 256: round 5; d = 160: round 6): the
// input is either h (h_in given, ln_in_* unused) or the residual stream normalised in the kernel
// with ln_in (h_in NULL); h_out NULL writes x only (gamma / beta / eps then unused).
int dk_net_qkv_attn_ln_f32x3_ex_async(const float* h_in, float* x_io, const float* ln_in_gamma, const float* ln_in_beta,
                                      float ln_in_eps, const void* wqkv_hi, const void* wqkv_lo, const float* bqkv,
                                      const void* wp_hi, const void* wp_lo, const float* bp, uint32_t batch, uint32_t heads,
                                      uint32_t head_dim, const float* gamma, const float* beta, float eps, float* h_out,
                                      const float* stats_in, float* stats_out, float* x_out, void* stream) {
    const bool xin = h_in == nullptr;
    if (x_out == x_io) x_out = nullptr;   // (in place)
    if (!x_io || !wqkv_hi || !wqkv_lo || !bqkv || !wp_hi || !wp_lo || !bp || (xin && (!ln_in_gamma || !ln_in_beta)) ||
        (h_out && (!gamma || !beta || h_out == h_in || h_out == x_io || h_out == x_out)) || (h_in && h_in == x_io) ||
        (x_out && x_out == h_in) || heads != 4u ||
        (head_dim != 64u && head_dim != 40u) || (head_dim == 40u && !xin) ||
        (head_dim == 64u && (stats_in || stats_out)))   // (row statistics: the d = 160 chain only)
        return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    const float scale = 1.0f / sqrtf((float)head_dim);
    if (head_dim == 40u)
        hipLaunchKernelGGL((dk::net::qkv_attn_ln_f32x3_kernel<40, true>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                           (const float*)nullptr, x_io, (const uint16_t*)wqkv_hi, (const uint16_t*)wqkv_lo, bqkv,
                           (const uint16_t*)wp_hi, (const uint16_t*)wp_lo, bp, scale, gamma, beta, eps, h_out, ln_in_gamma,
                           ln_in_beta, ln_in_eps, (const float2*)stats_in, (float2*)stats_out, x_out);
    else if (xin)
        hipLaunchKernelGGL((dk::net::qkv_attn_ln_f32x3_kernel<64, true>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                           (const float*)nullptr, x_io, (const uint16_t*)wqkv_hi, (const uint16_t*)wqkv_lo, bqkv,
                           (const uint16_t*)wp_hi, (const uint16_t*)wp_lo, bp, scale, gamma, beta, eps, h_out, ln_in_gamma,
                           ln_in_beta, ln_in_eps, (const float2*)nullptr, (float2*)nullptr, x_out);
    else
        hipLaunchKernelGGL((dk::net::qkv_attn_ln_f32x3_kernel<64, false>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                           h_in, x_io, (const uint16_t*)wqkv_hi, (const uint16_t*)wqkv_lo, bqkv, (const uint16_t*)wp_hi,
                           (const uint16_t*)wp_lo, bp, scale, gamma, beta, eps, h_out, (const float*)nullptr,
                           (const float*)nullptr, 0.0f, (const float2*)nullptr, (float2*)nullptr, x_out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_mlp_ln_f32x3_ex_async(const float* h_in, float* x_io, const float* ln_in_gamma, const float* ln_in_beta,
                                 float ln_in_eps, const void* w1_hi, const void* w1_lo, const float* b1, const void* w2_hi,
                                 const void* w2_lo, const float* b2, uint32_t rows, uint32_t d, uint32_t n_hidden,
                                 const float* gamma, const float* beta, float eps, float* h_out, const float* stats_in,
                                 float* stats_out, void* stream) {
    const bool xin = h_in == nullptr;
    if (!x_io || !w1_hi || !w1_lo || !b1 || !w2_hi || !w2_lo || !b2 || (xin && (!ln_in_gamma || !ln_in_beta)) ||
        (h_out && (!gamma || !beta || h_out == h_in || h_out == x_io)) || (h_in && h_in == x_io) ||
        (d != 256u && d != 160u) || (d == 160u && (!xin || !stats_in)) || (d == 256u && (stats_in || stats_out)) ||
        n_hidden == 0 || n_hidden > dk::net::MLP_MAX_HIDDEN || n_hidden % 64u)
        return DK_E_INVALID;
    if (rows == 0) return DK_OK;
    const dim3 grid((rows + 127u) / 128u);
    if (d == 160u)   // (4 waves x 32 rows, mlp_ln_f32x3_kernel: x normalised with the producer's row statistics)
        hipLaunchKernelGGL((dk::net::mlp_ln_f32x3_kernel<160, 32, 4, true>), grid, dim3(256u), 0, (hipStream_t)stream,
                           (const float*)nullptr, x_io, (const uint16_t*)w1_hi, (const uint16_t*)w1_lo, b1,
                           (const uint16_t*)w2_hi, (const uint16_t*)w2_lo, b2, rows, n_hidden, gamma, beta, eps, h_out,
                           ln_in_gamma, ln_in_beta, (const float2*)stats_in, (float2*)stats_out);
    else if (xin)
        hipLaunchKernelGGL((dk::net::mlp16_ln_f32x3_kernel<256, 32, true>), grid, dim3(512u), 0, (hipStream_t)stream,
                           (const float*)nullptr, x_io, (const uint16_t*)w1_hi, (const uint16_t*)w1_lo, b1,
                           (const uint16_t*)w2_hi, (const uint16_t*)w2_lo, b2, rows, n_hidden, gamma, beta, eps, h_out,
                           ln_in_gamma, ln_in_beta, ln_in_eps);
    else
        hipLaunchKernelGGL((dk::net::mlp16_ln_f32x3_kernel<256, 32, false>), grid, dim3(512u), 0, (hipStream_t)stream,
                           h_in, x_io, (const uint16_t*)w1_hi, (const uint16_t*)w1_lo, b1, (const uint16_t*)w2_hi,
                           (const uint16_t*)w2_lo, b2, rows, n_hidden, gamma, beta, eps, h_out, (const float*)nullptr,
                           (const float*)nullptr, 0.0f);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_class_pool_ln_f32_async(const float* x, uint32_t batch, uint32_t d, const float* queries, uint32_t classes,
                                   float scale, const float* ln_w, const float* ln_b, float eps, float* out, void* stream) {
    if (!x || !queries || !ln_w || !ln_b || !out || classes == 0 || classes > 64u || (d != 160u && d != 256u))
        return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    static const bool small_off = getenv("DK_POOL_SMALL") && atoi(getenv("DK_POOL_SMALL")) == 0;   // (measurement switch)
    if (classes <= 8u && !small_off) {   // (few classes: f32 FMAs, class_pool_small_ln_f32_kernel)
        if (d == 160u)
            hipLaunchKernelGGL((dk::net::class_pool_small_ln_f32_kernel<160>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                               x, batch, queries, classes, scale, ln_w, ln_b, eps, out);
        else
            hipLaunchKernelGGL((dk::net::class_pool_small_ln_f32_kernel<256>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                               x, batch, queries, classes, scale, ln_w, ln_b, eps, out);
    } else if (d == 160u)
        hipLaunchKernelGGL((dk::net::class_pool_ln_f32x3_kernel<160>), dim3(batch), dim3(256), 0, (hipStream_t)stream, x,
                           batch, queries, classes, scale, ln_w, ln_b, eps, out);
    else
        hipLaunchKernelGGL((dk::net::class_pool_ln_f32x3_kernel<256>), dim3(batch), dim3(256), 0, (hipStream_t)stream, x,
                           batch, queries, classes, scale, ln_w, ln_b, eps, out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_class_mlp_bf16_async(const void* pooled, uint32_t batch, uint32_t d, uint32_t classes, const void* w1,
                                const void* b1, const void* w2, const void* b2, void* out, void* stream) {
    if (!pooled || !w1 || !b1 || !w2 || !b2 || !out || classes == 0 || classes > 65535u || (d != 160u && d != 256u))
        return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    const dim3 grid((batch + 127u) / 128u, classes);
    if (d == 160u)
        hipLaunchKernelGGL((dk::net::class_mlp_bf16_kernel<160>), grid, dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)pooled, batch, classes, (const uint16_t*)w1, (const uint16_t*)b1,
                           (const uint16_t*)w2, (const uint16_t*)b2, (uint16_t*)out);
    else
        hipLaunchKernelGGL((dk::net::class_mlp_bf16_kernel<256>), grid, dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)pooled, batch, classes, (const uint16_t*)w1, (const uint16_t*)b1,
                           (const uint16_t*)w2, (const uint16_t*)b2, (uint16_t*)out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_class_mlp_f32x3_async(const float* pooled, uint32_t batch, uint32_t d, uint32_t classes, const void* w1_hi,
                                 const void* w1_lo, const float* b1, const float* w2, const float* b2, float* out,
                                 void* stream) {
    if (!pooled || !w1_hi || !w1_lo || !b1 || !w2 || !b2 || !out || classes == 0 || classes > 65535u ||
        (d != 160u && d != 256u))
        return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    const dim3 grid((batch + 127u) / 128u, classes);
    if (d == 160u)
        hipLaunchKernelGGL((dk::net::class_mlp_f32x3_kernel<160>), grid, dim3(256), 0, (hipStream_t)stream, pooled, batch,
                           classes, (const uint16_t*)w1_hi, (const uint16_t*)w1_lo, b1, w2, b2, out);
    else
        hipLaunchKernelGGL((dk::net::class_mlp_f32x3_kernel<256>), grid, dim3(256), 0, (hipStream_t)stream, pooled, batch,
                           classes, (const uint16_t*)w1_hi, (const uint16_t*)w1_lo, b1, w2, b2, out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

#ifdef DK_NET_PROF
// profiling builds: the summed phase clocks of qkv_attn_ln_kernel since the last read (then cleared)
extern "C" int dk_net_prof_read(uint64_t* out8) {
    DK_HIP(hipMemcpyFromSymbol(out8, HIP_SYMBOL(dk::net::dk_net_prof_acc), 8 * sizeof(uint64_t)));
    const uint64_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    DK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dk::net::dk_net_prof_acc), z, sizeof(z)));
    return DK_OK;
}
// the same for mlp_ln_kernel: [wave 0 (early group) | wave 4 (late group)][phase], 16 words
extern "C" int dk_net_mlp_prof_read(uint64_t* out16) {
    DK_HIP(hipMemcpyFromSymbol(out16, HIP_SYMBOL(dk::net::dk_mlp_prof_acc), 16 * sizeof(uint64_t)));
    const uint64_t z[16] = {};
    DK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dk::net::dk_mlp_prof_acc), z, sizeof(z)));
    return DK_OK;
}
#endif
int dk_net_class_pool_ln_bf16_async(const void* x, uint32_t batch, uint32_t d, const void* queries, uint32_t classes,
                                    float scale, const void* ln_w, const void* ln_b, float eps, void* out, void* stream) {
    if (!x || !queries || !ln_w || !ln_b || !out || classes == 0 || classes > 64u || (d != 160u && d != 256u))
        return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    if (d == 160u)
        hipLaunchKernelGGL((dk::net::class_pool_ln_kernel<160>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)x, batch, (const uint16_t*)queries, classes, scale, (const uint16_t*)ln_w,
                           (const uint16_t*)ln_b, eps, (uint16_t*)out);
    else
        hipLaunchKernelGGL((dk::net::class_pool_ln_kernel<256>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)x, batch, (const uint16_t*)queries, classes, scale, (const uint16_t*)ln_w,
                           (const uint16_t*)ln_b, eps, (uint16_t*)out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_qkv_attn_ln_bf16_async(const void* h, void* x_io, const void* wqkv, const void* bqkv, const void* wp, const void* bp,
                                  uint32_t batch, uint32_t heads, uint32_t head_dim, const void* gamma, const void* beta,
                                  float eps, void* h_out, void* stream) {
    if (!h || !x_io || !wqkv || !bqkv || !wp || !bp || !gamma || !beta || !h_out || h == h_out || heads != 4u ||
        (head_dim != 40u && head_dim != 64u))
        return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    const float scale = 1.0f / sqrtf((float)head_dim);
    if (head_dim == 40u)
        hipLaunchKernelGGL((dk::net::qkv_attn_ln_kernel<40>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)h, (uint16_t*)x_io, (const uint16_t*)wqkv, (const uint16_t*)bqkv,
                           (const uint16_t*)wp, (const uint16_t*)bp, batch, scale, (const uint16_t*)gamma,
                           (const uint16_t*)beta, eps, (uint16_t*)h_out);
    else
        hipLaunchKernelGGL((dk::net::qkv_attn_ln_kernel<64>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)h, (uint16_t*)x_io, (const uint16_t*)wqkv, (const uint16_t*)bqkv,
                           (const uint16_t*)wp, (const uint16_t*)bp, batch, scale, (const uint16_t*)gamma,
                           (const uint16_t*)beta, eps, (uint16_t*)h_out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_attn_ln_bf16_async(const void* qkv, void* x_io, const void* wp, const void* bp, uint32_t batch, uint32_t heads,
                              uint32_t head_dim, const void* gamma, const void* beta, float eps, void* h_out, void* stream) {
    if (!qkv || !x_io || !wp || !bp || !gamma || !beta || !h_out || heads != 4u || (head_dim != 40u && head_dim != 64u))
        return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    const float scale = 1.0f / sqrtf((float)head_dim);
    if (head_dim == 40u)
        hipLaunchKernelGGL((dk::net::attn_ln_kernel<40, 4>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)qkv, (uint16_t*)x_io, (const uint16_t*)wp, (const uint16_t*)bp, batch, scale,
                           (const uint16_t*)gamma, (const uint16_t*)beta, eps, (uint16_t*)h_out);
    else
        hipLaunchKernelGGL((dk::net::attn_ln_kernel<64, 4>), dim3(batch), dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)qkv, (uint16_t*)x_io, (const uint16_t*)wp, (const uint16_t*)bp, batch, scale,
                           (const uint16_t*)gamma, (const uint16_t*)beta, eps, (uint16_t*)h_out);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_attn62_bf16_async(const void* qkv, void* y, uint32_t batch, uint32_t heads, uint32_t head_dim, void* stream) {
    if (!qkv || !y || heads != 4u || (head_dim != 40u && head_dim != 64u)) return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    if ((uint64_t)batch * heads > 0xFFFFFFFFull) return DK_E_INVALID;
    const uint32_t waves = batch * heads;
    const float scale = 1.0f / sqrtf((float)head_dim);
    if (head_dim == 40u)
        hipLaunchKernelGGL((dk::net::attn62_kernel<40, 4>), dim3((waves + 3u) / 4u), dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)qkv, (uint16_t*)y, batch, scale);
    else
        hipLaunchKernelGGL((dk::net::attn62_kernel<64, 4>), dim3((waves + 3u) / 4u), dim3(256), 0, (hipStream_t)stream,
                           (const uint16_t*)qkv, (uint16_t*)y, batch, scale);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

// ---------------------------------------------------------------- f32 network row kernels (az_net_f32_kernels.h)
namespace {
int p4_of(uint32_t d) { return (d % 4u == 0u && d >= 4u && d <= 128u * (uint32_t)dk::net::LN4_MAX) ? (int)((d / 4u + 31u) / 32u) : 0; }
}  // namespace
#define DK_P4_CASES(M) M(1) M(2) M(3) M(4)

int dk_net_embed_ln_f32_async(const int32_t* d_tokens, uint32_t batch, const void* const* tables, uint32_t d,
                              const void* gamma, const void* beta, float eps, void* x_out, void* h_out, void* stream) {
    const int p4 = p4_of(d);
    // (h_out NULL: x only)
    if (!tables || !d_tokens || !x_out || (h_out && (!gamma || !beta)) || p4 == 0) return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    const uint32_t rows = batch * 62u;
    hipStream_t st = (hipStream_t)stream;
    const float* const* t = (const float* const*)tables;
    if (!h_out) {   // x only: one lane per float4
        const uint64_t n = (uint64_t)rows * (d / 4u);
        hipLaunchKernelGGL(dk::net::embed_f32_kernel, dim3((uint32_t)((n + 255u) / 256u)), dim3(256), 0, st, d_tokens, batch,
                           (int)d, t[0], t[1], t[2], t[3], t[4], t[5], (float*)x_out);
        DK_HIP(hipGetLastError());
        return DK_OK;
    }
    const dim3 grid((rows + 7u) / 8u), block(256);
    switch (p4) {
#define M(P) case P: hipLaunchKernelGGL(dk::net::embed_ln_f32_kernel<P>, grid, block, 0, st, d_tokens, batch, (int)d, t[0], t[1], \
                                        t[2], t[3], t[4], t[5], (const float*)gamma, (const float*)beta, eps, (float*)x_out,      \
                                        (float*)h_out); break;
        DK_P4_CASES(M)
#undef M
    }
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_add_ln_f32_async(void* x_io, const void* delta, uint32_t rows, uint32_t d, const void* gamma, const void* beta,
                            float eps, void* h_out, void* stream) {
    return dk_net_add_bias_ln_f32_async(x_io, delta, nullptr, rows, d, gamma, beta, eps, h_out, stream);
}
int dk_net_add_bias_ln_f32_async(void* x_io, const void* delta, const void* bias, uint32_t rows, uint32_t d,
                                 const void* gamma, const void* beta, float eps, void* h_out, void* stream) {
    const int p4 = p4_of(d);
    if (!x_io || !h_out || !gamma || !beta || p4 == 0) return DK_E_INVALID;
    if (rows == 0) return DK_OK;
    const dim3 grid((rows + 7u) / 8u), block(256);
    hipStream_t st = (hipStream_t)stream;
    switch (p4) {
#define M(P) case P: hipLaunchKernelGGL(dk::net::add_ln_f32_kernel<P>, grid, block, 0, st, (float*)x_io, (const float*)delta, \
                                        rows, (int)d, (const float*)gamma, (const float*)beta, eps, (float*)h_out,          \
                                        (const float*)bias); break;
        DK_P4_CASES(M)
#undef M
    }
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_gelu_f32_async(void* y, uint64_t n, void* stream) { return dk_net_gelu_bias_f32_async(y, nullptr, n, 4u, stream); }
int dk_net_gelu_bias_f32_async(void* y, const void* bias, uint64_t n, uint32_t width, void* stream) {
    if (!y || n % 4u || width == 0 || width % 4u || n % width) return DK_E_INVALID;
    if (n == 0) return DK_OK;
    const uint64_t n4 = n / 4u;
    hipLaunchKernelGGL(dk::net::gelu_f32_kernel, dim3((unsigned)((n4 + 255u) / 256u)), dim3(256), 0, (hipStream_t)stream,
                       (float*)y, (size_t)n4, (const float*)bias, width / 4u);
    DK_HIP(hipGetLastError());
    return DK_OK;
}

#ifndef DK_ATTN_F32_MFMA
#define DK_ATTN_F32_MFMA 1
#endif
int dk_net_attn62_f32_async(const void* qkv, void* y, uint32_t batch, uint32_t heads, uint32_t head_dim, void* stream) {
    return dk_net_attn62_bias_f32_async(qkv, nullptr, y, batch, heads, head_dim, stream);
}
int dk_net_attn62_bias_f32_async(const void* qkv, const void* bqkv, void* y, uint32_t batch, uint32_t heads, uint32_t head_dim,
                                 void* stream) {
    if (!qkv || !y || heads == 0 || (head_dim != 40u && head_dim != 64u)) return DK_E_INVALID;
    if (batch == 0) return DK_OK;
    if ((uint64_t)batch * heads > 0x7FFFFFFFull) return DK_E_INVALID;
    const float scale = 1.0f / sqrtf((float)head_dim);
#if DK_ATTN_F32_MFMA   // f32 matrix cores (default); 0: the VALU kernel
    if (head_dim == 40u)
        hipLaunchKernelGGL((dk::net::attn62_f32_mfma_kernel<40>), dim3(batch * heads), dim3(64), 0, (hipStream_t)stream,
                           (const float*)qkv, (float*)y, batch, heads, scale, (const float*)bqkv);
    else
        hipLaunchKernelGGL((dk::net::attn62_f32_mfma_kernel<64>), dim3(batch * heads), dim3(64), 0, (hipStream_t)stream,
                           (const float*)qkv, (float*)y, batch, heads, scale, (const float*)bqkv);
#else
    if (bqkv) return DK_E_INVALID;   // (the VALU kernel takes the biased qkv only)
    if (head_dim == 40u)
        hipLaunchKernelGGL((dk::net::attn62_f32_kernel<40>), dim3(batch * heads), dim3(64), 0, (hipStream_t)stream,
                           (const float*)qkv, (float*)y, batch, heads, scale);
    else
        hipLaunchKernelGGL((dk::net::attn62_f32_kernel<64>), dim3(batch * heads), dim3(64), 0, (hipStream_t)stream,
                           (const float*)qkv, (float*)y, batch, heads, scale);
#endif
    DK_HIP(hipGetLastError());
    return DK_OK;
}

int dk_net_add_ln_bf16_async(void* x_io, const void* delta, uint32_t rows, uint32_t d, const void* gamma, const void* beta,
                             float eps, void* h_out, void* stream) {
    const int per = ln_per(d);
    if (!x_io || !h_out || !gamma || !beta || per == 0) return DK_E_INVALID;
    if (rows == 0) return DK_OK;
    const uint32_t rows_per_block = 8u * (uint32_t)dk::net::ADD_LN_ROWS;
    const dim3 grid((rows + rows_per_block - 1u) / rows_per_block), block(256);
    hipStream_t st = (hipStream_t)stream;
    switch (per) {
#define M(P) case P: hipLaunchKernelGGL(dk::net::add_ln_kernel<P>, grid, block, 0, st, (uint16_t*)x_io,                  \
                                        (const uint16_t*)delta, rows, (int)d, (const uint16_t*)gamma, (const uint16_t*)beta, eps, \
                                        (uint16_t*)h_out); break;
        DK_LN_CASES(M)
#undef M
    }
    DK_HIP(hipGetLastError());
    return DK_OK;
}

}  // extern "C"
