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
// MI355X layout (not the reference's pointer tree).  Every node owns a
// contiguous child block reserved at its first expansion (size = number of
// actions it allows).  A node is split into
//   hot  (32 B): stats (visits low 32 | integer win_score high 32), child_base, info,
//                the exact f64 mean and an f32 1/sqrt(visits), both refreshed at backup
//   cold (16 B): unexpanded actions, parent, action   -- touched at expansion only
// so one tree level of the selection is ONE round trip: the child block's hot
// records (contiguous) are loaded together, the UCT pick is computed in
// registers and the picked record is already the next level's node.  The
// stats read on the way down are kept in the LDS path, so the backup is
// store-only (no loads, no atomics): only this lane ever touches this tree.
// Forced chains (nodes with a single allowed action, e.g. the NoAnnouncement
// passes after every card) are walked in ONE step: the chain head (a child of
// a branching node or of the root) keeps in child_base a pointer to the chain
// end, updated whenever the chain grows.  The reference reads a node's
// win_score only when its parent has >= 2 children (UCT) or it is a root child,
// and a node's visits only as ln(N) of a branching node or as a root child, so
// the interior of a chain needs no bookkeeping; which nodes exist, and every
// value that is read, stay identical to the reference's.
// Chain ends keep no statistics: a chain end is passed on every visit of its chain head
// since the end was created, so its visit count is the head's minus the head's count at
// that time, which the end's record holds instead (its win_score is never read: its
// parent has a single child).  The backup therefore writes no chain end.
// Sibling min/max is computed once per level (identical values to the
// reference's per-child recomputation).  ln(N) comes from a host-built table
// of glibc `log` values, which is what Rust's f64::ln calls, so UCT values are
// bit-exact.
#pragma once
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <type_traits>
#include "common.h"
#include "rng.h"

namespace dk {

// Phase timers (profiling builds only): wave-uniform shader-clock stamps taken at
// the reconvergence points between select / expand / rollout / backup.
#if defined(DK_PHASE_PROF) && defined(__HIP_DEVICE_COMPILE__)
#define DK_STAMP(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#define DK_PROF(mem, k, v) prof_acc[k] += (v)
#define DK_PROF_DECL uint64_t prof_acc[PROF_SLOTS] = {}
#define DK_PROF_FLUSH(mem) for (int k_ = 0; k_ < PROF_SLOTS; ++k_) mem.prof_add(k_, prof_acc[k_])
#define DK_STAMP_DRAINED(t) __builtin_amdgcn_s_waitcnt(0); const uint64_t t = __builtin_amdgcn_s_memtime()
#define DK_PROF_WAVEMAX(k, v) do { int m_ = (v); for (int o_ = 32; o_ >= 1; o_ >>= 1) { const int t_ = __shfl_xor(m_, o_); m_ = t_ > m_ ? t_ : m_; } prof_acc[k] += (uint64_t)m_; } while (0)
// a wave-level event counted once (by the lowest active lane): the trip of a loop, with a histogram
// of its active lanes (slots k+1 .. k+5: <= 8, <= 16, <= 32, <= 48, <= 64) and their sum (k+6)
#define DK_PROF_TRIP(k) do { const uint64_t b_ = __builtin_amdgcn_ballot_w64(true); const int na_ = popc64(b_); \
    if ((int)__lane_id() == ctz64(b_)) { prof_acc[k] += 1; \
        prof_acc[(k) + 1 + (na_ <= 8 ? 0 : na_ <= 16 ? 1 : na_ <= 32 ? 2 : na_ <= 48 ? 3 : 4)] += 1; \
        prof_acc[(k) + 6] += (uint64_t)na_; } } while (0)
#else
#define DK_STAMP(t) [[maybe_unused]] const uint64_t t = 0
#define DK_PROF(mem, k, v) ((void)0)
#define DK_PROF_DECL
#define DK_PROF_FLUSH(mem) ((void)0)
#define DK_PROF_WAVEMAX(k, v) ((void)0)
#define DK_PROF_TRIP(k) ((void)0)
#define DK_STAMP_DRAINED(t) [[maybe_unused]] const uint64_t t = 0
#endif

// Two hot-record layouts; the launch picks one per batch (doko_amd.hip, hot_layout):
//  NodeHot16 (16 B): stats, child_base, info.  The pick derives the sibling min / max
//    exactly from 64-bit cross products of the stats and divides in f64 only for the
//    candidates, so a scanned child and a backed-up node cost 16 B.  Faster when the
//    launch has several waves per SIMD (C3: 6 %, C2d: 4 %): the halved bytes win.
//  NodeHot32 (32 B): also the exact mean and an f32 1/sqrt(visits) written by the
//    backup.  Faster at one wave per SIMD (C2's 32,768 roots: 7 %), where the pick's
//    dependent chain is exposed and a cached mean shortens it.
#ifndef DK_HOT16_WAVES
#define DK_HOT16_WAVES 3
#endif
struct alignas(16) NodeHot16 {
    uint64_t stats;       // visits (low 32) | win_score (high 32, two's complement)
    uint32_t child_base;  // first slot of the child block (valid when nchild > 0)
    uint32_t info;        // nchild:6 | player:2 | has_unexpanded:1 | chain_head:1 | state_idx:22
    static constexpr bool CACHED_MEAN = false;
    static constexpr int MIN_WAVES = DK_HOT16_WAVES;   // search-kernel register budget (3 waves per SIMD: <= 168 VGPRs)
    static constexpr bool WIDE = false;                // pool offsets: 32-bit (a wave's regions < 4 GiB)
    static constexpr bool PAIR = false;                // two lanes per root (NodeHot16P)
    static constexpr bool LONG = false;                // 64-bit cross products (NodeHot16L)
};
// 16-B records searched by lane PAIRS: launches of at most 32 roots per wave (a single wave per
// SIMD, half of its lanes otherwise idle) give every root two lanes, lane l and l + 32.  Both
// run the root's whole search on identical data (same control flow, the same loads and stores),
// except the pick, which they split: each scans half of the child block and the halves combine
// their partial minima / maxima / candidates through v_permlane32_swap, keeping the reference's
// first-strict-maximum order (pick_child_pair).
struct alignas(16) NodeHot16P : NodeHot16 {
    static constexpr int MIN_WAVES = 1;
    static constexpr bool PAIR = true;
};
// 16-B records for searches beyond P24_MAX_ITERS iterations (the production shape: 200,000
// iterations per sample, compare_impi/run.rs:270-291): the same record and pick, with the sibling
// means compared by 64-bit cross products (|w| <= 123 v, v < 2^22: products < 2^53).  Until round
// 4 such searches took the 32-B records (NodeHot32); these halve the hot pool per slot.
struct alignas(16) NodeHot16L : NodeHot16 {
    static constexpr int MIN_WAVES = 2;
    static constexpr bool LONG = true;
};
struct alignas(16) NodeHot16PL : NodeHot16P {
    static constexpr bool LONG = true;
};
struct alignas(32) NodeHot32 {
    uint64_t stats;
    uint32_t child_base;
    uint32_t info;
    double q;             // win_score / visits exactly as the reference computes it (0 if unvisited)
    float isv;            // ~1/sqrt(visits) (f32 estimate for the UCT filter)
    uint32_t pad;
    static constexpr bool CACHED_MEAN = true;
    static constexpr int MIN_WAVES = 1;   // no budget (its launches have one wave per SIMD)
    static constexpr bool WIDE = false;
    static constexpr bool PAIR = false;
    static constexpr bool LONG = false;   // (its pick compares the cached exact means)
};
// NodeHot32 addressed with 64-bit offsets: contexts whose per-wave pool regions reach 4 GiB
// (very long searches: the fallback pool's 32-B records at >= ~175 K iterations, node states
// at >= ~1 M iterations), where 32-bit byte offsets would wrap into a neighbour lane's tree.
struct alignas(32) NodeHot32W : NodeHot32 {
    static constexpr bool WIDE = true;
};
// 8-B records (launches of <= P8_MAX_ITERS iterations): everything packed into two words
//   w0 = win_score << 11 | visits                         (the stats: the backup stores w0 only)
//   w1 = child_base/2 : 13 | nchild : 4 | player : 2 | open : 1 | head : 1 | state : 11
// Child blocks start at even slots, so one 16-B load fetches two children and a block of
// twelve is 96 B.  The root's record is never stored (nchild <= 39 does not fit 4 bits):
// the root lives in registers, its stats are the iteration count.  In registers a node is
// carried in the 16-B logical form (NodeHot16 fields); GpuMem / HostMem decode on load.
struct alignas(16) U4 { uint32_t x, y, z, w; };   // one 16-B load: two 8-B records
struct alignas(8) NodeHot8 {
    uint32_t w0, w1;
    static constexpr bool CACHED_MEAN = false;
    static constexpr int MIN_WAVES = DK_HOT16_WAVES;
    static constexpr bool WIDE = false;
    static constexpr bool PAIR = false;
    static constexpr bool LONG = false;
};
// visits < 2^11, slots < 2^14, state indices < 2^10 (bit 10 of the state field marks a
// resolved chain head, below)
static constexpr uint32_t P8_MAX_ITERS = 1023;
// proven slot bound with even-aligned blocks: the root and its padding slot, the root block
// (<= 39 children, padded to 40) and one block of <= 12 children per iteration
static constexpr uint32_t P8_SLOT_BOUND(uint32_t iters) { return 42u + 12u * iters; }
static_assert(P8_SLOT_BOUND(P8_MAX_ITERS) <= (1u << 14), "8-B child_base field");
DK_HD uint32_t p8_w0(uint64_t stats) { return ((uint32_t)(stats >> 32) << 11) | ((uint32_t)stats & 2047u); }
DK_HD uint32_t p8_w1(uint32_t child_base, uint32_t info) {
    return (child_base >> 1) | (info & 15u) << 13 | ((info >> 6) & 15u) << 17 | (info >> 10) << 21;
}
DK_HD uint32_t p8_visits(uint32_t w0) { return w0 & 2047u; }
DK_HD int32_t p8_win(uint32_t w0) { return (int32_t)w0 >> 11; }
DK_HD uint64_t p8_stats(uint32_t w0) { return (uint64_t)(uint32_t)p8_win(w0) << 32 | p8_visits(w0); }
DK_HD uint32_t p8_cb(uint32_t w1) { return (w1 & 0x1FFFu) << 1; }
DK_HD uint32_t p8_info(uint32_t w1) { return ((w1 >> 13) & 15u) | ((w1 >> 17) & 15u) << 6 | (w1 >> 21) << 10; }
DK_HD bool p8_forced(uint32_t w1) { return (w1 & (15u << 13 | 1u << 19)) == 1u << 13; }   // nchild == 1 && !open
// A resolved chain head: a forced chain head whose chain end is fully expanded stores the
// end's child block, child count and player in place of its own (never used again) state,
// marked by bit 10 of the state field, so that the selection descends from the head to the
// end's children without loading the end's record.  The end's visit count, the ln(N) of its
// pick, is 1 + the sum of its children's visits (every simulation through a non-terminal
// node after the one that created it goes on to one of its children).
static constexpr uint32_t P8_RESOLVED = 0x400u;
DK_HD bool ni_resolved(uint32_t info) { return ((info >> 10) & P8_RESOLVED) != 0; }   // (state field: info >> 10)
template <class H> struct is_p8 { static constexpr bool value = false; };
template <> struct is_p8<NodeHot8> { static constexpr bool value = true; };

// the layout of host builds (test harnesses); -DDK_HOT16=0 selects the 32-B one
#ifndef DK_HOT16
#define DK_HOT16 1
#endif
#if defined(DK_HOT16L) && DK_HOT16L
using NodeHot = NodeHot16L;   // (host builds of the long 16-B records: 64-bit cross products)
#elif DK_HOT16
using NodeHot = NodeHot16;
#else
using NodeHot = NodeHot32;
#endif
struct alignas(16) NodeCold {
    uint64_t unexpanded;  // actions not yet expanded
    uint32_t parent;      // parent slot (0xFFFFFFFF for the root)
    uint32_t action;      // action that led here
};

DK_HD uint32_t ni_nchild(uint32_t info) { return info & 63u; }
DK_HD uint32_t ni_player(uint32_t info) { return (info >> 6) & 3u; }
DK_HD bool ni_open(uint32_t info) { return (info >> 8) & 1u; }
DK_HD bool ni_head(uint32_t info) { return (info >> 9) & 1u; }
DK_HD uint32_t ni_state(uint32_t info) { return info >> 10; }
DK_HD uint32_t ni_make(uint32_t nchild, uint32_t player, bool open, bool head, uint32_t state) {
    return nchild | (player << 6) | (open ? 1u << 8 : 0u) | (head ? 1u << 9 : 0u) | (state << 10);
}
static constexpr uint32_t NI_MAX_STATES = 1u << 22;
#ifndef DK_DEFER_BACKUP
#define DK_DEFER_BACKUP 0
#endif
static constexpr int PROF_SLOTS = 40;   // per-root counters of the profiling build (DK_PHASE_PROF)
// Child-block placement (GpuMem::balign / HostMem::balign): a power of two A >= 1 starts every block
// at a multiple of A slots; BALIGN_LINE | L (L a power of two: the slots of one 128-B line) packs
// blocks but moves one that would straddle a line boundary to the next line, so that a block of at
// most L slots is one line -- one DRAM line per selection level instead of 1.6 on average with
// 8-B records (a random 8 / 16-B access moves a whole 128-B line) -- and a larger one starts a line.  `pb`: the block's slots (8-B
// records: rounded up to even).  Placement never changes results, only slot indices.
static constexpr uint32_t BALIGN_LINE = 0x80000000u;
DK_HD uint32_t block_base(uint32_t next, uint32_t pb, uint32_t balign) {
    if (balign & BALIGN_LINE) {
        const uint32_t line = balign & 0xFFFFu;
        const uint32_t off = next & (line - 1u);
        if (pb > line) return off ? next + (line - off) : next;        // (a larger block: whole lines)
        return off + pb > line ? next + (line - off) : next;
    }
    return (next + balign - 1u) & ~(balign - 1u);
}
static constexpr int MAX_DEPTH = 512;   // selection path bound (LDS part + global overflow)

DK_HD int sel4i(const int r[4], int p) { return p == 0 ? r[0] : (p == 1 ? r[1] : (p == 2 ? r[2] : r[3])); }

static constexpr double DK_F64_EPSILON = 2.220446049250313e-16;
static constexpr int SCAN_REG = 12;  // child blocks up to this size are scanned from registers

// Outcome codes of search_root
enum { SR_OK = 0, SR_CAPACITY = 1, SR_STATE = 2 };

DK_HD double mean_of(uint64_t st) {
    const uint32_t v = (uint32_t)st;
    return v > 0 ? (double)(int32_t)(st >> 32) / (double)v : 0.0;
}

// Exact UCT value of one child (node.rs:238-277), the reference's f64 ops in order.
// (q = the child's mean as computed by mean_of)
DK_HD double uct_exact(uint64_t st, double q, bool flat, double min_q, double max_q, double lnN, double c) {
    const uint32_t v = (uint32_t)st;
    if (v == 0) return INFINITY;
    const double nq = flat ? 1.0 : 2.0 * (q - min_q) / (max_q - min_q) - 1.0;
    return nq + c * sqrt(lnN / (double)v);
}

#if defined(__HIP_DEVICE_COMPILE__)
DK_HD float rcp_approx(float x) { return __builtin_amdgcn_rcpf(x); }
DK_HD float sqrt_approx(float x) { return __builtin_amdgcn_sqrtf(x); }
DK_HD float rsqrt_approx(float x) { return __builtin_amdgcn_rsqf(x); }
#elif defined(DK_APPROX_HOOKS)   // host tests: adversarially perturbed approximations
float rcp_approx(float x);
float sqrt_approx(float x);
float rsqrt_approx(float x);
#else
DK_HD float rcp_approx(float x) { return 1.0f / x; }
DK_HD float sqrt_approx(float x) { return sqrtf(x); }
DK_HD float rsqrt_approx(float x) { return 1.0f / sqrtf(x); }
#endif

template <class H>
DK_HD H make_hot(uint64_t stats, uint32_t child_base, uint32_t info) {
    H h;
    h.stats = stats; h.child_base = child_base; h.info = info;
    if constexpr (H::CACHED_MEAN) {
        h.q = mean_of(stats); h.isv = (uint32_t)stats ? rsqrt_approx((float)(uint32_t)stats) : 0.0f; h.pad = 0;
    }
    return h;
}
// the backup's store: stats, plus the cached mean of a 32-B record
template <class H>
DK_HD void hot_backup(H& h, uint64_t stats, double q, float isv) {
    h.stats = stats;
    if constexpr (H::CACHED_MEAN) { h.q = q; h.isv = isv; }
    else { (void)q; (void)isv; }
}
// the exact mean (mean_of) and the f32 1/sqrt(visits) estimate of a hot record
DK_HD double hot_q(const NodeHot16& h) { return mean_of(h.stats); }
DK_HD double hot_q(const NodeHot32& h) { return h.q; }
DK_HD float hot_isv(const NodeHot16& h) { return (uint32_t)h.stats ? rsqrt_approx((float)(uint32_t)h.stats) : 0.0f; }
DK_HD float hot_isv(const NodeHot32& h) { return h.isv; }

// Child block of n <= SCAN_REG records held in registers, structure of arrays
// (constant indices only, so everything stays in VGPRs).
struct Block {
    uint64_t st[SCAN_REG];
    uint32_t cb[SCAN_REG], inf[SCAN_REG];
    double q[SCAN_REG];
    float isv[SCAN_REG];
};

// UCT pick over a register block (32-B records); returns the index and the picked node's
// stats / child_base / info.  Bit-exact with the reference's first-strict-
// maximum over f64 UCT values:
//  1. sibling min / max over the stored exact means (the reference's values);
//  2. every child's UCT value estimated in f32 from the same f64 differences
//     and the stored 1/sqrt(v): |u_f32 - u_f64| <= B with
//     B ~ 4e-7 * (2 + c*sqrt(ln N)) + 5e-7 (derivation in DESIGN.md);
//  3. exact f64 UCT only for children whose estimate is within 2B (taken
//     with a x3.7 safety factor) of the best estimate -- all others are
//     strictly below the maximum -- first strict maximum among them, and only
//     when their statistics differ (equal statistics: the first one wins).
// Every scanned child has been visited (see pick_child_x).
//
// Chain-end prefetch: the chain end of the leading candidate, if it is an expanded
// single-action node (a forced chain head), is loaded while the exact evaluation
// runs; *end_ok tells whether *end holds the picked child's chain end.
template <class Mem>
DK_HD uint32_t pick_child_reg(const Block& b, uint32_t n, double lnN, double c, Mem& mem, uint64_t* p_st, uint32_t* p_cb,
                              uint32_t* p_inf, NodeHot32* end, bool* end_ok) {
#if !defined(__HIP_DEVICE_COMPILE__)
    for (uint32_t j = 0; j < n; ++j)
        if ((uint32_t)b.st[j] == 0) { fprintf(stderr, "pick_child_reg: unvisited child\n"); abort(); }
#endif
    double min_q = INFINITY, max_q = -INFINITY;
#pragma unroll
    for (int j = 0; j < SCAN_REG; ++j) {
        if ((uint32_t)j < n) {
            min_q = b.q[j] < min_q ? b.q[j] : min_q;
            max_q = b.q[j] > max_q ? b.q[j] : max_q;
        }
    }
    const double range = max_q - min_q;
    const bool flat = fabs(range) < DK_F64_EPSILON;
    const float inv_r = flat ? 0.0f : 2.0f * rcp_approx((float)range);
    const float ex = (float)c * sqrt_approx((float)lnN);
    // the first maximum of the estimates, tracked with its record
    float ue[SCAN_REG];
    float umax = -INFINITY;
    uint32_t jm = 0, cbm = b.cb[0], inm = b.inf[0];
    uint64_t sm = b.st[0];
#pragma unroll
    for (int j = 0; j < SCAN_REG; ++j) {
        ue[j] = -INFINITY;
        if (wave_any((uint32_t)j < n)) {
            const float nq = flat ? 1.0f : (float)(b.q[j] - min_q) * inv_r - 1.0f;
            ue[j] = (uint32_t)j < n ? nq + ex * b.isv[j] : -INFINITY;
            const bool gt = ue[j] > umax;
            umax = gt ? ue[j] : umax;
            jm = gt ? (uint32_t)j : jm;
            sm = gt ? b.st[j] : sm; cbm = gt ? b.cb[j] : cbm; inm = gt ? b.inf[j] : inm;
        }
    }
    const float cut = umax - 3e-6f * (3.0f + fabsf(ex));
    uint32_t cmask = 0;
#pragma unroll
    for (int j = 0; j < SCAN_REG; ++j) cmask |= (ue[j] >= cut ? 1u : 0u) << j;   // implies j < n
    const uint32_t nc = (uint32_t)popc32(cmask);
    // prefetch the chain end of the leading candidate if it is a forced chain head
    const bool f1 = ni_nchild(inm) == 1 && !ni_open(inm);
    NodeHot32 e1;
    if (f1) e1 = mem.load_hot(cbm);
    // As in pick_child_x: candidates sharing the leader's statistics (equal f64 values, the
    // first of them wins) need no exact evaluation; otherwise the f64 formula decides among
    // all candidates, first strict maximum.
    uint32_t pick = jm, pc = cbm, pi = inm;
    uint64_t ps = sm;
    uint32_t emask = jm != (uint32_t)ctz32(cmask) ? 1u : 0u;
    if (nc >= 2) {
#pragma unroll
        for (int j = 0; j < SCAN_REG; ++j) emask |= (((cmask >> j) & 1u) && b.st[j] != sm ? 1u : 0u) << j;
    }
    if (emask) {
        double best = -INFINITY;
#pragma unroll
        for (int j = 0; j < SCAN_REG; ++j) {
            if ((cmask >> j) & 1u) {
                const double u = uct_exact(b.st[j], b.q[j], flat, min_q, max_q, lnN, c);
                if (u > best) { best = u; pick = (uint32_t)j; ps = b.st[j]; pc = b.cb[j]; pi = b.inf[j]; }
            }
        }
    }
    *p_st = ps; *p_cb = pc; *p_inf = pi;
    *end_ok = pick == jm && f1;
    if (*end_ok) *end = e1;
    return pick;
}

// Exact comparison of two means w_a/v_a < w_b/v_b (v > 0) by cross products in 24-bit
// multiplies (v_mul_i32_i24, full rate): exact while |w| < 2^23, v < 2^23 and |w| v < 2^31.
// A simulation's reward is a player_points value, |r| <= 123 for every engine (DKV scoring:
// 25 basic + 10 extra points, x3 for a solo, stats/**), so |w| <= 123 v and v <= iterations;
// the launch takes 16-B records only for iterations <= P24_MAX_ITERS (doko_amd.hip).
static constexpr uint32_t P24_MAX_ITERS = 4095;
static_assert((uint64_t)P24_MAX_ITERS * P24_MAX_ITERS * 123u < (1ull << 31), "cross products exceed 31 bits");
static_assert((uint64_t)P24_MAX_ITERS * 123u < (1ull << 23), "win scores exceed 24-bit operands");
DK_HD int mul24(int a, int b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __mul24(a, b);
#else
    return a * b;
#endif
}
DK_HD bool mean_lt(int32_t wa, uint32_t va, int32_t wb, uint32_t vb) { return mul24(wa, (int)vb) < mul24(wb, (int)va); }
// the comparison of the long records (NodeHot16L): 64-bit cross products, exact for |w| <= 123 v and
// v < NI_MAX_STATES (iterations are bounded by the state index field): |w| v < 123 * 2^44 < 2^51
template <bool LONG>
DK_HD bool mean_lt_t(int32_t wa, uint32_t va, int32_t wb, uint32_t vb) {
    if constexpr (LONG) return (int64_t)wa * (int64_t)vb < (int64_t)wb * (int64_t)va;
    else return mean_lt(wa, va, wb, vb);
}
// The spread of the sibling means as D = wmax vmin - wmin vmax >= 0 (exact), returned as f32
// (D == 0 <=> the reference's `range < f64::EPSILON`: distinct fractions with denominators below
// 2^22 differ by more than 2^-44, which their f64 quotients keep).
template <bool LONG>
DK_HD float spread_d(int32_t wmax, uint32_t vmax, int32_t wmin, uint32_t vmin, bool* flat) {
    if constexpr (LONG) {
        const int64_t D = (int64_t)wmax * (int64_t)vmin - (int64_t)wmin * (int64_t)vmax;
        *flat = D == 0;
        return (float)D;
    } else {
        // >= 0 and < 2^32: exact in u32 arithmetic (each product is < 2^31 in magnitude, mean_lt)
        const uint32_t D = (uint32_t)mul24(wmax, (int)vmin) - (uint32_t)mul24(wmin, (int)vmax);
        *flat = D == 0;
        return (float)D;
    }
}

// Blocks of 8-B records held as raw words.
struct Block8 {
    uint32_t w0[SCAN_REG], w1[SCAN_REG];
};

// Record accessors of the shared pick (pick_child_x): a child's raw fields as the block
// holds them, its visits / win_score, and the in-register decode of the picked child.
struct Raw16 {
    static constexpr bool LONG = false;
    uint64_t st; uint32_t cb, inf;
    DK_HD static Raw16 at(const Block& b, int j) { return Raw16{b.st[j], b.cb[j], b.inf[j]}; }
    DK_HD uint32_t vis() const { return (uint32_t)st; }
    DK_HD int32_t win() const { return (int32_t)(st >> 32); }
    DK_HD uint64_t stats() const { return st; }
    DK_HD uint64_t key() const { return st; }        // equal keys <=> equal statistics
    DK_HD uint32_t child_base() const { return cb; }
    DK_HD uint32_t info() const { return inf; }
    DK_HD bool forced() const { return ni_nchild(inf) == 1 && !ni_open(inf); }
};
struct Raw16L : Raw16 {   // (NodeHot16L: 64-bit cross products)
    static constexpr bool LONG = true;
    DK_HD static Raw16L at(const Block& b, int j) { Raw16L r; r.st = b.st[j]; r.cb = b.cb[j]; r.inf = b.inf[j]; return r; }
};
struct Raw8 {
    static constexpr bool LONG = false;
    uint32_t w0, w1;
    DK_HD static Raw8 at(const Block8& b, int j) { return Raw8{b.w0[j], b.w1[j]}; }
    DK_HD uint32_t vis() const { return p8_visits(w0); }
    DK_HD int32_t win() const { return p8_win(w0); }
    DK_HD uint64_t stats() const { return p8_stats(w0); }
    DK_HD uint32_t key() const { return w0; }        // equal keys <=> equal statistics
    DK_HD uint32_t child_base() const { return p8_cb(w1); }
    DK_HD uint32_t info() const { return p8_info(w1); }
    DK_HD bool forced() const { return p8_forced(w1) && !(w1 >> 31); }   // (resolved heads need no prefetch)
};
template <class R>
DK_HD R sel_raw(bool p, const R& a, const R& b);
template <>
DK_HD Raw16 sel_raw(bool p, const Raw16& a, const Raw16& b) { return Raw16{p ? a.st : b.st, p ? a.cb : b.cb, p ? a.inf : b.inf}; }
template <>
DK_HD Raw8 sel_raw(bool p, const Raw8& a, const Raw8& b) { return Raw8{p ? a.w0 : b.w0, p ? a.w1 : b.w1}; }
template <>
DK_HD Raw16L sel_raw(bool p, const Raw16L& a, const Raw16L& b) {
    Raw16L r; r.st = p ? a.st : b.st; r.cb = p ? a.cb : b.cb; r.inf = p ? a.inf : b.inf; return r;
}


// The pick for 8-B and 16-B records (no stored mean), bit-exact with the reference's first
// strict maximum of the f64 UCT values (node.rs:238-277):
//  1. the sibling min / max EXACTLY, by comparing means w/v as 24-bit cross products
//     (mean_lt; an unvisited child's mean is 0/1).  The spread is D / (vmin vmax) with the
//     integer D = wmax vmin - wmin vmax, so the reference's `range < f64::EPSILON` is D == 0:
//     two distinct fractions of denominators <= 4095 differ by >= 6e-8 (the f64 quotients
//     keep that gap), equal ones give range 0.
//  2. every child's UCT value estimated in f32: with r = rsq(v), the mean is w r^2 and the
//     exploration term c sqrt(ln N) r, so one transcendental per child; the normalisation
//     2 (q - min) / range - 1 is one fma with A = 2 vmin vmax / D, B = -(A min + 1).  The
//     estimate's error stays under the cut's margin: the f32 mean carries
//     a relative error of a few ulp (<= 1e-6 with rsq perturbed by 4 ulp), covered by the
//     4e-6 |q|max / range term.
//  3. the exact f64 formula only for the children within the margin of the best estimate
//     (a 12-bit candidate mask): none with one candidate; the f64 min / max quotients are
//     computed only then.
// A child index j that no lane's block reaches is skipped wave-uniformly (wave_any), so a
// wave whose blocks are all narrow pays for its widest block, not for twelve children.
// Chain-end prefetch as in pick_child_reg.
// Every child it scans has been visited: the selection descends only into fully expanded
// nodes, and each child was backed up by the simulation that created it (the reference's
// +inf for an unvisited child never arises; host builds check this).
template <class R, class B, class Mem>
DK_HD uint32_t pick_child_x(const B& b, uint32_t n, double lnN, double c, Mem& mem, uint64_t* p_st, uint32_t* p_cb,
                            uint32_t* p_inf, NodeHot16* end, bool* end_ok, uint32_t cbx) {
#if !defined(__HIP_DEVICE_COMPILE__)
    for (uint32_t j = 0; j < n; ++j)
        if (R::at(b, (int)j).vis() == 0) { fprintf(stderr, "pick_child_x: unvisited child\n"); abort(); }
#endif
    int32_t wmin = R::at(b, 0).win(), wmax = wmin;
    uint32_t vmin = R::at(b, 0).vis(), vmax;
    vmax = vmin;
    // (a branch per child, not a select: a wave whose blocks are all narrower than j skips it)
#pragma unroll
    for (int j = 1; j < SCAN_REG; ++j) {
        if ((uint32_t)j < n) {
            const R r = R::at(b, j);
            const int32_t w = r.win();
            const uint32_t v = r.vis();
            const bool lt = mean_lt_t<R::LONG>(w, v, wmin, vmin);
            const bool gt = mean_lt_t<R::LONG>(wmax, vmax, w, v);
            wmin = lt ? w : wmin; vmin = lt ? v : vmin;
            wmax = gt ? w : wmax; vmax = gt ? v : vmax;
        }
    }
    bool flat;
    const float Df = spread_d<R::LONG>(wmax, vmax, wmin, vmin, &flat);
    const float vv = (float)vmin * (float)vmax;                           // exact below 2^24 (LONG: one rounding)
    const float A = flat ? 0.0f : 2.0f * vv * rcp_approx(Df);
    const float minf = (float)wmin * rcp_approx((float)vmin);
    const float maxf = (float)wmax * rcp_approx((float)vmax);
    const float Bc = flat ? 1.0f : -(minf * A + 1.0f);
    const float qabs = fmaxf(fabsf(minf), fabsf(maxf));
    const float ex = (float)c * sqrt_approx((float)lnN);
    // The first maximum of the estimates is tracked with its record, so no per-index
    // selection is needed afterwards.
    float ue[SCAN_REG];
    float umax = -INFINITY;
    uint32_t jm = 0;
    R rm = R::at(b, 0);
#pragma unroll
    for (int j = 0; j < SCAN_REG; ++j) {
        ue[j] = -INFINITY;
        if (wave_any((uint32_t)j < n)) {
            const R r = R::at(b, j);
            const uint32_t vis = r.vis();
            const float rs = rsqrt_approx((float)vis);
            const float nq = fmaf((float)r.win() * (rs * rs), A, Bc);
            ue[j] = (uint32_t)j < n ? fmaf(ex, rs, nq) : -INFINITY;
            const bool gt = ue[j] > umax;
            umax = gt ? ue[j] : umax;
            jm = gt ? (uint32_t)j : jm;
            rm = sel_raw(gt, r, rm);
        }
    }
    // the leading candidate is the pick but in the rare exact case: start its next load now
    mem.touch_next(cbx + jm, rm.child_base(), rm.info());
    const float cut = umax - (3e-6f * (3.0f + fabsf(ex)) + 4e-6f * qabs * A);
    uint32_t cmask = 0;
#pragma unroll
    for (int j = 0; j < SCAN_REG; ++j) cmask |= (ue[j] >= cut ? 1u : 0u) << j;   // implies j < n
    const uint32_t nc = (uint32_t)popc32(cmask);
#ifdef DK_PICK_CENSUS
    dk_pick_census(n, nc);
    { uint32_t c1 = (uint32_t)ctz32(cmask), dif = 0;
      for (int j = 0; j < SCAN_REG; ++j) dif |= ((cmask >> j) & 1u) && R::at(b, j).key() != R::at(b, (int)c1).key();
      dk_pick_tie(dif == 0); }
#endif
    // prefetch the chain end of the leading candidate if it is a forced chain head
    const bool f1 = rm.forced();
    NodeHot16 e1;
    if (f1) e1 = mem.load_hot(rm.child_base());
    uint32_t pick = jm;
    R rp = rm;
    // When every candidate has the leading one's statistics, their f64 values are equal and
    // the first candidate wins, which is jm (equal statistics give equal estimates; the test
    // jm == first candidate keeps this exact even where they would not).  Otherwise (0.09 %
    // of the picks at C3) the reference's f64 formula decides among all candidates, first
    // strict maximum.
    uint32_t emask = jm != (uint32_t)ctz32(cmask) ? 1u : 0u;
    if (nc >= 2) {
#pragma unroll
        for (int j = 0; j < SCAN_REG; ++j) emask |= (((cmask >> j) & 1u) && R::at(b, j).key() != rm.key() ? 1u : 0u) << j;
    }
    if (emask) {
        const double min_q = (double)wmin / (double)vmin, max_q = (double)wmax / (double)vmax;
        double best = -INFINITY;
#pragma unroll
        for (int j = 0; j < SCAN_REG; ++j) {
            if ((cmask >> j) & 1u) {
                const R r = R::at(b, j);
                const uint64_t sj = r.stats();
                const double u = uct_exact(sj, mean_of(sj), flat, min_q, max_q, lnN, c);
                if (u > best) { best = u; pick = (uint32_t)j; rp = r; }
            }
        }
    }
    *p_st = rp.stats(); *p_cb = rp.child_base(); *p_inf = rp.info();
    *end_ok = pick == jm && f1;
    if (*end_ok) *end = e1;
    return pick;
}

#ifndef DK_TOUCH_EARLY
#define DK_TOUCH_EARLY 0
#endif
// ---- lane pairs (NodeHot16P) ----------------------------------------------------------
static constexpr int SCAN_HALF = SCAN_REG / 2;   // children per lane of a pair
// Half a child block (16-B records) in registers.
struct BlockH {
    uint64_t st[SCAN_HALF];
    uint32_t cb[SCAN_HALF], inf[SCAN_HALF];
};
// The partner lane's value (lane ^ 32): one v_permlane32_swap (a half exchange) and a select.
DK_HD uint32_t pair_x(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return __lane_id() < 32 ? r[1] : r[0];
#else
    return v;   // (host builds never search in pairs)
#endif
}
DK_HD uint64_t pair_x64(uint64_t v) { return (uint64_t)pair_x((uint32_t)(v >> 32)) << 32 | pair_x((uint32_t)v); }
DK_HD int32_t pair_xi(int32_t v) { return (int32_t)pair_x((uint32_t)v); }
DK_HD float pair_xf(float v) { union { float f; uint32_t u; } a; a.f = v; a.u = pair_x(a.u); return a.f; }
DK_HD double pair_xd(double v) { union { double d; uint64_t u; } a; a.d = v; a.u = pair_x64(a.u); return a.d; }

// pick_child_x for a lane pair: this lane holds children j0 .. j0 + 5 of the block (j0 = 0 in the
// lower half of the wave, 6 in the upper), its partner the others.  Every step keeps the
// sequential order of pick_child_x: a partial result of the upper half (later children) replaces
// the lower half's only when it is STRICTLY smaller (sibling minimum), strictly larger (sibling
// maximum, first estimate maximum, first exact maximum), so both lanes end with the reference's
// first strict maximum (node.rs:258-277) and the same record.
template <bool LONG, class Mem>
DK_HD uint32_t pick_child_pair(const BlockH& b, uint32_t n, uint32_t j0, double lnN, double c, Mem& mem,
                               uint64_t* p_st, uint32_t* p_cb, uint32_t* p_inf, NodeHot16* end, bool* end_ok,
                               uint32_t cbx) {
    const bool upper = j0 != 0;
    const bool have = j0 < n;                 // the lower half always holds child 0
#if DK_TOUCH_EARLY
    // 0. before the pick: each lane requests what the next step would load for its half's most
    // visited child (UCT's pick converges to the most visited), so that the real load of the
    // picked child's block / state finds it on its way while the pick runs
    if (have) {
        uint32_t vb = (uint32_t)b.st[0], jb = 0, cbb = b.cb[0], inb = b.inf[0];
#pragma unroll
        for (int k = 1; k < SCAN_HALF; ++k) {
            const bool better = j0 + (uint32_t)k < n && (uint32_t)b.st[k] > vb;
            vb = better ? (uint32_t)b.st[k] : vb; jb = better ? (uint32_t)k : jb;
            cbb = better ? b.cb[k] : cbb; inb = better ? b.inf[k] : inb;
        }
        mem.touch_early(cbx + j0 + jb, cbb, inb);
    }
#endif
    // 1. sibling min / max (exact, cross products) over this half, then the pair
    int32_t wmin = have ? (int32_t)(b.st[0] >> 32) : 0, wmax = wmin;
    uint32_t vmin = have ? (uint32_t)b.st[0] : 1u, vmax = vmin;
#pragma unroll
    for (int k = 1; k < SCAN_HALF; ++k) {
        if (j0 + (uint32_t)k < n) {
            const int32_t w = (int32_t)(b.st[k] >> 32);
            const uint32_t v = (uint32_t)b.st[k];
            const bool lt = mean_lt_t<LONG>(w, v, wmin, vmin);
            const bool gt = mean_lt_t<LONG>(wmax, vmax, w, v);
            wmin = lt ? w : wmin; vmin = lt ? v : vmin;
            wmax = gt ? w : wmax; vmax = gt ? v : vmax;
        }
    }
    {
        const int32_t pwmin = pair_xi(wmin), pwmax = pair_xi(wmax);
        const uint32_t pvmin = pair_x(vmin), pvmax = pair_x(vmax);
        const bool phave = upper || n > (uint32_t)SCAN_HALF;   // the partner holds a child
        // lower-half (a) and upper-half (b) partials: b replaces a only when strictly beyond it
        const int32_t awmin = upper ? pwmin : wmin, awmax = upper ? pwmax : wmax;
        const uint32_t avmin = upper ? pvmin : vmin, avmax = upper ? pvmax : vmax;
        const int32_t bwmin = upper ? wmin : pwmin, bwmax = upper ? wmax : pwmax;
        const uint32_t bvmin = upper ? vmin : pvmin, bvmax = upper ? vmax : pvmax;
        const bool bh = upper ? have : phave;
        const bool bmin = bh && mean_lt_t<LONG>(bwmin, bvmin, awmin, avmin);
        const bool bmax = bh && mean_lt_t<LONG>(awmax, avmax, bwmax, bvmax);
        wmin = bmin ? bwmin : awmin; vmin = bmin ? bvmin : avmin;
        wmax = bmax ? bwmax : awmax; vmax = bmax ? bvmax : avmax;
    }
    bool flat;
    const float Df = spread_d<LONG>(wmax, vmax, wmin, vmin, &flat);
    const float vv = (float)vmin * (float)vmax;
    const float A = flat ? 0.0f : 2.0f * vv * rcp_approx(Df);
    const float minf = (float)wmin * rcp_approx((float)vmin);
    const float maxf = (float)wmax * rcp_approx((float)vmax);
    const float Bc = flat ? 1.0f : -(minf * A + 1.0f);
    const float qabs = fmaxf(fabsf(minf), fabsf(maxf));
    const float ex = (float)c * sqrt_approx((float)lnN);
    // 2. estimates of this half, first maximum with its record
    float ue[SCAN_HALF];
    float umax = -INFINITY;
    uint32_t jm = j0, cbm = b.cb[0], inm = b.inf[0];
    uint64_t sm = b.st[0];
#pragma unroll
    for (int k = 0; k < SCAN_HALF; ++k) {
        ue[k] = -INFINITY;
        if (wave_any(j0 + (uint32_t)k < n)) {
            const uint32_t vis = (uint32_t)b.st[k];
            const float rs = rsqrt_approx((float)vis);
            const float nq = fmaf((float)(int32_t)(b.st[k] >> 32) * (rs * rs), A, Bc);
            ue[k] = j0 + (uint32_t)k < n ? fmaf(ex, rs, nq) : -INFINITY;
            const bool gt = ue[k] > umax;
            umax = gt ? ue[k] : umax;
            jm = gt ? j0 + (uint32_t)k : jm;
            sm = gt ? b.st[k] : sm; cbm = gt ? b.cb[k] : cbm; inm = gt ? b.inf[k] : inm;
        }
    }
    {
        const float pu = pair_xf(umax);
        const uint32_t pj = pair_x(jm), pcb = pair_x(cbm), pin = pair_x(inm);
        const uint64_t ps = pair_x64(sm);
        // the upper half's maximum wins only when strictly larger (its children come later)
        const bool take = upper ? !(umax > pu) : pu > umax;
        umax = take ? pu : umax; jm = take ? pj : jm; cbm = take ? pcb : cbm; inm = take ? pin : inm; sm = take ? ps : sm;
    }
    mem.touch_next(cbx + jm, cbm, inm);   // (see pick_child_x)
    const float cut = umax - (3e-6f * (3.0f + fabsf(ex)) + 4e-6f * qabs * A);
    uint32_t cmask = 0;
#pragma unroll
    for (int k = 0; k < SCAN_HALF; ++k) cmask |= (ue[k] >= cut ? 1u : 0u) << (j0 + (uint32_t)k);
    cmask |= pair_x(cmask);
    const uint32_t nc = (uint32_t)popc32(cmask);
    // prefetch the chain end of the leading candidate if it is a forced chain head
    const bool f1 = ni_nchild(inm) == 1 && !ni_open(inm);
    NodeHot16 e1;
    if (f1) e1 = mem.load_hot(cbm);
    uint32_t pick = jm, pc = cbm, pi = inm;
    uint64_t ps = sm;
    uint32_t emask = jm != (uint32_t)ctz32(cmask) ? 1u : 0u;
    if (nc >= 2) {
        uint32_t em = 0;
#pragma unroll
        for (int k = 0; k < SCAN_HALF; ++k) em |= (((cmask >> (j0 + k)) & 1u) && b.st[k] != sm ? 1u : 0u);
        emask |= em | pair_x(em);
    }
    if (emask) {
        // the exact f64 values of this half's candidates, first strict maximum, then the pair's
        const double min_q = (double)wmin / (double)vmin, max_q = (double)wmax / (double)vmax;
        double best = -INFINITY;
        uint32_t bj = 0, bcb = 0, binf = 0;
        uint64_t bst = 0;
#pragma unroll
        for (int k = 0; k < SCAN_HALF; ++k) {
            if ((cmask >> (j0 + k)) & 1u) {
                const double u = uct_exact(b.st[k], mean_of(b.st[k]), flat, min_q, max_q, lnN, c);
                if (u > best) { best = u; bj = j0 + (uint32_t)k; bst = b.st[k]; bcb = b.cb[k]; binf = b.inf[k]; }
            }
        }
        const double pb = pair_xd(best);
        const uint32_t pj = pair_x(bj), pcb = pair_x(bcb), pin = pair_x(binf);
        const uint64_t pst = pair_x64(bst);
        const bool take = upper ? !(best > pb) : pb > best;
        pick = take ? pj : bj; ps = take ? pst : bst; pc = take ? pcb : bcb; pi = take ? pin : binf;
    }
    *p_st = ps; *p_cb = pc; *p_inf = pi;
    *end_ok = pick == jm && f1;
    if (*end_ok) *end = e1;
    return pick;
}

template <class E, class Mem>
DK_HD int search_root(const typename E::Work& root, Rng& rng, uint32_t iters, double c,
                      Mem& mem, uint32_t* visits39, double* values39, uint8_t* best_out, uint64_t* ctr_scanned,
                      uint32_t* used = nullptr) {
    using Work = typename E::Work;
    using NodeHot = typename Mem::Hot;   // the in-register form of a node (8-B records: NodeHot16)
    constexpr bool P8 = is_p8<typename Mem::Rec>::value;
    // the root's structure (child_base, info) lives in registers: it changes only
    // when the root itself is expanded, and its visits are the iteration count
    uint32_t root_cb = 0, root_info;
    if (!E::node_ok(root)) {   // a root whose fields the 64-B node record cannot hold (malformed)
        for (int a = 0; a < 39; ++a) { visits39[a] = 0; values39[a] = 0.0; }
        *best_out = 0xFF;
        return SR_STATE;
    }
    {
        const uint64_t ra = E::allowed(root, true);
        const NodeHot h = make_hot<NodeHot>(0, 0, ni_make(0, (uint32_t)E::current_player(root), ra != 0, false, 0));
        root_info = h.info;
        NodeCold cd;
        cd.unexpanded = ra; cd.parent = 0xFFFFFFFFu; cd.action = 0xFFu;
        if constexpr (!P8) mem.store_hot(0, h);   // 8-B records: the root is never stored
        mem.store_cold(0, cd);
        mem.store_state(0, E::pack_node(root));
    }
    // 8-B records: child blocks start at even slots (slot 1 is padding)
    uint32_t next_slot = P8 ? 2 : 1, next_state = 1;
    int status = SR_OK;
    uint64_t scanned = 0;
    DK_PROF_DECL;
    // Deferred backup (8-B records, DK_DEFER_BACKUP): a simulation's backup writes the updated
    // statistics into its LDS path entries only; the global stores are issued by the NEXT
    // simulation's selection, entry k right before the load of the block that holds it (the
    // block of entry k - 1's node), the rest after the selection.  Every VMEM wait counts the
    // wave's earlier stores (vmcnt on gfx9), so stores issued right before the selection's
    // first load put their completion latency on every simulation's critical path; issued one
    // level ahead, each completes under the previous level's load.  A lane's loads see its own
    // earlier stores (program order), so every read is the value the immediate stores gave.
    // (8-B records and lane pairs; the 16- / 32-B three-wave kernels would spill the extra state)
    constexpr bool DEFER = DK_DEFER_BACKUP && (P8 || Mem::Rec::PAIR);
    uint32_t pend = 0;                      // pending entries: n | kc << 8 | kx << 16 (0xFF: none)
    uint32_t pend_ci = 0, pend_xi = 0;      // structure words of the new leaf / the expanded node
    uint32_t pend_xcb = 0;                  // (16- / 32-B records: the expanded node's child base)
    auto flush = [&](int k) {
        uint64_t ns;
        const uint32_t e = mem.path_get_lds(k, &ns);
        const uint32_t s = e & 0x3FFFFFFFu;
        const int kc_ = (int)((pend >> 8) & 0xFFu), kx_ = (int)((pend >> 16) & 0xFFu);
        if constexpr (P8) {
            if (k == kc_ || k == kx_) mem.store_rec8(s, p8_w0(ns), k == kc_ ? pend_ci : pend_xi);
            else mem.store_backup(s, ns, 0.0, 0.0f);
        } else {
            if (k == kc_) mem.store_hot(s, make_hot<NodeHot>(ns, 0, pend_ci));
            else if (k == kx_) mem.store_hot(s, make_hot<NodeHot>(ns, pend_xcb, pend_xi));
            else mem.store_backup(s, ns, mean_of(ns), rsqrt_approx((float)(uint32_t)ns));
        }
    };
    int fl = 1;                             // next pending entry to store
    auto flush_upto = [&](int k) {
        if constexpr (DEFER) {
            const int pn = (int)(pend & 0xFFu);
            const int hi = k < pn ? k : pn;
            for (; fl <= hi; ++fl) flush(fl);
        }
    };

    for (uint32_t it = 0; it < iters; ++it) {
        DK_STAMP(t0);
        fl = 1;
        // ---------------- selection
        uint32_t slot = 0;
        NodeHot x;
        x.stats = (uint64_t)it; x.child_base = root_cb; x.info = root_info;
        uint32_t x_visits = it;   // root visits == completed iterations
        int depth = 0;
        uint32_t chain_head = 0xFFFFFFFFu;   // head whose skip pointer led to x
        uint32_t chain_info = 0;             // its info (8-B records rewrite both fields)
        uint32_t chain_visits = 0;           // visits of the last chain head passed
        constexpr uint32_t N_FROM_BLOCK = 0xFFFFFFFFu;   // x_visits of a resolved chain end
        bool x_end = false;                  // x is a chain end (no stats of its own)
        mem.path_set(0, 0u, x.stats);
        // One trip per BRANCHING level: a lane first hops through single-child nodes
        // (a chain head jumps to its chain end), then picks among its children.  A wave
        // whose lanes sit at forced and branching levels at the same time thus pays one
        // pick per trip, not one trip per tree level.
        [[maybe_unused]] int hops = 0;   // dependent chain loads of this simulation (profiling)
        for (;;) {
            DK_STAMP_DRAINED(tf0);
            while (ni_nchild(x.info) == 1 && !ni_open(x.info)) {
                chain_head = ni_head(x.info) ? slot : 0xFFFFFFFFu;
                chain_info = x.info;
                if (P8 && slot != 0 && ni_resolved(x.info)) {
                    // resolved chain head: its chain end's children directly (no load)
                    scanned += 1;
                    DK_PROF(mem, 5, 1);
                    chain_visits = x_visits;
                    x_visits = N_FROM_BLOCK;
                    x_end = true;
                    x.info = ni_make(ni_state(x.info) & 15u, ni_player(x.info), false, false, 0);
                    slot = 0xFFFFFFFFu;
                    break;
                }
                flush_upto(depth + 1);
                const NodeHot y = mem.load_hot(x.child_base);
                scanned += 1;
                DK_PROF(mem, 5, 1);
#ifdef DK_PHASE_PROF
                hops += 1;
#endif
                if (slot == 0) {
                    // the root's only child: a root child, whose stats are the result
                    depth += 1;
                    if (depth >= MAX_DEPTH - 1) { status = SR_CAPACITY; break; }
                    mem.path_set(depth, x.child_base | (ni_player(x.info) << 30), y.stats);
                    x_visits = (uint32_t)y.stats;
                    x_end = false;
                } else {
                    // a chain head's skip to its chain end (derived visits, no path entry)
                    chain_visits = x_visits;
                    x_visits -= (uint32_t)y.stats;
                    x_end = true;
                }
                slot = x.child_base;
                x = y;
            }
            DK_STAMP_DRAINED(tf1);
            DK_PROF(mem, 19, tf1 - tf0);   // forced-chain hops
            if (status != SR_OK || ni_nchild(x.info) == 0 || ni_open(x.info)) break;
            const uint32_t n = ni_nchild(x.info);
            DK_PROF_TRIP(21);   // branching-level trips of the wave (slots 21-27)
            uint32_t pick;
            NodeHot y, end;
            bool end_ok = false;
            if (n <= (uint32_t)SCAN_REG) {
                if constexpr (P8) {
                    // blocks start at even slots: one 16-B load per pair of children
                    flush_upto(depth + 1);
                    DK_STAMP_DRAINED(tl0);
                    const double lnN = x_visits == N_FROM_BLOCK ? 0.0 : mem.ln(x_visits);
                    Block8 blk;
#pragma unroll
                    for (int j = 0; j < SCAN_REG / 2; ++j) {
                        if ((uint32_t)(2 * j) < n) {
                            const U4 q = mem.load_pair((x.child_base >> 1) + (uint32_t)j);
                            blk.w0[2 * j] = q.x; blk.w1[2 * j] = q.y; blk.w0[2 * j + 1] = q.z; blk.w1[2 * j + 1] = q.w;
                        } else {
                            blk.w0[2 * j] = 0; blk.w1[2 * j] = 0; blk.w0[2 * j + 1] = 0; blk.w1[2 * j + 1] = 0;
                        }
                    }
                    DK_STAMP_DRAINED(tl1);
                    DK_PROF(mem, 8, tl1 - tl0);
                    double lnN_x = lnN;
                    if (x_visits == N_FROM_BLOCK) {
                        uint32_t N = 1;
#pragma unroll
                        for (int j = 0; j < SCAN_REG; ++j) N += (uint32_t)j < n ? p8_visits(blk.w0[j]) : 0u;
                        x_visits = N;
                        lnN_x = mem.ln(N);
                    }
                    pick = pick_child_x<Raw8>(blk, n, lnN_x, c, mem, &y.stats, &y.child_base, &y.info, &end, &end_ok, x.child_base);
#if defined(DK_PICK_DOUBLE) && defined(__HIP_DEVICE_COMPILE__)
                    // measurement builds: the pick computed a second time (result discarded) in the trips
                    // with at most DK_PICK_DOUBLE active lanes: the time it adds is those picks' cost
                    if (popc64(__builtin_amdgcn_ballot_w64(true)) <= DK_PICK_DOUBLE) {
                        uint64_t s2; uint32_t c2, i2; NodeHot e2; bool o2 = false;
                        const uint32_t p2 = pick_child_x<Raw8>(blk, n, lnN_x * 1.0000000001, c, mem, &s2, &c2, &i2, &e2, &o2, x.child_base);
                        asm volatile("" :: "v"(p2), "v"((uint32_t)s2), "v"(c2), "v"(i2), "v"((uint32_t)o2));   // keep it
                    }
#endif
                    DK_STAMP_DRAINED(tl2);
                    DK_PROF(mem, 9, tl2 - tl1);
                } else if constexpr (Mem::Rec::PAIR) {
                    // lane pairs: this lane loads and scans its half of the block
                    flush_upto(depth + 1);
                    DK_STAMP_DRAINED(tl0);
                    const double lnN = mem.ln(x_visits);
                    const uint32_t j0 = mem.half ? (uint32_t)SCAN_HALF : 0u;
                    BlockH blk;
#pragma unroll
                    for (int k = 0; k < SCAN_HALF; ++k) {
                        if (j0 + (uint32_t)k < n) {
                            const NodeHot h = mem.load_hot(x.child_base + j0 + (uint32_t)k);
                            blk.st[k] = h.stats; blk.cb[k] = h.child_base; blk.inf[k] = h.info;
                        } else {
                            blk.st[k] = 0; blk.cb[k] = 0; blk.inf[k] = 0;
                        }
                    }
                    DK_STAMP_DRAINED(tl1);
                    DK_PROF(mem, 8, tl1 - tl0);
                    pick = pick_child_pair<Mem::Rec::LONG>(blk, n, j0, lnN, c, mem, &y.stats, &y.child_base, &y.info, &end, &end_ok, x.child_base);
                    DK_STAMP_DRAINED(tl2);
                    DK_PROF(mem, 9, tl2 - tl1);
                } else {
                    flush_upto(depth + 1);
                    DK_STAMP_DRAINED(tl0);
                    const double lnN = mem.ln(x_visits);
                    Block blk;
#pragma unroll
                    for (int j = 0; j < SCAN_REG; ++j) {
                        if ((uint32_t)j < n) {
                            const NodeHot h = mem.load_hot(x.child_base + (uint32_t)j);
                            blk.st[j] = h.stats; blk.cb[j] = h.child_base; blk.inf[j] = h.info; blk.q[j] = hot_q(h); blk.isv[j] = hot_isv(h);
                        } else {
                            blk.st[j] = 0; blk.cb[j] = 0; blk.inf[j] = 0; blk.q[j] = 0.0; blk.isv[j] = 0.0f;
                        }
                    }
                    DK_STAMP_DRAINED(tl1);
                    DK_PROF(mem, 8, tl1 - tl0);
                    if constexpr (NodeHot::CACHED_MEAN)
                        pick = pick_child_reg(blk, n, lnN, c, mem, &y.stats, &y.child_base, &y.info, &end, &end_ok);
                    else
                        pick = pick_child_x<typename std::conditional<Mem::Rec::LONG, Raw16L, Raw16>::type>(
                            blk, n, lnN, c, mem, &y.stats, &y.child_base, &y.info, &end, &end_ok, x.child_base);
                    DK_STAMP_DRAINED(tl2);
                    DK_PROF(mem, 9, tl2 - tl1);
                }
            } else {
                // generic block (never produced by the doko engines, whose nodes offer <= 12 actions)
                flush_upto(depth + 1);
                const double lnN = mem.ln(x_visits);
                double min_q = INFINITY, max_q = -INFINITY;
                for (uint32_t j = 0; j < n; ++j) {
                    const double q = mean_of(mem.load_hot(x.child_base + j).stats);
                    min_q = q < min_q ? q : min_q;
                    max_q = q > max_q ? q : max_q;
                }
                const bool flat = fabs(max_q - min_q) < DK_F64_EPSILON;
                double best = -INFINITY;
                pick = 0;
                y = mem.load_hot(x.child_base);
                for (uint32_t j = 0; j < n; ++j) {
                    const NodeHot r = mem.load_hot(x.child_base + j);
                    const double u = uct_exact(r.stats, mean_of(r.stats), flat, min_q, max_q, lnN, c);
                    if (u > best) { best = u; pick = j; y = r; }
                }
            }
            chain_head = 0xFFFFFFFFu;
            scanned += n;
            DK_PROF(mem, 6, 1);
            const uint32_t child = x.child_base + pick;
            depth += 1;
            if (depth >= MAX_DEPTH - 1) { status = SR_CAPACITY; break; }
            mem.path_set(depth, child | (ni_player(x.info) << 30), y.stats);
            slot = child;
            x_visits = (uint32_t)y.stats;
            x = y;
            x_end = false;
            if (P8 && ni_nchild(x.info) == 1 && !ni_open(x.info) && ni_resolved(x.info)) {
                // the picked child is a resolved chain head: on to its chain end's children
                chain_head = slot;
                chain_info = x.info;
                scanned += 1;
                DK_PROF(mem, 5, 1);
                chain_visits = x_visits;
                x_visits = N_FROM_BLOCK;
                x_end = true;
                x.info = ni_make(ni_state(x.info) & 15u, ni_player(x.info), false, false, 0);
                slot = 0xFFFFFFFFu;
            } else if (end_ok) {
                // the picked child is a forced chain head: its prefetched chain end
                chain_head = ni_head(x.info) ? slot : 0xFFFFFFFFu;
                chain_info = x.info;
                scanned += 1;
                DK_PROF(mem, 5, 1);
                chain_visits = x_visits;
                x_visits -= (uint32_t)end.stats;
                x_end = true;
                slot = x.child_base;
                x = end;
            }
        }
        if (status != SR_OK) break;
        flush_upto(1 << 30);
        DK_STAMP(t1);
        DK_PROF(mem, 0, t1 - t0);
        DK_PROF(mem, 4, (uint64_t)depth);
        DK_PROF_WAVEMAX(7, depth);
        DK_PROF_WAVEMAX(20, hops);
        // ---------------- expansion
        // path entries whose whole record the backup writes: the new leaf (kc = depth) and the
        // expanded node (kx); 8-B records carry their structure words pre-encoded
        int kx = -1, kc = -1;
        uint32_t x_cb = 0, x_info = 0, c_info = 0;
        Work w;
        if (ni_open(x.info)) {
            // A node's action set is computed at its first expansion, from its state (a
            // node is created with its open flag only: allowed != 0 <=> not terminal), and
            // kept in its cold record from then on; the root's comes from dk_create's
            // first-expansion mask.  Both loads in flight together.
            uint32_t nch = ni_nchild(x.info);
            const bool first = nch == 0 && slot != 0;
            NodeCold cd;
            if (!first) cd = mem.load_cold(slot);
            const auto packed = mem.load_state(ni_state(x.info));
            DK_STAMP_DRAINED(tx0);
            w = E::unpack_node(packed);
            DK_STAMP_DRAINED(tx1);
            if (first) cd.unexpanded = E::allowed(w, false);
            DK_STAMP_DRAINED(tx2);
            DK_PROF(mem, 14, tx0 - t1);   // cold record + state loads
            DK_PROF(mem, 15, tx1 - tx0);  // unpack
            DK_PROF(mem, 16, tx2 - tx1);  // first-expansion action set
            DK_PROF(mem, 17, first ? 1 : 0);
            const uint64_t bit = random_single(cd.unexpanded, rng);
            const int a = ctz64(bit);
            const uint32_t block = nch + (uint32_t)popc64(cd.unexpanded);
            if (nch == 0) {
                // (8-B records: blocks start at even slots, next_slot stays even; mem.balign may align
                // them further or keep them within one 128-B line, block_base)
                const uint32_t base = block_base(next_slot, P8 ? (block + 1u) & ~1u : block, mem.balign);
                if (base + block > mem.cap_slots || next_state >= mem.cap_states || next_state >= NI_MAX_STATES) {
                    status = SR_CAPACITY;
                    break;
                }
                x.child_base = base;
                next_slot = base + (P8 ? (block + 1u) & ~1u : block);
            }
            cd.unexpanded &= ~bit;
            const uint32_t child = x.child_base + nch;
            nch += 1;
            // a chain end that is now fully expanded with >= 2 children: resolve its head
            if (P8 && x_end && chain_head != 0xFFFFFFFFu && cd.unexpanded == 0 && nch >= 2)
                mem.store_node_tail(chain_head, x.child_base, ni_make(1, ni_player(x.info), false, true, P8_RESOLVED | nch));
            const uint32_t new_info = ni_make(nch, ni_player(x.info), cd.unexpanded != 0, ni_head(x.info), ni_state(x.info));
            if (slot == 0) { root_cb = x.child_base; root_info = new_info; }
            if (slot != 0 && !x_end) {
                // x is on the path: its new structure is stored with its backup (one store)
                kx = depth;
                if constexpr (P8) x_info = p8_w1(x.child_base, new_info);
                else { x_cb = x.child_base; x_info = new_info; }
            } else if (!P8 || slot != 0) {
                mem.store_node_tail(slot, x.child_base, new_info);
            }
            // (a node left without unexpanded actions is never expanded again: no store)
            if (cd.unexpanded != 0) mem.store_unexpanded(slot, cd.unexpanded);
            // a forced chain grew: its head now points at the new end
            if (block == 1 && chain_head != 0xFFFFFFFFu) mem.store_child_base(chain_head, child, chain_info);
            DK_STAMP_DRAINED(te0);
#if defined(DK_EXP_DOUBLE) && defined(__HIP_DEVICE_COMPILE__)
            {   // measurement builds: the expansion's transition and action set once more on a copy
                Work w2 = E::unpack_node(packed);
                const uint64_t al2 = E::allowed(w2, false);
                E::step(w2, a);
                const auto n2 = E::pack_node(w2);
                uint32_t k2 = (uint32_t)al2 ^ (uint32_t)(al2 >> 32), wd[sizeof(n2) / 4];
                __builtin_memcpy(wd, &n2, sizeof(wd));
                for (uint32_t i = 0; i < sizeof(n2) / 4; ++i) k2 ^= wd[i];
                asm volatile("" :: "v"(k2));
            }
#endif
            E::step(w, a);
            DK_STAMP_DRAINED(te1);
            DK_PROF(mem, 12, te1 - te0);
            const bool child_open = !E::terminal(w);   // == (E::allowed(w, false) != 0)
            // a single child of a non-root node is a chain end: its record holds the chain
            // head's visits before this simulation's backup (x itself, or the head x is the end of)
            const bool child_end = block == 1 && slot != 0;
            const uint64_t child_stats = child_end ? (uint64_t)(x_end ? chain_visits : x_visits) : 0ULL;
            const uint32_t child_info = ni_make(0, (uint32_t)E::current_player(w), child_open, slot == 0 || block >= 2, next_state);
            // the new leaf's record is written by the backup, with its first statistics
            if (child_end) mem.store_hot(child, make_hot<NodeHot>(child_stats, 0, child_info));
            else c_info = P8 ? p8_w1(0, child_info) : child_info;
            if (slot == 0) {
                // a root child: its action is part of the result
                NodeCold cc;
                cc.unexpanded = 0; cc.parent = slot; cc.action = (uint32_t)a;
                mem.store_cold(child, cc);
            }
            DK_STAMP_DRAINED(te2);
            DK_PROF(mem, 13, te2 - te1);
            mem.store_state(next_state, E::pack_node(w));
            DK_STAMP_DRAINED(te3);
            DK_PROF(mem, 18, te3 - te2);  // pack + state store
            next_state += 1;
            if (!child_end) {
                depth += 1;
                mem.path_set(depth, child | (ni_player(x.info) << 30), 0ULL);
                kc = depth;
            }
            slot = child;
        } else {
            w = E::unpack_node(mem.load_state(ni_state(x.info)));
        }
        DK_STAMP(t2);
        DK_PROF(mem, 1, t2 - t1);
        // ---------------- rollout
        int r[4];
#if defined(DK_ROLL_DOUBLE) && defined(__HIP_DEVICE_COMPILE__)
        {   // measurement builds: the rollout played a second time on copies (result discarded, kept
            // alive): the VALU instructions / time it adds are the rollout's (profiles/r06/valu_by_phase.json)
            Rng r2 = rng; int q[4];
            const int p2 = E::rollout(w, r2, q);
            asm volatile("" :: "v"(p2), "v"(q[0]), "v"(q[1]), "v"(q[2]), "v"(q[3]), "v"((uint32_t)r2.s0));
        }
#endif
        [[maybe_unused]] const int rplies = E::rollout(w, rng, r);
        DK_PROF(mem, 10, (uint64_t)rplies);
        DK_PROF_WAVEMAX(11, rplies);
        DK_STAMP(t3);
        DK_PROF(mem, 2, t3 - t2);
        // ---------------- backup (leaf -> root): stores of the stats read on the way down
        // (two loops: the global overflow part and the LDS part keep distinct address spaces)
        // The expanded node and the new leaf get their whole record in this one store
        // (structure from the expansion, statistics from the backup).
        auto put = [&](int k, uint32_t e, uint64_t ns) {
            const uint32_t s = e & 0x3FFFFFFFu;
            if constexpr (P8) {
                if (k == kc || k == kx) mem.store_rec8(s, p8_w0(ns), k == kc ? c_info : x_info);
                else mem.store_backup(s, ns, 0.0, 0.0f);
            } else {
                if (k == kc) mem.store_hot(s, make_hot<NodeHot>(ns, 0, c_info));
                else if (k == kx) mem.store_hot(s, make_hot<NodeHot>(ns, x_cb, x_info));
                else mem.store_backup(s, ns, mean_of(ns), rsqrt_approx((float)(uint32_t)ns));
            }
        };
        const int k_lds = depth < mem.lds_entries() - 1 ? depth : mem.lds_entries() - 1;
        for (int k = depth; k > k_lds; --k) {
            uint64_t st;
            const uint32_t e = mem.path_get_ovf(k, &st);
            put(k, e, st + (((uint64_t)(uint32_t)sel4i(r, (int)(e >> 30)) << 32) | 1ULL));
        }
        if constexpr (DEFER) {
            for (int k = k_lds; k >= 1; --k) {
                uint64_t st;
                const uint32_t e = mem.path_get_lds(k, &st);
                mem.path_set(k, e, st + (((uint64_t)(uint32_t)sel4i(r, (int)(e >> 30)) << 32) | 1ULL));
            }
            const uint32_t pkc = kc >= 1 && kc <= k_lds ? (uint32_t)kc : 0xFFu;
            const uint32_t pkx = kx >= 1 && kx <= k_lds ? (uint32_t)kx : 0xFFu;
            pend = (uint32_t)(k_lds > 0 ? k_lds : 0) | pkc << 8 | pkx << 16;
            pend_ci = c_info; pend_xi = x_info; pend_xcb = x_cb;
        } else {
            for (int k = k_lds; k >= 1; --k) {
                uint64_t st;
                const uint32_t e = mem.path_get_lds(k, &st);
                put(k, e, st + (((uint64_t)(uint32_t)sel4i(r, (int)(e >> 30)) << 32) | 1ULL));
            }
        }
        // (the root's own record is read by nothing but the result: deferred, once at the end)
        if constexpr (!P8 && !DEFER) mem.store_stats(0, (uint64_t)(it + 1));
        if (it + 1 == iters) (void)rng.next_u64();  // random_bool((1f32/1000f32) as f64)
        DK_STAMP_DRAINED(t4);   // (drained: the backup owns its store completion)
        DK_PROF(mem, 3, t4 - t3);
    }
    if (status == SR_OK) {   // the last simulation's statistics
        fl = 1;
        flush_upto(1 << 30);
        if constexpr (!P8 && DEFER) mem.store_stats(0, (uint64_t)iters);
    }
    if (ctr_scanned) *ctr_scanned = scanned;
    if (used) { used[0] = next_slot; used[1] = next_state; }   // pool high-water of this root
    DK_PROF_FLUSH(mem);

    // ---------------- result: root children in expansion order
    for (int a = 0; a < 39; ++a) { visits39[a] = 0; values39[a] = 0.0; }
    int best = -1; uint32_t bv = 0;
    for (uint32_t j = 0; j < ni_nchild(root_info); ++j) {
        const uint64_t st = mem.load_hot(root_cb + j).stats;
        const uint32_t act = mem.load_cold(root_cb + j).action;
        const uint32_t v = (uint32_t)st;
        visits39[act] = v;
        values39[act] = (double)(int32_t)(st >> 32) / (double)v;
        if (best < 0 || v >= bv) { best = (int)act; bv = v; }   // max_by_key: last maximum
    }
    *best_out = best < 0 ? (uint8_t)0xFF : (uint8_t)best;
    return status;
}

}  // namespace dk
