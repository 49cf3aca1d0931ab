// ORACLE — test infrastructure only. Never linked into the product library.
//
// Policy fusion of rs-doko-py-bridge/src/compare_impi/policy_fusion.rs:
//   PolicyFusionMaxN::fuse            :23-74
//   PolicyFusionAverageStrategy::fuse :77-123
#pragma once
#include <algorithm>
#include <cstdint>
#include <vector>

namespace oracle {

static constexpr int FUSE_ACTIONS = 39;

// visits: S rows of 39 counts; allowed: FdoAllowedActions bits.
inline int fuse_maxn(const uint32_t* visits, int S, uint64_t allowed, uint32_t* ranks_out) {
    uint32_t cum[FUSE_ACTIONS];
    for (int a = 0; a < FUSE_ACTIONS; ++a) cum[a] = (allowed >> a & 1) ? 0u : 0xFFFFFFFFu;
    for (int s = 0; s < S; ++s) {
        std::vector<std::pair<int, uint32_t>> pairs;
        for (int a = 0; a < FUSE_ACTIONS; ++a) if (allowed >> a & 1) pairs.push_back({a, visits[s * FUSE_ACTIONS + a]});
        std::stable_sort(pairs.begin(), pairs.end(), [](const std::pair<int, uint32_t>& x, const std::pair<int, uint32_t>& y) {
            return x.second > y.second;  // sort_by_key(Reverse(visits)), stable
        });
        for (size_t r = 0; r < pairs.size(); ++r) cum[pairs[r].first] += (uint32_t)r + 1u;
    }
    int best = 0;
    for (int a = 1; a < FUSE_ACTIONS; ++a) if (cum[a] < cum[best]) best = a;  // min_by_key: first minimum
    if (ranks_out) for (int a = 0; a < FUSE_ACTIONS; ++a) ranks_out[a] = cum[a];
    return best;
}

inline int fuse_avg(const uint32_t* visits, int S, float* probs_out) {
    float sum[FUSE_ACTIONS];
    for (int a = 0; a < FUSE_ACTIONS; ++a) sum[a] = 0.0f;
    for (int s = 0; s < S; ++s) {
        uint64_t total = 0;
        for (int a = 0; a < FUSE_ACTIONS; ++a) total += visits[s * FUSE_ACTIONS + a];
        for (int a = 0; a < FUSE_ACTIONS; ++a) sum[a] += (float)visits[s * FUSE_ACTIONS + a] / (float)total;
    }
    int best = 0;  // max_by: the LAST maximum wins; incomparable (NaN) counts as Equal
    for (int a = 1; a < FUSE_ACTIONS; ++a) if (!(sum[best] > sum[a])) best = a;
    if (probs_out) for (int a = 0; a < FUSE_ACTIONS; ++a) probs_out[a] = sum[a];
    return best;
}

}  // namespace oracle
