// ORACLE — test infrastructure only. Never linked into the product library.
#pragma once
#include "full_doko.hpp"

namespace oracle {
namespace fdo {

void gather_impossible_colors(const State& s, uint32_t out[4]);
void played_club_queens(const State& s, int out[4]);
void card_matching(const State& s, SmallRng& rng, Hand out_hands[4], int out_res[4]);
State card_matching_full(const State& s, SmallRng& rng);
bool sample_consistent(const State& orig, const State& sample);

}  // namespace fdo
}  // namespace oracle
