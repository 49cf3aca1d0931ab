// ORACLE — test infrastructure only. Never linked into the product library.
//
// CPU restatement of the rs-doko rule-based determinization sampler
// (rs-doko-assignment/src/assignment.rs:12-581), kept in the reference's own
// Vec-of-cards form so the intermediate lists can be compared with the
// reference's unit tests (assignment.rs:593-1190).
#pragma once
#include <cstdint>
#include <vector>
#include "doko.hpp"
#include "rand09.hpp"

namespace oracle {
namespace dko {

using CardVec = std::vector<int>;   // DoCard as its bit index 0..23

// hand/hand.rs:135-181 — ascending DoCard order, both copies adjacent.
CardVec hand_to_vec(uint64_t hand);
// hand/hand.rs:183-195
uint64_t hand_from_vec(const CardVec& cards);

// assignment.rs:13-39
uint64_t calc_remaining_cards(const Trick tricks[12], uint64_t observing_hand);
// assignment.rs:79-287 (marriage = -1 for None)
void player_allowed_to_have(int marriage, const Trick tricks[12], uint64_t observing_hand, int observing_player,
                            CardVec out[4]);
// assignment.rs:507-580. Returns false where the reference would panic
// (a card no player may hold: the `unwrap` at :430-433).
bool sample_assignment(int marriage, const Trick tricks[12], uint64_t observing_hand, const int lengths[4],
                       int observing_player, SmallRng& rng, CardVec out[4]);
// assignment.rs:472-505 with observation_for_current_player() (rs-doko/src/state/state.rs:336-410):
// observer = current player (BOTTOM when finished), marriage = the wedding
// player of a (un)solved wedding; only the hands change (clone_with_different_hands).
bool sample_assignment_full(const State& s, SmallRng& rng, State& out);

}  // namespace dko
}  // namespace oracle
