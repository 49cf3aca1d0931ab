// ORACLE — test infrastructure only. Never linked into the product library.
//
// Faithful CPU restatement of the simplified rs-doko rule engine
// (/root/reference/rs-doko/src): normal game + wedding + silent solo, 26 actions,
// no announcements. Plus the env adapter McDokoEnvState, whose
// allowed_actions/by_action are `todo!()` in the reference
// (rs-doko-mcts/src/env/envs/env_state_doko.rs:138-144): defined here through the
// identity DoAction bits 0-25 == FdoAction bits 0-25.
#pragma once
#include <cstdint>
#include "rand09.hpp"

namespace oracle {
namespace dko {

enum Phase : int { Reservation = 0, PlayCard = 1, Finished = 2 };   // basic/phase.rs
enum Res : int { Wedding = 0, Healthy = 1 };                        // reservation/reservation.rs
static constexpr int A_Healthy = 24, A_Wedding = 25;

struct Trick { int cards[4] = {-1, -1, -1, -1}; int start = 0; bool present = false; };

enum TeamKind : int { InReservations = 0, WeddingUnsolved, WeddingSolved, NoWedding };
struct TeamState { int kind = InReservations; int wedding_player = 0; int solved = 0; uint8_t re = 0; };

struct Stats { int winning_team; uint8_t re_players; bool is_solo; uint32_t re_eyes, kontra_eyes;
               int32_t re_points, kontra_points, player_points[4]; };

struct State {
    int res[4] = {-1, -1, -1, -1};
    int res_start = 0;
    Trick tricks[12];
    uint64_t hands[4] = {0, 0, 0, 0};
    int current_player = 0;   // -1 None
    int phase = Reservation;
    int trick_index = 0;
    bool has_rr = false; int rr_wedding = -1;   // DoReservationResult: -1 NoReservation, else wedding player
    uint32_t eyes[4] = {0, 0, 0, 0};
    uint32_t ntricks[4] = {0, 0, 0, 0};
    TeamState team;
    bool has_stats = false;
    Stats stats;
};

uint64_t hand_add(uint64_t h, int c);
uint64_t hand_remove(uint64_t h, int c);   // removes the LOW copy first (hand/hand.rs:38-46)
enum Color { Trump = 0, Heart, Spade, Club };
int card_color(int c);                      // card/card_to_color.rs (normal game)
uint64_t calculate_allowed_actions(int phase, int trick_color, uint64_t hand);
int winning_player_in_trick(const Trick& t);
State new_game(SmallRng& rng);
State from_hands(const uint64_t hands[4], int start);
void play_action(State& s, int action_idx);
bool random_action_for_current_player(State& s, SmallRng& rng);
uint64_t observation_allowed(const State& s);
Stats calculate_stats(uint8_t re, const uint32_t eyes[4], const uint32_t ntricks[4]);
TeamState resolve_team(const State& s);   // teams/team_logic.rs:69-143

struct Env {
    State doko;
    int last_action = -1;
    int current_player() const { return doko.current_player < 0 ? 0 : doko.current_player; }
    bool is_terminal() const { return doko.phase == Finished; }
    uint64_t allowed_actions(bool /*first_expansion*/) const { return observation_allowed(doko); }
    Env by_action(int a) const { Env e; e.doko = doko; play_action(e.doko, a); e.last_action = a; return e; }
    bool rewards_or_none(double out[4]) const;
    void random_rollout(SmallRng& rng, double out[4]) const;
};

}  // namespace dko
}  // namespace oracle
