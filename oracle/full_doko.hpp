// ORACLE — test infrastructure only. Never linked into the product library.
//
// Faithful CPU restatement of the rs-full-doko rule engine
// (/root/reference/rs-full-doko/src).  Data structures mirror the Rust ones
// (heapless vectors of tricks, announcement occurrence lists, Option<> fields
// as has_/-1 sentinels) so each function can be read side by side with the
// reference file:line cited above it in full_doko.cpp.
#pragma once
#include <cstdint>
#include <cstring>
#include "rand09.hpp"

namespace oracle {
namespace fdo {

// ---- enums (discriminants as in the reference) -----------------------------
// FdoCard: card kind k in 0..23, bit = 1 << k   (card/cards.rs:8-36)
enum Card : int {
    DiamondNine = 0, DiamondTen, DiamondJack, DiamondQueen, DiamondKing, DiamondAce,
    HeartNine, HeartTen, HeartJack, HeartQueen, HeartKing, HeartAce,
    ClubNine, ClubTen, ClubJack, ClubQueen, ClubKing, ClubAce,
    SpadeNine, SpadeTen, SpadeJack, SpadeQueen, SpadeKing, SpadeAce,
};
// FdoAction: bit index 0..38 (action/action.rs:9-54). Cards are 0..23.
enum ActionIdx : int {
    A_ReservationHealthy = 24, A_ReservationWedding, A_ReservationDiamondsSolo, A_ReservationHeartsSolo,
    A_ReservationSpadesSolo, A_ReservationClubsSolo, A_ReservationTrumplessSolo, A_ReservationQueensSolo,
    A_ReservationJacksSolo,
    A_AnnouncementReContra = 33, A_AnnouncementNo90, A_AnnouncementNo60, A_AnnouncementNo30,
    A_AnnouncementBlack, A_NoAnnouncement = 38,
};
static constexpr int ACTION_COUNT = 39;
inline uint64_t abit(int idx) { return 1ULL << idx; }

// FdoReservation (reservation/reservation.rs:11-23) — EnumSet order.
enum Reservation : int { Healthy = 0, Wedding, DiamondsSolo, HeartsSolo, SpadesSolo, ClubsSolo, QueensSolo, JacksSolo, TrumplessSolo };
// FdoVisibleReservation (reservation.rs:62-77)
enum VisibleReservation : int { V_Wedding = 0, V_Healthy, V_NotRevealed, V_DiamondsSolo, V_HeartsSolo, V_SpadesSolo,
                                V_ClubsSolo, V_QueensSolo, V_JacksSolo, V_TrumplessSolo, V_NoneYet };
// FdoGameType (game_type/game_type.rs:6-20)
enum GameType : int { Normal = 0, GWedding, GDiamondsSolo, GHeartsSolo, GSpadesSolo, GClubsSolo, GTrumplessSolo, GQueensSolo, GJacksSolo };
// FdoColor (basic/color.rs)
enum Color : int { Trump = 0, Diamond, Heart, Spade, Club };
// FdoPhase (basic/phase.rs)
enum Phase : int { Reservation = 0, Announcement = 1, PlayCard = 2, Finished = 3 };
// FdoAnnouncement bits (announcement/announcement.rs:11-21)
enum Ann : uint32_t { ReContra = 1, No90 = 2, No60 = 4, No30 = 8, Black = 16, CounterReContra = 32, NoAnnouncement = 64 };

// ---- hand (hand/hand.rs:20-550) --------------------------------------------
static constexpr int SECOND = 24;
struct Hand {
    uint64_t bits = 0;
    bool contains(int c) const { return (bits >> c & 1) || (bits >> (c + SECOND) & 1); }
    bool contains_both(int c) const { return (bits >> c & 1) && (bits >> (c + SECOND) & 1); }
    void add(int c);
    void remove(int c);          // removes the HIGH copy first (hand.rs:235-247)
    void remove_ignore(int c) { if (contains(c)) remove(c); }
    void remove_both(int c);
    int len() const { return __builtin_popcountll(bits); }
    void remove_color(int color, int game_type);
    Hand plus_hand(const Hand& other) const;
    // FdoHandIter (hand_iter.rs:11-39): ascending bit order, each copy separately.
    int iter(int out[48]) const {
        int n = 0; uint64_t b = bits;
        while (b) { int pos = __builtin_ctzll(b); b &= b - 1; out[n++] = pos < SECOND ? pos : pos - SECOND; }
        return n;
    }
};

struct Trick {
    int cards[4] = {-1, -1, -1, -1};
    int len = 0;
    int start = 0;
    int winning_player = -1;
    int winning_card = -1;
    int player_at(int i) const { return (start + i) % 4; }
    bool is_completed() const { return len == 4; }
};

struct AnnOccurrence { int card_index; int player; uint32_t announcement; };

struct Announcements {
    AnnOccurrence list[12];
    int n = 0;
    int re_lowest = -1;        // Option<FdoAnnouncement> as bit or -1
    int contra_lowest = -1;
    int turns_without = 0;
    int starting_player = 0;
    uint32_t allowed = 0;       // current_player_allowed_announcements
};

enum TeamKind : int { InReservations = 0, WeddingUnsolved, WeddingSolved, NoWedding };
struct TeamState {
    int kind = InReservations;
    int wedding_player = 0;
    int solved_trick_index = 0;
    uint8_t re_players = 0;
    bool is_final() const { return kind == WeddingSolved || kind == NoWedding; }
    bool has_re() const { return kind == WeddingSolved || kind == NoWedding; }
};

enum ResKind : int { NoReservation = 0, Solo, RWedding };
struct ReservationResult { int kind = NoReservation; int player = 0; int reservation = 0; };

struct BasicWinningDetails { int v[23]; };
struct AdditionalDetails {
    bool against_club_queens; int doko_re, doko_kontra, fuchs_re, fuchs_kontra; bool karlchen_re, karlchen_kontra;
};
struct EndOfGameStats {
    uint8_t re_players; bool is_solo;
    uint32_t player_eyes[4]; uint32_t re_eyes, kontra_eyes;
    int32_t re_points, kontra_points, player_points[4];
    bool has_winning_details; bool has_draw_details; bool has_additional;
    AdditionalDetails additional;
    int win_details[23];     // FdoBasicWinningPointsDetails fields in declaration order
    int draw_details[14];    // FdoBasicDrawPointsDetails fields in declaration order
};

struct State {
    // reservations_round: PlayerOrientedVec<FdoReservation>
    int res[4] = {0, 0, 0, 0};
    int res_len = 0;
    int res_start = 0;
    Trick tricks[12];
    int n_tricks = 0;
    Hand hands[4];
    Announcements announcements;
    int card_index = 0;
    int current_player = 0;        // -1 == None
    int phase = Reservation;
    bool has_reservation_result = false;
    ReservationResult reservation_result;
    int game_type = -1;             // -1 == None
    uint32_t player_eyes[4] = {0, 0, 0, 0};
    uint32_t player_num_tricks[4] = {0, 0, 0, 0};
    TeamState team_state;
    bool has_stats = false;
    EndOfGameStats stats;
};

// rules
int card_to_color(int card, int game_type);
uint32_t card_eyes(int card);
void color_masks(int game_type, uint64_t out[5]);
bool is_greater_in_trick(int cur, int prev, int trick_color, int game_type);
void trick_play_card(Trick& t, int card, int game_type);
int trick_color(const Trick& t, int game_type);  // -1 == None
uint64_t select_by_rank(uint64_t v, uint64_t r);
uint64_t random_single(uint64_t mask, SmallRng& rng);
uint64_t calculate_allowed_actions(int phase, int trick_color, Hand hand, int game_type, uint32_t allowed_announcements);
uint32_t all_higher_than(int lowest);
uint32_t calc_allowed_announcements(int player, int n_cards, const TeamState& ts, int re_lowest, int contra_lowest);
TeamState team_resolve(const ReservationResult& rr, const Trick* tricks, int n_tricks, const Hand* hands);
ReservationResult winning_player_in_reservation_round(const State& s);
int reservation_to_game_type(const ReservationResult& rr);
EndOfGameStats calculate_stats(const uint32_t eyes[4], const uint32_t ntricks[4], uint8_t re_players,
                               int re_lowest, int contra_lowest, const Trick* tricks, int n_tricks);

// stats building blocks (stats/win_conditions, stats/basic_points, stats/additional_points)
bool re_won(uint32_t re_eyes, uint32_t re_prev, uint32_t ko_prev, bool re_all, bool ko_all);
bool kontra_won(uint32_t ko_eyes, uint32_t re_prev, uint32_t ko_prev, bool re_all, bool ko_all);
void basic_winning_points(uint32_t loser_eyes, bool winner_all, uint32_t re_prev, uint32_t ko_prev,
                          uint32_t re_eyes, uint32_t ko_eyes, int* win, int* lose, int* details);
void basic_draw_points(uint32_t re_prev, uint32_t ko_prev, uint32_t re_eyes, uint32_t ko_eyes, int* re, int* ko,
                       int* details);
AdditionalDetails additional_points(uint8_t re_players, int winning_team, const Trick* tricks, int n_tricks,
                                    int* re_add, int* ko_add);
// announcement rounds (announcement/announcement.rs:83-215); returns 0 NextPlayerIs / 1 RoundIsOver
int announcements_start_round(Announcements& a, int card_index, int start, const int hand_lens[4], const TeamState& ts,
                              int* next);
int announcements_play(Announcements& a, int player, uint32_t ann, int card_index, const int hand_lens[4],
                       const TeamState& ts, int* next);
int calc_cards_last_announcement_pub(uint32_t set, int wedding_solved, bool* some);
uint32_t internal_calc_allowed_pub(int n_cards, uint32_t prev, int wedding_solved, bool enemy_some, int enemy_cards);

State new_game_from_hand_and_start_player(const Hand hands[4], int start_player);
State new_game(SmallRng& rng);
void play_action(State& s, int action_idx);
int current_trick_color(const State& s);
bool random_action_for_current_player(State& s, SmallRng& rng);
bool random_action_for_current_player_no_announcement(State& s, SmallRng& rng);
uint64_t observation_allowed_actions(const State& s);
void visible_reservations(const State& s, int observing_player, int out[4]);

// rs-doko-mcts env adapter McFullDokoEnvState (env/envs/env_state_full_doko.rs)
struct Env {
    State doko;
    int last_action = -1;
    int current_player() const { return doko.phase == Finished ? 0 : doko.current_player; }
    bool is_terminal() const { return doko.phase == Finished; }
    uint64_t allowed_actions(bool first_expansion) const;
    Env by_action(int action_idx) const;
    bool rewards_or_none(double out[4]) const;
    void random_rollout(SmallRng& rng, double out[4]) const;
};

}  // namespace fdo
}  // namespace oracle
