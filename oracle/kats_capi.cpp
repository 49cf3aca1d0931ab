// ORACLE — test infrastructure only. Never linked into the product library.
//
// C entry points of the restatement's rule building blocks, one per function the
// reference's own unit tests call, so tests/test_rule_kats.py can check the restatement
// against every assertion tests/golden/make_rule_kats.py extracted from those tests:
//   card order / colour / colour masks / eyes  rs-full-doko/src/card/*.rs
//   tricks (colour, eyes, winner, next player) rs-full-doko/src/trick/*.rs
//   team resolution                            rs-full-doko/src/team/team_logic.rs:37-122
//   reservation round winner, game type        rs-full-doko/src/reservation/reservation_winning_logic.rs
//   allowed announcements                      rs-full-doko/src/announcement/calc_announcement.rs:21-229
//   announcement rounds                        rs-full-doko/src/announcement/announcement.rs:83-215
//   DKV scoring and its parts                  rs-full-doko/src/stats/**
//   rs-doko allowed actions, teams, scoring    rs-doko/src/{action,teams,stats}
// Tricks are passed as int32 [n][5] = {start player, card0..card3 (-1 = none)}.
#include <cstdint>
#include <cstring>

#include "doko.hpp"
#include "full_doko.hpp"

using namespace oracle;

namespace {

void fdo_tricks(const int32_t* t, int n, int game_type, fdo::Trick out[12]) {
    for (int i = 0; i < n && i < 12; ++i) {
        out[i] = fdo::Trick();
        out[i].start = t[5 * i];
        for (int k = 0; k < 4; ++k)
            if (t[5 * i + 1 + k] >= 0) fdo::trick_play_card(out[i], t[5 * i + 1 + k], game_type);
    }
}

fdo::TeamState team_of(int kind, int wedding_player, int solved, int re_mask) {
    fdo::TeamState ts;
    ts.kind = kind;
    ts.wedding_player = wedding_player;
    ts.solved_trick_index = solved;
    ts.re_players = (uint8_t)re_mask;
    return ts;
}

int opt_ann(int bit) { return bit == 0 ? -1 : bit; }   // 0 = None in the C interface

}  // namespace

extern "C" {

uint32_t or_kat_card_eyes(int card) { return fdo::card_eyes(card); }
void or_kat_color_masks(int game_type, uint64_t* out) { fdo::color_masks(game_type, out); }

// out: [0] trick colour (-1 None) [1] next player (-1 None) [2] completed [3] eyes (completed)
//      [4] winning player [5] winning card (-1 while open)
void or_kat_trick(const int32_t* trick, int game_type, int32_t* out) {
    fdo::Trick t;
    fdo_tricks(trick, 1, game_type, &t);
    out[0] = fdo::trick_color(t, game_type);
    out[1] = t.is_completed() ? -1 : t.player_at(t.len);
    out[2] = t.is_completed();
    uint32_t e = 0;
    for (int i = 0; i < t.len; ++i) e += fdo::card_eyes(t.cards[i]);
    out[3] = (int32_t)e;
    out[4] = t.winning_player;
    out[5] = t.winning_card;
}

// FdoTeamState::resolve(reservation_result, tricks, hands): out = kind, wedding_player, solved, re mask
void or_kat_team_resolve(int rr_kind, int rr_player, int rr_res, const int32_t* tricks, int n_tricks,
                         const uint64_t* hands, int32_t* out) {
    fdo::ReservationResult rr;
    rr.kind = rr_kind; rr.player = rr_player; rr.reservation = rr_res;
    fdo::Trick t[12];
    fdo_tricks(tricks, n_tricks, fdo::Normal, t);    // FdoTrick::existing plays them as a normal game (trick.rs:55-68)
    fdo::Hand h[4];
    for (int p = 0; p < 4; ++p) h[p].bits = hands[p];
    const fdo::TeamState ts = fdo::team_resolve(rr, t, n_tricks, h);
    out[0] = ts.kind; out[1] = ts.wedding_player; out[2] = ts.solved_trick_index; out[3] = ts.re_players;
}

// winning_player_in_reservation_round + to_game_type: out = kind, player, reservation, game type
void or_kat_reservation_winner(int start, const int32_t* res, int n, int32_t* out) {
    fdo::State s;
    s.res_start = start; s.res_len = n;
    for (int i = 0; i < n; ++i) s.res[i] = res[i];
    const fdo::ReservationResult rr = fdo::winning_player_in_reservation_round(s);
    out[0] = rr.kind; out[1] = rr.player; out[2] = rr.reservation; out[3] = fdo::reservation_to_game_type(rr);
}
int or_kat_game_type_of(int kind, int player, int reservation) {
    fdo::ReservationResult rr;
    rr.kind = kind; rr.player = player; rr.reservation = reservation;
    return fdo::reservation_to_game_type(rr);
}

uint32_t or_kat_all_higher_than(int lowest_bit) { return fdo::all_higher_than(opt_ann(lowest_bit)); }
uint32_t or_kat_calc_allowed(int player, int n_cards, int team_kind, int wedding_player, int solved, int re_mask,
                             int re_lowest_bit, int contra_lowest_bit) {
    return fdo::calc_allowed_announcements(player, n_cards, team_of(team_kind, wedding_player, solved, re_mask),
                                           opt_ann(re_lowest_bit), opt_ann(contra_lowest_bit));
}
// internal_calc_allowed_annoucements(n, prev set, wedding solved index (-1 None), enemy cards (-1 None))
uint32_t or_kat_internal_calc_allowed(int n_cards, uint32_t prev, int wedding_solved, int enemy_cards) {
    return fdo::internal_calc_allowed_pub(n_cards, prev, wedding_solved < 0 ? 0 : wedding_solved, enemy_cards >= 0,
                                          enemy_cards < 0 ? 0 : enemy_cards);
}
// calc_number_of_cards_announcement_possible_for_last_announcement(set, wedding solved (-1 None)) -> -1 None
int or_kat_cards_last_announcement(uint32_t set, int wedding_solved) {
    bool some = false;
    const int v = fdo::calc_cards_last_announcement_pub(set, wedding_solved < 0 ? 0 : wedding_solved, &some);
    return some ? v : -1;
}

// An announcement round: ops = (player, announcement bit) pairs; op 0 is start_round with
// player = the round's starting player.  After every op out[21*i ..] = result (0 NextPlayerIs,
// 1 RoundIsOver), its player, number of occurrences, starting player, turns without announcement,
// re lowest (0 None), contra lowest, allowed set, 0, then the occurrences
// (card_index << 8 | player << 4 | announcement bit index), -1 beyond the count
void or_kat_announcement_round(const int32_t* hand_lens, int team_kind, int wedding_player, int solved, int re_mask,
                               int card_index, const int32_t* ops, int n_ops, int32_t* out) {
    fdo::Announcements a;
    const fdo::TeamState ts = team_of(team_kind, wedding_player, solved, re_mask);
    int hl[4];
    for (int p = 0; p < 4; ++p) hl[p] = hand_lens[p];
    for (int i = 0; i < n_ops; ++i) {
        int next = -1, r;
        if (i == 0) r = fdo::announcements_start_round(a, card_index, ops[0], hl, ts, &next);
        else r = fdo::announcements_play(a, ops[2 * i], (uint32_t)ops[2 * i + 1], card_index, hl, ts, &next);
        int32_t* o = out + 21 * i;
        o[0] = r; o[1] = next; o[2] = a.n; o[3] = a.starting_player; o[4] = a.turns_without;
        o[5] = a.re_lowest < 0 ? 0 : a.re_lowest; o[6] = a.contra_lowest < 0 ? 0 : a.contra_lowest;
        o[7] = (int32_t)a.allowed; o[8] = 0;
        for (int k = 0; k < 12; ++k)
            o[9 + k] = k < a.n ? (a.list[k].card_index << 8 | a.list[k].player << 4 | __builtin_ctz(a.list[k].announcement)) : -1;
    }
}

// FdoEndOfGameStats::calculate (stats.rs:46-243).  out: [0] re mask [1] is_solo [2] re eyes [3] kontra eyes
// [4] re points [5] kontra points [6..9] player points [10] has winning details [11..33] its 23 fields
// [34] has draw details [35..48] its 14 fields [49] has additional details [50..56] its 7 fields
void or_kat_stats(const uint32_t* eyes, const uint32_t* ntricks, int re_mask, int re_lowest_bit, int contra_lowest_bit,
                  const int32_t* tricks, int n_tricks, int32_t* out) {
    fdo::Trick t[12];
    fdo_tricks(tricks, n_tricks, fdo::Normal, t);
    const fdo::EndOfGameStats s = fdo::calculate_stats(eyes, ntricks, (uint8_t)re_mask, opt_ann(re_lowest_bit),
                                                       opt_ann(contra_lowest_bit), t, n_tricks);
    memset(out, 0, 57 * sizeof(int32_t));
    out[0] = s.re_players; out[1] = s.is_solo; out[2] = (int32_t)s.re_eyes; out[3] = (int32_t)s.kontra_eyes;
    out[4] = s.re_points; out[5] = s.kontra_points;
    for (int p = 0; p < 4; ++p) out[6 + p] = s.player_points[p];
    out[10] = s.has_winning_details;
    if (s.has_winning_details) for (int i = 0; i < 23; ++i) out[11 + i] = s.win_details[i];
    out[34] = s.has_draw_details;
    if (s.has_draw_details) for (int i = 0; i < 14; ++i) out[35 + i] = s.draw_details[i];
    out[49] = s.has_additional;
    const fdo::AdditionalDetails& d = s.additional;
    out[50] = d.against_club_queens; out[51] = d.doko_re; out[52] = d.doko_kontra; out[53] = d.fuchs_re;
    out[54] = d.fuchs_kontra; out[55] = d.karlchen_re; out[56] = d.karlchen_kontra;
}

int or_kat_re_won(uint32_t eyes, uint32_t re_prev, uint32_t ko_prev, int re_all, int ko_all) {
    return fdo::re_won(eyes, re_prev, ko_prev, re_all != 0, ko_all != 0);
}
int or_kat_kontra_won(uint32_t eyes, uint32_t re_prev, uint32_t ko_prev, int re_all, int ko_all) {
    return fdo::kontra_won(eyes, re_prev, ko_prev, re_all != 0, ko_all != 0);
}
// FdoBasicWinningPointsDetails::calculate(winner eyes, loser eyes, winner won all, re prev, kontra prev, re eyes,
// kontra eyes): out = winner points, loser points, 23 detail fields
void or_kat_basic_winning(uint32_t winner_eyes, uint32_t loser_eyes, int winner_all, uint32_t re_prev, uint32_t ko_prev,
                          uint32_t re_eyes, uint32_t ko_eyes, int32_t* out) {
    (void)winner_eyes;
    int w, l;
    fdo::basic_winning_points(loser_eyes, winner_all != 0, re_prev, ko_prev, re_eyes, ko_eyes, &w, &l, out + 2);
    out[0] = w; out[1] = l;
}
// FdoBasicDrawPointsDetails::calculate(re prev, kontra prev, re eyes, kontra eyes): out = re, kontra, 14 fields
void or_kat_basic_draw(uint32_t re_prev, uint32_t ko_prev, uint32_t re_eyes, uint32_t ko_eyes, int32_t* out) {
    int r, k;
    fdo::basic_draw_points(re_prev, ko_prev, re_eyes, ko_eyes, &r, &k, out + 2);
    out[0] = r; out[1] = k;
}
// FdoAdditionalPointsDetails::calculate(re players, winning team (0 Re, 1 Kontra, -1 None), tricks):
// out = re, kontra, against_club_queens, doko re, doko kontra, fuchs re, fuchs kontra, karlchen re, karlchen kontra
void or_kat_additional(int re_mask, int winning_team, const int32_t* tricks, int n_tricks, int32_t* out) {
    fdo::Trick t[12];
    fdo_tricks(tricks, n_tricks, fdo::Normal, t);
    int ra, ka;
    const fdo::AdditionalDetails d = fdo::additional_points((uint8_t)re_mask, winning_team, t, n_tricks, &ra, &ka);
    out[0] = ra; out[1] = ka; out[2] = d.against_club_queens; out[3] = d.doko_re; out[4] = d.doko_kontra;
    out[5] = d.fuchs_re; out[6] = d.fuchs_kontra; out[7] = d.karlchen_re; out[8] = d.karlchen_kontra;
}

// rs-doko ---------------------------------------------------------------------------------
// calculate_allowed_actions_in_normal_game(phase, trick colour (-1 None; DoColor 0 Trump 1 Heart
// 2 Spade 3 Club), hand)
uint64_t or_kat_do_allowed(int phase, int trick_color, uint64_t hand) {
    return dko::calculate_allowed_actions(phase, trick_color, hand);
}
// resolve_team_state(reservation result (-1 NoReservation, else wedding player), tricks[12] (start -1 = None), hands)
void or_kat_do_team_resolve(int wedding_player, const int32_t* tricks, const uint64_t* hands, int32_t* out) {
    dko::State s;
    s.rr_wedding = wedding_player;
    s.has_rr = true;
    for (int i = 0; i < 12; ++i) {
        s.tricks[i] = dko::Trick();
        if (tricks[5 * i] < 0) continue;
        s.tricks[i].present = true;
        s.tricks[i].start = tricks[5 * i];
        for (int k = 0; k < 4; ++k) s.tricks[i].cards[k] = tricks[5 * i + 1 + k];
    }
    for (int p = 0; p < 4; ++p) s.hands[p] = hands[p];
    const dko::TeamState t = dko::resolve_team(s);
    out[0] = t.kind; out[1] = t.wedding_player; out[2] = t.solved; out[3] = t.re;
}
// calculate_end_of_game_stats(re players, eyes, tricks won): out = winning team, is_solo, re eyes, kontra eyes,
// re points, kontra points, player points[4]
void or_kat_do_stats(int re_mask, const uint32_t* eyes, const uint32_t* ntricks, int32_t* out) {
    const dko::Stats s = dko::calculate_stats((uint8_t)re_mask, eyes, ntricks);
    out[0] = s.winning_team; out[1] = s.is_solo; out[2] = (int32_t)s.re_eyes; out[3] = (int32_t)s.kontra_eyes;
    out[4] = s.re_points; out[5] = s.kontra_points;
    for (int p = 0; p < 4; ++p) out[6 + p] = s.player_points[p];
}
uint64_t or_kat_do_hand_add(uint64_t h, int c) { return dko::hand_add(h, c); }
uint64_t or_kat_fdo_hand_add(uint64_t h, int c) { fdo::Hand x; x.bits = h; x.add(c); return x.bits; }

}  // extern "C"
