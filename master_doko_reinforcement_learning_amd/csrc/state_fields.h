// Host-side state packer of the C-ABI: dk_fdo_from_fields / dk_fdo_to_fields and the
// rs-doko pair (include/doko_amd.h).  A caller that holds the reference's FdoState /
// DoState (rs-full-doko/src/state/state.rs:24-75, rs-doko/src/state/state.rs:28-76)
// copies its fields into dk_fdo_fields / dk_do_fields and gets the 128-B wire format the
// kernels read; nothing here touches the device.  Trick winners are recomputed with the
// engine's trick order (fdo::trick_key, the same function the kernels use), so a packed
// state never disagrees with the rules that step it.
#pragma once
#include <string.h>

#include "../../include/doko_amd.h"
#include "engine/do_engine.h"
#include "engine/fdo_engine.h"

namespace dk {
namespace fields {

inline bool in_range(int v, int lo, int hi) { return v >= lo && v <= hi; }

// winner of a complete trick (trick_winning_player_logic.rs:15-44): first strict maximum
inline int trick_winner(const int8_t cards[4], int start, uint32_t game_type) {
    const uint32_t tc = fdo::card_color(cards[0], game_type);
    int best_key = -2, best_i = 0;
    for (int i = 0; i < 4; ++i) {
        const int k = fdo::trick_key(cards[i], tc, game_type);
        if (k > best_key) { best_key = k; best_i = i; }
    }
    return (start + best_i) & 3;
}

// card multiplicities of hands + played cards: every kind at most twice, no stray hand bits
inline bool card_counts_ok(const uint64_t hands[4], const int8_t* played, int n_played) {
    int cnt[24] = {0};
    for (int p = 0; p < 4; ++p) {
        if (hands[p] >> 48) return false;
        for (int c = 0; c < 24; ++c) cnt[c] += (int)((hands[p] >> c) & 1) + (int)((hands[p] >> (c + 24)) & 1);
    }
    for (int i = 0; i < n_played; ++i) {
        if (!in_range(played[i], 0, 23)) return false;
        cnt[played[i]] += 1;
    }
    for (int c = 0; c < 24; ++c) if (cnt[c] > 2) return false;
    return true;
}

inline bool ann_bit_ok(int b, bool allow_none) {
    return (allow_none && b == 0) || b == 1 || b == 2 || b == 4 || b == 8 || b == 16 || b == 32;
}

inline int fdo_from_fields(const dk_fdo_fields* f, dk_state* out) {
    if (!f || !out) return DK_E_INVALID;
    const int nt = f->n_tricks, gt = f->game_type;
    if (!in_range(f->res_start, 0, 3) || !in_range(f->res_len, 0, 4) || !in_range(nt, 0, 12) ||
        !in_range(f->phase, 0, 3) || !in_range(f->current_player, -1, 3) || !in_range(gt, -1, 8) ||
        !in_range(f->rr_kind, -1, 2) || !in_range(f->rr_player, 0, 3) || !in_range(f->rr_reservation, 0, 8) ||
        !in_range(f->team_kind, 0, 3) || !in_range(f->wedding_player, 0, 3) || !in_range(f->solved_trick, 0, 11) ||
        f->re_players > 15 || !in_range(f->ann_n, 0, 12) || !in_range(f->ann_turns_without, 0, 4) ||
        !in_range(f->ann_start, 0, 3) || f->ann_allowed > 63 || !in_range(f->card_index, 0, 48) ||
        !ann_bit_ok(f->re_lowest, true) || !ann_bit_ok(f->contra_lowest, true))
        return DK_E_STATE;
    if ((f->current_player < 0) != (f->phase == fdo::PH_FINISHED)) return DK_E_STATE;
    for (int i = 0; i < f->res_len; ++i) if (!in_range(f->reservations[i], 0, 8)) return DK_E_STATE;
    if (nt > 0 && gt < 0) return DK_E_STATE;
    dk_fdo_state d;
    memset(&d, 0, sizeof(d));
    memset(d.cards, DK_NONE, sizeof(d.cards));
    int ci = 0, prev_winner = f->res_start;
    for (int t = 0; t < nt; ++t) {
        if (f->trick_start[t] != prev_winner) return DK_E_STATE;   // trick 0: the round's starter; then the winners
        int len = 0;
        while (len < 4 && f->trick_cards[t][len] >= 0) {
            if (f->trick_cards[t][len] > 23) return DK_E_STATE;
            d.cards[ci++] = (uint8_t)f->trick_cards[t][len];
            ++len;
        }
        for (int k = len; k < 4; ++k) if (f->trick_cards[t][k] >= 0) return DK_E_STATE;
        if (len < 4 && t != nt - 1) return DK_E_STATE;              // only the last trick may be open
        if (len == 4) {
            prev_winner = trick_winner(f->trick_cards[t], f->trick_start[t], (uint32_t)gt);
            d.trick_winners |= (uint32_t)prev_winner << (2 * t);
        }
    }
    if (ci != f->card_index) return DK_E_STATE;
    {
        int8_t played[48];
        for (int i = 0; i < ci; ++i) played[i] = (int8_t)d.cards[i];
        if (!card_counts_ok(f->hands, played, ci)) return DK_E_STATE;
    }
    uint8_t ann_players = 0;
    for (int k = 0; k < f->ann_n; ++k) {
        if (!in_range(f->ann_player[k], 0, 3) || !in_range(f->ann_card_index[k], 0, 48) ||
            !ann_bit_ok(f->ann_announcement[k], false))
            return DK_E_STATE;
        ann_players |= (uint8_t)(1u << f->ann_player[k]);
    }
    for (int p = 0; p < 4; ++p) {
        if (f->player_eyes[p] > 240 || f->player_num_tricks[p] > 12) return DK_E_STATE;
        d.hands[p] = f->hands[p];
        d.eyes[p] = (uint8_t)f->player_eyes[p];
        d.ntricks[p] = (uint8_t)f->player_num_tricks[p];
    }
    memset(d.res, DK_NONE, sizeof(d.res));
    for (int i = 0; i < f->res_len; ++i) d.res[i] = (uint8_t)f->reservations[i];
    d.res_start = (uint8_t)f->res_start;
    d.res_len = (uint8_t)f->res_len;
    d.card_index = (uint8_t)f->card_index;
    d.phase = (uint8_t)f->phase;
    d.current_player = f->current_player < 0 ? (uint8_t)DK_NONE : (uint8_t)f->current_player;
    d.game_type = gt < 0 ? (uint8_t)DK_NONE : (uint8_t)gt;
    d.rr_kind = f->rr_kind < 0 ? (uint8_t)DK_NONE : (uint8_t)f->rr_kind;
    d.rr_player = (uint8_t)f->rr_player;
    d.rr_reservation = (uint8_t)f->rr_reservation;
    d.team_kind = (uint8_t)f->team_kind;
    d.wedding_player = (uint8_t)f->wedding_player;
    d.solved_trick = (uint8_t)f->solved_trick;
    d.re_players = f->re_players;
    d.re_lowest = f->re_lowest;
    d.contra_lowest = f->contra_lowest;
    d.ann_turns = (uint8_t)f->ann_turns_without;
    d.ann_start = (uint8_t)f->ann_start;
    d.ann_allowed = f->ann_allowed;
    d.ann_count = (uint8_t)f->ann_n;
    d.ann_players = ann_players;
    d.n_tricks = (uint8_t)nt;
    d.game = DK_GAME_FULL_DOKO;
    memcpy(out, &d, sizeof(d));
    return DK_OK;
}

inline int fdo_to_fields(const dk_state* s, dk_fdo_fields* f) {
    if (!s || !f) return DK_E_INVALID;
    const dk_fdo_state& d = s->fdo;
    if (d.game != DK_GAME_FULL_DOKO || d.n_tricks > 12 || d.card_index > 48 || d.res_len > 4) return DK_E_STATE;
    memset(f, 0, sizeof(*f));
    for (int p = 0; p < 4; ++p) {
        f->hands[p] = d.hands[p];
        f->player_eyes[p] = d.eyes[p];
        f->player_num_tricks[p] = d.ntricks[p];
    }
    f->res_start = (int8_t)d.res_start;
    f->res_len = (int8_t)d.res_len;
    for (int i = 0; i < 4; ++i) f->reservations[i] = i < d.res_len ? (int8_t)d.res[i] : (int8_t)-1;
    f->n_tricks = (int8_t)d.n_tricks;
    memset(f->trick_start, -1, sizeof(f->trick_start));
    memset(f->trick_cards, -1, sizeof(f->trick_cards));
    for (int t = 0; t < d.n_tricks; ++t) {
        f->trick_start[t] = (int8_t)(t == 0 ? d.res_start : (d.trick_winners >> (2 * (t - 1))) & 3);
        for (int i = 0; i < 4; ++i) {
            const int ci = 4 * t + i;
            if (ci < d.card_index) f->trick_cards[t][i] = (int8_t)d.cards[ci];
        }
    }
    f->ann_n = (int8_t)d.ann_count;
    memset(f->ann_card_index, -1, sizeof(f->ann_card_index));
    memset(f->ann_player, -1, sizeof(f->ann_player));
    f->re_lowest = d.re_lowest;
    f->contra_lowest = d.contra_lowest;
    f->ann_turns_without = (int8_t)d.ann_turns;
    f->ann_start = (int8_t)d.ann_start;
    f->ann_allowed = d.ann_allowed;
    f->card_index = (int8_t)d.card_index;
    f->current_player = d.current_player == DK_NONE ? (int8_t)-1 : (int8_t)d.current_player;
    f->phase = (int8_t)d.phase;
    f->rr_kind = d.rr_kind == DK_NONE ? (int8_t)-1 : (int8_t)d.rr_kind;
    f->rr_player = (int8_t)d.rr_player;
    f->rr_reservation = (int8_t)d.rr_reservation;
    f->game_type = d.game_type == DK_NONE ? (int8_t)-1 : (int8_t)d.game_type;
    f->team_kind = (int8_t)d.team_kind;
    f->wedding_player = (int8_t)d.wedding_player;
    f->solved_trick = (int8_t)d.solved_trick;
    f->re_players = d.re_players;
    return DK_OK;
}

inline int do_from_fields(const dk_do_fields* f, dk_state* out) {
    if (!f || !out) return DK_E_INVALID;
    if (!in_range(f->res_start, 0, 3) || !in_range(f->current_player, -1, 3) || !in_range(f->phase, 0, 2) ||
        !in_range(f->trick_index, 0, 12) || (f->rr_kind != -1 && f->rr_kind != 0 && f->rr_kind != 2) ||
        !in_range(f->rr_player, 0, 3) || !in_range(f->team_kind, 0, 3) || !in_range(f->wedding_player, 0, 3) ||
        !in_range(f->solved_trick, 0, 11) || f->re_players > 15)
        return DK_E_STATE;
    dk_do_state d;
    memset(&d, 0, sizeof(d));
    memset(d.cards, DK_NONE, sizeof(d.cards));
    int rl = 0;
    for (int i = 0; i < 4; ++i) {
        const int r = f->reservations[i];
        if (!in_range(r, -1, 1) || (r >= 0 && i != rl)) return DK_E_STATE;   // played ones first, in round order
        d.res[i] = r < 0 ? (uint8_t)DK_NONE : (uint8_t)r;
        rl += r >= 0;
    }
    int ci = 0, prev_winner = f->res_start;
    bool open_seen = false;
    int8_t played[48];
    for (int t = 0; t < 12; ++t) {
        if (f->trick_start[t] < 0) {
            for (int k = 0; k < 4; ++k) if (f->trick_cards[t][k] >= 0) return DK_E_STATE;
            open_seen = true;
            continue;
        }
        if (open_seen || f->trick_start[t] != prev_winner || f->trick_start[t] > 3) return DK_E_STATE;
        int len = 0;
        while (len < 4 && f->trick_cards[t][len] >= 0) {
            if (f->trick_cards[t][len] > 23) return DK_E_STATE;
            played[ci] = f->trick_cards[t][len];
            d.cards[ci++] = (uint8_t)f->trick_cards[t][len];
            ++len;
        }
        for (int k = len; k < 4; ++k) if (f->trick_cards[t][k] >= 0) return DK_E_STATE;
        if (len == 4) {
            prev_winner = trick_winner(f->trick_cards[t], f->trick_start[t], fdo::GT_NORMAL);
            d.trick_winners |= (uint32_t)prev_winner << (2 * t);
        } else {
            open_seen = true;   // an open trick is the last present one
        }
    }
    if (!card_counts_ok(f->hands, played, ci)) return DK_E_STATE;
    if ((f->current_player < 0) != (f->phase == dko::PH_FINISHED)) return DK_E_STATE;
    for (int p = 0; p < 4; ++p) {
        if (f->player_eyes[p] > 240 || f->player_num_tricks[p] > 12) return DK_E_STATE;
        d.hands[p] = f->hands[p];
        d.eyes[p] = (uint8_t)f->player_eyes[p];
        d.ntricks[p] = (uint8_t)f->player_num_tricks[p];
    }
    d.res_start = (uint8_t)f->res_start;
    d.res_len = (uint8_t)rl;
    d.card_index = (uint8_t)ci;
    d.phase = (uint8_t)f->phase;
    d.current_player = f->current_player < 0 ? (uint8_t)DK_NONE : (uint8_t)f->current_player;
    d.rr_kind = f->rr_kind < 0 ? (uint8_t)DK_NONE : (uint8_t)f->rr_kind;
    d.rr_player = (uint8_t)f->rr_player;
    d.team_kind = (uint8_t)f->team_kind;
    d.wedding_player = (uint8_t)f->wedding_player;
    d.solved_trick = (uint8_t)f->solved_trick;
    d.re_players = f->re_players;
    d.trick_index = (uint8_t)f->trick_index;
    d.game = DK_GAME_DOKO;
    memcpy(out, &d, sizeof(d));
    return DK_OK;
}

inline int do_to_fields(const dk_state* s, dk_do_fields* f) {
    if (!s || !f) return DK_E_INVALID;
    const dk_do_state& d = s->dk;
    if (d.game != DK_GAME_DOKO || d.card_index > 48 || d.trick_index > 12) return DK_E_STATE;
    memset(f, 0, sizeof(*f));
    for (int p = 0; p < 4; ++p) {
        f->hands[p] = d.hands[p];
        f->player_eyes[p] = d.eyes[p];
        f->player_num_tricks[p] = d.ntricks[p];
    }
    f->res_start = (int8_t)d.res_start;
    for (int i = 0; i < 4; ++i) f->reservations[i] = d.res[i] == DK_NONE ? (int8_t)-1 : (int8_t)d.res[i];
    memset(f->trick_start, -1, sizeof(f->trick_start));
    memset(f->trick_cards, -1, sizeof(f->trick_cards));
    // present tricks: trick 0 opens when the reservations end, each later one when its
    // predecessor completes (rs-doko/src/state/state.rs:189-309)
    const int present = d.phase == dko::PH_RESERVATION ? 0 : (d.trick_index < 12 ? d.trick_index + 1 : 12);
    for (int t = 0; t < present; ++t) {
        f->trick_start[t] = (int8_t)(t == 0 ? d.res_start : (d.trick_winners >> (2 * (t - 1))) & 3);
        for (int i = 0; i < 4; ++i) {
            const int ci = 4 * t + i;
            if (ci < d.card_index) f->trick_cards[t][i] = (int8_t)d.cards[ci];
        }
    }
    f->current_player = d.current_player == DK_NONE ? (int8_t)-1 : (int8_t)d.current_player;
    f->phase = (int8_t)d.phase;
    f->trick_index = (int8_t)d.trick_index;
    f->rr_kind = d.rr_kind == DK_NONE ? (int8_t)-1 : (int8_t)d.rr_kind;
    f->rr_player = (int8_t)d.rr_player;
    f->team_kind = (int8_t)d.team_kind;
    f->wedding_player = (int8_t)d.wedding_player;
    f->solved_trick = (int8_t)d.solved_trick;
    f->re_players = d.re_players;
    return DK_OK;
}

}  // namespace fields
}  // namespace dk

extern "C" {
int dk_fdo_from_fields(const dk_fdo_fields* f, dk_state* out) { return dk::fields::fdo_from_fields(f, out); }
int dk_fdo_to_fields(const dk_state* s, dk_fdo_fields* f) { return dk::fields::fdo_to_fields(s, f); }
int dk_do_from_fields(const dk_do_fields* f, dk_state* out) { return dk::fields::do_from_fields(f, out); }
int dk_do_to_fields(const dk_state* s, dk_do_fields* f) { return dk::fields::do_to_fields(s, f); }
}
