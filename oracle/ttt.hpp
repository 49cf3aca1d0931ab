// ORACLE — test infrastructure only. Never linked into the product library.
//
// Tic-tac-toe of rs-doko-mcts/src/example/tic_tac_toe.rs:29-193 and its env
// adapter tic_tac_toe_impl.rs:17-63 (allowed_actions/by_action are `todo!()`
// there; defined here as "empty cells as action bits 0-8").
#pragma once
#include <cstdint>
#include "rand09.hpp"

namespace oracle {
namespace ttt {

enum Finish : int { NotFinished = 0, Xwon = 1, Owon = 2, Draw = 3 };

// tic_tac_toe.rs:29-80
inline int calc_finish_state(const int b[9]) {
    static const int lines[8][3] = {{0, 1, 2}, {3, 4, 5}, {6, 7, 8}, {0, 3, 6}, {1, 4, 7}, {2, 5, 8}, {0, 4, 8}, {2, 4, 6}};
    bool remaining = false;
    for (int l = 0; l < 8; ++l) {
        bool all_x = true, all_o = true;
        for (int k = 0; k < 3; ++k) {
            const int v = b[lines[l][k]];
            if (v != 1) all_x = false;
            if (v != 2) all_o = false;
            if (v == 0) remaining = true;
        }
        if (all_x) return Xwon;
        if (all_o) return Owon;
    }
    return remaining ? NotFinished : Draw;
}

struct Env {
    int board[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // 0 empty, 1 X, 2 O
    int finish = NotFinished;
    int last_action = -1;

    // tic_tac_toe.rs:109-130
    int current_player() const {
        int x = 0, o = 0;
        for (int i = 0; i < 9; ++i) { x += board[i] == 1; o += board[i] == 2; }
        return x == o ? 0 : 1;
    }
    bool is_terminal() const { return finish != NotFinished; }
    uint64_t allowed_actions(bool) const {
        if (finish != NotFinished) return 0;
        uint64_t m = 0;
        for (int i = 0; i < 9; ++i) if (board[i] == 0) m |= 1ULL << i;
        return m;
    }
    // tic_tac_toe.rs:90-108
    Env by_action(int index) const {
        Env e = *this;
        e.board[index] = current_player() == 0 ? 1 : 2;
        e.finish = calc_finish_state(e.board);
        e.last_action = index;
        return e;
    }
    // tic_tac_toe.rs:132-141
    void rewards(double out[4]) const {
        out[0] = out[1] = 0.0; out[2] = out[3] = 0.0;
        if (finish == Xwon) { out[0] = 1.0; out[1] = -1.0; }
        else if (finish == Owon) { out[0] = -1.0; out[1] = 1.0; }
    }
    bool rewards_or_none(double out[4]) const { if (finish == NotFinished) return false; rewards(out); return true; }
    // tic_tac_toe.rs:143-165 + tic_tac_toe_impl.rs:52-61
    void random_rollout(SmallRng& rng, double out[4]) const {
        Env s = *this;
        while (s.finish == NotFinished) {
            int empties[9], n = 0;
            for (int i = 0; i < 9; ++i) if (s.board[i] == 0) empties[n++] = i;
            const int ri = (int)rng.random_range_usize(0, n);
            s.board[empties[ri]] = s.current_player() == 0 ? 1 : 2;
            s.finish = calc_finish_state(s.board);
            s.last_action = ri;
        }
        s.rewards(out);
    }
};

}  // namespace ttt
}  // namespace oracle
