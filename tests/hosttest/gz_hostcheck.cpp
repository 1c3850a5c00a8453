// TEST-ONLY: a host build of the per-lane device logic (csrc/gz_bitboard.h, through
// gz_hosttest.cpp) checked against the C oracle (oracle/gz_oracle.c), both compiled with
// -fsanitize=address,undefined by tests/test_hostcheck_cpu.py (the
// sanitizer build of the host and oracle code; GPU sanitizers are not available).
//
// On positions reached by random legal play from the empty board:
//   * one move of the offensive rollout policy (ai_agent.py:251-430): the bitboard
//     policy_move == or_offensive_move, with the same number of RNG draws;
//   * a whole rollout (_simulate, ai_agent.py:265-304): value, final board and draws;
// then a few MCTS searches (or_get_move, ai_agent.py:109-222) and one self-play game
// (or_play_game, training.py:141-218) run through the oracle's tree code.
// Exit status 0 = every comparison equal and no sanitizer report.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../oracle/gz_oracle.h"

extern "C" int ht_policy_move(const int8_t* cells, int player, uint64_t key, uint32_t* draws);
extern "C" double ht_rollout(const int8_t* cells, int n_moves, int mover, int ai, int max_depth, uint64_t key,
                             uint32_t* draws, int8_t* out_cells, int* out_n, int* out_over, int* out_winner);

static uint64_t lcg(uint64_t& s) {
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    return s >> 11;
}

int main(int argc, char** argv) {
    const int n_pos = argc > 1 ? std::atoi(argv[1]) : 600;
    uint64_t s = 20251003;
    int fails = 0, checked = 0;
    for (int i = 0; i < n_pos; i++) {
        or_board b;
        or_board_init(&b);
        const int plies = (int)(lcg(s) % 90);
        for (int k = 0; k < plies && !b.over; k++) {
            uint64_t m[4];
            const int n = or_legal_mask(&b, m);
            if (n == 0) break;
            int pick = (int)(lcg(s) % (uint64_t)n), cell = -1;
            for (int c = 0; c < OR_CELLS; c++)
                if ((m[c >> 6] >> (c & 63)) & 1ULL) {
                    if (pick-- == 0) {
                        cell = c;
                        break;
                    }
                }
            or_make_move(&b, cell / OR_N, cell % OR_N);
        }
        if (b.over) continue;
        const uint64_t key = or_stream_key(7, i, plies, 1 + (int)(lcg(s) % 200));
        uint64_t d64 = 0;
        uint32_t d32 = 0;
        const int mo = or_offensive_move(&b, key, &d64);
        const int mg = ht_policy_move(b.cell, b.player, key, &d32);
        if (mo != mg || d64 != d32) {
            std::printf("policy mismatch at position %d: oracle %d (%llu draws), bitboard %d (%u draws)\n", i, mo,
                        (unsigned long long)d64, mg, d32);
            fails++;
        }
        const int ai = 1 + (int)(lcg(s) & 1);
        or_board fin;
        d64 = 0;
        d32 = 0;
        const double vo = or_rollout(&b, ai, 100, key, &d64, &fin);
        int8_t cells[OR_CELLS];
        int n_out = 0, over = 0, winner = 0;
        const double vg = ht_rollout(b.cell, b.n_moves, b.player, ai, 100, key, &d32, cells, &n_out, &over, &winner);
        if (std::memcmp(&vo, &vg, sizeof vo) != 0 || d64 != d32 || std::memcmp(cells, fin.cell, OR_CELLS) != 0 ||
            n_out != fin.n_moves || over != fin.over || winner != fin.winner) {
            std::printf("rollout mismatch at position %d: value %.17g / %.17g, draws %llu / %u\n", i, vo, vg,
                        (unsigned long long)d64, d32);
            fails++;
        }
        checked++;
    }
    // MCTS searches and one game through the oracle's tree code (sanitized)
    or_params p;
    std::memset(&p, 0, sizeof p);
    p.num_simulations = 50;
    p.c_puct = 1.6;
    p.exploration = 0.05;
    p.beta = 0.2;
    p.max_depth = 100;
    p.seed = 11;
    static int32_t parent[512], move[512], visits[512];
    static double value[512];
    for (int g = 0; g < 4; g++) {
        or_board b;
        or_board_init(&b);
        const int32_t opening[10] = {112, 113, 97, 128, 98, 140, 82, 66, 126 + g, 154 - g};
        or_replay(&b, opening, 6 + g);  // past the opening book (ply < 6, ai_agent.py:132-166)
        or_tree_info info;
        std::memset(&info, 0, sizeof info);
        info.parent = parent;
        info.move = move;
        info.visits = visits;
        info.value = value;
        info.cap = 512;
        const int mv = or_get_move(&b, b.player, &p, g, &info);
        if (mv < 0 || mv >= OR_CELLS || b.cell[mv] != 0 || info.n_nodes < 2 || info.n_nodes > 512) {
            std::printf("search %d: move %d, %d nodes\n", g, mv, info.n_nodes);
            fails++;
        }
    }
    p.num_simulations = 8;
    static int8_t cells_out[200 * OR_CELLS], players[200], z[200];
    static int32_t moves[200];
    int winner = 0;
    int64_t predicts = 0;
    const int n = or_play_game(&p, &p, 3, cells_out, moves, players, z, 200, &winner, &predicts, 0);
    if (n <= 0 || n > 200) {
        std::printf("game: %d plies\n", n);
        fails++;
    }
    std::printf("hostcheck: %d positions compared, %d mismatches, game of %d plies\n", checked, fails, n);
    return fails == 0 && checked > n_pos / 2 ? 0 : 1;
}
