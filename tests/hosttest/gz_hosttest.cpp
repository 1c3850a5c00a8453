// TEST-ONLY host build of the per-lane device logic in csrc/gz_bitboard.h, so the
// CPU test suite can compare the bitboard rollout policy with the C oracle
// without a GPU.  Never loaded by the product path.
#include "../../alphazero-gomoku_amd/csrc/gz_bitboard.h"

using namespace gz;

static void from_cells(const int8_t* cells, BB& black, BB& white) {
    black = bb_zero();
    white = bb_zero();
    for (int i = 0; i < GZ_CELLS; i++) {
        if (cells[i] == 1) bb_set(black, cell_to_bit(i));
        if (cells[i] == 2) bb_set(white, cell_to_bit(i));
    }
}

static void to_cells(const BB& black, const BB& white, int8_t* cells) {
    for (int i = 0; i < GZ_CELLS; i++) {
        int b = cell_to_bit(i);
        cells[i] = bb_test(black, b) ? 1 : (bb_test(white, b) ? 2 : 0);
    }
}

extern "C" int ht_policy_move(const int8_t* cells, int player, uint64_t key, uint32_t* draws) {
    BB black, white;
    from_cells(cells, black, white);
    BB me = player == 1 ? black : white, op = player == 1 ? white : black;
    BB e = empties(me, op);
    Centre cb = centre_buckets();
    bool won;
    int b = policy_move(me, op, e, cb, key, draws, &won);
    return bit_to_cell(b);
}

extern "C" double ht_rollout(const int8_t* cells, int n_moves, int mover, int ai, int max_depth,
                             uint64_t key, uint32_t* draws, int8_t* out_cells, int* out_n, int* out_over,
                             int* out_winner) {
    BB black, white;
    from_cells(cells, black, white);
    RolloutResult r = rollout(black, white, n_moves, mover, ai, max_depth, key, draws);
    to_cells(r.black, r.white, out_cells);
    *out_n = r.n_moves;
    *out_over = r.over;
    *out_winner = r.winner;
    return r.value;
}

extern "C" void ht_threats(const int8_t* cells, int player, uint64_t* win4, uint64_t* make3_4, int* has3) {
    BB black, white;
    from_cells(cells, black, white);
    BB me = player == 1 ? black : white;
    Threats t = threats(me);
    BB e = empties(black, white);
    BB w = t.win & e, m = t.make3 & e;
    for (int k = 0; k < 4; k++) win4[k] = make3_4[k] = 0;
    for (int i = 0; i < GZ_CELLS; i++) {
        int b = cell_to_bit(i);
        if (bb_test(w, b)) win4[i >> 6] |= 1ULL << (i & 63);
        if (bb_test(m, b)) make3_4[i >> 6] |= 1ULL << (i & 63);
    }
    *has3 = has_run3(me);
}
