// gz_search.h -- device pieces shared by the search kernels (gz_selfplay.hip,
// gz_plan.hip): the SoA tree, wave helpers, the pattern-score grid, the leaf
// sink and MCTSNode.ucb1.
#pragma once
#include <hip/hip_runtime.h>

#include <climits>

#include "gz_bitboard.h"
#ifndef GZ_TABLE_QUAL
#define GZ_TABLE_QUAL static __device__ const
#endif
#include "gz_tables.h"
#include "../../include/gzero.h"

namespace gz {

constexpr int WAVE = 64;
constexpr int GRID_W = 23;  // 15 + 2*4 padding for 9-cell pattern windows
constexpr int GRID_CELLS = GRID_W * GRID_W;
constexpr int GRID_BYTES = 544;

// ---------------------------------------------------------------- tree (LDS)
struct Tree {
    double* value;
    double* bg;
    int32_t* visits;
    int16_t* parent;
    int16_t* bound;  // exclusive bit bound of the node's unexplored moves
    uint8_t* move;   // row-major cell (255 for the root)
    uint8_t* term;   // 0 live, 1/2 winner colour, 3 draw
};

__host__ __device__ inline size_t tree_bytes_for(int S) {
    size_t mn = (size_t)S + 1;
    return (mn * 26 + 255) & ~(size_t)255;
}

__device__ inline Tree tree_at(char* base, int S) {
    size_t mn = (size_t)S + 1;
    Tree t;
    t.value = (double*)base;
    t.bg = (double*)(base + 8 * mn);
    t.visits = (int32_t*)(base + 16 * mn);
    t.parent = (int16_t*)(base + 20 * mn);
    t.bound = (int16_t*)(base + 22 * mn);
    t.move = (uint8_t*)(base + 24 * mn);
    t.term = (uint8_t*)(base + 25 * mn);
    return t;
}

// ---------------------------------------------------------------- wave helpers
__device__ inline int lane_id() { return threadIdx.x & (WAVE - 1); }
__device__ inline uint64_t ballot(bool p) { return __ballot(p ? 1 : 0); }
__device__ inline int rank_in(uint64_t m) {
    return __popcll(m & ((1ull << lane_id()) - 1ull));
}

// argmax with first-index tie break (Python max keeps the first maximum)
__device__ inline void wave_argmax(double& v, int& id) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        double ov = __shfl_xor(v, off);
        int oi = __shfl_xor(id, off);
        if (ov > v || (ov == v && oi < id)) {
            v = ov;
            id = oi;
        }
    }
}

__device__ inline void wave_argmax_int(int& v, int& id) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        int ov = __shfl_xor(v, off);
        int oi = __shfl_xor(id, off);
        if (ov > v || (ov == v && oi < id)) {
            v = ov;
            id = oi;
        }
    }
}

__device__ inline long long wave_sum_ll(long long v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

__device__ inline BB bb_bcast(const BB& x) {
    BB o;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) o.w[i] = __shfl(x.w[i], 0);
    return o;
}

__device__ inline double term_value(int term, int ai) {
    // _get_terminal_value, ai_agent.py:287-304
    return term == 3 ? 0.1 : (term == ai ? 1.0 : -1.0);
}

// ---------------------------------------------------------------- pattern score
// grid: 23x23 bytes, 0 empty / 1 black / 2 white / 3 off-board, cell (r,c) at (r+4)*23+c+4
__device__ __forceinline__ void write_grid(uint8_t* grid, const BB& black, const BB& white) {
    for (int idx = lane_id(); idx < GRID_CELLS; idx += WAVE) {
        int r = idx / GRID_W - 4, c = idx % GRID_W - 4;
        uint8_t v = 3;
        if (r >= 0 && r < GZ_N && c >= 0 && c < GZ_N) {
            int b = r * 16 + c;
            v = bb_test(black, b) ? 1 : (bb_test(white, b) ? 2 : 0);
        }
        grid[idx] = v;
    }
    __syncthreads();
}

// _pattern_score (bg_planner.py:133-155) over the player's stones `pstones` on the
// board in `grid`, with cell `ov_idx` (grid index, -1 for none) overridden to `player`.
__device__ __forceinline__ long long pattern_score_lane(const uint8_t* grid, const BB& pstones, int player, int ov_idx) {
    const int DR[4] = {1, 0, 1, 1}, DC[4] = {0, 1, 1, -1};  // bg_planner.py:147
    long long total = 0;
    // walk the stones in ascending bit order: word index from a select chain
    // (no dynamic register indexing)
    int wi = 0;
    uint32_t w = pstones.w[0];
    while (true) {
        while (w == 0 && wi < GZ_W - 1) {
            wi++;
            w = bb_word(pstones, wi);
        }
        if (w == 0) break;
        {
            int b = wi * 32 + ctz(w);
            w &= w - 1;
            int r = b >> 4, c = b & 15;
            int g0 = (r + 4) * GRID_W + (c + 4);
#pragma unroll
            for (int d = 0; d < 4; d++) {
                int step = DR[d] * GRID_W + DC[d];
                int code = 0, pw = 1;
#pragma unroll
                for (int k = -4; k <= 4; k++) {
                    if (k == 0) continue;
                    int gi = g0 + k * step;
                    int v = grid[gi];
                    v = (gi == ov_idx) ? player : v;
                    int dig = v == player ? 0 : (v == 0 ? 1 : 2);
                    code += dig * pw;
                    pw *= 3;
                }
                total += GZ_PATTERN_LUT[code];
            }
        }
    }
    return total;
}

__device__ inline double bg_from_score(long long s) {
    long long k = s / 50;  // every pattern weight is a multiple of 50
    return k >= GZ_TANH_N ? 1.0 : GZ_TANH_TABLE[k];
}

__device__ inline int grid_index_of_bit(int bit) { return ((bit >> 4) + 4) * GRID_W + (bit & 15) + 4; }

// ---------------------------------------------------------------- leaves
struct LeafSink {
    uint32_t* leaves;
    int32_t cap;
    int32_t* count;
    int32_t* meta;  // optional, per leaf: -1 root, >= 0 the parent's leaf index (a root
                    // child, or a child of one), -2 any other node (gz_pv_forward_tree)
};

__device__ inline void leaf_meta(const LeafSink& s, int idx, int32_t v) {
    if (s.meta && idx >= 0 && idx < s.cap) s.meta[idx] = v;
}

__device__ inline int leaf_reserve(const LeafSink& s, int n) {
    int base = 0;
    if (lane_id() == 0 && n > 0) base = atomicAdd(s.count, n);
    return __shfl(base, 0);
}

__device__ inline void leaf_write(const LeafSink& s, int idx, const BB& black, const BB& white) {
    if (idx < 0 || idx >= s.cap) return;
    uint4* dst = (uint4*)(s.leaves + (size_t)idx * 16);
    dst[0] = make_uint4(black.w[0], black.w[1], black.w[2], black.w[3]);
    dst[1] = make_uint4(black.w[4], black.w[5], black.w[6], black.w[7]);
    dst[2] = make_uint4(white.w[0], white.w[1], white.w[2], white.w[3]);
    dst[3] = make_uint4(white.w[4], white.w[5], white.w[6], white.w[7]);
}

// ---------------------------------------------------------------- UCB
// MCTSNode.ucb1, ai_agent.py:532-562 (time_reward == 0: the model object never
// carries _last_decision_time, ai_agent.py:553).
__device__ inline double ucb1(const Tree& t, int i, double mlog, const gz_search_params& p) {
    int n = t.visits[i];
    if (n == 0) return __builtin_inf();
    double exploitation = t.value[i] / (double)n;
    double exploration = p.c_puct * __builtin_sqrt(mlog / (double)n);
    double base = exploitation + exploration;
    double bg_bonus = p.beta * t.bg[i];
    double time_reward = 0.0;
    return base + bg_bonus + time_reward;
}

__device__ inline void load_bb(BB& x, const uint32_t* src) {
#pragma unroll
    for (int i = 0; i < GZ_W; i++) x.w[i] = src[i];
}
__device__ inline void store_bb(uint32_t* dst, const BB& x) {
#pragma unroll
    for (int i = 0; i < GZ_W; i++) dst[i] = x.w[i];
}

}  // namespace gz
