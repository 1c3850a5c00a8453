// gz_plan.hip -- MCTS with BG-planner rollout plies (planner_steps > 0) on gfx950.
//
// _simulate (ai_agent.py:251-285) starts every rollout with planner_steps plies of
// BGPlannerAI.get_move (bg_planner.py:232-269), each of which needs GraphNet and
// OpponentDQN on the rollout board.  Those nets are batched across all rollouts of
// all games (gz_gnet.hip), so the search runs as a host-driven pipeline of
// launches over per-game contexts kept in the workspace:
//
//   begin   (wave per game)   root, root children, one rollout job per simulation
//                             of the parallel phase (simulations 1..min(S, L+1))
//   repeat until no game has a pending job:
//     planner_steps x [ collect  (thread per job) active jobs -> GN input rows
//                       gz_gn_forward over the collected rows
//                       step     (wave per job)  knowledge search + compose + move ]
//     collect  (final: jobs past their planner plies -> rollout)
//     rollout  (thread per job)  offensive policy to the end (_simulate :276-285)
//     resume   (wave per game)   back up; run sequential simulations (UCB select,
//                                expand) until one needs a rollout -> 1 new job;
//                                after the last simulation: pick the move
//
// Every draw, tree update and tie-break follows the fused search of
// gz_selfplay.hip (and the reference), so with the same net outputs the moves
// and trees are identical to the C oracle's (tests/test_gpu_plan.py).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>
#include <vector>

#include "gz_gnet.h"
#include "gz_search.h"

using namespace gz;
using gzgn::GnTag;

namespace {

// ---------------------------------------------------------------- workspace
struct PlanCtx {  // 256-byte header, then the tree (tree_bytes_for(S))
    uint32_t black[8], white[8];
    int64_t game_id;
    int64_t sim_draws;
    int32_t n_moves, player, L, n_par;
    int32_t phase;  // 0 done, 1 parallel jobs pending, 2 sequential job pending
    int32_t k;      // next sequential simulation
    int32_t x;      // leaf of the pending sequential simulation
    int32_t n_nodes, predicts, main_draws, move;
    uint32_t dm;
    int32_t root_leaf;  // the root's leaf index (leaf tags for gz_pv_forward_tree), -1 none
    int32_t pad[31];
};
static_assert(sizeof(PlanCtx) == 256, "ctx header");

struct PlanJob {  // 128 bytes
    uint32_t black[8], white[8];
    uint64_t key;
    double value;
    uint32_t cnt;
    int32_t game;
    int32_t sim;
    int32_t row;      // GN batch row of the current planner ply
    int16_t n_moves;
    int8_t mover, ai;
    int8_t state;     // 0 none, 1 planner plies, 2 rollout, 3 done
    int8_t steps;
    int8_t pad[2];
    // incremental GraphNet chain (gn_inc_kernel): the stones added since the base
    // maps whose squares are in the job's map slot, whether the base is that slot
    // (after a full forward) rather than the search root's, and the planner move
    // the next planner ply's board adds
    uint8_t st[gzgn::TAG_STONES];
    uint8_t nst, bj, pend, pad3;
    int32_t pad2[3];
};
static_assert(sizeof(PlanJob) == 128, "job");

struct Counters {
    int32_t rows;         // GN rows collected this round
    int32_t nfull, ninc;  // this planner step's full-forward / incremental rows
    int32_t ihead;        // gn_inc_kernel's chunk queue head (cleared with rows, nfull, ninc)
    // games with a job after resume: only w.ctr's is used, cleared by the host right
    // before plan_resume_kernel and never by the per-step resets of (rows, nfull, ninc)
    int32_t pending;
    int32_t pad[59];
};
// never cleared by a search: gz_plan_gn_stats reads (and resets) them
struct GnStats {
    int64_t full, inc, mismatch, checked;
    int64_t pad[4];
};

__host__ __device__ inline size_t ctx_stride(int S) { return sizeof(PlanCtx) + tree_bytes_for(S); }

constexpr size_t GN_REC_BYTES = 928 * 4;  // a net record (gz_gnet.h REC)
// gz_gn_workspace_bytes(1): the record + the split heads' scratch (3 x 256 floats), checked at run time
constexpr size_t GN_WS_BYTES = GN_REC_BYTES + 3 * 256 * 4;

struct Workspace {
    char* ctx;
    PlanJob* jobs;
    uint32_t* gn_in;   // [C][16] (C = chunk_rows: the GN rows of one planner step)
    float* gn_p;       // [C][225]
    float* gn_q;
    float* gn_rec;     // gz_gn_forward's workspace for C rows (records, then the heads' scratch)
    int32_t* rows;     // row -> job
    Counters* ctr;
    Counters* ctr2;    // a planner step's rows / nfull / ninc alternate between ctr and ctr2
    GnStats* stats;
    GnTag* tags;       // [C] incremental tags of the rows
    int32_t* full_list, *inc_list;  // [C] rows by kind
    float *chk_p, *chk_q, *chk_rec;  // GZ_FLAG_GN_CHECK: the full forward of the same rows
    char* slots;       // map slots: [n] search roots, then [C] jobs (gzgn::SLOT_BYTES each)
    size_t end;
};

__host__ __device__ inline size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

// Round 0 (the parallel phase: up to n * S rollouts at once) runs its jobs in chunks
// of C: a chunk's planner plies, then the next chunk's; jobs are independent, so
// this only bounds the row buffers and the map slots (one per job of a chunk)
constexpr size_t PLAN_CHUNK = 65536;
__host__ __device__ inline size_t chunk_rows(int n, int S) {
    const size_t nj = (size_t)n * (S > 0 ? S : 1);
    const size_t c = (size_t)n > PLAN_CHUNK ? (size_t)n : PLAN_CHUNK;
    return nj < c ? nj : c;
}

__host__ __device__ inline Workspace carve(void* base, int n, int S) {
    char* p = (char*)base;
    const size_t nj = (size_t)n * (S > 0 ? S : 1), C = chunk_rows(n, S);
    Workspace w;
    w.ctr = (Counters*)p;
    w.ctr2 = w.ctr + 1;
    p += align256(2 * sizeof(Counters));
    w.stats = (GnStats*)p;
    p += align256(sizeof(GnStats));
    w.ctx = p;
    p += align256(ctx_stride(S) * (size_t)n);
    w.jobs = (PlanJob*)p;
    p += align256(sizeof(PlanJob) * nj);
    w.gn_in = (uint32_t*)p;
    p += align256(C * 16 * 4);
    w.gn_p = (float*)p;
    p += align256(C * 225 * 4);
    w.gn_q = (float*)p;
    p += align256(C * 225 * 4);
    w.gn_rec = (float*)p;
    p += align256(C * GN_WS_BYTES);
    w.rows = (int32_t*)p;
    p += align256(C * 4);
    w.tags = (GnTag*)p;
    p += align256(C * sizeof(GnTag));
    w.full_list = (int32_t*)p;
    p += align256(C * 4);
    w.inc_list = (int32_t*)p;
    p += align256(C * 4);
    w.chk_p = (float*)p;
    p += align256(C * 225 * 4);
    w.chk_q = (float*)p;
    p += align256(C * 225 * 4);
    w.chk_rec = (float*)p;
    p += align256(C * GN_WS_BYTES);
    w.slots = p;
    p += align256(((size_t)n + C) * gzgn::SLOT_BYTES);
    w.end = (size_t)(p - (char*)base);
    return w;
}

__host__ inline size_t workspace_bytes(int n, int S) { return carve(nullptr, n, S).end; }

__device__ inline PlanCtx* ctx_at(const Workspace& w, int g, int S) {
    return (PlanCtx*)(w.ctx + (size_t)g * ctx_stride(S));
}
__device__ inline Tree ctx_tree(PlanCtx* c, int S) { return tree_at((char*)c + sizeof(PlanCtx), S); }

__device__ inline void job_set(PlanJob& j, const BB& black, const BB& white, int n_moves, int mover, int ai,
                               uint64_t key, int game, int sim) {
    store_bb(j.black, black);
    store_bb(j.white, white);
    j.key = key;
    j.value = 0.0;
    j.cnt = 0;
    j.game = game;
    j.sim = sim;
    j.row = -1;
    j.n_moves = (int16_t)n_moves;
    j.mover = (int8_t)mover;
    j.ai = (int8_t)ai;
    j.state = 1;
    j.steps = 0;
}

// ---------------------------------------------------------------- planner move
// KnowledgeSearch.score_move / top_k_moves (bg_planner.py:90-131) + the compose
// and exploration of BGPlannerAI.get_move (:242-269), one wave per board.
//
// Pattern term: pattern(temp, P) = pattern(board, P) + delta(m).  The window
// code (8 cells around a centre, base 3: 0 = P's stone, 1 = empty, 2 = other or
// off-board; digit i <-> offsets -4..-1, +1..+4) of every cell and direction is
// tabulated once per board; placing a stone on the empty cell m changes only the
// windows of P's stones within 4 cells of m on the 4 lines through m (digit
// 1 -> 0 or 2), plus m's own windows when the stone is P's.
struct PlanShared {
    uint16_t code[GZ_CELLS][4];  // window code of every cell (centre excluded)
    int32_t top[16];
    uint8_t grid[GRID_BYTES];
    int32_t base;
};
// plan_step_kernel's workgroup of PW waves: the cells' scores and the waves' pattern parts
constexpr int PW = 4;
struct PlanShared4 {
    PlanShared s;
    double sc[PW * WAVE];
    int32_t part[PW];
};

__device__ inline int pow3(int i) {
    const int P3[8] = {1, 3, 9, 27, 81, 243, 729, 2187};
    int r = 1;
#pragma unroll
    for (int k = 0; k < 8; k++) r = (k == i) ? P3[k] : r;
    return r;
}

// After `who` plays the empty cell at grid index g0: is there an empty cell f != g0
// where `who` then completes five with g0 inside the five?  (A five through f that
// avoids g0 was already a threat before the move.)  Every 5-window along the 4
// lines through g0 (border cells read 3: blocked) with 3 of who's stones and one
// empty cell besides g0 gives such an f.
__device__ inline bool new_five_through(const uint8_t* grid, int g0, int who) {
    const int STEP[4] = {GRID_W, 1, GRID_W + 1, GRID_W - 1};  // (1,0) (0,1) (1,1) (1,-1)
#pragma unroll
    for (int d = 0; d < 4; d++) {
        int st[9], em[9];
#pragma unroll
        for (int k = -4; k <= 4; k++) {
            const int v = k == 0 ? who : grid[g0 + k * STEP[d]];
            st[k + 4] = v == who;
            em[k + 4] = v == 0;
        }
#pragma unroll
        for (int s0 = 0; s0 <= 4; s0++) {
            int ns = 0, ne = 0;
#pragma unroll
            for (int k = 0; k < 5; k++) {
                ns += st[s0 + k];
                ne += em[s0 + k];
            }
            if (ns == 4 && ne == 1) return true;  // g0 + 3 stones, one empty cell
        }
    }
    return false;
}

// window codes (wrt P) of `cell` into sh->code; returns its pattern(board, P) part
__device__ __forceinline__ int cell_codes(PlanShared* sh, int cell, const BB& Pst, int P) {
    const int DR[4] = {1, 0, 1, 1}, DC[4] = {0, 1, 1, -1};  // bg_planner.py:147
    const int r = cell / GZ_N, c = cell % GZ_N;
    const int g0 = (r + 4) * GRID_W + (c + 4);
    const bool isP = bb_test(Pst, r * 16 + c);
    int part = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const int step = DR[d] * GRID_W + DC[d];
        int code = 0, pw = 1;
#pragma unroll
        for (int k = -4; k <= 4; k++) {
            if (k == 0) continue;
            const int v = sh->grid[g0 + k * step];
            code += (v == P ? 0 : (v == 0 ? 1 : 2)) * pw;
            pw *= 3;
        }
        sh->code[cell][d] = (uint16_t)code;
        if (isP) part += GZ_PATTERN_LUT[code];
    }
    return part;
}

// KnowledgeSearch.score_move(board, m, P) (bg_planner.py:90-106) of one cell (-inf
// for occupied / off-board cells), given the codes of every cell and pattern(board, P)
struct KsCtx {
    BB E, Wm, Fo, Pst;
    int mover, P, oppP, n_moves, ne;
};
__device__ __forceinline__ KsCtx ks_ctx(const BB& black, const BB& white, int mover, int n_moves, int P) {
    KsCtx k;
    k.E = empties(black, white);
    k.ne = bb_count(k.E);
    const BB mine = mover == 1 ? black : white;
    k.Pst = P == 1 ? black : white;
    k.oppP = 3 - P;
    const BB Ost = k.oppP == 1 ? black : white;
    k.Wm = threats(mine).win & k.E;  // cells where the mover completes five
    k.Fo = threats(Ost).win & k.E;   // cells where P's opponent completes five
    k.mover = mover;
    k.P = P;
    k.n_moves = n_moves;
    return k;
}
__device__ __forceinline__ double cell_score(const PlanShared* sh, int cell, const KsCtx& k, int base) {
    const int DR[4] = {1, 0, 1, 1}, DC[4] = {0, 1, 1, -1};
    if (cell >= GZ_CELLS) return -__builtin_inf();
    const int r = cell / GZ_N, c = cell % GZ_N, bit = r * 16 + c;
    if (!bb_test(k.E, bit)) return -__builtin_inf();
    const bool win = bb_test(k.Wm, bit);
    if (win && k.mover == k.P) return 1e6;
    bool opp_wins;
    if (win || k.n_moves + 1 >= 200 || k.ne == 1) {
        // the move ends the game: make_move fails on the copies, which keep
        // the old winner -- P's opponent iff it just won (and a cell is left)
        opp_wins = win && k.ne > 1;
    } else if (k.mover == k.P) {
        BB f = k.Fo;
        f.w[bit >> 5] &= ~(1u << (bit & 31));
        opp_wins = bb_any(f);
    } else {
        // the mover is P's opponent: after m it completes five at a cell f != m
        // iff f already did (Fo) or a five-window through m holds 3 of its
        // stones, m and the empty f (new_five_through)
        BB f = k.Fo;
        f.w[bit >> 5] &= ~(1u << (bit & 31));
        opp_wins = bb_any(f) || new_five_through(sh->grid, (r + 4) * GRID_W + (c + 4), k.oppP);
    }
    if (opp_wins) return -1e5;
    const int nd = k.mover == k.P ? 0 : 2;  // digit of the new stone wrt P
    int delta = 0;
#pragma unroll
    for (int d = 0; d < 4; d++) {
#pragma unroll
        for (int q = -4; q <= 4; q++) {
            if (q == 0) continue;
            const int rr = r + q * DR[d], cc = c + q * DC[d];
            if (rr < 0 || rr >= GZ_N || cc < 0 || cc >= GZ_N) continue;
            if (!bb_test(k.Pst, rr * 16 + cc)) continue;
            const int code = sh->code[rr * GZ_N + cc][d];
            const int j = 4 - q;  // m's slot in the window of the stone at offset q
            const int i = j < 4 ? j : j - 1;
            delta += GZ_PATTERN_LUT[code + (nd - 1) * pow3(i)] - GZ_PATTERN_LUT[code];
        }
        if (k.mover == k.P) delta += GZ_PATTERN_LUT[sh->code[cell][d]];
    }
    const int dist = (r > 7 ? r - 7 : 7 - r) + (c > 7 ? c - 7 : 7 - c);
    const double cb = (6 - dist) * 0.5;
    return (double)(base + delta) + (cb > 0.0 ? cb : 0.0);
}

// KnowledgeSearch.score_move(board, m, P) (bg_planner.py:90-106) of every cell, one wave
// (cell_codes / cell_score's work, kept as one body: split, the one-wave kernel spilled more),
// lane-strided: sc[s] is cell lane + 64 s (-inf for occupied / off-board cells);
// returns the number of empty cells.
__device__ __forceinline__ int knowledge_scores(PlanShared* sh, const BB& black, const BB& white, int mover,
                                                int n_moves, int P, double (&sc)[4]) {
    const int lane = lane_id();
    const int DR[4] = {1, 0, 1, 1}, DC[4] = {0, 1, 1, -1};  // bg_planner.py:147
    const BB E = empties(black, white);
    const int ne = bb_count(E);
    const BB mine = mover == 1 ? black : white;
    const BB Pst = P == 1 ? black : white;
    const int oppP = 3 - P;
    const BB Ost = oppP == 1 ? black : white;
    const BB Wm = threats(mine).win & E;  // cells where the mover completes five
    const BB Fo = threats(Ost).win & E;   // cells where P's opponent completes five

    // window codes of every cell (wrt P) and pattern(board, P)
    write_grid(sh->grid, black, white);
    int part = 0;
    for (int cell = lane; cell < GZ_CELLS; cell += WAVE) {
        const int r = cell / GZ_N, c = cell % GZ_N;
        const int g0 = (r + 4) * GRID_W + (c + 4);
        const bool isP = bb_test(Pst, r * 16 + c);
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const int step = DR[d] * GRID_W + DC[d];
            int code = 0, pw = 1;
#pragma unroll
            for (int k = -4; k <= 4; k++) {
                if (k == 0) continue;
                const int v = sh->grid[g0 + k * step];
                code += (v == P ? 0 : (v == 0 ? 1 : 2)) * pw;
                pw *= 3;
            }
            sh->code[cell][d] = (uint16_t)code;
            if (isP) part += GZ_PATTERN_LUT[code];
        }
    }
    int base = (int)wave_sum_ll(part);
    __syncthreads();

    // score of every legal cell (lane-strided, row-major)
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const int cell = lane + 64 * s;
        sc[s] = -__builtin_inf();
        if (cell >= GZ_CELLS) continue;
        const int r = cell / GZ_N, c = cell % GZ_N, bit = r * 16 + c;
        if (!bb_test(E, bit)) continue;
        const bool win = bb_test(Wm, bit);
        double score;
        if (win && mover == P) {
            score = 1e6;
        } else {
            bool opp_wins;
            if (win || n_moves + 1 >= 200 || ne == 1) {
                // the move ends the game: make_move fails on the copies, which keep
                // the old winner -- P's opponent iff it just won (and a cell is left)
                opp_wins = win && ne > 1;
            } else if (mover == P) {
                BB f = Fo;
                f.w[bit >> 5] &= ~(1u << (bit & 31));
                opp_wins = bb_any(f);
            } else {
                // the mover is P's opponent: after m it completes five at a cell f != m
                // iff f already did (Fo) or a five-window through m holds 3 of its
                // stones, m and the empty f (new_five_through)
                BB f = Fo;
                f.w[bit >> 5] &= ~(1u << (bit & 31));
                opp_wins = bb_any(f) || new_five_through(sh->grid, (r + 4) * GRID_W + (c + 4), oppP);
            }
            if (opp_wins) {
                score = -1e5;
            } else {
                const int nd = mover == P ? 0 : 2;  // digit of the new stone wrt P
                int delta = 0;
#pragma unroll
                for (int d = 0; d < 4; d++) {
#pragma unroll
                    for (int k = -4; k <= 4; k++) {
                        if (k == 0) continue;
                        const int rr = r + k * DR[d], cc = c + k * DC[d];
                        if (rr < 0 || rr >= GZ_N || cc < 0 || cc >= GZ_N) continue;
                        if (!bb_test(Pst, rr * 16 + cc)) continue;
                        const int code = sh->code[rr * GZ_N + cc][d];
                        const int j = 4 - k;  // m's slot in the window of the stone at offset k
                        const int i = j < 4 ? j : j - 1;
                        delta += GZ_PATTERN_LUT[code + (nd - 1) * pow3(i)] - GZ_PATTERN_LUT[code];
                    }
                    if (mover == P) delta += GZ_PATTERN_LUT[sh->code[cell][d]];
                }
                const int dist = (r > 7 ? r - 7 : 7 - r) + (c > 7 ? c - 7 : 7 - c);
                const double cb = (6 - dist) * 0.5;
                score = (double)(base + delta) + (cb > 0.0 ? cb : 0.0);
            }
        }
        sc[s] = score;
    }
    return ne;
}

__device__ int planner_pick(PlanShared* sh, const BB& black, const BB& white, int mover, int n_moves, int P,
                            const gz_planner_params& pp, const float* __restrict__ pv, const float* __restrict__ qv,
                            uint64_t key, uint32_t* cnt) {
    const int lane = lane_id();
    double sc[4];
    int cl[4];
#pragma unroll
    for (int s = 0; s < 4; s++) cl[s] = lane + 64 * s;
    const int ne = knowledge_scores(sh, black, white, mover, n_moves, P, sc);
    // top-k: Python's stable sort, descending (score desc, row-major asc)
    const int m = ne < pp.k ? ne : pp.k;
    for (int rnk = 0; rnk < m; rnk++) {
        double bv = -__builtin_inf();
        int bi = INT_MAX;
#pragma unroll
        for (int s = 0; s < 4; s++)
            if (sc[s] > bv || (sc[s] == bv && cl[s] < bi && sc[s] != -__builtin_inf())) {
                bv = sc[s];
                bi = cl[s];
            }
        wave_argmax(bv, bi);
#pragma unroll
        for (int s = 0; s < 4; s++)
            if (cl[s] == bi) sc[s] = -__builtin_inf();
        if (lane == 0) sh->top[rnk] = bi;
    }
    __syncthreads();
    // compose: first strict maximum of alpha*p - (1-alpha)*q in top-k order (fp64)
    double cv = -__builtin_inf();
    int ci = INT_MAX;
    if (lane < m) {
        const int cell = sh->top[lane];
        cv = pp.alpha * (double)pv[cell] - (1 - pp.alpha) * (double)qv[cell];
        ci = lane;
    }
    wave_argmax(cv, ci);
    int best = sh->top[ci];
    if (to_unit(draw(key, (*cnt)++)) < pp.explore) best = sh->top[below(draw(key, (*cnt)++), (uint32_t)m)];
    __syncthreads();
    return best;
}

// planner_pick with PW waves: the window codes and the cells' scores one cell per
// thread (the heavy part, 4 cells per lane with one wave), then wave 0 alone as
// planner_pick: top-k, compose, explore -- the same scores, so the same move and draws.
// Returns the move in wave 0 (-1 elsewhere).
__device__ int planner_pick4(PlanShared4* sh4, const BB& black, const BB& white, int mover, int n_moves, int P,
                             const gz_planner_params& pp, const float* __restrict__ pv, const float* __restrict__ qv,
                             uint64_t key, uint32_t* cnt) {
    PlanShared* sh = &sh4->s;
    const int lane = lane_id(), wave = threadIdx.x / WAVE, t = threadIdx.x;
    const KsCtx k = ks_ctx(black, white, mover, n_moves, P);
    for (int idx = t; idx < GRID_CELLS; idx += PW * WAVE) {
        const int r = idx / GRID_W - 4, c = idx % GRID_W - 4;
        uint8_t v = 3;
        if (r >= 0 && r < GZ_N && c >= 0 && c < GZ_N) {
            const int b = r * 16 + c;
            v = bb_test(black, b) ? 1 : (bb_test(white, b) ? 2 : 0);
        }
        sh->grid[idx] = v;
    }
    __syncthreads();
    const int part = t < GZ_CELLS ? cell_codes(sh, t, k.Pst, P) : 0;
    const long long wp = wave_sum_ll(part);
    if (lane == 0) sh4->part[wave] = (int)wp;
    __syncthreads();
    int base = 0;
#pragma unroll
    for (int w = 0; w < PW; w++) base += sh4->part[w];
    sh4->sc[t] = cell_score(sh, t, k, base);
    __syncthreads();
    int best = -1;
    if (wave == 0) {
        double sc[4];
        int cl[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
            cl[s] = lane + 64 * s;
            sc[s] = sh4->sc[cl[s]];
        }
        // top-k: Python's stable sort, descending (score desc, row-major asc)
        const int m = k.ne < pp.k ? k.ne : pp.k;
        for (int rnk = 0; rnk < m; rnk++) {
            double bv = -__builtin_inf();
            int bi = INT_MAX;
#pragma unroll
            for (int s = 0; s < 4; s++)
                if (sc[s] > bv || (sc[s] == bv && cl[s] < bi && sc[s] != -__builtin_inf())) {
                    bv = sc[s];
                    bi = cl[s];
                }
            wave_argmax(bv, bi);
#pragma unroll
            for (int s = 0; s < 4; s++)
                if (cl[s] == bi) sc[s] = -__builtin_inf();
            if (lane == 0) sh->top[rnk] = bi;
        }
        // (the top-k list is this wave's: its LDS writes are visible to it)
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        // compose: first strict maximum of alpha*p - (1-alpha)*q in top-k order (fp64)
        double cv = -__builtin_inf();
        int ci = INT_MAX;
        if (lane < m) {
            const int cell = sh->top[lane];
            cv = pp.alpha * (double)pv[cell] - (1 - pp.alpha) * (double)qv[cell];
            ci = lane;
        }
        wave_argmax(cv, ci);
        best = sh->top[ci];
        if (to_unit(draw(key, (*cnt)++)) < pp.explore) best = sh->top[below(draw(key, (*cnt)++), (uint32_t)m)];
    }
    return best;
}

// ---------------------------------------------------------------- kernels
// root + root children + one job per parallel simulation (mcts() of gz_selfplay.hip)
__global__ __launch_bounds__(WAVE) void plan_begin_kernel(const gz_board_state* boards, const int64_t* game_ids, int n,
                                                          gz_search_params p, Workspace w, LeafSink sink, int gather) {
    __shared__ uint8_t grid[GRID_BYTES];
    const int g = blockIdx.x;
    if (g >= n) return;
    const int lane = lane_id();
    const int S = p.num_simulations;
    PlanCtx* cx = ctx_at(w, g, S);
    Tree t = ctx_tree(cx, S);
    if (lane == 0) cx->root_leaf = -1;
    const gz_board_state bs = boards[g];
    BB black, white;
    load_bb(black, bs.black);
    load_bb(white, bs.white);
    const int player = bs.player, n_moves = bs.n_moves;
    const int64_t game_id = game_ids[g];
    const BB E = empties(black, white);
    const int L = bb_count(E);
    const BB me = player == 1 ? black : white, op = player == 1 ? white : black;
    const BB Wm = threats(me).win & E;
    const uint64_t kmain = stream_key(p.seed, game_id, n_moves, 0);
    uint32_t dm = 0;
    int move = -1, phase = 0, n_par = 0, predicts = 0;
    if (!bs.over && L > 0) {
        if (n_moves == 0 && bb_test(E, 7 * 16 + 7)) {
            move = 7 * GZ_N + 7;
        } else {
            bool search = true;
            if (n_moves < 6) {  // _opening_move, ai_agent.py:138-166
                const BB k3 = GZ_MASK_K3, k5 = GZ_MASK_K5;
                BB s = k3 & E;
                if (!bb_any(s)) s = k5 & E;
                if (bb_any(s)) {
                    move = bit_to_cell(select_bit(s, (int)below(draw(kmain, dm++), (uint32_t)bb_count(s))));
                    search = false;
                }
            }
            if (search) {
                const bool use_bg = p.beta != 0.0;
                n_par = S < L + 1 ? S : L + 1;
                if (use_bg) write_grid(grid, black, white);
                if (lane == 0) {
                    t.parent[0] = -1;
                    t.move[0] = 255;
                    t.term[0] = 0;
                    t.bound[0] = 256;
                    t.visits[0] = 0;
                    t.value[0] = 0.0;
                    t.bg[0] = 0.0;
                }
                int nonterm = 0;
                for (int base = 1; base < n_par; base += WAVE) {
                    const int j = base + lane;
                    const bool valid = j < n_par;
                    int term = 0;
                    if (valid) {
                        const int bit = select_bit(E, L - j);
                        const bool win = bb_test(Wm, bit);
                        term = win ? player : ((n_moves + 1 >= 200 || L == 1) ? 3 : 0);
                        t.parent[j] = 0;
                        t.move[j] = (uint8_t)bit_to_cell(bit);
                        t.term[j] = (uint8_t)term;
                        t.bound[j] = 256;
                        t.visits[j] = term ? 1 : 0;
                        t.value[j] = term ? term_value(term, player) : 0.0;
                        double bgv = 0.0;
                        if (use_bg) {
                            BB ps = me;
                            bb_set(ps, bit);
                            bgv = bg_from_score(pattern_score_lane(grid, ps, player, grid_index_of_bit(bit)));
                        }
                        t.bg[j] = bgv;
                        PlanJob& jb = w.jobs[(size_t)g * S + j];
                        if (!term) {
                            BB cb = op, cm = me;
                            bb_set(cm, bit);
                            job_set(jb, player == 1 ? cm : cb, player == 1 ? cb : cm, n_moves + 1, 3 - player, player,
                                    stream_key(p.seed, game_id, n_moves, j + 1), g, j + 1);
                        } else {
                            jb.state = 0;
                        }
                    }
                    nonterm += __popcll(ballot(valid && term == 0));
                }
                __syncthreads();
                predicts = 1 + nonterm;
                if (gather) {
                    const int bidx = leaf_reserve(sink, 1 + nonterm);
                    if (lane == 0) {
                        leaf_write(sink, bidx, black, white);
                        leaf_meta(sink, bidx, -1);
                        cx->root_leaf = bidx;
                    }
                    int off = 1;
                    for (int base = 1; base < n_par; base += WAVE) {
                        const int j = base + lane;
                        const bool live = j < n_par && t.term[j] == 0;
                        const uint64_t msk = ballot(live);
                        if (live) {
                            const int bit = cell_to_bit(t.move[j]);
                            BB cbk = black, cwh = white;
                            if (player == 1) bb_set(cbk, bit);
                            else bb_set(cwh, bit);
                            leaf_write(sink, bidx + off + rank_in(msk), cbk, cwh);
                            leaf_meta(sink, bidx + off + rank_in(msk), bidx);
                        }
                        off += __popcll(msk);
                    }
                }
                if (lane == 0) {
                    if (n_par >= 2) t.bound[0] = (int16_t)cell_to_bit(t.move[n_par - 1]);
                    if (n_par >= 1)  // simulation 1: rollout from the root
                        job_set(w.jobs[(size_t)g * S], black, white, n_moves, player, player,
                                stream_key(p.seed, game_id, n_moves, 1), g, 1);
                }
                phase = n_par >= 1 ? 1 : 0;
                if (n_par == 0)  // no simulation: _mcts_search's no-children fallback (:204)
                    move = bit_to_cell(select_bit(E, (int)below(draw(kmain, dm++), (uint32_t)L)));
            }
        }
    }
    if (lane == 0) {
        store_bb(cx->black, black);
        store_bb(cx->white, white);
        cx->game_id = game_id;
        cx->sim_draws = 0;
        cx->n_moves = n_moves;
        cx->player = player;
        cx->L = L;
        cx->n_par = n_par;
        cx->phase = phase;
        cx->k = n_par + 1;
        cx->x = -1;
        cx->n_nodes = n_par;
        cx->predicts = predicts;
        cx->main_draws = 0;
        cx->move = move;
        cx->dm = dm;
        if (phase) atomicAdd(&w.ctr->pending, 1);
    }
}

// jobs [j0, j1) in their planner plies -> GN rows; jobs past them -> rollout.
// inc: also tag each row for the incremental GraphNet (gn_inc_kernel): a rollout's
// first board that is the search root plus one stone, and every later planner ply's
// board (its predecessor plus the planner's move), add one stone to maps that are
// kept; any other board runs the full forward and keeps its maps in the job's slot.
// Job slot: n + (job - j0) in round 0's chunks (slot_game 0), n + game afterwards
// (one job per game).
// one atomic per wave: lane's slot among the wave's `take` lanes in *ctr's range
__device__ inline int wave_slot(bool take, int32_t* ctr) {
    const uint64_t m = ballot(take);
    if (!m) return -1;
    const int lane = lane_id(), leader = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(ctr, __popcll(m));
    base = __shfl(base, leader);
    return take ? base + __popcll(m & ((1ull << lane) - 1)) : -1;
}

__global__ void plan_collect_kernel(Workspace w, int S, int n, int j0, int count, int stride, int planner_steps,
                                    int final_round, int inc, int slot_game) {
    // (every lane reaches the wave-wide slot allocations: no early returns)
    const int t_ = blockIdx.x * blockDim.x + threadIdx.x;
    const int i = j0 + t_ * stride;
    PlanJob* jp = t_ < count ? &w.jobs[i] : nullptr;
    const bool st1 = jp && jp->state == 1;
    // (a planner move that ends the game sets state 3 itself, in plan_step_kernel)
    const bool want = st1 && !final_round && jp->steps < planner_steps;
    if (st1 && !want) jp->state = 2;
    const int row = wave_slot(want, &w.ctr->rows);
    GnTag t;
    t.mode = -1;
    if (want) {
        PlanJob& j = *jp;
        BB black, white;
        load_bb(black, j.black);
        load_bb(white, j.white);
        j.row = row;
        w.rows[row] = i;
        uint4* dst = (uint4*)(w.gn_in + (size_t)row * 16);
        dst[0] = make_uint4(black.w[0], black.w[1], black.w[2], black.w[3]);
        dst[1] = make_uint4(black.w[4], black.w[5], black.w[6], black.w[7]);
        dst[2] = make_uint4(white.w[0], white.w[1], white.w[2], white.w[3]);
        dst[3] = make_uint4(white.w[4], white.w[5], white.w[6], white.w[7]);
        if (inc) {
            t.job = n + (slot_game ? j.game : t_);
            t.mode = 1;
            t.nst = 0;
            t.cell = -1;
            if (j.steps == 0) {  // one stone from the root?
                const PlanCtx* cx = ctx_at(w, j.game, S);
                BB rb, rw;
                load_bb(rb, cx->black);
                load_bb(rw, cx->white);
                int nd = 0, bit = -1;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    const uint32_t db = black.w[k] ^ rb.w[k], dw = white.w[k] ^ rw.w[k];
                    nd += __popc(db) + __popc(dw);
                    const uint32_t add = (db & black.w[k]) | (dw & white.w[k]);
                    if (add) bit = k * 32 + __ffs(add) - 1;
                }
                if (nd == 1 && bit >= 0) {
                    t.cell = bit_to_cell(bit);
                    t.base = j.game;
                    j.bj = 0;
                    j.nst = 0;
                } else {
                    t.mode = 0;
                }
            } else if (j.bj) {  // the job's own full maps
                t.cell = j.pend;
                t.base = t.job;
            } else if (j.nst < gzgn::TAG_STONES) {  // the root's maps + the job's squares
                t.cell = j.pend;
                t.base = j.game;
                t.nst = j.nst;
#pragma unroll
                for (int k = 0; k < gzgn::TAG_STONES; k++) t.st[k] = j.st[k];
            } else {
                t.mode = 0;
            }
            if (t.mode == 0) {
                t.base = t.job;
                j.bj = 1;
                j.nst = 0;
            } else if (!j.bj) {
                j.st[j.nst++] = (uint8_t)t.cell;
            }
            w.tags[row] = t;
        }
    }
    if (inc) {
        const int f = wave_slot(t.mode == 0, &w.ctr->nfull), k = wave_slot(t.mode == 1, &w.ctr->ninc);
        if (f >= 0) w.full_list[f] = row;
        if (k >= 0) w.inc_list[k] = row;
    }
}

// GZ_FLAG_GN_CHECK: rows whose incremental record (policy-conv outputs), p or q
// differ in any bit from the full forward's
__global__ void plan_gn_check_kernel(Workspace w) {
    const int row = blockIdx.x;
    if (row >= w.ctr->rows) return;
    bool bad = false;
    for (int e = threadIdx.x; e < 450; e += blockDim.x)
        bad |= __float_as_uint(w.gn_rec[(size_t)row * 928 + e]) != __float_as_uint(w.chk_rec[(size_t)row * 928 + e]);
    for (int e = threadIdx.x; e < 225; e += blockDim.x) {
        bad |= __float_as_uint(w.gn_p[(size_t)row * 225 + e]) != __float_as_uint(w.chk_p[(size_t)row * 225 + e]);
        bad |= __float_as_uint(w.gn_q[(size_t)row * 225 + e]) != __float_as_uint(w.chk_q[(size_t)row * 225 + e]);
    }
    bad = __syncthreads_or(bad);
    if (threadIdx.x == 0) {
        atomicAdd((unsigned long long*)&w.stats->checked, 1ull);
        if (bad) atomicAdd((unsigned long long*)&w.stats->mismatch, 1ull);
    }
}

// one planner ply (BGPlannerAI.get_move + make_move) per collected row
// (at least 3 waves per SIMD: 178 -> 168 VGPRs, config 4 +4.5 %)
__global__ void plan_gn_count_kernel(Workspace w) {
    atomicAdd((unsigned long long*)&w.stats->full, (unsigned long long)w.ctr->nfull);
    atomicAdd((unsigned long long*)&w.stats->inc, (unsigned long long)w.ctr->ninc);
}

// one planner ply of row blockIdx.x; with PW waves (count_rows) it also adds the
// incremental planner nets' row counts to the search statistics (the GN forward of this
// step is complete): plan_gn_count_kernel without a launch (in the one-wave kernel the
// atomics cost it 30 more spilled registers)
template <int NWV, class SH>
__device__ __forceinline__ void plan_step_row(Workspace& w, const gz_planner_params& pp, int count_rows, SH* sh) {
    const int row = blockIdx.x;
    if (NWV > 1 && count_rows && row == 0 && threadIdx.x == 0) {
        atomicAdd((unsigned long long*)&w.stats->full, (unsigned long long)w.ctr->nfull);
        atomicAdd((unsigned long long*)&w.stats->inc, (unsigned long long)w.ctr->ninc);
    }
    if (row >= w.ctr->rows) return;
    PlanJob& j = w.jobs[w.rows[row]];
    BB black, white;
    load_bb(black, j.black);
    load_bb(white, j.white);
    const int mover = j.mover, n_moves = j.n_moves, P = j.ai;
    uint32_t cnt = j.cnt;
    int mv;
    if constexpr (NWV == 1)
        mv = planner_pick(sh, black, white, mover, n_moves, P, pp, w.gn_p + (size_t)row * 225,
                          w.gn_q + (size_t)row * 225, j.key, &cnt);
    else
        mv = planner_pick4(sh, black, white, mover, n_moves, P, pp, w.gn_p + (size_t)row * 225,
                           w.gn_q + (size_t)row * 225, j.key, &cnt);
    if (threadIdx.x == 0) {  // make_move (gomoku_board.py:84-113)
        const int bit = cell_to_bit(mv);
        BB& mine = mover == 1 ? black : white;
        const BB E = empties(black, white);
        const bool win = bb_test(threats(mine).win, bit);
        const int ne = bb_count(E);
        bb_set(mine, bit);
        store_bb(j.black, black);
        store_bb(j.white, white);
        j.n_moves = (int16_t)(n_moves + 1);
        j.mover = (int8_t)(3 - mover);
        j.cnt = cnt;
        j.steps = (int8_t)(j.steps + 1);
        j.pend = (uint8_t)mv;
        if (win || ne == 1 || n_moves + 1 >= 200) {  // game over: straight to the value
            j.state = 3;
            j.value = win ? (mover == P ? 1.0 : -1.0) : 0.1;
        }
        j.row = -1;
    }
}
// large launches (round 0): a wave per row, at least 3 waves per SIMD (178 -> 168
// VGPRs, config 4 +4.5 %)
__global__ __launch_bounds__(WAVE) __attribute__((amdgpu_waves_per_eu(3, 8))) void plan_step_kernel(
    Workspace w, gz_planner_params pp, int count_rows) {
    __shared__ PlanShared sh;
    plan_step_row<1>(w, pp, count_rows, &sh);
}
// small launches (the sequential rounds: a row per game): PW waves per row
__global__ __launch_bounds__(PW * WAVE) void plan_step4_kernel(Workspace w, gz_planner_params pp, int count_rows,
                                                               Counters* next) {
    __shared__ PlanShared4 sh;
    // the next planner step's counters (the other set: every kernel of the step that used
    // it is done) -- hipMemsetAsync's work, without a launch
    if (blockIdx.x == 0 && threadIdx.x < 4) (&next->rows)[threadIdx.x] = 0;  // rows, nfull, ninc, ihead (not pending)
    plan_step_row<PW>(w, pp, count_rows, &sh);
}

// offensive rollout (_simulate :276-285) of every job past its planner plies
__global__ void plan_rollout_kernel(Workspace w, int count, int stride, int max_depth) {
    const int t_ = blockIdx.x * blockDim.x + threadIdx.x;
    if (t_ >= count) return;
    const int i = t_ * stride;
    PlanJob& j = w.jobs[i];
    if (j.state != 2) return;
    BB black, white;
    load_bb(black, j.black);
    load_bb(white, j.white);
    uint32_t cnt = j.cnt;
    RolloutResult r = rollout(black, white, j.n_moves, j.mover, j.ai, max_depth, j.key, &cnt, j.steps);
    j.value = r.value;
    j.cnt = cnt;
    j.state = 3;
}

// back up, then sequential simulations until one needs a rollout (or the search ends)
__global__ __launch_bounds__(WAVE) void plan_resume_kernel(int n, gz_search_params p, Workspace w, LeafSink sink,
                                                           int gather, int32_t* moves, gz_search_stats* stats) {
    __shared__ uint8_t grid[GRID_BYTES];
    const int g = blockIdx.x;
    if (g >= n) return;
    const int lane = lane_id();
    const int S = p.num_simulations;
    PlanCtx* cx = ctx_at(w, g, S);
    Tree t = ctx_tree(cx, S);
    int phase = cx->phase;
    if (phase == 0) return;
    const int player = cx->player, n_moves = cx->n_moves, L = cx->L, n_par = cx->n_par;
    const int64_t game_id = cx->game_id;
    BB rblack, rwhite;
    load_bb(rblack, cx->black);
    load_bb(rwhite, cx->white);
    const bool use_bg = p.beta != 0.0;
    long long draws = 0;
    int n_nodes = cx->n_nodes, k = cx->k, predicts = cx->predicts;
    if (phase == 1) {  // parallel phase: every child got one update; the root sums in order
        for (int s = 1 + lane; s <= n_par; s += WAVE) {
            const PlanJob& j = w.jobs[(size_t)g * S + (s - 1)];
            if (s == 1 || t.term[s - 1] == 0) draws += j.cnt;
            if (s > 1 && t.term[s - 1] == 0) {
                t.value[s - 1] = j.value;
                t.visits[s - 1] = 1;
            }
        }
        __syncthreads();
        if (lane == 0) {
            double acc = w.jobs[(size_t)g * S].value;
            for (int j = 1; j < n_par; j++) acc += t.value[j];
            t.value[0] = acc;
            t.visits[0] = n_par;
        }
        __syncthreads();
    } else {  // the pending sequential simulation
        const PlanJob& j = w.jobs[(size_t)g * S];
        if (lane == 0) {
            draws += j.cnt;
            const double v = j.value;
            for (int y = cx->x; y >= 0; y = t.parent[y]) {
                t.visits[y] += 1;
                t.value[y] += v;
            }
        }
        k++;
        __syncthreads();
    }
    draws = wave_sum_ll(draws);
    phase = 0;
    for (; k <= S; k++) {
        int x = 0;
        BB cbk = rblack, cwh = rwhite;
        int cm = player, cn = n_moves;
        while (true) {  // _select, ai_agent.py:224-232
            if (t.term[x]) break;
            if (highest_bit_below(empties(cbk, cwh), t.bound[x]) >= 0) break;
            int pv = t.visits[x];
            pv = pv < 1 ? 1 : pv;
            const double lg = GZ_LOG_TABLE[pv];
            const double mlog = lg > 1.0 ? lg : 1.0;
            double bv = -__builtin_inf();
            int bi = INT_MAX;
            for (int i = 1 + lane; i < n_nodes; i += WAVE) {
                if (t.parent[i] == x) {
                    const double u = ucb1(t, i, mlog, p);
                    if (u > bv || bi == INT_MAX) {
                        bv = u;
                        bi = i;
                    }
                }
            }
            wave_argmax(bv, bi);
            if (bi == INT_MAX) break;
            x = bi;
            const int bit = cell_to_bit(t.move[x]);
            if (cm == 1) bb_set(cbk, bit);
            else bb_set(cwh, bit);
            cm = 3 - cm;
            cn++;
        }
        if (!t.term[x] && t.visits[x] > 0) {  // _expand, ai_agent.py:234-249
            const BB ex = empties(cbk, cwh);
            const int hb = highest_bit_below(ex, t.bound[x]);
            if (hb >= 0) {
                const int c = n_nodes++;
                const bool win = bb_test(threats(cm == 1 ? cbk : cwh).win, hb);
                const int term = win ? cm : ((cn + 1 >= 200 || bb_count(ex) == 1) ? 3 : 0);
                __syncthreads();
                if (lane == 0) {
                    t.bound[x] = (int16_t)hb;
                    t.parent[c] = (int16_t)x;
                    t.move[c] = (uint8_t)bit_to_cell(hb);
                    t.term[c] = (uint8_t)term;
                    t.bound[c] = 256;
                    t.visits[c] = 0;
                    t.value[c] = 0.0;
                    t.bg[c] = 0.0;
                }
                if (cm == 1) bb_set(cbk, hb);
                else bb_set(cwh, hb);
                cm = 3 - cm;
                cn++;
                if (use_bg) {
                    write_grid(grid, cbk, cwh);
                    if (lane == 0)
                        t.bg[c] = bg_from_score(pattern_score_lane(grid, player == 1 ? cbk : cwh, player, -1));
                }
                if (term == 0) {
                    predicts++;
                    if (gather) {
                        const int bidx = leaf_reserve(sink, 1);
                        // a child of a root child: its parent's leaf index (root + 1 + the
                        // parent's rank among the live root children), as mcts() does
                        int tag = -2;
                        const int rl = cx->root_leaf, np = cx->n_par;
                        if (sink.meta && rl >= 0 && x >= 1 && x < np) {
                            int rank = 0;
                            for (int base = 1; base < x; base += WAVE) {
                                const int j = base + lane;
                                rank += __popcll(ballot(j < x && t.term[j] == 0));
                            }
                            if (rl + 1 + rank < sink.cap) tag = rl + 1 + rank;
                        }
                        if (lane == 0) {
                            leaf_write(sink, bidx, cbk, cwh);
                            leaf_meta(sink, bidx, tag);
                        }
                    }
                }
                x = c;
                __syncthreads();
            }
        }
        const int tx = t.term[x];
        if (tx) {  // _simulate on a terminal node: no rollout
            const double v = term_value(tx, player);
            if (lane == 0)
                for (int y = x; y >= 0; y = t.parent[y]) {
                    t.visits[y] += 1;
                    t.value[y] += v;
                }
            __syncthreads();
            continue;
        }
        if (lane == 0) {
            job_set(w.jobs[(size_t)g * S], cbk, cwh, cn, cm, player, stream_key(p.seed, game_id, n_moves, k), g, k);
            cx->x = x;
        }
        phase = 2;
        break;
    }
    if (lane == 0) {
        cx->sim_draws += draws;
        cx->n_nodes = n_nodes;
        cx->predicts = predicts;
        cx->k = k;
        cx->phase = phase;
        if (phase) atomicAdd(&w.ctr->pending, 1);
    }
    if (phase == 0) {  // result: first root child with the most visits; exploration (ai_agent.py:128-129,199-204)
        const uint64_t kmain = stream_key(p.seed, game_id, n_moves, 0);
        uint32_t dm = cx->dm;
        const BB E = empties(rblack, rwhite);
        int best;
        if (n_par >= 2) {
            int bv = -1, bi = INT_MAX;
            for (int j = 1 + lane; j < n_par; j += WAVE) {
                const int v = t.visits[j];
                if (v > bv) {
                    bv = v;
                    bi = j;
                }
            }
            wave_argmax_int(bv, bi);
            best = t.move[bi];
        } else {
            best = bit_to_cell(select_bit(E, (int)below(draw(kmain, dm++), (uint32_t)L)));
        }
        if (n_moves >= 6 && to_unit(draw(kmain, dm++)) < p.exploration)
            best = bit_to_cell(select_bit(E, (int)below(draw(kmain, dm++), (uint32_t)L)));
        if (lane == 0) {
            cx->move = best;
            cx->dm = dm;
        }
    }
}

// final outputs (and the tree in gz_search's layout when requested)
__global__ __launch_bounds__(WAVE) void plan_finish_kernel(int n, int S, Workspace w, int32_t* moves,
                                                           gz_search_stats* stats, char* trees) {
    const int g = blockIdx.x;
    if (g >= n) return;
    PlanCtx* cx = ctx_at(w, g, S);
    const int lane = lane_id();
    if (trees) {
        const size_t tb = tree_bytes_for(S);
        const uint32_t* src = (const uint32_t*)((char*)cx + sizeof(PlanCtx));
        uint32_t* dst = (uint32_t*)(trees + (size_t)g * tb);
        for (size_t i = lane; i < tb / 4; i += WAVE) dst[i] = src[i];
    }
    if (lane == 0) {
        moves[g] = cx->move;
        if (stats) {
            gz_search_stats st;
            st.n_nodes = cx->n_nodes;
            st.predicts = cx->predicts;
            st.main_draws = (int32_t)cx->dm;
            st.pad = 0;
            st.sim_draws = cx->sim_draws;
            stats[g] = st;
        }
    }
}

// BGPlannerAI.get_move on a batch of boards (no search): GN rows are the boards
__global__ __launch_bounds__(WAVE) void planner_move_kernel(const gz_board_state* boards, const int32_t* ai,
                                                            const uint64_t* keys, int n, gz_planner_params pp,
                                                            const float* gp, const float* gq, int32_t* moves,
                                                            uint32_t* draws) {
    __shared__ PlanShared sh;
    const int i = blockIdx.x;
    if (i >= n) return;
    const gz_board_state b = boards[i];
    BB black, white;
    load_bb(black, b.black);
    load_bb(white, b.white);
    uint32_t cnt = 0;
    int mv = -1;
    if (bb_any(empties(black, white)))
        mv = planner_pick(&sh, black, white, b.player, b.n_moves, ai[i], pp, gp + (size_t)i * 225,
                          gq + (size_t)i * 225, keys[i], &cnt);
    if (lane_id() == 0) {
        moves[i] = mv;
        draws[i] = cnt;
    }
}

// KnowledgeSearch.score_move for every cell of every board (bg_planner.py:90-106):
// -1e9 where the move is invalid (occupied), as the reference returns
__global__ __launch_bounds__(WAVE) void knowledge_scores_kernel(const gz_board_state* boards, const int32_t* player,
                                                                int n, double* scores) {
    __shared__ PlanShared sh;
    const int i = blockIdx.x;
    if (i >= n) return;
    const gz_board_state b = boards[i];
    BB black, white;
    load_bb(black, b.black);
    load_bb(white, b.white);
    double sc[4];
    knowledge_scores(&sh, black, white, b.player, b.n_moves, player[i], sc);
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const int cell = lane_id() + 64 * s;
        if (cell < GZ_CELLS) scores[(size_t)i * GZ_CELLS + cell] = sc[s] == -__builtin_inf() ? -1e9 : sc[s];
    }
}

__global__ void boards_to_rows_kernel(const gz_board_state* boards, int n, uint32_t* rows) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int k = 0; k < 8; k++) {
        rows[(size_t)i * 16 + k] = boards[i].black[k];
        rows[(size_t)i * 16 + 8 + k] = boards[i].white[k];
    }
}

}  // namespace

extern "C" void gz_internal_set_error(const char* msg);
extern "C" int gz_gn_forward(const float* d_weights, const uint32_t* d_boards, int32_t n, const int32_t* d_count,
                             float* d_p, float* d_q, float* d_logits, void* d_workspace, void* stream);
extern "C" size_t gz_gn_workspace_bytes(int32_t n);
extern "C" int gz_internal_gn_roots(const float* d_weights, const uint32_t* d_rows, int32_t n, void* d_slots,
                                    float* d_rec, void* stream);
extern "C" int gz_internal_gn_forward_tagged(const float* d_weights, const uint32_t* d_rows, int32_t max_rows,
                                             const int32_t* d_count, const int32_t* d_full_list,
                                             const int32_t* d_full_count, const int32_t* d_inc_list,
                                             const int32_t* d_inc_count, const void* d_tags, void* d_slots,
                                             float* d_p, float* d_q, float* d_rec, float* d_hscratch,
                                             int32_t* d_queue, void* stream);

static int plan_fail(int code, const char* msg) {
    gz_internal_set_error(msg);
    return code;
}

static int plan_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return plan_fail(GZ_ERR_HIP, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
    return GZ_OK;
}

extern "C" size_t gz_plan_workspace_bytes(int32_t n, int32_t num_simulations) {
    return workspace_bytes(n < 1 ? 1 : n, num_simulations);
}

// gz_plan_search with optional leaf tags (d_leaf_meta, [leaf_cap]: gz_selfplay_plan_run)
extern "C" int gz_internal_plan_search(const gz_board_state* d_boards, const int64_t* d_game_ids, int32_t n,
                                       const gz_search_params* p, const gz_planner_params* pp,
                                       const float* d_gn_weights, void* d_workspace, void* d_trees, int32_t* d_moves,
                                       gz_search_stats* d_stats, uint32_t* d_leaves, int32_t leaf_cap,
                                       int32_t* d_leaf_count, int32_t* d_leaf_meta, void* stream) {
    if (!p || !pp) return plan_fail(GZ_ERR_ARG, "gz_plan_search: params are NULL");
    if (p->num_simulations < 1 || p->num_simulations > GZ_MAX_SIMULATIONS)
        return plan_fail(GZ_ERR_ARG, "gz_plan_search: num_simulations out of range [1, 4095]");
    if (p->planner_steps < 0 || p->planner_steps > 100 || pp->k < 1 || pp->k > 16)
        return plan_fail(GZ_ERR_ARG, "gz_plan_search: planner_steps must be in [0, 100] and k in [1, 16]");
    if (n < 0 || (n > 0 && (!d_boards || !d_game_ids || !d_moves || !d_workspace || !d_gn_weights)))
        return plan_fail(GZ_ERR_ARG, "gz_plan_search: bad arguments");
    const bool gather = (p->flags & GZ_FLAG_GATHER_LEAVES) != 0;
    if (gather && (!d_leaves || !d_leaf_count || leaf_cap < 0))
        return plan_fail(GZ_ERR_ARG, "gz_plan_search: leaf gathering needs d_leaves and d_leaf_count");
    if (n == 0) return GZ_OK;
    if (gz_gn_workspace_bytes(1) != GN_WS_BYTES)
        return plan_fail(GZ_ERR_INTERNAL, "gz_plan_search: planner-net record size mismatch");
    hipStream_t s = (hipStream_t)stream;
    const int S = p->num_simulations;
    Workspace w = carve(d_workspace, n, S);
    LeafSink sink{d_leaves, leaf_cap, d_leaf_count, gather ? d_leaf_meta : nullptr};
    const int n_jobs = n * S;
    const int C = (int)chunk_rows(n, S);
    // incremental GraphNet (gn_inc_kernel) unless GZ_GN_INC=0; GZ_FLAG_GN_CHECK also
    // runs the full forward on every row and counts the rows that differ
    const char* env = getenv("GZ_GN_INC");
    const bool inc = p->planner_steps > 0 && !(env && env[0] == '0');
    const bool check = inc && (p->flags & GZ_FLAG_GN_CHECK) != 0;
    int rc;
    if (hipMemsetAsync(w.ctr, 0, 2 * sizeof(Counters), s) != hipSuccess)
        return plan_fail(GZ_ERR_HIP, "gz_plan_search: memset");
    if (hipMemsetAsync(w.jobs, 0, sizeof(PlanJob) * (size_t)n_jobs, s) != hipSuccess)
        return plan_fail(GZ_ERR_HIP, "gz_plan_search: memset");
    plan_begin_kernel<<<n, WAVE, 0, s>>>(d_boards, d_game_ids, n, *p, w, sink, gather ? 1 : 0);
    if ((rc = plan_check("plan_begin_kernel"))) return rc;
    if (inc) {  // the roots' maps and policy-conv outputs -> root slots 0..n-1
        boards_to_rows_kernel<<<(n + 255) / 256, 256, 0, s>>>(d_boards, n, w.gn_in);
        if ((rc = plan_check("boards_to_rows_kernel"))) return rc;
        if ((rc = gz_internal_gn_roots(d_gn_weights, w.gn_in, n, w.slots, w.gn_rec, stream))) return rc;
    }
    // one planner step over jobs [j0, j1): collect -> GraphNet + DQN -> planner move
    // planner step k uses counter set k & 1 (rows, nfull, ninc; pending is w.ctr's, read
    // only around resume); the set is zeroed by the previous step's plan_step4_kernel, or
    // here when that step ran the one-wave kernel
    int step_no = 0;
    bool zeroed = true;  // (both sets cleared above)
    auto planner_step = [&](int j0, int j1, int max_rows, int slot_game) -> int {
        int r;
        Workspace wk = w;
        wk.ctr = (step_no & 1) ? w.ctr2 : w.ctr;
        Counters* next = (step_no & 1) ? w.ctr : w.ctr2;
        step_no++;
        // rows, nfull, ninc, ihead (pending is left alone: the resume's own memset clears it)
        if (!zeroed && hipMemsetAsync(&wk.ctr->rows, 0, 4 * sizeof(int32_t), s) != hipSuccess)
            return plan_fail(GZ_ERR_HIP, "memset");
        // jobs j0 .. j1-1 (round 0's chunk), or (slot_game) the one job per game at g * S
        const int cnt = slot_game ? n : j1 - j0, stride = slot_game ? S : 1;
        plan_collect_kernel<<<(cnt + 255) / 256, 256, 0, s>>>(wk, S, n, j0, cnt, stride, p->planner_steps, 0,
                                                               inc ? 1 : 0, slot_game);
        if ((r = plan_check("plan_collect_kernel"))) return r;
        if (!inc) {
            if ((r = gz_gn_forward(d_gn_weights, w.gn_in, max_rows, &wk.ctr->rows, w.gn_p, w.gn_q, nullptr, w.gn_rec,
                                   stream)))
                return r;
        } else {
            if ((r = gz_internal_gn_forward_tagged(d_gn_weights, w.gn_in, max_rows, &wk.ctr->rows, w.full_list,
                                                   &wk.ctr->nfull, w.inc_list, &wk.ctr->ninc, w.tags, w.slots, w.gn_p,
                                                   w.gn_q, w.gn_rec, w.gn_rec + (size_t)max_rows * 928, &wk.ctr->ihead,
                                                   stream)))
                return r;
            if (check) {
                if ((r = gz_gn_forward(d_gn_weights, w.gn_in, max_rows, &wk.ctr->rows, w.chk_p, w.chk_q, nullptr,
                                       w.chk_rec, stream)))
                    return r;
                plan_gn_check_kernel<<<max_rows, 256, 0, s>>>(wk);
                if ((r = plan_check("plan_gn_check_kernel"))) return r;
            }
        }
        // PW waves per row when the launch leaves CUs idle (GZ_PLAN_STEP4: that row cap, A/B)
        static const int cap4 = [] {
            const char* e = getenv("GZ_PLAN_STEP4");
            return e ? atoi(e) : 4096;
        }();
        if (max_rows <= cap4) {
            plan_step4_kernel<<<max_rows, PW * WAVE, 0, s>>>(wk, *pp, inc ? 1 : 0, next);
            zeroed = true;
        } else {
            if (inc) plan_gn_count_kernel<<<1, 1, 0, s>>>(wk);
            plan_step_kernel<<<max_rows, WAVE, 0, s>>>(wk, *pp, 0);
            zeroed = false;
        }
        return plan_check("plan_step_kernel");
    };
    // The pending count is read (one host synchronisation) every `every` rounds only: a
    // round after the last is a no-op (no job is collected, rolled out or resumed when no
    // game has a pending simulation), so the rounds in between are launched unread.
    static const int every = [] {
        const char* e = getenv("GZ_PLAN_SYNC_EVERY");
        const int v = e ? atoi(e) : 2;
        return v < 1 ? 1 : v;
    }();
    for (int round = 0;; round++) {
        if (round % every == 0) {
            int32_t pending = 0;
            if (hipMemcpyAsync(&pending, &w.ctr->pending, 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                hipStreamSynchronize(s) != hipSuccess)
                return plan_fail(GZ_ERR_HIP, "gz_plan_search: reading the pending count");
            if (pending == 0) break;
        }
        if (round > S + 1 + every) return plan_fail(GZ_ERR_INTERNAL, "gz_plan_search: search did not terminate");
        if (round == 0) {  // every job of the parallel phase, C at a time
            for (int j0 = 0; j0 < n_jobs; j0 += C) {
                const int j1 = j0 + C < n_jobs ? j0 + C : n_jobs;
                for (int st = 0; st < p->planner_steps; st++)
                    if ((rc = planner_step(j0, j1, j1 - j0, 0))) return rc;
            }
        } else {  // one job per game
            for (int st = 0; st < p->planner_steps; st++)
                if ((rc = planner_step(0, n_jobs, n, 1))) return rc;
        }
        // after round 0 the only jobs are the sequential simulations' (job g * S)
        const int cnt = round == 0 ? n_jobs : n, stride = round == 0 ? 1 : S;
        plan_collect_kernel<<<(cnt + 255) / 256, 256, 0, s>>>(w, S, n, 0, cnt, stride, p->planner_steps, 1, 0, 0);
        if ((rc = plan_check("plan_collect_kernel"))) return rc;
        plan_rollout_kernel<<<(cnt + 255) / 256, 256, 0, s>>>(w, cnt, stride, p->max_depth);
        if ((rc = plan_check("plan_rollout_kernel"))) return rc;
        if (hipMemsetAsync(&w.ctr->pending, 0, 4, s) != hipSuccess) return plan_fail(GZ_ERR_HIP, "memset");
        plan_resume_kernel<<<n, WAVE, 0, s>>>(n, *p, w, sink, gather ? 1 : 0, d_moves, d_stats);
        if ((rc = plan_check("plan_resume_kernel"))) return rc;
    }
    plan_finish_kernel<<<n, WAVE, 0, s>>>(n, S, w, d_moves, d_stats, (char*)d_trees);
    return plan_check("plan_finish_kernel");
}

// out[4] (host int64) = rows that ran the full forward / the incremental forward /
// were checked / differed from the full forward (GZ_FLAG_GN_CHECK), summed over the
// searches since the last reset
extern "C" int gz_plan_gn_stats(void* d_workspace, int32_t n, int32_t num_simulations, int64_t* out, int32_t reset,
                                void* stream) {
    if (!d_workspace || n < 1 || num_simulations < 1) return plan_fail(GZ_ERR_ARG, "gz_plan_gn_stats: bad arguments");
    Workspace w = carve(d_workspace, n, num_simulations);
    hipStream_t s = (hipStream_t)stream;
    GnStats h;
    if (out) {
        if (hipMemcpyAsync(&h, w.stats, sizeof(h), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return plan_fail(GZ_ERR_HIP, "gz_plan_gn_stats: copy");
        out[0] = h.full;
        out[1] = h.inc;
        out[2] = h.checked;
        out[3] = h.mismatch;
    }
    if (reset && hipMemsetAsync(w.stats, 0, sizeof(GnStats), s) != hipSuccess)
        return plan_fail(GZ_ERR_HIP, "gz_plan_gn_stats: reset");
    return GZ_OK;
}

extern "C" int gz_plan_search(const gz_board_state* d_boards, const int64_t* d_game_ids, int32_t n,
                              const gz_search_params* p, const gz_planner_params* pp, const float* d_gn_weights,
                              void* d_workspace, void* d_trees, int32_t* d_moves, gz_search_stats* d_stats,
                              uint32_t* d_leaves, int32_t leaf_cap, int32_t* d_leaf_count, void* stream) {
    return gz_internal_plan_search(d_boards, d_game_ids, n, p, pp, d_gn_weights, d_workspace, d_trees, d_moves,
                                   d_stats, d_leaves, leaf_cap, d_leaf_count, nullptr, stream);
}

extern "C" int gz_planner_move(const gz_board_state* d_boards, const int32_t* d_ai, const uint64_t* d_keys,
                               int32_t n, const gz_planner_params* pp, const float* d_gn_weights, void* d_workspace,
                               int32_t* d_moves, uint32_t* d_draws, void* stream) {
    if (!pp || n < 0 || (n > 0 && (!d_boards || !d_ai || !d_keys || !d_gn_weights || !d_workspace || !d_moves ||
                                   !d_draws)))
        return plan_fail(GZ_ERR_ARG, "gz_planner_move: bad arguments");
    if (pp->k < 1 || pp->k > 16) return plan_fail(GZ_ERR_ARG, "gz_planner_move: k must be in [1, 16]");
    if (n == 0) return GZ_OK;
    hipStream_t s = (hipStream_t)stream;
    char* base = (char*)d_workspace;
    uint32_t* rows = (uint32_t*)base;
    float* gp = (float*)(base + align256((size_t)n * 64));
    float* gq = gp + (size_t)n * 225;
    float* rec = (float*)((char*)base + align256((size_t)n * 64) + align256((size_t)n * 225 * 4 * 2));
    boards_to_rows_kernel<<<(n + 255) / 256, 256, 0, s>>>(d_boards, n, rows);
    int rc;
    if ((rc = plan_check("boards_to_rows_kernel"))) return rc;
    if ((rc = gz_gn_forward(d_gn_weights, rows, n, nullptr, gp, gq, nullptr, rec, stream))) return rc;
    planner_move_kernel<<<n, WAVE, 0, s>>>(d_boards, d_ai, d_keys, n, *pp, gp, gq, d_moves, d_draws);
    return plan_check("planner_move_kernel");
}

extern "C" size_t gz_planner_move_workspace_bytes(int32_t n) {
    const size_t m = (size_t)(n < 1 ? 1 : n);
    return align256(m * 64) + align256(m * 225 * 4 * 2) + gz_gn_workspace_bytes((int32_t)m);
}

extern "C" int gz_knowledge_scores(const gz_board_state* d_boards, const int32_t* d_player, int32_t n,
                                   double* d_scores, void* stream) {
    if (n < 0 || (n > 0 && (!d_boards || !d_player || !d_scores)))
        return plan_fail(GZ_ERR_ARG, "gz_knowledge_scores: bad arguments");
    if (n == 0) return GZ_OK;
    knowledge_scores_kernel<<<n, WAVE, 0, (hipStream_t)stream>>>(d_boards, d_player, n, d_scores);
    return plan_check("knowledge_scores_kernel");
}
