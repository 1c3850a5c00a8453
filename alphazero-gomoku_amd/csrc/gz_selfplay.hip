// gz_selfplay.hip -- MCTS self-play engine for gfx950 (MI355X).
//
// One 64-lane wavefront (one workgroup) owns one game.  The reference's search
// (ai_agent.py:168-222) has two regimes, handled differently:
//
//  * parallel phase.  While the root still has unexplored moves, _select
//    (ai_agent.py:224-232) returns the root and _expand pops the root's
//    highest-index empty cell, so simulations 1..min(S, L+1) are a rollout from
//    the root followed by one rollout from each root child, children created in
//    reverse row-major order.  Their rollouts are independent (each simulation
//    draws from its own RNG sub-stream), so the 64 lanes run them concurrently,
//    each lane holding its own bit-plane board in VGPRs and pulling the next
//    simulation from a wave-local counter when its rollout ends.
//  * sequential phase.  Simulations L+2..S descend by UCB; the wave computes the
//    UCB of all children in parallel, expands, runs the rollout on one lane and
//    backs up.  Results are bit-identical to running the simulations in order.
//
// The tree lives in LDS (26 bytes per node, SoA).  UCB arithmetic is fp64 with
// -ffp-contract=off so every rounding matches CPython/numpy; np.log / np.tanh
// values come from tables generated with numpy (gz_tables.h).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>
#include <string>

#include "gz_search.h"

using namespace gz;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(GZ_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return GZ_OK;
}

struct SearchOut {
    int n_nodes;
    int predicts;
    int main_draws;
    long long sim_draws;
};

// Wave-uniform state of the position being searched, kept in LDS so that the
// rollout loop's VGPR budget goes to the per-lane boards.
struct RootShared {
    BB black, white;  // position
    BB me, op;        // stones of the side to move (the AI) / of the opponent
    BB E;             // empty cells
    BB W;             // cells where the side to move completes five
    double v1;        // value of simulation 1 (rollout from the root)
    int n_moves, player;
};

__device__ inline BB lds_bb(const BB& x) {
    BB o;
#pragma unroll
    for (int i = 0; i < GZ_W; i++) o.w[i] = x.w[i];
    return o;
}

// ---------------------------------------------------------------- MCTS (one wave)
// _mcts_search (ai_agent.py:168-204) after the root's setup; returns the chosen
// cell.  The no-children fallback (:204) draws from the main stream.
__device__ __forceinline__ int mcts(RootShared* rs, int64_t game_id, const gz_search_params& p, Tree t, const LeafSink& sink,
                    bool gather, uint8_t* grid, int L, uint64_t kmain, uint32_t& dm, SearchOut& so) {
    const int lane = lane_id();
    const int S = p.num_simulations;
    const bool use_bg = p.beta != 0.0;
    const int n_moves = rs->n_moves, player = rs->player;
    const int n_par = S < L + 1 ? S : L + 1;
    long long lane_draws = 0;

    if (use_bg) write_grid(grid, lds_bb(rs->black), lds_bb(rs->white));

    // ---- root (MCTSNode.__init__, ai_agent.py:494-523) and its children in
    // expansion order: child j takes the j-th highest empty cell (_expand pops
    // the last entry of the row-major list, ai_agent.py:241)
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
        int j = base + lane;
        bool valid = j < n_par;
        int term = 0;
        if (valid) {
            int bit = select_bit(lds_bb(rs->E), L - j);
            bool win = bb_test(lds_bb(rs->W), bit);
            term = win ? player : ((n_moves + 1 >= 200 || L == 1) ? 3 : 0);
            t.parent[j] = 0;
            t.move[j] = (uint8_t)bit_to_cell(bit);
            t.term[j] = (uint8_t)term;
            t.bound[j] = 256;
            t.visits[j] = 0;
            t.value[j] = 0.0;
            double bgv = 0.0;
            if (use_bg) {
                BB ps = lds_bb(rs->me);
                bb_set(ps, bit);
                bgv = bg_from_score(pattern_score_lane(grid, ps, player, grid_index_of_bit(bit)));
            }
            t.bg[j] = bgv;
        }
        nonterm += __popcll(ballot(valid && term == 0));
    }
    __syncthreads();
    so.predicts = 1 + nonterm;  // root + every non-terminal child runs predict
    int root_bidx = -1;  // the root's leaf index (the tree forward's tags)
    if (gather) {
        int bidx = leaf_reserve(sink, 1 + nonterm);
        root_bidx = bidx;
        if (lane == 0) {
            leaf_write(sink, bidx, lds_bb(rs->black), lds_bb(rs->white));
            leaf_meta(sink, bidx, -1);
        }
        int off = 1;
        for (int base = 1; base < n_par; base += WAVE) {
            int j = base + lane;
            bool live = j < n_par && t.term[j] == 0;
            uint64_t m = ballot(live);
            if (live) {
                int bit = cell_to_bit(t.move[j]);
                BB cbk = lds_bb(rs->black), cwh = lds_bb(rs->white);
                if (player == 1) bb_set(cbk, bit);
                else bb_set(cwh, bit);
                leaf_write(sink, bidx + off + rank_in(m), cbk, cwh);
                leaf_meta(sink, bidx + off + rank_in(m), bidx);
            }
            off += __popcll(m);
        }
    }
    if (lane == 0 && n_par >= 2) t.bound[0] = (int16_t)cell_to_bit(t.move[n_par - 1]);
    __syncthreads();

    // ---- parallel phase: simulations 1..n_par, one rollout per lane at a time
    {
        const Centre cb = centre_buckets();
        BB rme = bb_zero(), rop = bb_zero();
        int rmover = 0, rn = 0, rsteps = 0, rsim = 0;
        uint64_t rkey = 0;
        uint32_t rcnt = 0;
        int next_sim = 1;
        while (true) {
            while (true) {  // hand simulations to idle lanes
                bool need = rsim == 0;
                uint64_t m = ballot(need);
                if (next_sim > n_par || m == 0) break;
                int s = next_sim + rank_in(m);
                next_sim += __popcll(m);
                if (need && s <= n_par) {
                    bool start = true;
                    if (s == 1) {
                        rme = lds_bb(rs->me);
                        rop = lds_bb(rs->op);
                        rmover = player;
                        rn = n_moves;
                    } else {
                        int j = s - 1;
                        int term = t.term[j];
                        if (term) {  // _simulate on a terminal node: no rollout, no draws
                            t.value[j] = term_value(term, player);
                            t.visits[j] = 1;
                            start = false;
                        } else {
                            int bit = cell_to_bit(t.move[j]);
                            rme = lds_bb(rs->op);
                            rop = lds_bb(rs->me);
                            bb_set(rop, bit);
                            rmover = 3 - player;
                            rn = n_moves + 1;
                        }
                    }
                    if (start) {
                        if (p.max_depth <= 0) {  // loop never entered: board not over -> 0.0
                            if (s == 1) rs->v1 = 0.0;
                            else {
                                t.value[s - 1] = 0.0;
                                t.visits[s - 1] = 1;
                            }
                        } else {
                            rsim = s;
                            rsteps = 0;
                            rkey = stream_key(p.seed, game_id, n_moves, s);
                            rcnt = 0;
                        }
                    }
                }
            }
            bool active = rsim != 0;
            if (ballot(active) == 0) break;
            if (active) {  // one ply of _simulate (ai_agent.py:273-282)
                BB e = empties(rme, rop);
                int ne = bb_count(e);
                bool done = false;
                double v = 0.0;
                if (ne == 0) {
                    done = true;
                } else {
                    bool won;
                    int b = policy_move(rme, rop, e, cb, rkey, &rcnt, &won);
                    bb_set(rme, b);
                    rn++;
                    rsteps++;
                    if (won) {
                        done = true;
                        v = rmover == player ? 1.0 : -1.0;
                    } else if (ne == 1 || rn >= 200) {
                        done = true;
                        v = 0.1;
                    } else if (rsteps >= p.max_depth) {
                        done = true;
                        v = 0.0;
                    }
                    BB tmp = rme;
                    rme = rop;
                    rop = tmp;
                    rmover = 3 - rmover;
                }
                if (done) {
                    if (rsim == 1) rs->v1 = v;
                    else {
                        t.value[rsim - 1] = v;
                        t.visits[rsim - 1] = 1;
                    }
                    lane_draws += rcnt;
                    rsim = 0;
                }
            }
        }
    }
    __syncthreads();
    // _backpropagate of the parallel phase: each child got exactly one update;
    // the root sums the values in simulation order (fp64, like node.value += v)
    if (lane == 0) {
        double acc = 0.0;
        if (n_par >= 1) acc += rs->v1;
        for (int j = 1; j < n_par; j++) acc += t.value[j];
        t.value[0] = acc;
        t.visits[0] = n_par;
    }
    __syncthreads();
    int n_nodes = n_par;

    // ---- sequential phase: simulations n_par+1..S
    for (int k = n_par + 1; k <= S; k++) {
        int x = 0;
        BB cbk = lds_bb(rs->black), cwh = lds_bb(rs->white);
        int cm = player, cn = n_moves;
        while (true) {  // _select, ai_agent.py:224-232
            if (t.term[x]) break;
            if (highest_bit_below(empties(cbk, cwh), t.bound[x]) >= 0) break;  // unexplored moves left
            int pv = t.visits[x];
            pv = pv < 1 ? 1 : pv;
            double lg = GZ_LOG_TABLE[pv];
            double mlog = lg > 1.0 ? lg : 1.0;
            double bv = -__builtin_inf();
            int bi = INT_MAX;
            for (int i = 1 + lane; i < n_nodes; i += WAVE) {
                if (t.parent[i] == x) {
                    double u = ucb1(t, i, mlog, p);
                    if (u > bv || bi == INT_MAX) {
                        bv = u;
                        bi = i;
                    }
                }
            }
            wave_argmax(bv, bi);
            if (bi == INT_MAX) break;  // no children
            x = bi;
            int bit = cell_to_bit(t.move[x]);
            if (cm == 1) bb_set(cbk, bit);
            else bb_set(cwh, bit);
            cm = 3 - cm;
            cn++;
        }
        if (!t.term[x] && t.visits[x] > 0) {  // _expand, ai_agent.py:234-249
            BB ex = empties(cbk, cwh);
            int hb = highest_bit_below(ex, t.bound[x]);
            if (hb >= 0) {
                int c = n_nodes++;
                bool win = bb_test(threats(cm == 1 ? cbk : cwh).win, hb);
                int term = win ? cm : ((cn + 1 >= 200 || bb_count(ex) == 1) ? 3 : 0);
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
                    so.predicts++;
                    if (gather) {
                        int bidx = leaf_reserve(sink, 1);
                        // a child of a root child of the parallel phase: tag it with
                        // that node's leaf index (root + 1 + its rank among the live
                        // root children), else -2
                        int tag = -2;
                        if (sink.meta && root_bidx >= 0 && x >= 1 && x < n_par) {
                            int rank = 0;
                            for (int base = 1; base < x; base += WAVE) {
                                const int j = base + lane;
                                rank += __popcll(ballot(j < x && t.term[j] == 0));
                            }
                            const int pidx = root_bidx + 1 + rank;
                            if (pidx < sink.cap) tag = pidx;
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
        double v;
        int tx = t.term[x];
        if (tx) {
            v = term_value(tx, player);
        } else {  // rollout on lane 0
            double vv = 0.0;
            if (lane == 0) {
                uint32_t cnt = 0;
                uint64_t key = stream_key(p.seed, game_id, n_moves, k);
                RolloutResult r = rollout(cbk, cwh, cn, cm, player, p.max_depth, key, &cnt);
                vv = r.value;
                lane_draws += cnt;
            }
            v = __shfl(vv, 0);
        }
        if (lane == 0) {  // _backpropagate, ai_agent.py:441-448
            int y = x;
            while (y >= 0) {
                t.visits[y] += 1;
                t.value[y] += v;
                y = t.parent[y];
            }
        }
        __syncthreads();
    }
    so.n_nodes = n_nodes;
    so.sim_draws = wave_sum_ll(lane_draws);

    // ---- result: first root child with the most visits (ai_agent.py:199-201)
    int best;
    if (n_par >= 2) {
        int bv = -1, bi = INT_MAX;
        for (int j = 1 + lane; j < n_par; j += WAVE) {
            int v = t.visits[j];
            if (v > bv) {
                bv = v;
                bi = j;
            }
        }
        wave_argmax_int(bv, bi);
        best = t.move[bi];
    } else {
        best = bit_to_cell(select_bit(lds_bb(rs->E), (int)below(draw(kmain, dm++), (uint32_t)L)));
    }
    return best;
}

// AlphaZeroGomokuAI.get_move + _opening_move (ai_agent.py:109-166) for the
// position already stored in rs->black / rs->white / rs->n_moves / rs->player.
__device__ __forceinline__ int search_move(RootShared* rs, int64_t game_id, const gz_search_params& p, Tree t, const LeafSink& sink,
                           bool gather, uint8_t* grid, SearchOut& so) {
    const int lane = lane_id();
    const int n_moves = rs->n_moves, player = rs->player;
    {
        BB black = lds_bb(rs->black), white = lds_bb(rs->white);
        BB E = empties(black, white);
        BB me = player == 1 ? black : white;
        BB W = threats(me).win & E;
        __syncthreads();
        if (lane == 0) {
            rs->E = E;
            rs->W = W;
            rs->me = me;
            rs->op = player == 1 ? white : black;
        }
        __syncthreads();
    }
    const BB E = lds_bb(rs->E);
    const int L = bb_count(E);
    uint64_t kmain = stream_key(p.seed, game_id, n_moves, 0);
    uint32_t dm = 0;
    so.n_nodes = 0;
    so.predicts = 0;
    so.sim_draws = 0;
    so.main_draws = 0;
    int best = -1;
    if (L == 0) return -1;
    if (n_moves < 6) {
        if (n_moves == 0 && bb_test(E, 7 * 16 + 7)) return 7 * GZ_N + 7;
        const BB k3 = GZ_MASK_K3, k5 = GZ_MASK_K5;
        BB s = k3 & E;
        if (!bb_any(s)) s = k5 & E;
        if (bb_any(s)) {
            best = bit_to_cell(select_bit(s, (int)below(draw(kmain, dm++), (uint32_t)bb_count(s))));
            so.main_draws = dm;
            return best;
        }
        best = mcts(rs, game_id, p, t, sink, gather, grid, L, kmain, dm, so);
        so.main_draws = dm;
        return best;
    }
    best = mcts(rs, game_id, p, t, sink, gather, grid, L, kmain, dm, so);
    if (to_unit(draw(kmain, dm++)) < p.exploration)  // ai_agent.py:128-129
        best = bit_to_cell(select_bit(lds_bb(rs->E), (int)below(draw(kmain, dm++), (uint32_t)L)));
    so.main_draws = dm;
    return best;
}


// ---------------------------------------------------------------- kernels
__global__ __launch_bounds__(WAVE, 4) void search_kernel(const gz_board_state* boards, const int64_t* game_ids, int n,
                                                         gz_search_params p, char* trees, size_t tree_stride,
                                                         int32_t* moves, gz_search_stats* stats, LeafSink sink,
                                                         int gather) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ RootShared rs;
    __shared__ uint8_t grid[GRID_BYTES];
    int i = blockIdx.x;
    if (i >= n) return;
    const gz_board_state& bs = boards[i];
    if (lane_id() == 0) {
        load_bb(rs.black, bs.black);
        load_bb(rs.white, bs.white);
        rs.n_moves = bs.n_moves;
        rs.player = bs.player;
    }
    __syncthreads();
    Tree t = tree_at(smem, p.num_simulations);
    SearchOut so;
    int mv;
    if (bs.over) {  // callers never search a finished board
        mv = -1;
        so.n_nodes = so.predicts = so.main_draws = 0;
        so.sim_draws = 0;
    } else {
        mv = search_move(&rs, game_ids[i], p, t, sink, gather != 0, grid, so);
    }
    __syncthreads();
    if (trees) {  // export the tree for inspection
        size_t tb = tree_bytes_for(p.num_simulations);
        const uint32_t* src = (const uint32_t*)smem;
        uint32_t* dst = (uint32_t*)(trees + (size_t)i * tree_stride);
        for (size_t w = lane_id(); w < tb / 4; w += WAVE) dst[w] = src[w];
    }
    if (lane_id() == 0) {
        moves[i] = mv;
        if (stats) {
            gz_search_stats st;
            st.n_nodes = so.n_nodes;
            st.predicts = so.predicts;
            st.main_draws = so.main_draws;
            st.pad = 0;
            st.sim_draws = so.sim_draws;
            stats[i] = st;
        }
    }
}

struct SlotHeader {  // 128 bytes
    uint32_t black[8];
    uint32_t white[8];
    int64_t game_id;
    int64_t game_id_stride;
    int32_t n_moves;
    int32_t player;
    int64_t game_id_end;  // the slot is idle once game_id >= game_id_end (no new game starts)
    int64_t games_done;
    // totals over every search this slot ran since init: predict() calls and RNG
    // draws (main stream, simulation streams).  The checker compares them with the
    // oracle's per-ply counts (gz_selfplay_draws): they see the rollout and planner
    // decisions a game's moves hide
    int64_t predicts;
    int64_t main_draws;
    int64_t sim_draws;
};
static_assert(sizeof(SlotHeader) == 128, "slot header");

__host__ __device__ inline size_t slot_stride_bytes() {
    size_t b = sizeof(SlotHeader) + (size_t)GZ_MAX_GAME_PLIES * sizeof(gz_record);
    return (b + 255) & ~(size_t)255;
}

__global__ void selfplay_init_kernel(char* slots, int n_slots, int64_t base, int64_t stride) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    SlotHeader* h = (SlotHeader*)(slots + (size_t)s * slot_stride_bytes());
    for (int i = 0; i < 8; i++) h->black[i] = h->white[i] = 0;
    h->game_id = base + s;
    h->game_id_stride = stride;
    h->n_moves = 0;
    h->player = 1;
    h->game_id_end = INT64_MAX;
    h->games_done = 0;
    h->predicts = h->main_draws = h->sim_draws = 0;
}

// training.play_one_game (training.py:141-218) for one slot, n_plies plies,
// restarting finished games.
#ifndef GZ_SP_WPE
#define GZ_SP_WPE 3  // selfplay_kernel: waves per SIMD the register allocation targets (4: 96 spilled VGPRs, 7 % slower)
#endif
__global__ __launch_bounds__(WAVE, GZ_SP_WPE) void selfplay_kernel(char* slots, int n_slots, gz_search_params p, int n_plies,
                                                           gz_record* records, int rec_cap, LeafSink sink, int gather,
                                                           gz_selfplay_counters* ctr) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    __shared__ RootShared rs;
    __shared__ uint8_t grid[GRID_BYTES];
    const int s = blockIdx.x;
    if (s >= n_slots) return;
    const int lane = lane_id();
    SlotHeader* h = (SlotHeader*)(slots + (size_t)s * slot_stride_bytes());
    gz_record* rec = (gz_record*)(h + 1);
    if (lane == 0) {
        load_bb(rs.black, h->black);
        load_bb(rs.white, h->white);
        rs.n_moves = h->n_moves;
        rs.player = h->player;
    }
    int64_t game_id = h->game_id;
    const int64_t gstride = h->game_id_stride, gend = h->game_id_end;
    if (game_id >= gend) return;  // idle: its games are done
    long long games = 0, moves_played = 0, mcts_played = 0, npred = 0, dmain = 0, dsim = 0;
    Tree t = tree_at(smem, p.num_simulations);
    __syncthreads();
    for (int it = 0; it < n_plies; it++) {
        SearchOut so;
        int mv = search_move(&rs, game_id, p, t, sink, gather != 0, grid, so);
        __syncthreads();
        if (mv < 0) break;  // unreachable: live games always have an empty cell
        npred += so.predicts;
        dmain += so.main_draws;
        dsim += so.sim_draws;
        const int n_moves = rs.n_moves, player = rs.player;
        const int bit = cell_to_bit(mv);
        const bool win = bb_test(lds_bb(rs.W), bit);  // rs.W = winning cells of the mover
        const int ne = bb_count(lds_bb(rs.E));
        if (lane == 0) {  // buf.add(planes, move_idx, player), training.py:203-206
            gz_record& r = rec[n_moves];
            store_bb(r.black, rs.black);
            store_bb(r.white, rs.white);
            r.game_id = game_id;
            r.ply = (int16_t)n_moves;
            r.move = (int16_t)mv;
            r.player = (int8_t)player;
            r.z = 0;
            // board.make_move (gomoku_board.py:84-113)
            if (player == 1) bb_set(rs.black, bit);
            else bb_set(rs.white, bit);
            rs.n_moves = n_moves + 1;
            rs.player = 3 - player;
        }
        __syncthreads();
        const int over = win ? player : ((ne == 1 || n_moves + 1 >= 200) ? 3 : 0);
        moves_played++;
        mcts_played += n_moves >= 6;  // (plies 0-5: _opening_move, never a search)
        if (over) {  // buf.finalize_with_winner (training.py:89-94) and restart
            const int winner = over == 3 ? 0 : over;
            const int n = n_moves + 1;
            int base = 0;
            if (lane == 0) base = atomicAdd(&ctr->records, n);
            base = __shfl(base, 0);
            for (int i = lane; i < n; i += WAVE) {
                if (base + i < rec_cap) {
                    gz_record r = rec[i];
                    r.z = (int8_t)(winner == 0 ? 0 : (r.player == winner ? 1 : -1));
                    records[base + i] = r;
                }
            }
            if (lane == 0 && base + n > rec_cap) {
                int lost = base + n - (base > rec_cap ? base : rec_cap);
                atomicAdd(&ctr->records_dropped, lost);
            }
            games++;
            game_id += gstride;
            __syncthreads();
            if (lane == 0) {
                rs.black = bb_zero();
                rs.white = bb_zero();
                rs.n_moves = 0;
                rs.player = 1;
            }
            __syncthreads();
            if (game_id >= gend) break;  // no next game: the slot goes idle
        }
    }
    if (lane == 0) {
        store_bb(h->black, rs.black);
        store_bb(h->white, rs.white);
        h->game_id = game_id;
        h->n_moves = rs.n_moves;
        h->player = rs.player;
        h->games_done += games;
        h->predicts += npred;
        h->main_draws += dmain;
        h->sim_draws += dsim;
        atomicAdd((unsigned long long*)&ctr->moves, (unsigned long long)moves_played);
        atomicAdd((unsigned long long*)&ctr->games, (unsigned long long)games);
        atomicAdd((unsigned long long*)&ctr->mcts_moves, (unsigned long long)mcts_played);
    }
}

// The move-application half of selfplay_kernel for searches run elsewhere
// (gz_plan_search): record, make_move, finish / restart (training.py:141-218).
__global__ __launch_bounds__(WAVE) void selfplay_commit_kernel(char* slots, int n_slots, const int32_t* moves,
                                                              const gz_search_stats* stats, gz_record* records,
                                                              int rec_cap, gz_selfplay_counters* ctr) {
    const int s = blockIdx.x;
    if (s >= n_slots) return;
    const int lane = lane_id();
    SlotHeader* h = (SlotHeader*)(slots + (size_t)s * slot_stride_bytes());
    if (h->game_id >= h->game_id_end) return;  // idle (its search ran on a dead board; nothing is recorded)
    gz_record* rec = (gz_record*)(h + 1);
    BB black, white;
    load_bb(black, h->black);
    load_bb(white, h->white);
    const int n_moves = h->n_moves, player = h->player;
    const int mv = moves[s];
    if (mv < 0) return;  // unreachable: live games always have an empty cell
    const int bit = cell_to_bit(mv);
    BB& mine = player == 1 ? black : white;
    const BB E = empties(black, white);
    const bool win = bb_test(threats(mine).win, bit);
    const int ne = bb_count(E);
    if (lane == 0) {
        gz_record& r = rec[n_moves];
        store_bb(r.black, black);
        store_bb(r.white, white);
        r.game_id = h->game_id;
        r.ply = (int16_t)n_moves;
        r.move = (int16_t)mv;
        r.player = (int8_t)player;
        r.z = 0;
    }
    bb_set(mine, bit);
    const int over = win ? player : ((ne == 1 || n_moves + 1 >= 200) ? 3 : 0);
    __syncthreads();
    long long games = 0;
    int64_t game_id = h->game_id;
    if (over) {
        const int winner = over == 3 ? 0 : over;
        const int n = n_moves + 1;
        int base = 0;
        if (lane == 0) base = atomicAdd(&ctr->records, n);
        base = __shfl(base, 0);
        for (int i = lane; i < n; i += WAVE) {
            if (base + i < rec_cap) {
                gz_record r = rec[i];
                r.z = (int8_t)(winner == 0 ? 0 : (r.player == winner ? 1 : -1));
                records[base + i] = r;
            }
        }
        if (lane == 0 && base + n > rec_cap) {
            int lost = base + n - (base > rec_cap ? base : rec_cap);
            atomicAdd(&ctr->records_dropped, lost);
        }
        games = 1;
        game_id += h->game_id_stride;
        black = bb_zero();
        white = bb_zero();
    }
    if (lane == 0) {
        store_bb(h->black, black);
        store_bb(h->white, white);
        h->game_id = game_id;
        h->n_moves = over ? 0 : n_moves + 1;
        h->player = over ? 1 : 3 - player;
        h->games_done += games;
        h->predicts += stats[s].predicts;
        h->main_draws += stats[s].main_draws;
        h->sim_draws += stats[s].sim_draws;
        atomicAdd((unsigned long long*)&ctr->moves, 1ull);
        if (n_moves >= 6) atomicAdd((unsigned long long*)&ctr->mcts_moves, 1ull);
        if (games) atomicAdd((unsigned long long*)&ctr->games, 1ull);
    }
}

__global__ void selfplay_boards_kernel(const char* slots, int n_slots, gz_board_state* out, int64_t* gids) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    const SlotHeader* h = (const SlotHeader*)(slots + (size_t)s * slot_stride_bytes());
    gz_board_state b;
    for (int i = 0; i < 8; i++) {
        b.black[i] = h->black[i];
        b.white[i] = h->white[i];
    }
    b.n_moves = h->n_moves;
    b.player = h->player;
    b.over = 0;
    b.winner = 0;
    out[s] = b;
    if (gids) gids[s] = h->game_id;
}

// K1: GomokuBoard.make_move + get_valid_moves, one board per lane
__device__ inline void legal_rowmajor(const BB& e, uint64_t out[4]) {
    out[0] = out[1] = out[2] = out[3] = 0;
    for (int r = 0; r < GZ_N; r++) {
        uint64_t row = (e.w[r >> 1] >> ((r & 1) * 16)) & 0x7FFFu;
        int off = r * GZ_N;
        out[off >> 6] |= row << (off & 63);
        if ((off & 63) + GZ_N > 64) out[(off >> 6) + 1] |= row >> (64 - (off & 63));
    }
}

__global__ void board_step_kernel(gz_board_state* boards, const int32_t* moves, int n, int32_t* ok,
                                  uint64_t* legal) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    gz_board_state b = boards[i];
    BB black, white;
    load_bb(black, b.black);
    load_bb(white, b.white);
    int m = moves[i];
    int res = 0;
    BB E = empties(black, white);
    if (m >= 0 && m < GZ_CELLS && !b.over) {  // is_valid_move (gomoku_board.py:67-82)
        int bit = cell_to_bit(m);
        if (bb_test(E, bit)) {
            BB& mine = b.player == 1 ? black : white;
            bool win = bb_test(threats(mine).win, bit);
            int ne = bb_count(E);
            bb_set(mine, bit);
            b.n_moves++;
            if (win) {
                b.over = 1;
                b.winner = b.player;
            } else if (ne == 1 || b.n_moves >= 200) {
                b.over = 1;
                b.winner = 0;
            }
            b.player = 3 - b.player;
            res = 1;
            E = empties(black, white);
        }
    }
    store_bb(b.black, black);
    store_bb(b.white, white);
    boards[i] = b;
    if (ok) ok[i] = res;
    if (legal) {
        uint64_t lm[4];
        legal_rowmajor(E, lm);
        for (int k = 0; k < 4; k++) legal[(size_t)i * 4 + k] = lm[k];
    }
}

__global__ void policy_kernel(const gz_board_state* boards, const uint64_t* keys, int n, int32_t* moves,
                              uint32_t* draws) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const gz_board_state& b = boards[i];
    BB black, white;
    load_bb(black, b.black);
    load_bb(white, b.white);
    BB me = b.player == 1 ? black : white, op = b.player == 1 ? white : black;
    BB e = empties(me, op);
    uint32_t cnt = 0;
    int mv = -1;
    if (bb_any(e)) {
        bool won;
        mv = bit_to_cell(policy_move(me, op, e, centre_buckets(), keys[i], &cnt, &won));
    }
    moves[i] = mv;
    draws[i] = cnt;
}

__global__ void rollout_kernel(const gz_board_state* boards, const int32_t* ai, const uint64_t* keys, int n,
                               int max_depth, double* values, gz_board_state* fin, uint32_t* draws) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    gz_board_state b = boards[i];
    BB black, white;
    load_bb(black, b.black);
    load_bb(white, b.white);
    uint32_t cnt = 0;
    double v;
    if (b.over) {
        v = b.winner == 0 ? 0.1 : (b.winner == ai[i] ? 1.0 : -1.0);
    } else {
        RolloutResult r = rollout(black, white, b.n_moves, b.player, ai[i], max_depth, keys[i], &cnt);
        v = r.value;
        black = r.black;
        white = r.white;
        b.n_moves = r.n_moves;
        b.over = r.over;
        b.winner = r.winner;
        b.player = (r.n_moves % 2) ? 2 : 1;
    }
    values[i] = v;
    if (fin) {
        store_bb(b.black, black);
        store_bb(b.white, white);
        fin[i] = b;
    }
    draws[i] = cnt;
}

__global__ __launch_bounds__(WAVE) void pattern_kernel(const gz_board_state* boards, const int32_t* player, int n,
                                                       int64_t* score, double* bg) {
    __shared__ uint8_t grid[GRID_BYTES];
    int i = blockIdx.x;
    if (i >= n) return;
    BB black, white;
    load_bb(black, boards[i].black);
    load_bb(white, boards[i].white);
    write_grid(grid, black, white);
    if (lane_id() == 0) {
        int pl = player[i];
        long long s = pattern_score_lane(grid, pl == 1 ? black : white, pl, -1);
        score[i] = s;
        bg[i] = bg_from_score(s);
    }
}

inline hipStream_t as_stream(void* s) { return (hipStream_t)s; }

int validate_params(const gz_search_params* p) {
    if (!p) return fail(GZ_ERR_ARG, "params is NULL");
    if (p->num_simulations < 0 || p->num_simulations > GZ_MAX_SIMULATIONS)
        return fail(GZ_ERR_ARG, "num_simulations out of range [0, 4095]");
    if (p->planner_steps != 0)
        return fail(GZ_ERR_UNSUPPORTED, "planner_steps > 0 runs through gz_plan_search / gz_selfplay_plan_run");
    return GZ_OK;
}

size_t smem_bytes(int S) { return tree_bytes_for(S); }

}  // namespace

extern "C" {

const char* gz_last_error(void) { return g_last_error.c_str(); }

// shared by the other translation units of libgzero (not part of gzero.h)
void gz_internal_set_error(const char* msg) { g_last_error = msg ? msg : ""; }

int gz_version(void) { return 1; }

size_t gz_tree_bytes(int32_t num_simulations) { return tree_bytes_for(num_simulations); }

size_t gz_slot_bytes(int32_t num_simulations) {
    (void)num_simulations;
    return slot_stride_bytes();
}

int gz_board_step(gz_board_state* d_boards, const int32_t* d_moves, int32_t n, int32_t* d_ok, uint64_t* d_legal,
                  void* stream) {
    if (n < 0 || (n > 0 && (!d_boards || !d_moves))) return fail(GZ_ERR_ARG, "gz_board_step: bad arguments");
    if (n == 0) return GZ_OK;
    board_step_kernel<<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(d_boards, d_moves, n, d_ok, d_legal);
    return check_launch("board_step_kernel");
}

int gz_policy_move(const gz_board_state* d_boards, const uint64_t* d_keys, int32_t n, int32_t* d_moves,
                   uint32_t* d_draws, void* stream) {
    if (n < 0 || (n > 0 && (!d_boards || !d_keys || !d_moves || !d_draws)))
        return fail(GZ_ERR_ARG, "gz_policy_move: bad arguments");
    if (n == 0) return GZ_OK;
    policy_kernel<<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(d_boards, d_keys, n, d_moves, d_draws);
    return check_launch("policy_kernel");
}

int gz_rollout(const gz_board_state* d_boards, const int32_t* d_ai, const uint64_t* d_keys, int32_t n,
               int32_t max_depth, double* d_values, gz_board_state* d_final, uint32_t* d_draws, void* stream) {
    if (n < 0 || (n > 0 && (!d_boards || !d_ai || !d_keys || !d_values || !d_draws)))
        return fail(GZ_ERR_ARG, "gz_rollout: bad arguments");
    if (n == 0) return GZ_OK;
    rollout_kernel<<<(n + 255) / 256, 256, 0, as_stream(stream)>>>(d_boards, d_ai, d_keys, n, max_depth, d_values,
                                                                   d_final, d_draws);
    return check_launch("rollout_kernel");
}

int gz_pattern_score(const gz_board_state* d_boards, const int32_t* d_player, int32_t n, int64_t* d_score,
                     double* d_bg, void* stream) {
    if (n < 0 || (n > 0 && (!d_boards || !d_player || !d_score || !d_bg)))
        return fail(GZ_ERR_ARG, "gz_pattern_score: bad arguments");
    if (n == 0) return GZ_OK;
    pattern_kernel<<<n, WAVE, 0, as_stream(stream)>>>(d_boards, d_player, n, d_score, d_bg);
    return check_launch("pattern_kernel");
}

int gz_search(const gz_board_state* d_boards, const int64_t* d_game_ids, int32_t n, const gz_search_params* p,
              void* d_trees, int32_t* d_moves, gz_search_stats* d_stats, uint32_t* d_leaves, int32_t leaf_cap,
              int32_t* d_leaf_count, void* stream) {
    int rc = validate_params(p);
    if (rc) return rc;
    if (n < 0 || (n > 0 && (!d_boards || !d_game_ids || !d_moves)))
        return fail(GZ_ERR_ARG, "gz_search: bad arguments");
    bool gather = (p->flags & GZ_FLAG_GATHER_LEAVES) != 0;
    if (gather && (!d_leaves || !d_leaf_count || leaf_cap < 0))
        return fail(GZ_ERR_ARG, "gz_search: leaf gathering needs d_leaves and d_leaf_count");
    if (n == 0) return GZ_OK;
    LeafSink sink{d_leaves, leaf_cap, d_leaf_count, nullptr};
    size_t tb = tree_bytes_for(p->num_simulations);
    search_kernel<<<n, WAVE, smem_bytes(p->num_simulations), as_stream(stream)>>>(
        d_boards, d_game_ids, n, *p, (char*)d_trees, tb, d_moves, d_stats, sink, gather ? 1 : 0);
    return check_launch("search_kernel");
}

int gz_selfplay_init(void* d_slots, int32_t n_slots, int32_t num_simulations, int64_t game_id_base,
                     int64_t game_id_stride, void* stream) {
    (void)num_simulations;
    if (!d_slots || n_slots <= 0) return fail(GZ_ERR_ARG, "gz_selfplay_init: bad arguments");
    selfplay_init_kernel<<<(n_slots + 255) / 256, 256, 0, as_stream(stream)>>>((char*)d_slots, n_slots, game_id_base,
                                                                               game_id_stride);
    return check_launch("selfplay_init_kernel");
}

int gz_selfplay_run(void* d_slots, int32_t n_slots, const gz_search_params* p, int32_t n_plies,
                    gz_record* d_records, int32_t record_cap, uint32_t* d_leaves, int32_t leaf_cap,
                    int32_t* d_leaf_meta, gz_selfplay_counters* d_counters, void* stream) {
    int rc = validate_params(p);
    if (rc) return rc;
    if (!d_slots || n_slots <= 0 || n_plies < 0 || !d_counters || !d_records || record_cap < 0)
        return fail(GZ_ERR_ARG, "gz_selfplay_run: bad arguments");
    bool gather = (p->flags & GZ_FLAG_GATHER_LEAVES) != 0;
    if (gather && (!d_leaves || leaf_cap < 0)) return fail(GZ_ERR_ARG, "gz_selfplay_run: leaf buffer missing");
    if (n_plies == 0) return GZ_OK;
    LeafSink sink{d_leaves, leaf_cap, &d_counters->leaves, gather ? d_leaf_meta : nullptr};
    selfplay_kernel<<<n_slots, WAVE, smem_bytes(p->num_simulations), as_stream(stream)>>>(
        (char*)d_slots, n_slots, *p, n_plies, d_records, record_cap, sink, gather ? 1 : 0, d_counters);
    return check_launch("selfplay_kernel");
}

size_t gz_selfplay_plan_workspace_bytes(int32_t n_slots, int32_t num_simulations) {
    size_t a = ((size_t)n_slots * sizeof(gz_board_state) + 255) & ~(size_t)255;
    size_t b = ((size_t)n_slots * 8 + 255) & ~(size_t)255;
    size_t c = ((size_t)n_slots * 4 + 255) & ~(size_t)255;
    size_t d = ((size_t)n_slots * sizeof(gz_search_stats) + 255) & ~(size_t)255;
    return a + b + c + d + gz_plan_workspace_bytes(n_slots, num_simulations);
}

// gz_plan_search with leaf tags (gz_plan.hip)
int gz_internal_plan_search(const gz_board_state* d_boards, const int64_t* d_game_ids, int32_t n,
                            const gz_search_params* p, const gz_planner_params* pp, const float* d_gn_weights,
                            void* d_workspace, void* d_trees, int32_t* d_moves, gz_search_stats* d_stats,
                            uint32_t* d_leaves, int32_t leaf_cap, int32_t* d_leaf_count, int32_t* d_leaf_meta,
                            void* stream);

int gz_selfplay_plan_run(void* d_slots, int32_t n_slots, const gz_search_params* p, const gz_planner_params* pp,
                         const float* d_gn_weights, void* d_workspace, int32_t n_plies, gz_record* d_records,
                         int32_t record_cap, uint32_t* d_leaves, int32_t leaf_cap, int32_t* d_leaf_meta,
                         gz_selfplay_counters* d_counters, void* stream) {
    if (!p || !pp || !d_slots || n_slots <= 0 || n_plies < 0 || !d_counters || !d_records || record_cap < 0 ||
        !d_workspace || !d_gn_weights)
        return fail(GZ_ERR_ARG, "gz_selfplay_plan_run: bad arguments");
    bool gather = (p->flags & GZ_FLAG_GATHER_LEAVES) != 0;
    if (gather && (!d_leaves || leaf_cap < 0)) return fail(GZ_ERR_ARG, "gz_selfplay_plan_run: leaf buffer missing");
    char* ws = (char*)d_workspace;
    gz_board_state* d_boards = (gz_board_state*)ws;
    ws += ((size_t)n_slots * sizeof(gz_board_state) + 255) & ~(size_t)255;
    int64_t* d_gids = (int64_t*)ws;
    ws += ((size_t)n_slots * 8 + 255) & ~(size_t)255;
    int32_t* d_moves = (int32_t*)ws;
    ws += ((size_t)n_slots * 4 + 255) & ~(size_t)255;
    gz_search_stats* d_stats = (gz_search_stats*)ws;
    ws += ((size_t)n_slots * sizeof(gz_search_stats) + 255) & ~(size_t)255;
    hipStream_t st = as_stream(stream);
    for (int it = 0; it < n_plies; it++) {
        selfplay_boards_kernel<<<(n_slots + 255) / 256, 256, 0, st>>>((const char*)d_slots, n_slots, d_boards, d_gids);
        int rc = check_launch("selfplay_boards_kernel");
        if (rc) return rc;
        rc = gz_internal_plan_search(d_boards, d_gids, n_slots, p, pp, d_gn_weights, ws, nullptr, d_moves, d_stats,
                                     gather ? d_leaves : nullptr, leaf_cap, gather ? &d_counters->leaves : nullptr,
                                     gather ? d_leaf_meta : nullptr, stream);
        if (rc) return rc;
        selfplay_commit_kernel<<<n_slots, WAVE, 0, st>>>((char*)d_slots, n_slots, d_moves, d_stats, d_records,
                                                         record_cap, d_counters);
        rc = check_launch("selfplay_commit_kernel");
        if (rc) return rc;
    }
    return GZ_OK;
}

int gz_plan_gn_stats(void* d_workspace, int32_t n, int32_t num_simulations, int64_t* out, int32_t reset, void* stream);

int gz_selfplay_plan_gn_stats(void* d_workspace, int32_t n_slots, int32_t num_simulations, int64_t* out,
                              int32_t reset, void* stream) {
    if (!d_workspace || n_slots <= 0) return fail(GZ_ERR_ARG, "gz_selfplay_plan_gn_stats: bad arguments");
    char* ws = (char*)d_workspace;
    ws += ((size_t)n_slots * sizeof(gz_board_state) + 255) & ~(size_t)255;
    ws += ((size_t)n_slots * 8 + 255) & ~(size_t)255;
    ws += ((size_t)n_slots * 4 + 255) & ~(size_t)255;
    ws += ((size_t)n_slots * sizeof(gz_search_stats) + 255) & ~(size_t)255;
    return gz_plan_gn_stats(ws, n_slots, num_simulations, out, reset, stream);
}

__global__ void selfplay_limit_kernel(char* slots, int n_slots, int64_t end) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    SlotHeader* h = (SlotHeader*)(slots + (size_t)s * slot_stride_bytes());
    h->game_id_end = end;
}

// the new slot index of every slot: the active ones (game_id < game_id_end) first, then
// the idle ones, each in slot order; one workgroup scans the flags in tiles of 1024
__global__ __launch_bounds__(1024) void selfplay_order_kernel(const char* slots, int n_slots, int32_t* order,
                                                              int32_t* n_active) {
    __shared__ int wsum[16];
    __shared__ int carry, total;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // pass 0 counts the active slots, pass 1 places both classes
    for (int pass = 0; pass < 2; pass++) {
        if (tid == 0) carry = 0;
        __syncthreads();
        for (int t0 = 0; t0 < n_slots; t0 += 1024) {
            const int s = t0 + tid;
            bool act = false;
            if (s < n_slots) {
                const SlotHeader* h = (const SlotHeader*)(slots + (size_t)s * slot_stride_bytes());
                act = h->game_id < h->game_id_end;
            }
            const uint64_t m = __ballot(act);
            if (lane == 0) wsum[wave] = __popcll(m);
            __syncthreads();
            int before = carry;
            for (int w = 0; w < wave; w++) before += wsum[w];
            const int rank = before + __popcll(m & ((1ull << lane) - 1));  // active slots before s
            if (pass == 1 && s < n_slots) order[s] = act ? rank : total + (s - rank);
            __syncthreads();
            if (tid == 0) {
                int c = 0;
                for (int w = 0; w < 16; w++) c += wsum[w];
                carry += c;
            }
            __syncthreads();
        }
        if (tid == 0 && pass == 0) {
            total = carry;
            *n_active = carry;
        }
        __syncthreads();
    }
}

// slot s -> dst slot order[s] (16-B words, one workgroup per slot)
__global__ __launch_bounds__(256) void selfplay_move_kernel(const char* slots, const int32_t* order, char* dst) {
    const size_t sb = slot_stride_bytes();
    const uint4* a = (const uint4*)(slots + (size_t)blockIdx.x * sb);
    uint4* b = (uint4*)(dst + (size_t)order[blockIdx.x] * sb);
    for (size_t i = threadIdx.x; i < sb / 16; i += 256) b[i] = a[i];
}

__global__ void selfplay_draws_kernel(const char* slots, int n_slots, int64_t* out) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n_slots) return;
    const SlotHeader* h = (const SlotHeader*)(slots + (size_t)s * slot_stride_bytes());
    out[3 * s] = h->predicts;
    out[3 * s + 1] = h->main_draws;
    out[3 * s + 2] = h->sim_draws;
}

int gz_selfplay_set_game_end(void* d_slots, int32_t n_slots, int64_t game_id_end, void* stream) {
    if (!d_slots || n_slots <= 0) return fail(GZ_ERR_ARG, "gz_selfplay_set_game_end: bad arguments");
    selfplay_limit_kernel<<<(n_slots + 255) / 256, 256, 0, as_stream(stream)>>>((char*)d_slots, n_slots, game_id_end);
    return check_launch("selfplay_limit_kernel");
}

size_t gz_selfplay_compact_workspace_bytes(int32_t n_slots) { return (size_t)(n_slots > 0 ? n_slots : 0) * 4; }

int gz_selfplay_compact(const void* d_slots, int32_t n_slots, void* d_dst, int32_t* d_n_active, void* d_workspace,
                        void* stream) {
    if (!d_slots || n_slots <= 0 || !d_dst || d_dst == d_slots || !d_n_active || !d_workspace)
        return fail(GZ_ERR_ARG, "gz_selfplay_compact: bad arguments");
    int32_t* order = (int32_t*)d_workspace;
    selfplay_order_kernel<<<1, 1024, 0, as_stream(stream)>>>((const char*)d_slots, n_slots, order, d_n_active);
    int rc = check_launch("selfplay_order_kernel");
    if (rc) return rc;
    selfplay_move_kernel<<<n_slots, 256, 0, as_stream(stream)>>>((const char*)d_slots, order, (char*)d_dst);
    return check_launch("selfplay_move_kernel");
}

int gz_selfplay_draws(const void* d_slots, int32_t n_slots, int64_t* d_out, void* stream) {
    if (!d_slots || n_slots <= 0 || !d_out) return fail(GZ_ERR_ARG, "gz_selfplay_draws: bad arguments");
    selfplay_draws_kernel<<<(n_slots + 255) / 256, 256, 0, as_stream(stream)>>>((const char*)d_slots, n_slots, d_out);
    return check_launch("selfplay_draws_kernel");
}

int gz_selfplay_boards(const void* d_slots, int32_t n_slots, int32_t num_simulations, gz_board_state* d_out,
                       int64_t* d_game_ids, void* stream) {
    (void)num_simulations;
    if (!d_slots || n_slots <= 0 || !d_out) return fail(GZ_ERR_ARG, "gz_selfplay_boards: bad arguments");
    selfplay_boards_kernel<<<(n_slots + 255) / 256, 256, 0, as_stream(stream)>>>((const char*)d_slots, n_slots, d_out,
                                                                                 d_game_ids);
    return check_launch("selfplay_boards_kernel");
}

}  // extern "C"
