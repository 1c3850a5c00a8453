/*
 * gz_oracle.c -- TEST INFRASTRUCTURE ONLY (see gz_oracle.h).
 *
 * CPU restatement of the reference self-play path.  Every function cites the
 * reference lines it follows.  Build: oracle/Makefile (gcc -O2 -ffp-contract=off;
 * no FMA contraction so fp64 UCB arithmetic rounds exactly like CPython/numpy).
 */
#include "gz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "gz_tables.h"

#define N OR_N
#define CELLS OR_CELLS

/* ------------------------------------------------------------------ rng */
static const uint64_t GOLDEN = 0x9E3779B97F4A7C15ULL;

uint64_t or_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

uint64_t or_stream_key(uint64_t seed, int64_t game_id, int32_t ply, int32_t sim) {
    uint64_t k = or_mix64(seed + GOLDEN);
    k = or_mix64(k ^ ((uint64_t)game_id * GOLDEN));
    k = or_mix64(k + ((uint64_t)(uint32_t)ply << 32) + (uint64_t)(uint32_t)sim);
    return k;
}

uint64_t or_draw(uint64_t key, uint64_t i) { return or_mix64(key + GOLDEN * (i + 1)); }

static double to_unit(uint64_t x) { return (double)(x >> 11) * (1.0 / 9007199254740992.0); }

static int below(uint64_t x, int n) {
    return (int)(((unsigned __int128)x * (uint64_t)n) >> 64);
}

/* random.choice(seq) on stream (key, *cnt) */
static int choice_idx(uint64_t key, uint64_t* cnt, int n) {
    uint64_t x = or_draw(key, (*cnt)++);
    return below(x, n);
}

/* ---------------------------------------------------------------- board */
static const int DIRS[4][2] = {{0, 1}, {1, 0}, {1, 1}, {1, -1}}; /* gomoku_board.py:33-38 */

void or_board_init(or_board* b) {
    memset(b->cell, 0, sizeof(b->cell));
    b->n_moves = 0;
    b->player = 1;
    b->over = 0;
    b->winner = 0;
}

/* _count_consecutive, gomoku_board.py:167-190 */
static int count_consec(const or_board* b, int r, int c, int dr, int dc, int p) {
    int n = 0;
    r += dr;
    c += dc;
    while (r >= 0 && r < N && c >= 0 && c < N && b->cell[r * N + c] == p) {
        n++;
        r += dr;
        c += dc;
    }
    return n;
}

/* longest run of p through (r,c) if (r,c) held p */
static int run_through(const or_board* b, int r, int c, int p) {
    int best = 0;
    for (int d = 0; d < 4; d++) {
        int cnt = 1 + count_consec(b, r, c, DIRS[d][0], DIRS[d][1], p) +
                  count_consec(b, r, c, -DIRS[d][0], -DIRS[d][1], p);
        if (cnt > best) best = cnt;
    }
    return best;
}

/* check_win, gomoku_board.py:139-165 */
static int check_win(const or_board* b, int r, int c) {
    return run_through(b, r, c, b->cell[r * N + c]) >= 5;
}

static int board_full(const or_board* b) {
    for (int i = 0; i < CELLS; i++)
        if (b->cell[i] == 0) return 0;
    return 1;
}

/* make_move, gomoku_board.py:84-113 */
int or_make_move(or_board* b, int r, int c) {
    if (!(r >= 0 && r < N && c >= 0 && c < N)) return 0;
    if (b->cell[r * N + c] != 0 || b->over) return 0;
    b->cell[r * N + c] = b->player;
    b->n_moves++;
    if (check_win(b, r, c)) {
        b->over = 1;
        b->winner = b->player;
    } else if (board_full(b) || b->n_moves >= 200) {
        b->over = 1;
        b->winner = 0;
    }
    b->player = (int8_t)(3 - b->player);
    return 1;
}

/* get_valid_moves, gomoku_board.py:201-213 (row-major, ignores game_over) */
static int legal_list(const or_board* b, int* out) {
    int n = 0;
    for (int i = 0; i < CELLS; i++)
        if (b->cell[i] == 0) out[n++] = i;
    return n;
}

int or_legal_mask(const or_board* b, uint64_t out[4]) {
    int n = 0;
    out[0] = out[1] = out[2] = out[3] = 0;
    for (int i = 0; i < CELLS; i++)
        if (b->cell[i] == 0) {
            out[i >> 6] |= 1ULL << (i & 63);
            n++;
        }
    return n;
}

int or_replay(or_board* b, const int32_t* moves, int n) {
    int ok = 0;
    for (int i = 0; i < n; i++) ok += or_make_move(b, moves[i] / N, moves[i] % N);
    return ok;
}

/* ------------------------------------------------------- rollout policy */
/* _evaluate_threat_level(board, p) >= 3  (ai_agent.py:403-430): some run of 3 */
static int has_run3(const or_board* b, int p) {
    for (int r = 0; r < N; r++)
        for (int c = 0; c < N; c++) {
            if (b->cell[r * N + c] != p) continue;
            for (int d = 0; d < 4; d++) {
                int r1 = r + DIRS[d][0], c1 = c + DIRS[d][1];
                int r2 = r + 2 * DIRS[d][0], c2 = c + 2 * DIRS[d][1];
                if (r2 < 0 || r2 >= N || c2 < 0 || c2 >= N) continue;
                if (b->cell[r1 * N + c1] == p && b->cell[r2 * N + c2] == p) return 1;
            }
        }
    return 0;
}

/* _select_offensive_move, ai_agent.py:306-361.
 * Step 2 (ai_agent.py:321-326) can never fire: the test stone is the mover's.
 * Step 3 (_find_defensive_moves, :363-381) placing the mover's stone never changes the
 * opponent's runs, so it yields all legal moves or none.  Step 4 (:383-401) is
 * "mover already has a run >= 3" or "the run through m reaches 3". */
int or_offensive_move(const or_board* b, uint64_t key, uint64_t* draws) {
    int L[CELLS], S[CELLS];
    int n = legal_list(b, L);
    int me = b->player, op = 3 - me;
    for (int k = 0; k < n; k++) /* step 1: first immediate win, row-major */
        if (run_through(b, L[k] / N, L[k] % N, me) >= 5) return L[k];
    if (has_run3(b, op)) return L[choice_idx(key, draws, n)];   /* step 3 */
    if (has_run3(b, me)) return L[choice_idx(key, draws, n)];   /* step 4, all */
    int ns = 0;
    for (int k = 0; k < n; k++)
        if (run_through(b, L[k] / N, L[k] % N, me) >= 3) S[ns++] = L[k];
    if (ns) return S[choice_idx(key, draws, ns)];
    /* step 5: Manhattan buckets <=2, <=4, else (ai_agent.py:339-361) */
    int c2[CELLS], c4[CELLS], ce[CELLS], n2 = 0, n4 = 0, ne = 0;
    for (int k = 0; k < n; k++) {
        int r = L[k] / N, c = L[k] % N;
        int d = abs(r - 7) + abs(c - 7);
        if (d <= 2) c2[n2++] = L[k];
        else if (d <= 4) c4[n4++] = L[k];
        else ce[ne++] = L[k];
    }
    if (n2) return c2[choice_idx(key, draws, n2)];
    if (n4) return c4[choice_idx(key, draws, n4)];
    return ce[choice_idx(key, draws, ne)];
}

/* _get_terminal_value, ai_agent.py:287-304 */
static double terminal_value(const or_board* b, int ai) {
    if (!b->over) return 0.0;
    if (b->winner == ai) return 1.0;
    if (b->winner != 0) return -1.0;
    return 0.1;
}

/* _simulate with planner_steps = 0, ai_agent.py:251-285 */
double or_rollout(const or_board* start, int ai, int max_depth, uint64_t key, uint64_t* draws,
                  or_board* final_out) {
    or_board b = *start;
    if (!b.over) {
        int steps = 0;
        int tmp[CELLS];
        while (!b.over && steps < max_depth) {
            if (legal_list(&b, tmp) == 0) break;
            int mv = or_offensive_move(&b, key, draws);
            or_make_move(&b, mv / N, mv % N);
            steps++;
        }
    }
    if (final_out) *final_out = b;
    return terminal_value(&b, ai);
}

/* -------------------------------------------------------- pattern score */
/* KnowledgeSearch._eval_segment, bg_planner.py:169-196, restated on a char window.
 * Built once into a LUT keyed by the 8 non-centre cells (0 me, 1 empty, 2 blocked). */
static int lut_ready = 0;
static int lut[6561];

static int count_nonoverlap(const char* s, const char* pat) {
    int n = 0;
    size_t lp = strlen(pat);
    const char* p = s;
    while ((p = strstr(p, pat)) != NULL) {
        n++;
        p += lp;
    }
    return n;
}

static int eval_window(const char* s) {
    int v = 0;
    if (strstr(s, "XXXXX")) v += 100000;
    if (strstr(s, ".XXXX.")) v += 10000;
    if (strstr(s, "XXXX.") || strstr(s, ".XXXX")) v += 5000;
    if (strstr(s, ".XXX.")) v += 1000;
    if (strstr(s, "XX.X") || strstr(s, "X.XX")) v += 300;
    if (strstr(s, ".XX.")) v += 50;
    if (count_nonoverlap(s, ".XXX.") >= 2) v += 3000;
    return v;
}

static void build_lut(void) {
    for (int code = 0; code < 6561; code++) {
        char s[10];
        int x = code;
        for (int j = 0; j < 8; j++) {
            char ch = "X.O"[x % 3];
            x /= 3;
            s[j < 4 ? j : j + 1] = ch;
        }
        s[4] = 'X';
        s[9] = 0;
        lut[code] = eval_window(s);
    }
    lut_ready = 1;
}

/* _pattern_score, bg_planner.py:133-155: all own stones x dirs (1,0),(0,1),(1,1),(1,-1) */
int64_t or_pattern_score(const or_board* b, int player) {
    static const int PD[4][2] = {{1, 0}, {0, 1}, {1, 1}, {1, -1}};
    if (!lut_ready) build_lut();
    int64_t total = 0;
    for (int r = 0; r < N; r++)
        for (int c = 0; c < N; c++) {
            if (b->cell[r * N + c] != player) continue;
            for (int d = 0; d < 4; d++) {
                int code = 0, pw = 1;
                for (int k = -4; k <= 4; k++) {
                    if (k == 0) continue;
                    int rr = r + k * PD[d][0], cc = c + k * PD[d][1];
                    int dig;
                    if (rr < 0 || rr >= N || cc < 0 || cc >= N) dig = 2;
                    else if (b->cell[rr * N + cc] == player) dig = 0;
                    else if (b->cell[rr * N + cc] == 0) dig = 1;
                    else dig = 2;
                    code += dig * pw;
                    pw *= 3;
                }
                total += lut[code];
            }
        }
    return total;
}

/* _bg_score, ai_agent.py:432-439: float(np.tanh(score / 10000.0)) */
double or_bg_score(const or_board* b, int player) {
    int64_t s = or_pattern_score(b, player);
    int64_t k = s / 50; /* every pattern weight is a multiple of 50 */
    return k >= GZ_TANH_N ? 1.0 : GZ_TANH_TABLE[k];
}

/* -------------------------------------------------------- BG planner */
/* KnowledgeSearch._opponent_can_win_next, bg_planner.py:116-125: for every empty
 * cell (get_valid_moves ignores game_over) a copy with current_player forced to
 * the opponent tries the move; make_move fails on a finished board, whose copy
 * then still reports the old game_over / winner. */
static int opp_can_win_next(const or_board* b, int opp) {
    for (int i = 0; i < CELLS; i++) {
        if (b->cell[i]) continue;
        or_board t = *b;
        t.player = (int8_t)opp;
        or_make_move(&t, i / N, i % N);
        if (t.over && t.winner == opp) return 1;
    }
    return 0;
}

/* KnowledgeSearch.score_move, bg_planner.py:90-106 (the stone placed is the side to move's) */
double or_ks_score(const or_board* b, int move, int P) {
    if (move < 0 || move >= CELLS || b->cell[move] != 0 || b->over) return -1e9;
    or_board t = *b;
    or_make_move(&t, move / N, move % N);
    if (t.over && t.winner == P) return 1e6;
    int opp = (P == 2) ? 1 : 2;
    if (opp_can_win_next(&t, opp)) return -1e5;
    double line = (double)or_pattern_score(&t, P);
    int dr = abs(move / N - 7), dc = abs(move % N - 7);
    double cb = (6 - (dr + dc)) * 0.5;
    return line + (cb > 0.0 ? cb : 0.0);
}

/* top_k_moves, bg_planner.py:108-114: Python's stable sort, descending */
int or_topk(const or_board* b, int P, int k, int32_t* out) {
    int L[CELLS];
    int n = legal_list(b, L);
    double sc[CELLS];
    for (int i = 0; i < n; i++) sc[i] = or_ks_score(b, L[i], P);
    int taken[CELLS] = {0};
    int m = n < k ? n : k;
    for (int r = 0; r < m; r++) {
        int bi = -1;
        for (int i = 0; i < n; i++)
            if (!taken[i] && (bi < 0 || sc[i] > sc[bi])) bi = i;
        taken[bi] = 1;
        out[r] = L[bi];
    }
    return m;
}

/* BGPlannerAI.get_move, bg_planner.py:232-269, with the nets' p / q given */
int or_planner_move(const or_board* b, int P, const or_planner_params* pp, const float* p, const float* q,
                    uint64_t key, uint64_t* draws) {
    int L[CELLS];
    int n = legal_list(b, L);
    if (n == 0) return -1;
    int32_t top[CELLS];
    int m = or_topk(b, P, pp->k, top);
    if (m == 0) return L[choice_idx(key, draws, n)];
    int best = -1;
    double bs = -1e18;
    for (int i = 0; i < m; i++) {
        double composed = pp->alpha * (double)p[top[i]] - (1 - pp->alpha) * (double)q[top[i]];
        if (composed > bs) {
            bs = composed;
            best = top[i];
        }
    }
    if (to_unit(or_draw(key, (*draws)++)) < pp->explore) return top[choice_idx(key, draws, m)];
    return best >= 0 ? best : L[choice_idx(key, draws, n)];
}

/* GraphNet / OpponentDQN in plain fp32 loops (bg_planner.py:22-78).  Offsets of
 * gzero/planner_nets.py's blob, recomputed here (or_gnet_layout lets the tests
 * check the two agree). */
#define GH 64
#define GDQ 256
enum { G_K3 = 9 * GH };
static void gnet_offsets(int32_t* o) {
    int off = 0;
    o[0] = off;            /* embed W [28][64] */
    off += 28 * GH;
    o[1] = off;            /* embed b */
    off += GH;
    for (int i = 0; i < 8; i++) {
        o[2 + i] = off;    /* layer i W, then bias */
        off += ((i % 2 == 0) ? G_K3 * GH : GH * GH) + GH;
    }
    o[10] = off;           /* policy conv W [2][64] */
    off += 2 * GH;
    o[11] = off;           /* policy conv b [2] (+2) */
    off += 4;
    o[12] = off;           /* policy fc W^T [450][225] */
    off += 450 * CELLS;
    o[13] = off;           /* policy fc b (+3) */
    off += 228;
    o[14] = off;           /* dqn fc0 W^T [675][256] */
    off += 3 * CELLS * GDQ;
    o[15] = off;
    off += GDQ;
    o[16] = off;           /* fc1 W^T [256][256] */
    off += GDQ * GDQ;
    o[17] = off;
    off += GDQ;
    o[18] = off;           /* fc2 W^T [256][225] */
    off += GDQ * CELLS;
    o[19] = off;           /* fc2 b (+3) */
}

int or_gnet_layout(int32_t* out, int cap) {
    int32_t o[20];
    gnet_offsets(o);
    for (int i = 0; i < 20 && i < cap; i++) out[i] = o[i];
    return 20;
}

static void planes_of(const or_board* b, float* x) { /* [3][225]: black, white, empty */
    for (int i = 0; i < CELLS; i++) {
        x[i] = b->cell[i] == 1;
        x[CELLS + i] = b->cell[i] == 2;
        x[2 * CELLS + i] = b->cell[i] == 0;
    }
}

/* 3x3 conv (padding 1) + bias + ReLU; W K-major [tap*cin_n + cin][cout] */
static void conv3(const float* in, int cin_n, const float* W, const float* bias, float* out) {
    for (int co = 0; co < GH; co++)
        for (int pos = 0; pos < CELLS; pos++) {
            int r = pos / N, c = pos % N;
            float acc = bias[co];
            for (int tap = 0; tap < 9; tap++) {
                int rr = r + tap / 3 - 1, cc = c + tap % 3 - 1;
                if (rr < 0 || rr >= N || cc < 0 || cc >= N) continue;
                for (int ci = 0; ci < cin_n; ci++)
                    acc += in[ci * CELLS + rr * N + cc] * W[(tap * cin_n + ci) * GH + co];
            }
            out[co * CELLS + pos] = acc > 0.f ? acc : 0.f;
        }
}

void or_gnet_forward(const float* blob, const or_board* b, float* logits, float* p, float* q) {
    int32_t o[20];
    gnet_offsets(o);
    float x[3 * CELLS];
    planes_of(b, x);
    float* h = (float*)malloc(sizeof(float) * GH * CELLS);
    float* g = (float*)malloc(sizeof(float) * GH * CELLS);
    conv3(x, 3, blob + o[0], blob + o[1], h);
    for (int i = 0; i < 8; i++) {
        const float* W = blob + o[2 + i];
        if (i % 2 == 0) {
            conv3(h, GH, W, W + G_K3 * GH, g);
        } else {
            const float* bias = W + GH * GH;
            for (int co = 0; co < GH; co++)
                for (int pos = 0; pos < CELLS; pos++) {
                    float acc = bias[co];
                    for (int ci = 0; ci < GH; ci++) acc += h[ci * CELLS + pos] * W[ci * GH + co];
                    g[co * CELLS + pos] = acc > 0.f ? acc : 0.f;
                }
        }
        float* t = h;
        h = g;
        g = t;
    }
    float pc[2 * CELLS]; /* policy conv, flattened channel-major (nn.Flatten) */
    for (int k = 0; k < 2; k++)
        for (int pos = 0; pos < CELLS; pos++) {
            float acc = blob[o[11] + k];
            for (int ci = 0; ci < GH; ci++) acc += blob[o[10] + k * GH + ci] * h[ci * CELLS + pos];
            pc[k * CELLS + pos] = acc;
        }
    float lg[CELLS], mx = -3.0e38f;
    for (int j = 0; j < CELLS; j++) {
        float acc = blob[o[13] + j];
        for (int i = 0; i < 2 * CELLS; i++) acc += blob[o[12] + i * CELLS + j] * pc[i];
        lg[j] = acc;
        if (acc > mx) mx = acc;
    }
    float sum = 0.f, e[CELLS];
    for (int j = 0; j < CELLS; j++) {
        e[j] = expf(lg[j] - mx);
        sum += e[j];
    }
    for (int j = 0; j < CELLS; j++) {
        if (logits) logits[j] = lg[j];
        if (p) p[j] = e[j] / sum;
    }
    if (q) {
        float a[GDQ], c[GDQ];
        for (int j = 0; j < GDQ; j++) {
            float acc = blob[o[15] + j];
            for (int i = 0; i < 3 * CELLS; i++) acc += blob[o[14] + i * GDQ + j] * x[i];
            a[j] = acc > 0.f ? acc : 0.f;
        }
        for (int j = 0; j < GDQ; j++) {
            float acc = blob[o[17] + j];
            for (int i = 0; i < GDQ; i++) acc += blob[o[16] + i * GDQ + j] * a[i];
            c[j] = acc > 0.f ? acc : 0.f;
        }
        for (int j = 0; j < CELLS; j++) {
            float acc = blob[o[19] + j];
            for (int i = 0; i < GDQ; i++) acc += blob[o[18] + i * CELLS + j] * c[i];
            q[j] = acc;
        }
    }
    free(h);
    free(g);
}

/* Test-side trace (NULL = off): every planner move made inside a rollout, and
   per played ply of or_play_game the search's (predicts, main_draws, sim_draws).
   Lets the checker compare decisions that never show in a game's moves. */
static int32_t* g_tr_mv;
static int g_tr_mv_cap, g_tr_mv_n;
static int64_t* g_tr_ply;
static int g_tr_ply_cap, g_tr_ply_n;

void or_trace_set(int32_t* planner_moves, int mv_cap, int64_t* ply_stats, int ply_cap) {
    g_tr_mv = planner_moves;
    g_tr_mv_cap = mv_cap;
    g_tr_mv_n = 0;
    g_tr_ply = ply_stats;
    g_tr_ply_cap = ply_cap;
    g_tr_ply_n = 0;
}

void or_trace_counts(int* n_moves, int* n_plies) {
    *n_moves = g_tr_mv_n;
    *n_plies = g_tr_ply_n;
}

/* _simulate, ai_agent.py:251-285: planner plies first, then the offensive policy */
double or_rollout_planner(const or_board* start, int ai, const or_params* p, int64_t game_id, int32_t sim,
                          uint64_t key, uint64_t* draws, or_board* final_out) {
    or_board b = *start;
    if (!b.over) {
        int steps = 0;
        int tmp[CELLS];
        float pv[CELLS], qv[CELLS];
        while (!b.over && steps < p->planner_steps) {
            /* NaN until filled: a callback that fails to write its outputs can never
               pass for valid net values (oracle.py re-raises its exception) */
            for (int i = 0; i < CELLS; i++) pv[i] = qv[i] = NAN;
            if (p->pq) p->pq(p->pq_ctx, &b, game_id, sim, steps, pv, qv);
            else or_gnet_forward(p->gn_blob, &b, NULL, pv, qv);
            int mv = or_planner_move(&b, ai, &p->planner, pv, qv, key, draws);
            if (g_tr_mv) {
                if (g_tr_mv_n < g_tr_mv_cap) g_tr_mv[g_tr_mv_n] = mv;
                g_tr_mv_n++;
            }
            if (mv < 0) break;
            or_make_move(&b, mv / N, mv % N);
            steps++;
        }
        while (!b.over && steps < p->max_depth) {
            if (legal_list(&b, tmp) == 0) break;
            int mv = or_offensive_move(&b, key, draws);
            or_make_move(&b, mv / N, mv % N);
            steps++;
        }
    }
    if (final_out) *final_out = b;
    return terminal_value(&b, ai);
}

/* ----------------------------------------------------------------- MCTS */
typedef struct {
    or_board b;
    int parent, move, visits, term;
    double value, bg;
    int16_t unexp[CELLS];
    int n_unexp;
    int16_t* kids;
    int n_kids;
} onode;

typedef struct {
    onode* nodes;
    int n, cap;
    int predicts;
} otree;

/* MCTSNode.__init__, ai_agent.py:494-523 */
static int new_node(otree* t, const or_board* b, int parent, int move, int ai, double beta) {
    onode* x = &t->nodes[t->n];
    x->b = *b;
    x->parent = parent;
    x->move = move;
    x->visits = 0;
    x->value = 0.0;
    x->term = b->over;
    x->n_unexp = 0;
    for (int i = 0; i < CELLS; i++)
        if (b->cell[i] == 0) x->unexp[x->n_unexp++] = (int16_t)i;
    x->n_kids = 0;
    x->kids = (int16_t*)malloc(sizeof(int16_t) * CELLS);
    /* the UCB's BG term is a pure function of the node's board: evaluate once */
    x->bg = (parent >= 0) ? or_bg_score(b, ai) : 0.0;
    (void)beta;
    if (!x->term) t->predicts++; /* GomokuModel.predict per non-terminal node (:522-523) */
    return t->n++;
}

/* MCTSNode.ucb1, ai_agent.py:532-562 (time_reward is always 0: the model never
 * carries _last_decision_time, :553) */
static double ucb1(const otree* t, const onode* x, const or_params* p) {
    if (x->visits == 0) return __builtin_inf();
    double exploitation = x->value / (double)x->visits;
    int pv = t->nodes[x->parent].visits;
    if (pv < 1) pv = 1;
    double lg = GZ_LOG_TABLE[pv];
    double m = (lg > 1.0) ? lg : 1.0;
    double exploration = p->c_puct * __builtin_sqrt(m / (double)x->visits);
    double base = exploitation + exploration;
    double bg_bonus = p->beta * x->bg;
    double time_reward = 0.0;
    return base + bg_bonus + time_reward;
}

/* _best_child, ai_agent.py:450-454: Python max keeps the first maximum */
static int best_child(const otree* t, const onode* x, const or_params* p) {
    int best = x->kids[0];
    double bv = ucb1(t, &t->nodes[best], p);
    for (int k = 1; k < x->n_kids; k++) {
        double v = ucb1(t, &t->nodes[x->kids[k]], p);
        if (v > bv) {
            bv = v;
            best = x->kids[k];
        }
    }
    return best;
}

/* _mcts_search + _mcts_simulation, ai_agent.py:168-222 */
static int mcts_search(const or_board* b, int ai, const or_params* p, int64_t game_id,
                       const int* L, int nL, uint64_t kmain, uint64_t* dmain, or_tree_info* info) {
    otree t;
    int S = p->num_simulations;
    t.cap = S + 2;
    t.nodes = (onode*)malloc(sizeof(onode) * (size_t)t.cap);
    t.n = 0;
    t.predicts = 0;
    int ply = b->n_moves;
    int64_t sim_draws = 0;
    new_node(&t, b, -1, -1, ai, p->beta);
    for (int k = 1; k <= S; k++) {
        uint64_t key = or_stream_key(p->seed, game_id, ply, k);
        uint64_t dk = 0;
        int x = 0; /* _select, :224-232 */
        while (!t.nodes[x].term && t.nodes[x].n_kids > 0) {
            if (t.nodes[x].n_unexp > 0) break;
            x = best_child(&t, &t.nodes[x], p);
        }
        if (!t.nodes[x].term && t.nodes[x].visits > 0 && t.nodes[x].n_unexp > 0) { /* _expand :234-249 */
            onode* par = &t.nodes[x];
            int mv = par->unexp[--par->n_unexp];
            or_board cb = par->b;
            or_make_move(&cb, mv / N, mv % N);
            int c = new_node(&t, &cb, x, mv, ai, p->beta);
            t.nodes[x].kids[t.nodes[x].n_kids++] = (int16_t)c;
            x = c;
        }
        double v; /* _simulate :251-285 */
        if (t.nodes[x].term) v = terminal_value(&t.nodes[x].b, ai);
        else if (p->planner_steps > 0) v = or_rollout_planner(&t.nodes[x].b, ai, p, game_id, k, key, &dk, NULL);
        else v = or_rollout(&t.nodes[x].b, ai, p->max_depth, key, &dk, NULL);
        sim_draws += (int64_t)dk;
        while (x >= 0) { /* _backpropagate :441-448 */
            t.nodes[x].visits += 1;
            t.nodes[x].value += v;
            x = t.nodes[x].parent;
        }
    }
    int best;
    onode* root = &t.nodes[0];
    if (root->n_kids > 0) { /* :199-201 */
        int bi = root->kids[0];
        for (int k = 1; k < root->n_kids; k++)
            if (t.nodes[root->kids[k]].visits > t.nodes[bi].visits) bi = root->kids[k];
        best = t.nodes[bi].move;
    } else {
        best = L[choice_idx(kmain, dmain, nL)]; /* :204 */
    }
    if (info) {
        info->n_nodes = t.n;
        info->predicts = t.predicts;
        info->sim_draws = sim_draws;
        for (int i = 0; i < t.n && i < info->cap; i++) {
            info->parent[i] = t.nodes[i].parent;
            info->move[i] = t.nodes[i].move;
            info->visits[i] = t.nodes[i].visits;
            info->value[i] = t.nodes[i].value;
        }
    }
    for (int i = 0; i < t.n; i++) free(t.nodes[i].kids);
    free(t.nodes);
    return best;
}

/* AlphaZeroGomokuAI.get_move + _opening_move, ai_agent.py:109-166 */
int or_get_move(const or_board* b, int ai, const or_params* p, int64_t game_id, or_tree_info* info) {
    int L[CELLS];
    int nL = legal_list(b, L);
    int ply = b->n_moves;
    uint64_t kmain = or_stream_key(p->seed, game_id, ply, 0), dmain = 0;
    if (info) {
        info->n_nodes = 0;
        info->predicts = 0;
        info->sim_draws = 0;
        info->main_draws = 0;
    }
    if (nL == 0) return -1;
    int best;
    if (ply < 6) {
        if (ply == 0 && b->cell[7 * N + 7] == 0) return 7 * N + 7;
        int C[CELLS], nc = 0;
        for (int k = 0; k < nL; k++)
            if (abs(L[k] / N - 7) <= 1 && abs(L[k] % N - 7) <= 1) C[nc++] = L[k];
        if (nc) {
            best = C[choice_idx(kmain, &dmain, nc)];
            if (info) info->main_draws = (int32_t)dmain;
            return best;
        }
        for (int k = 0; k < nL; k++)
            if (abs(L[k] / N - 7) <= 2 && abs(L[k] % N - 7) <= 2) C[nc++] = L[k];
        if (nc) {
            best = C[choice_idx(kmain, &dmain, nc)];
            if (info) info->main_draws = (int32_t)dmain;
            return best;
        }
        best = mcts_search(b, ai, p, game_id, L, nL, kmain, &dmain, info);
        if (info) info->main_draws = (int32_t)dmain;
        return best;
    }
    best = mcts_search(b, ai, p, game_id, L, nL, kmain, &dmain, info);
    if (to_unit(or_draw(kmain, dmain++)) < p->exploration) best = L[choice_idx(kmain, &dmain, nL)];
    if (info) info->main_draws = (int32_t)dmain;
    return best;
}

/* training.play_one_game (no timeouts) + SimpleReplay, training.py:77-97,141-218 */
int or_play_game(const or_params* black, const or_params* white, int64_t game_id, int8_t* cells_out,
                 int32_t* moves_out, int8_t* players_out, int8_t* z_out, int cap, int* winner,
                 int64_t* predicts, int max_plies) {
    or_board b;
    or_board_init(&b);
    int n = 0;
    int64_t pred = 0;
    int32_t parent[1], move[1], visits[1];
    double value[1];
    or_tree_info info = {0, 0, 0, 0, parent, move, visits, value, 0};
    while (!b.over && (max_plies <= 0 || n < max_plies)) {
        int pl = b.player;
        const or_params* p = (pl == 1) ? black : white;
        int mv = or_get_move(&b, pl, p, game_id, &info);
        pred += info.predicts;
        if (g_tr_ply) {
            if (g_tr_ply_n < g_tr_ply_cap) {
                g_tr_ply[3 * g_tr_ply_n] = info.predicts;
                g_tr_ply[3 * g_tr_ply_n + 1] = info.main_draws;
                g_tr_ply[3 * g_tr_ply_n + 2] = info.sim_draws;
            }
            g_tr_ply_n++;
        }
        if (mv < 0) break;
        if (n < cap) {
            if (cells_out) memcpy(cells_out + (size_t)n * CELLS, b.cell, CELLS);
            moves_out[n] = mv;
            players_out[n] = (int8_t)pl;
        }
        n++;
        or_make_move(&b, mv / N, mv % N);
    }
    for (int i = 0; i < n && i < cap; i++)
        z_out[i] = (int8_t)(b.winner == 0 ? 0 : (players_out[i] == b.winner ? 1 : -1));
    if (winner) *winner = b.winner;
    if (predicts) *predicts = pred;
    return n;
}
