/*
 * gzero.h -- C-ABI of libgzero.so, the MI355X (gfx950) self-play engine that
 * replaces the hot path of gitMasterLiujiahui/AlphaZero-Gomoku.
 *
 * The reference is pure Python with no FFI, so every entry point below
 * replaces a Python call site; the binding a maintainer would add (ctypes,
 * the same shape as cgo/JNI) is in INTEGRATION.md and in
 * alphazero-gomoku_amd/gzero/_lib.py.
 *
 * Conventions
 *  - All pointers named d_* are DEVICE pointers owned by the caller (torch
 *    tensors in the Python host).  `stream` is a hipStream_t passed as void*.
 *    Calls are stream-ordered and asynchronous; none allocates or synchronises.
 *  - Return value: GZ_OK (0) or a negative GZ_ERR_*; gz_last_error() holds a
 *    thread-local message.  Misuse (bad sizes) is rejected before any launch.
 *  - Boards are bit planes: row r in word r>>1, bits (r&1)*16 + c (c < 15);
 *    bit 15 of each row and row 15 are zero.  Cells are row-major r*15+c.
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GZ_OK 0
#define GZ_ERR_ARG -1
#define GZ_ERR_HIP -2
#define GZ_ERR_UNSUPPORTED -3
#define GZ_ERR_INTERNAL -4

#define GZ_MAX_SIMULATIONS 4095
#define GZ_MAX_GAME_PLIES 200

/* GomokuBoard state (gomoku_board.py:40-53): stones, len(move_history),
 * current_player (1/2), game_over, winner (0 = None). 80 bytes. */
typedef struct gz_board_state {
    uint32_t black[8];
    uint32_t white[8];
    int32_t n_moves;
    int32_t player;
    int32_t over;
    int32_t winner;
} gz_board_state;

/* AlphaZeroGomokuAI search knobs (ai_agent.py:29-31,65-90); difficulty maps
 * to num_simulations / c_puct / exploration exactly as the reference's table. */
typedef struct gz_search_params {
    int32_t num_simulations; /* params["num_simulations"] */
    int32_t max_depth;       /* rollout cap, _simulate max_depth (100) */
    double c_puct;           /* params["c_puct"] */
    double exploration;      /* params["exploration"] */
    double beta;             /* constructor beta: weight of tanh(pattern/1e4) in UCB */
    uint64_t seed;           /* RNG streams (gzero/rng.py) */
    int32_t planner_steps;   /* BG-planner plies per rollout (> 0: gz_plan_search / gz_selfplay_plan_run) */
    int32_t flags;           /* GZ_FLAG_* */
} gz_search_params;

#define GZ_FLAG_GATHER_LEAVES 1 /* append every non-terminal node's board for the PV forward */
#define GZ_FLAG_GN_CHECK 2      /* planner searches: also run the full GraphNet forward on every
                                   incremental row and count differing rows (gz_plan_gn_stats) */

/* BGPlannerAI.params (bg_planner.py:215-219): easy {8, 0.5, 0.2}, medium
 * {12, 0.65, 0.1}, hard {16, 0.75, 0.05}. */
typedef struct gz_planner_params {
    int32_t k;       /* knowledge-search top-k, 1..16 */
    int32_t pad;
    double alpha;    /* mix_alpha */
    double explore;  /* exploration probability */
} gz_planner_params;

/* One (s, pi, z) training tuple (training.py:77-97,203-210). 80 bytes. */
typedef struct gz_record {
    uint32_t black[8]; /* planes before the move (absolute colours) */
    uint32_t white[8];
    int64_t game_id;
    int16_t ply;    /* move number within the game */
    int16_t move;   /* r*15+c */
    int8_t player;  /* mover, 1/2 */
    int8_t z;       /* +1 mover won, -1 lost, 0 draw */
    int8_t pad[2];
} gz_record;

typedef struct gz_search_stats {
    int32_t n_nodes;
    int32_t predicts;   /* GomokuModel.predict calls the reference makes for this move */
    int32_t main_draws; /* draws on the (game, ply, 0) stream */
    int32_t pad;
    int64_t sim_draws;  /* draws summed over simulation streams */
} gz_search_stats;

typedef struct gz_selfplay_counters {
    int32_t records;         /* records written to d_records */
    int32_t leaves;          /* boards appended to d_leaves */
    int32_t records_dropped; /* records lost because d_records was full */
    int32_t leaves_dropped;
    int64_t moves;           /* plies played */
    int64_t games;           /* games finished */
    int64_t mcts_moves;      /* plies decided by MCTS (n_moves >= 6; the opening plies
                                0-5 of _opening_move do no search, ai_agent.py:138-166) */
} gz_selfplay_counters;

const char* gz_last_error(void);
int gz_version(void);

/* ---- K1: board step / legal mask / five-in-a-row (gomoku_board.py:84-213) ----
 * d_boards[i] <- make_move(d_moves[i]) (cell r*15+c, or any value outside
 * [0,225) which fails like an off-board move).  d_ok[i] = make_move's return.
 * d_legal (optional) = [n][4] uint64 row-major masks of empty cells after the
 * step (get_valid_moves, which ignores game_over). */
int gz_board_step(gz_board_state* d_boards, const int32_t* d_moves, int32_t n, int32_t* d_ok,
                  uint64_t* d_legal, void* stream);

/* ---- rollout policy and rollouts (ai_agent.py:251-430) ----
 * Component entry points used by the parity tests. keys = RNG stream keys. */
int gz_policy_move(const gz_board_state* d_boards, const uint64_t* d_keys, int32_t n, int32_t* d_moves,
                   uint32_t* d_draws, void* stream);
int gz_rollout(const gz_board_state* d_boards, const int32_t* d_ai, const uint64_t* d_keys, int32_t n,
               int32_t max_depth, double* d_values, gz_board_state* d_final, uint32_t* d_draws,
               void* stream);

/* ---- pattern score / _bg_score (bg_planner.py:133-196, ai_agent.py:432-439) ---- */
int gz_pattern_score(const gz_board_state* d_boards, const int32_t* d_player, int32_t n, int64_t* d_score,
                     double* d_bg, void* stream);

/* ---- K2+K3: one AlphaZeroGomokuAI.get_move per board (ai_agent.py:109-222) ----
 * One wavefront per board.  d_trees: n * gz_tree_bytes(num_simulations)
 * scratch holding each search tree (layout in DESIGN.md; readable by tests).
 * d_moves[i] = chosen cell or -1 (None).  Leaves are appended to d_leaves
 * ([leaf_cap][16] uint32: black[8], white[8]) when GZ_FLAG_GATHER_LEAVES. */
size_t gz_tree_bytes(int32_t num_simulations);
int gz_search(const gz_board_state* d_boards, const int64_t* d_game_ids, int32_t n,
              const gz_search_params* p, void* d_trees, int32_t* d_moves, gz_search_stats* d_stats,
              uint32_t* d_leaves, int32_t leaf_cap, int32_t* d_leaf_count, void* stream);

/* ---- self-play collector (training.py:141-218) over n_slots concurrent games ----
 * Slot s plays games game_id_base + s + g*game_id_stride, g = 0,1,2,...  Each
 * call advances every slot by n_plies plies; a finished game's tuples (with z)
 * are appended to d_records and the slot restarts from the empty board.
 * d_leaf_meta (optional, [leaf_cap] int32) tags every gathered leaf for
 * gz_pv_forward_tree: -1 = a search root, i >= 0 = a child of the node at leaf
 * index i (one stone more; that node is the root or one of its children), -2 =
 * any deeper node. */
size_t gz_slot_bytes(int32_t num_simulations);
int gz_selfplay_init(void* d_slots, int32_t n_slots, int32_t num_simulations, int64_t game_id_base,
                     int64_t game_id_stride, void* stream);
int gz_selfplay_run(void* d_slots, int32_t n_slots, const gz_search_params* p, int32_t n_plies,
                    gz_record* d_records, int32_t record_cap, uint32_t* d_leaves, int32_t leaf_cap,
                    int32_t* d_leaf_meta, gz_selfplay_counters* d_counters, void* stream);
/* gz_selfplay_run with BG-planner rollout plies (p->planner_steps > 0): each ply
 * is one gz_plan_search over all slots (host-driven, synchronises the stream
 * once per simulation round) followed by the same record / restart logic;
 * d_leaf_meta (optional) as for gz_selfplay_run.
 * d_workspace: gz_selfplay_plan_workspace_bytes(n_slots, num_simulations). */
size_t gz_selfplay_plan_workspace_bytes(int32_t n_slots, int32_t num_simulations);
int gz_selfplay_plan_run(void* d_slots, int32_t n_slots, const gz_search_params* p, const gz_planner_params* pp,
                         const float* d_gn_weights, void* d_workspace, int32_t n_plies, gz_record* d_records,
                         int32_t record_cap, uint32_t* d_leaves, int32_t leaf_cap, int32_t* d_leaf_meta,
                         gz_selfplay_counters* d_counters, void* stream);
/* per slot, totals over every search it ran since gz_selfplay_init: d_out[3s] =
 * predict() calls, d_out[3s+1] = main-stream RNG draws, d_out[3s+2] = simulation-
 * stream draws (the checker's view of rollout / planner decisions, ai_agent.py:168-285) */
int gz_selfplay_draws(const void* d_slots, int32_t n_slots, int64_t* d_out, void* stream);
/* A bounded game range (training.py:374-377 plays exactly its n games per iteration):
 * a slot whose next game id would be >= game_id_end goes idle instead of restarting --
 * gz_selfplay_run / gz_selfplay_plan_run skip it and record nothing for it (default:
 * no end, continuous refill). */
int gz_selfplay_set_game_end(void* d_slots, int32_t n_slots, int64_t game_id_end, void* stream);
/* Copies the slots into d_dst (another n_slots-slot buffer) with the active ones first
 * and the idle ones after, each in slot order; *d_n_active = the active count.  A slot
 * holds its whole game state, so the caller may then run the first *d_n_active slots
 * of d_dst only.  d_workspace: gz_selfplay_compact_workspace_bytes(n_slots). */
size_t gz_selfplay_compact_workspace_bytes(int32_t n_slots);
int gz_selfplay_compact(const void* d_slots, int32_t n_slots, void* d_dst, int32_t* d_n_active, void* d_workspace,
                        void* stream);
/* current board of every slot (for inspection / tests) */
int gz_selfplay_boards(const void* d_slots, int32_t n_slots, int32_t num_simulations,
                       gz_board_state* d_out, int64_t* d_game_ids, void* stream);

/* ---- K6: AlphaZeroGomokuNet forward (neural_network.py:94-159,214-252) ----
 * d_weights: packed blob of gz_pv_weight_floats() floats (layout in
 * csrc/gz_pvnet.h / gzero/weights.py).  Boards [n][16] uint32 bit planes.  If
 * d_count is not NULL it holds the number of valid boards on the device
 * (n = capacity).  Outputs: logits [n][225], value [n] (tanh), probs
 * [n][225] (softmax) or NULL; prior (optional, needs probs) = [n][225] float64
 * MCTSNode._get_prior_probability (ai_agent.py:564-582): the softmax at the empty
 * cells renormalised by their float64 sum (numpy's pairwise order), 0 at stones --
 * the reference's compact vector is prior[i][empty cells, row-major].
 * precision: GZ_PV_FP32 (exact f32 MFMA) or
 * GZ_PV_F16X3 (3-term fp16 split on the fp16 MFMA, ~22-bit operands, f32
 * accumulation).  d_workspace: gz_pv_workspace_bytes(n) bytes, required (fp32:
 * per-wave slabs; f16x3: the 1x1 head convs' outputs of every board, 2,816 B
 * each, passed from the tower kernel to the batched FC-heads kernel). */
#define GZ_PV_FP32 0
#define GZ_PV_F16X3 1
size_t gz_pv_weight_floats(void);
size_t gz_pv_workspace_bytes(int32_t n);
int gz_pv_forward(const float* d_weights, const uint32_t* d_boards, int32_t n, const int32_t* d_count,
                  float* d_logits, float* d_value, float* d_probs, double* d_prior, void* d_workspace,
                  int32_t precision, void* stream);

/* Incremental forward of the nodes of MCTS searches (MCTSNode.__init__ ->
 * GomokuModel.predict, ai_agent.py:522-523; neural_network.py:132-159), f16x3:
 * d_meta as written by gz_selfplay_run.  Roots and untagged nodes run the full
 * forward (roots also keep their intermediate maps and pre-BN accumulators, at
 * most root_cap of them) and are bit-identical to gz_pv_forward(..., GZ_PV_F16X3,
 * ...) of the same boards.  A root's children are the root's pre-BN accumulators
 * plus the convolution of their one-stone input differences (radius 1..4 per
 * layer's input): the same network in f16x3 arithmetic with fp32 accumulation in
 * another order, within 2e-5 of the full forward's logits / value (1e-4 of the
 * reference's fp32 forward).  The children of a root child (grandchildren)
 * recompute the windows around their stone from the root's maps overlaid with
 * their parent's recomputed squares (at most 16 * root_cap parents).  A tag whose
 * board does not differ from its parent's by exactly one cell is ignored (full
 * forward), so the tags only decide speed.  d_workspace:
 * gz_pv_tree_workspace_bytes(n, root_cap) bytes (~2.4 MB per root: maps 512 KB,
 * pre-BN accumulators 512 KB, 16 patches of 84 KB). */
size_t gz_pv_tree_workspace_bytes(int32_t n, int32_t root_cap);
int gz_pv_forward_tree(const float* d_weights, const uint32_t* d_boards, const int32_t* d_meta, int32_t n,
                       const int32_t* d_count, int32_t root_cap, float* d_logits, float* d_value, float* d_probs,
                       double* d_prior, void* d_workspace, void* stream);
/* d_out6 (device int32[6]) = the last tree forward's list sizes: roots seen, roots
 * with stored maps, incremental children, full-forward boards, incremental
 * grandchildren, parents that claimed a patch slot. */
int gz_pv_tree_stats(const void* d_workspace, int32_t n, int32_t* d_out6, void* stream);
/* d_out2 (device int32[2]) = the 16-row x 128-channel x 1152-deep MFMA tiles of the
 * residual convs the last tree forward's incremental kernels executed, for root
 * children and for grandchildren (measurement: bench.py's executed-FLOP roofline). */
int gz_pv_tree_exec_tiles(const void* d_workspace, int32_t n, int32_t* d_out2, void* stream);

/* ---- K7: BG planner nets (bg_planner.py:22-78, BGPlannerAI.get_move :243-250) ----
 * d_weights: packed blob of gz_gn_weight_floats() floats (csrc/gz_gnet.h,
 * gzero/planner_nets.py).  Boards [n][16] uint32 bit planes (d_count as above).
 * Outputs: p = softmax(GraphNet(planes)) [n][225], q = OpponentDQN(planes)
 * [n][225], logits [n][225] or NULL.  GraphNet convs in f16x3 (as GZ_PV_F16X3);
 * the policy FC and the DQN run batched over 32 boards per workgroup (fp32 MFMA);
 * a launch of fewer than 64 boards per CU without logits runs them split over output
 * tiles instead (16 boards x 4 tiles per workgroup, three launches, p and q the same
 * bits), the layers' outputs through the workspace.  GZ_GN_SMALL_HEADS=<rows> moves
 * that threshold (A/B knob).
 * d_workspace: gz_gn_workspace_bytes(n) bytes, required (per row a 3.6 KB net record,
 * then 3 KB of the split heads' scratch). */
size_t gz_gn_weight_floats(void);
size_t gz_gn_workspace_bytes(int32_t n);
int gz_gn_forward(const float* d_weights, const uint32_t* d_boards, int32_t n, const int32_t* d_count,
                  float* d_p, float* d_q, float* d_logits, void* d_workspace, void* stream);

/* ---- K4+K5+K7: MCTS with BG-planner rollout plies (planner_steps > 0) ----
 * gz_search's contract (ai_agent.py:109-222) for p->planner_steps >= 0 with the
 * planner of pp (BGPlannerAI for the searching AI's colour, bg_planner.py:199-269)
 * and its nets d_gn_weights (gz_gn_forward).  Host-driven: launches on `stream`
 * and synchronises it once per simulation round.  d_workspace:
 * gz_plan_workspace_bytes(n, num_simulations) bytes.  d_trees (optional) gets
 * gz_tree_bytes(num_simulations) bytes per game in gz_search's layout.
 * Footprint (C = max(n, 65536) GN rows per planner step, capped at n*S): per game
 * its context + tree and S 128-B jobs; per row 0.9 KB of p / q, a 6.6 KB net
 * workspace (gz_gn_workspace_bytes(1)) and, always reserved, the same again for
 * GZ_FLAG_GN_CHECK's full-forward copy (0.56 GB each at C = 65536); and n + C
 * incremental-GraphNet map slots of 232 KB (16.2 GB at n = 4096, S = 200 -- 17.4 GB
 * in all). */
size_t gz_plan_workspace_bytes(int32_t n, int32_t num_simulations);
int gz_plan_search(const gz_board_state* d_boards, const int64_t* d_game_ids, int32_t n,
                   const gz_search_params* p, const gz_planner_params* pp, const float* d_gn_weights,
                   void* d_workspace, void* d_trees, int32_t* d_moves, gz_search_stats* d_stats,
                   uint32_t* d_leaves, int32_t leaf_cap, int32_t* d_leaf_count, void* stream);

/* Incremental planner nets inside gz_plan_search / gz_selfplay_plan_run: a planner
 * ply's board is its predecessor plus the planner's move, and a rollout's first
 * board usually the search root plus one stone (bg_planner.py:243-250,
 * ai_agent.py:251-285), so GraphNet recomputes only the radius 1..5 squares around
 * the new stone from kept maps (the root's, or the rollout's own chain); the outputs
 * are bit-identical to gz_gn_forward's.  GZ_GN_INC=0 in the environment turns it
 * off.  out[4] (host) = rows run by the full forward, by the incremental forward,
 * rows checked against the full forward (GZ_FLAG_GN_CHECK) and rows that differed,
 * summed since the last reset (reset != 0 zeroes them after reading; the counters
 * start undefined until the first reset).  gz_selfplay_plan_gn_stats takes
 * gz_selfplay_plan_run's workspace. */
/* The incremental GraphNet on explicit chains (tests, tools): row i's 32-byte tag
 * (csrc/gz_gnet.h GnTag) = {mode, base, job, cell, nst, stones[6], pad}: mode 0 =
 * full forward, its maps and policy-conv outputs kept in slot `job`; mode 1 = the
 * board is the board of slot `base` plus the stone `cell`, with the squares of the
 * earlier stones stones[0..nst) (added since `base`) in slot `job`, where this row's
 * squares go too.  Slots: gz_gn_slot_bytes() each.  p, q as gz_gn_forward (bit-
 * identical).  Rows of one call must use distinct `job` slots, and no row's `job`
 * may be another row's `base`.  d_workspace: gz_gn_chain_workspace_bytes(n). */
size_t gz_gn_slot_bytes(void);
size_t gz_gn_chain_workspace_bytes(int32_t n);
int gz_gn_forward_chain(const float* d_weights, const uint32_t* d_boards, int32_t n, const void* d_tags,
                        void* d_slots, float* d_p, float* d_q, void* d_workspace, void* stream);
int gz_plan_gn_stats(void* d_workspace, int32_t n, int32_t num_simulations, int64_t* out, int32_t reset,
                     void* stream);
int gz_selfplay_plan_gn_stats(void* d_workspace, int32_t n_slots, int32_t num_simulations, int64_t* out,
                              int32_t reset, void* stream);

/* BGPlannerAI.get_move (bg_planner.py:232-269) for each board: d_ai = the
 * planner's colour P, d_keys = RNG stream; d_moves (-1 = None), d_draws.
 * d_workspace: gz_planner_move_workspace_bytes(n) bytes. */
size_t gz_planner_move_workspace_bytes(int32_t n);

/* KnowledgeSearch.score_move(board, (r, c), player) (bg_planner.py:90-106) for
 * every cell of every board, the side to move playing the stone: d_scores
 * [n][225] float64 -- 1e6 (the move wins for player), -1e5 (player's opponent can
 * then complete five, _opponent_can_win_next :116-125), else _pattern_score +
 * _center_bias (:127-196); -1e9 at occupied cells (is_valid_move fails).
 * top_k_moves (:108-114) = the first k cells of a stable descending sort. */
int gz_knowledge_scores(const gz_board_state* d_boards, const int32_t* d_player, int32_t n, double* d_scores,
                        void* stream);
int gz_planner_move(const gz_board_state* d_boards, const int32_t* d_ai, const uint64_t* d_keys, int32_t n,
                    const gz_planner_params* pp, const float* d_gn_weights, void* d_workspace,
                    int32_t* d_moves, uint32_t* d_draws, void* stream);

/* ---- K8 training-set materialisation (GomokuSelfPlayDataset, training.py:104-134;
 * augment_sample, training.py:44-71).  Samples [0, n) are the records as is;
 * sample n + 8j + 2k + f is record d_sel[j] under rot90^k (np.rot90, axes (1,2))
 * then, if f, np.flip(axis=2).  Outputs: d_x float32 [n+8m][3][15][15] planes
 * [black, white, empty]; d_y int64 move labels (the reference's label map, which
 * rotates the other way, unless GZ_AUG_FIX_LABELS); d_v float32 z.  d_sel values
 * must lie in [0, n) (others give zero planes and label -1). */
#define GZ_AUG_FIX_LABELS 1
int gz_dataset_build(const gz_record* d_records, int32_t n, const int32_t* d_sel, int32_t m, int32_t flags,
                     float* d_x, int64_t* d_y, float* d_v, void* stream);
/* The samples d_ids[0..count) of that dataset (a training batch, e.g. a DataLoader
 * permutation slice) without materialising the rest: outputs [count][...].
 * Ids outside [0, n+8m) give zero planes and label -1. */
int gz_dataset_gather(const gz_record* d_records, int32_t n, const int32_t* d_sel, int32_t m, const int64_t* d_ids,
                      int64_t count, int32_t flags, float* d_x, int64_t* d_y, float* d_v, void* stream);

/* ---- f1 training step: the policy-value net's convolutional part in training mode
 * (training.py:277-311 over neural_network.py:74-91, 132-159: BatchNorm on batch
 * statistics), forward and backward on the device (csrc/gz_sgd.hip):
 *   a0 = relu(BN0(conv0(x))); per block: h = relu(BN1(conv1(a) + b1)), a' = relu(BN2(conv2(h) + b2) + a);
 *   pin = policy_conv(a2) (flattened [boards][2 * 225]), vin = value_conv(a2) ([boards][225])
 * The FC heads (policy_fc, value_fc1/2), the loss and the optimiser stay with the caller
 * (gzero/sgd.py).  x = the model input planes float32 [boards][3][15][15]; activations
 * are fp32 NHWC [boards][225][128] in the workspace.  Weights in torch's layouts:
 * conv0 [128][3][3][3]; residual convs [128][128][3][3] (tower.0.conv1, tower.0.conv2,
 * tower.1.conv1, tower.1.conv2); policy_conv [2][128]; value_conv [1][128].  BN order:
 * bn, tower.0.bn1, tower.0.bn2, tower.1.bn1, tower.1.bn2.  gz_sgd_forward updates the
 * running statistics (momentum, unbiased variance) like torch.nn.BatchNorm2d.train();
 * the workspace (gz_sgd_workspace_bytes) carries the saved activations and statistics
 * from gz_sgd_forward to the gz_sgd_backward of the same batch. */
#define GZ_SGD_MAX_BOARDS 65535
typedef struct gz_sgd_net {
    const float* bn_weight[5];
    const float* bn_bias[5];
    float* bn_running_mean[5]; /* updated in place; NULL: not tracked */
    float* bn_running_var[5];
    const float* conv_weight[4];
    const float* conv_bias[4];
    float momentum, eps;
    const float* conv0_weight;
    const float* conv0_bias;
    const float* policy_weight;
    const float* policy_bias;
    const float* value_weight;
    const float* value_bias;
} gz_sgd_net;
typedef struct gz_sgd_grads { /* outputs (overwritten, not accumulated) */
    float* bn_weight[5];
    float* bn_bias[5];
    float* conv_weight[4];
    float* conv_bias[4];
    float* conv0_weight;
    float* conv0_bias;
    float* policy_weight;
    float* policy_bias;
    float* value_weight;
    float* value_bias;
} gz_sgd_grads;
size_t gz_sgd_workspace_bytes(int32_t boards);
/* d_pin [boards][450], d_vin [boards][225]: the heads' conv outputs of planes d_x */
int gz_sgd_forward(const gz_sgd_net* net, int32_t boards, const float* d_x, float* d_pin, float* d_vin,
                   void* d_workspace, void* stream);
/* from dL/dpin, dL/dvin: every parameter's gradient (d_x and the workspace are the
 * forward's) */
int gz_sgd_backward(const gz_sgd_net* net, int32_t boards, const float* d_x, const float* d_dpin,
                    const float* d_dvin, const gz_sgd_grads* grads, void* d_workspace, void* stream);
/* The FC heads and the loss of the training step (training.py:292-297 over
 * neural_network.py:150-159): logits = policy_fc(pin), val = tanh(value_fc2(relu(
 * value_fc1(vin)))), loss = CrossEntropy(logits, y) + MSE(val, v) (batch means), and
 * its backward: d_dpin [boards][450] and d_dvin [boards][225] for gz_sgd_backward and
 * the six FC gradients (overwritten), all multiplied by `scale` (1, or this rank's
 * share of a data-parallel global batch).  d_y int64 class labels [boards], d_v
 * [boards] targets; d_loss float[3] = {loss, mean cross-entropy, mean squared error}
 * (unscaled).  Weights in torch's layouts: policy_fc [225][450], value_fc1 [64][225],
 * value_fc2 [1][64].  d_ws: gz_sgd_fc_workspace_bytes(boards) bytes. */
typedef struct gz_sgd_fc {
    const float* policy_weight;
    const float* policy_bias;
    const float* value1_weight;
    const float* value1_bias;
    const float* value2_weight;
    const float* value2_bias;
} gz_sgd_fc;
typedef struct gz_sgd_fc_grads {
    float* policy_weight;
    float* policy_bias;
    float* value1_weight;
    float* value1_bias;
    float* value2_weight;
    float* value2_bias;
} gz_sgd_fc_grads;
size_t gz_sgd_fc_workspace_bytes(int32_t boards);
int gz_sgd_fc_loss(const gz_sgd_fc* fc, int32_t boards, const float* d_pin, const float* d_vin, const int64_t* d_y,
                   const float* d_v, float scale, float* d_dpin, float* d_dvin, const gz_sgd_fc_grads* grads,
                   float* d_loss, void* d_ws, void* stream);
/* checkers: a copy of a saved tensor of the last gz_sgd_forward on this workspace:
 * which 0..3 = the inputs of the four residual convs (a0, h1, a1, h2), 4..7 = their
 * outputs y1..y4, 8 = the tower output a2, 9 = y0 = conv0's output (fp32 NHWC) */
int gz_sgd_saved(const void* d_workspace, int32_t boards, int32_t which, float* d_out, void* stream);

/* The optimiser step of training.train_epoch (training.py:303-304): clip_grad_norm_(params,
 * max_norm) then Adam(lr, betas, eps, weight_decay) (torch.optim.Adam, L2 weight decay),
 * over up to GZ_ADAM_MAX_TENSORS tensors in two launches.  max_norm > 0: the gradients are
 * scaled by min(1, max_norm / (||g||_2 + 1e-6)) (the norm over every tensor, summed in
 * float64 in a fixed order: deterministic) -- in place, as clip_grad_norm_ does; max_norm
 * <= 0: no clipping.  step = the step number after this update (1 on the first).  Then per
 * element g' = g + wd p; m = b1 m + (1-b1) g'; v = b2 v + (1-b2) g'^2;
 * p -= (lr / (1-b1^step)) m / (sqrt(v) / sqrt(1-b2^step) + eps).  d_norm (optional): the
 * pre-clip norm (float32, as clip_grad_norm_ returns).  d_workspace:
 * gz_adam_workspace_bytes(). */
#define GZ_ADAM_MAX_TENSORS 48
typedef struct gz_adam_tensor {
    float* param;
    float* grad;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t numel;
} gz_adam_tensor;
size_t gz_adam_workspace_bytes(void);
int gz_adam_step(const gz_adam_tensor* tensors, int32_t n_tensors, float lr, float beta1, float beta2, float eps,
                 float weight_decay, int64_t step, float max_norm, float* d_norm, void* d_workspace, void* stream);

#ifdef __cplusplus
}
#endif
