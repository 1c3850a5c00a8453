"""Thin torch-owned-memory wrappers around the libgzero C-ABI.

Every buffer is a torch tensor on the current CUDA(HIP) device; raw pointers
and torch's current stream are handed to the library.  Nothing here runs on the
CPU as a substitute: without a GPU or the library the calls raise.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .boards import RECORD_DTYPE, STATE_DTYPE


def require_gpu():
    lib = _lib.load()
    if not torch.cuda.is_available():
        raise _lib.GzeroUnavailable("no HIP device visible: the gzero engine has no CPU fallback")
    return lib


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(None)


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def to_dev(arr):
    """numpy array (any dtype) -> uint8 device tensor holding the same bytes."""
    a = np.ascontiguousarray(arr)
    return torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).cuda()


def from_dev(t, dtype, count=None):
    a = t.cpu().numpy().view(dtype)
    return a if count is None else a[:count]


def search_params(num_simulations=200, c_puct=1.6, exploration=0.05, beta=0.2, seed=0, max_depth=100,
                  planner_steps=0, gather_leaves=False):
    return _lib.SearchParams(int(num_simulations), int(max_depth), float(c_puct), float(exploration),
                             float(beta), int(seed) & ((1 << 64) - 1), int(planner_steps),
                             _lib.GZ_FLAG_GATHER_LEAVES if gather_leaves else 0)


# ---------------------------------------------------------------- K1 board step
def board_step(states, moves):
    """Batched GomokuBoard.make_move: returns (new states, ok[int32], legal[n,4] uint64)."""
    lib = require_gpu()
    states = np.ascontiguousarray(states, dtype=STATE_DTYPE)
    n = len(states)
    d_states = to_dev(states)
    d_moves = torch.as_tensor(np.asarray(moves, np.int32)).cuda()
    d_ok = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_legal = torch.zeros(n * 4, dtype=torch.int64, device="cuda")
    _lib.check(lib.gz_board_step(ptr(d_states), ptr(d_moves), n, ptr(d_ok), ptr(d_legal), stream()), "gz_board_step")
    torch.cuda.synchronize()
    return (from_dev(d_states, STATE_DTYPE), d_ok.cpu().numpy(),
            d_legal.cpu().numpy().view(np.uint64).reshape(n, 4))


# ---------------------------------------------------------------- rollout policy
def policy_move(states, keys):
    lib = require_gpu()
    states = np.ascontiguousarray(states, dtype=STATE_DTYPE)
    n = len(states)
    d_states = to_dev(states)
    d_keys = torch.as_tensor(np.asarray(keys, np.uint64).view(np.int64)).cuda()
    d_moves = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_draws = torch.zeros(n, dtype=torch.int32, device="cuda")
    _lib.check(lib.gz_policy_move(ptr(d_states), ptr(d_keys), n, ptr(d_moves), ptr(d_draws), stream()),
               "gz_policy_move")
    torch.cuda.synchronize()
    return d_moves.cpu().numpy(), d_draws.cpu().numpy()


def rollout(states, ai, keys, max_depth=100):
    lib = require_gpu()
    states = np.ascontiguousarray(states, dtype=STATE_DTYPE)
    n = len(states)
    d_states = to_dev(states)
    d_ai = torch.as_tensor(np.asarray(ai, np.int32)).cuda()
    d_keys = torch.as_tensor(np.asarray(keys, np.uint64).view(np.int64)).cuda()
    d_vals = torch.zeros(n, dtype=torch.float64, device="cuda")
    d_fin = torch.zeros(n * STATE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    d_draws = torch.zeros(n, dtype=torch.int32, device="cuda")
    _lib.check(lib.gz_rollout(ptr(d_states), ptr(d_ai), ptr(d_keys), n, int(max_depth), ptr(d_vals), ptr(d_fin),
                              ptr(d_draws), stream()), "gz_rollout")
    torch.cuda.synchronize()
    return d_vals.cpu().numpy(), from_dev(d_fin, STATE_DTYPE), d_draws.cpu().numpy()


def pattern_score(states, players):
    lib = require_gpu()
    states = np.ascontiguousarray(states, dtype=STATE_DTYPE)
    n = len(states)
    d_states = to_dev(states)
    d_pl = torch.as_tensor(np.asarray(players, np.int32)).cuda()
    d_s = torch.zeros(n, dtype=torch.int64, device="cuda")
    d_bg = torch.zeros(n, dtype=torch.float64, device="cuda")
    _lib.check(lib.gz_pattern_score(ptr(d_states), ptr(d_pl), n, ptr(d_s), ptr(d_bg), stream()), "gz_pattern_score")
    torch.cuda.synchronize()
    return d_s.cpu().numpy(), d_bg.cpu().numpy()


# ---------------------------------------------------------------- MCTS get_move
def parse_tree(raw, num_simulations, n_nodes):
    """One exported search tree (LDS layout of gz_selfplay.hip) -> dict of arrays."""
    mn = num_simulations + 1
    b = np.asarray(raw, np.uint8)
    return {
        "value": b[0:8 * mn].view(np.float64)[:n_nodes],
        "bg": b[8 * mn:16 * mn].view(np.float64)[:n_nodes],
        "visits": b[16 * mn:20 * mn].view(np.int32)[:n_nodes],
        "parent": b[20 * mn:22 * mn].view(np.int16)[:n_nodes],
        "bound": b[22 * mn:24 * mn].view(np.int16)[:n_nodes],
        "move": b[24 * mn:25 * mn][:n_nodes],
        "term": b[25 * mn:26 * mn][:n_nodes],
    }


def search(states, game_ids, params, want_trees=False, leaf_cap=0):
    """One AlphaZeroGomokuAI.get_move per state.  Returns (moves, stats, trees, leaves)."""
    lib = require_gpu()
    states = np.ascontiguousarray(states, dtype=STATE_DTYPE)
    n = len(states)
    d_states = to_dev(states)
    d_gids = torch.as_tensor(np.asarray(game_ids, np.int64)).cuda()
    d_moves = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_stats = torch.zeros(n * ctypes.sizeof(_lib.SearchStats), dtype=torch.uint8, device="cuda")
    tb = lib.gz_tree_bytes(params.num_simulations)
    d_trees = torch.zeros(n * tb, dtype=torch.uint8, device="cuda") if want_trees else None
    gather = (params.flags & _lib.GZ_FLAG_GATHER_LEAVES) != 0
    d_leaves = torch.zeros(max(1, leaf_cap) * 16, dtype=torch.int32, device="cuda") if gather else None
    d_lc = torch.zeros(1, dtype=torch.int32, device="cuda") if gather else None
    _lib.check(lib.gz_search(ptr(d_states), ptr(d_gids), n, ctypes.byref(params), ptr(d_trees), ptr(d_moves),
                             ptr(d_stats), ptr(d_leaves), int(leaf_cap), ptr(d_lc), stream()), "gz_search")
    torch.cuda.synchronize()
    st = np.frombuffer(d_stats.cpu().numpy().tobytes(), dtype=np.dtype(
        [("n_nodes", "<i4"), ("predicts", "<i4"), ("main_draws", "<i4"), ("pad", "<i4"), ("sim_draws", "<i8")]))
    trees = None
    if want_trees:
        raw = d_trees.cpu().numpy().reshape(n, tb)
        trees = [parse_tree(raw[i], params.num_simulations, int(st["n_nodes"][i])) for i in range(n)]
    leaves = None
    if gather:
        cnt = int(d_lc.item())
        leaves = d_leaves.cpu().numpy().view(np.uint32).reshape(-1, 16)[:min(cnt, leaf_cap)]
    return d_moves.cpu().numpy(), st, trees, leaves


# ---------------------------------------------------------------- PV forward
class PVWeights:
    """Packed weight blob resident on the device (+ the fp32 kernel's scratch slab).

    precision: "fp32" (exact f32 MFMA) or "f16x3" (3-term fp16 split on the
    fp16 MFMA, f32 accumulation)."""

    def __init__(self, blob, precision="f16x3"):
        lib = require_gpu()
        if precision not in ("fp32", "f16x3"):
            raise ValueError(f"unknown precision {precision!r}")
        self.precision = precision
        self.mode = _lib.GZ_PV_FP32 if precision == "fp32" else _lib.GZ_PV_F16X3
        if isinstance(blob, torch.Tensor):  # (weights.pack_pv_weights_torch: packed on the device)
            blob = blob.detach().to(device="cuda", dtype=torch.float32).contiguous().reshape(-1)
        else:
            blob = torch.from_numpy(np.ascontiguousarray(blob, np.float32).reshape(-1))
        if blob.numel() != lib.gz_pv_weight_floats():
            raise ValueError(f"weight blob has {blob.numel()} floats, kernel expects {lib.gz_pv_weight_floats()}")
        self.tensor = blob.cuda()
        self.workspace = torch.empty(0, dtype=torch.uint8, device="cuda")

    def workspace_for(self, n):
        """gz_pv_workspace_bytes(n) bytes of scratch (the fp32 kernel's slabs, or the f16x3
        tower -> FC-heads records), grown on demand and kept."""
        need = _lib.load().gz_pv_workspace_bytes(int(max(1, n)))
        if self.workspace.numel() < need:
            self.workspace = torch.empty(need, dtype=torch.uint8, device="cuda")
        return self.workspace


def pv_forward_dev(weights, d_boards, n, d_count=None, d_logits=None, d_value=None, d_probs=None, d_prior=None):
    """Device-resident forward: d_boards int32/uint32 tensor [n,16]; returns output tensors.
    d_prior (float64 [n*225], needs d_probs): MCTSNode._get_prior_probability, dense."""
    lib = require_gpu()
    if d_logits is None:
        d_logits = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    if d_value is None:
        d_value = torch.empty(n, dtype=torch.float32, device="cuda")
    _lib.check(lib.gz_pv_forward(ptr(weights.tensor), ptr(d_boards), int(n), ptr(d_count), ptr(d_logits),
                                 ptr(d_value), ptr(d_probs), ptr(d_prior), ptr(weights.workspace_for(n)),
                                 weights.mode, stream()),
               "gz_pv_forward")
    return d_logits, d_value, d_probs


def pv_forward(weights, leaf_rows, want_prior=False):
    """Host convenience: [n,16] uint32 leaf rows -> (logits [n,225], value [n], probs [n,225])
    (+ prior [n,225] float64, dense over cells, 0 at stones, if want_prior)."""
    rows = np.ascontiguousarray(leaf_rows, np.uint32).reshape(-1, 16)
    n = rows.shape[0]
    d_b = torch.from_numpy(rows.view(np.int32).copy()).cuda()
    d_probs = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    d_prior = torch.empty(n * 225, dtype=torch.float64, device="cuda") if want_prior else None
    lg, v, pr = pv_forward_dev(weights, d_b, n, d_probs=d_probs, d_prior=d_prior)
    torch.cuda.synchronize()
    out = (lg.cpu().numpy().reshape(n, 225), v.cpu().numpy(), pr.cpu().numpy().reshape(n, 225))
    if want_prior:
        out += (d_prior.cpu().numpy().reshape(n, 225),)
    return out


def pv_forward_tree(weights, leaf_rows, meta, root_cap=None):
    """Host convenience for gz_pv_forward_tree: [n,16] uint32 leaf rows and their
    int32 meta (-1 root, >= 0 the parent's index for a root child or a child of
    one, -2 other) ->
    (logits [n,225], value [n], probs [n,225], prior [n,225], list sizes)."""
    lib = require_gpu()
    rows = np.ascontiguousarray(leaf_rows, np.uint32).reshape(-1, 16)
    n = rows.shape[0]
    meta = np.ascontiguousarray(meta, np.int32)
    if root_cap is None:
        root_cap = int((meta == -1).sum())
    d_b = torch.from_numpy(rows.view(np.int32).copy()).cuda()
    d_m = torch.from_numpy(meta.copy()).cuda()
    d_lg = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    d_v = torch.empty(n, dtype=torch.float32, device="cuda")
    d_p = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    d_pr = torch.empty(n * 225, dtype=torch.float64, device="cuda")
    ws = torch.empty(lib.gz_pv_tree_workspace_bytes(n, root_cap), dtype=torch.uint8, device="cuda")
    _lib.check(lib.gz_pv_forward_tree(ptr(weights.tensor), ptr(d_b), ptr(d_m), n, None, int(root_cap),
                                      ptr(d_lg), ptr(d_v), ptr(d_p), ptr(d_pr), ptr(ws), stream()),
               "gz_pv_forward_tree")
    st = torch.zeros(6, dtype=torch.int32, device="cuda")
    _lib.check(lib.gz_pv_tree_stats(ptr(ws), n, ptr(st), stream()), "gz_pv_tree_stats")
    torch.cuda.synchronize()
    return (d_lg.cpu().numpy().reshape(n, 225), d_v.cpu().numpy(), d_p.cpu().numpy().reshape(n, 225),
            d_pr.cpu().numpy().reshape(n, 225), [int(x) for x in st.cpu()])


class GNWeights:
    """BG planner nets (GraphNet + OpponentDQN) blob resident on the device."""

    def __init__(self, blob):
        lib = require_gpu()
        blob = np.ascontiguousarray(blob, np.float32)
        if blob.size != lib.gz_gn_weight_floats():
            raise ValueError(f"planner blob has {blob.size} floats, kernel expects {lib.gz_gn_weight_floats()}")
        self.tensor = torch.from_numpy(blob).cuda()
        self._ws = None

    def workspace_for(self, n):
        """Device workspace of gz_gn_forward for n boards (grown on demand, kept)."""
        need = int(require_gpu().gz_gn_workspace_bytes(max(1, int(n))))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device="cuda")
        return self._ws


def gn_forward_dev(weights, d_boards, n, d_count=None, d_p=None, d_q=None, d_logits=None):
    lib = require_gpu()
    if d_p is None:
        d_p = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    if d_q is None:
        d_q = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    _lib.check(lib.gz_gn_forward(ptr(weights.tensor), ptr(d_boards), int(n), ptr(d_count), ptr(d_p), ptr(d_q),
                                 ptr(d_logits), ptr(weights.workspace_for(n)), stream()), "gz_gn_forward")
    return d_p, d_q, d_logits


def gn_forward(weights, leaf_rows):
    """Host convenience: [n,16] uint32 rows -> (p [n,225], q [n,225], logits [n,225])."""
    rows = np.ascontiguousarray(leaf_rows, np.uint32).reshape(-1, 16)
    n = rows.shape[0]
    d_b = torch.from_numpy(rows.view(np.int32).copy()).cuda()
    d_lg = torch.empty(n * 225, dtype=torch.float32, device="cuda")
    p, q, lg = gn_forward_dev(weights, d_b, n, d_logits=d_lg)
    torch.cuda.synchronize()
    return p.cpu().numpy().reshape(n, 225), q.cpu().numpy().reshape(n, 225), lg.cpu().numpy().reshape(n, 225)


def plan_search(states, game_ids, params, pparams, gn_weights, want_trees=False, leaf_cap=0):
    """AlphaZeroGomokuAI.get_move with BG-planner rollout plies (gz_plan_search).
    Returns (moves, stats, trees, leaves) like search()."""
    lib = require_gpu()
    states = np.ascontiguousarray(states, dtype=STATE_DTYPE)
    n = len(states)
    d_states = to_dev(states)
    d_gids = torch.as_tensor(np.asarray(game_ids, np.int64)).cuda()
    d_moves = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_stats = torch.zeros(n * ctypes.sizeof(_lib.SearchStats), dtype=torch.uint8, device="cuda")
    S = params.num_simulations
    tb = lib.gz_tree_bytes(S)
    d_trees = torch.zeros(n * tb, dtype=torch.uint8, device="cuda") if want_trees else None
    gather = (params.flags & _lib.GZ_FLAG_GATHER_LEAVES) != 0
    d_leaves = torch.zeros(max(1, leaf_cap) * 16, dtype=torch.int32, device="cuda") if gather else None
    d_lc = torch.zeros(1, dtype=torch.int32, device="cuda") if gather else None
    ws = torch.empty(lib.gz_plan_workspace_bytes(n, S), dtype=torch.uint8, device="cuda")
    _lib.check(lib.gz_plan_search(ptr(d_states), ptr(d_gids), n, ctypes.byref(params), ctypes.byref(pparams),
                                  ptr(gn_weights.tensor), ptr(ws), ptr(d_trees), ptr(d_moves), ptr(d_stats),
                                  ptr(d_leaves), int(leaf_cap), ptr(d_lc), stream()), "gz_plan_search")
    torch.cuda.synchronize()
    st = np.frombuffer(d_stats.cpu().numpy().tobytes(), dtype=np.dtype(
        [("n_nodes", "<i4"), ("predicts", "<i4"), ("main_draws", "<i4"), ("pad", "<i4"), ("sim_draws", "<i8")]))
    trees = None
    if want_trees:
        raw = d_trees.cpu().numpy().reshape(n, tb)
        trees = [parse_tree(raw[i], S, int(st["n_nodes"][i])) for i in range(n)]
    leaves = None
    if gather:
        cnt = int(d_lc.item())
        leaves = d_leaves.cpu().numpy().view(np.uint32).reshape(-1, 16)[:min(cnt, leaf_cap)]
    return d_moves.cpu().numpy(), st, trees, leaves


def planner_move(states, ais, keys, pparams, gn_weights):
    """BGPlannerAI.get_move per state (gz_planner_move): returns (moves, draws)."""
    lib = require_gpu()
    states = np.ascontiguousarray(states, dtype=STATE_DTYPE)
    n = len(states)
    d_states = to_dev(states)
    d_ai = torch.as_tensor(np.asarray(ais, np.int32)).cuda()
    d_keys = torch.as_tensor(np.asarray(keys, np.uint64).view(np.int64)).cuda()
    d_moves = torch.zeros(n, dtype=torch.int32, device="cuda")
    d_draws = torch.zeros(n, dtype=torch.int32, device="cuda")
    ws = torch.empty(lib.gz_planner_move_workspace_bytes(n), dtype=torch.uint8, device="cuda")
    _lib.check(lib.gz_planner_move(ptr(d_states), ptr(d_ai), ptr(d_keys), n, ctypes.byref(pparams),
                                   ptr(gn_weights.tensor), ptr(ws), ptr(d_moves), ptr(d_draws), stream()),
               "gz_planner_move")
    torch.cuda.synchronize()
    return d_moves.cpu().numpy(), d_draws.cpu().numpy().view(np.uint32)


def knowledge_scores(states, players):
    """KnowledgeSearch.score_move(board, (r, c), player) for every cell of every
    state (gz_knowledge_scores): float64 [n, 225], -1e9 at occupied cells."""
    lib = require_gpu()
    states = np.ascontiguousarray(states, dtype=STATE_DTYPE)
    n = len(states)
    d_states = to_dev(states)
    d_pl = torch.as_tensor(np.asarray(players, np.int32)).cuda()
    d_sc = torch.empty(max(1, n) * 225, dtype=torch.float64, device="cuda")
    _lib.check(lib.gz_knowledge_scores(ptr(d_states), ptr(d_pl), n, ptr(d_sc), stream()), "gz_knowledge_scores")
    torch.cuda.synchronize()
    return d_sc[: n * 225].cpu().numpy().reshape(n, 225)
