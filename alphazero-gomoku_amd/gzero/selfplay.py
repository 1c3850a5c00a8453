"""Device-resident self-play collector: the batched form of
``training.play_one_game`` (training.py:141-218) over thousands of concurrent games.

One call of :meth:`SelfPlayEngine.step` advances every game slot by ``n_plies``
plies inside one kernel launch (one wavefront per game), then -- in
reference-work mode -- evaluates the policy-value network on every node the
searches created, exactly the ``GomokuModel.predict`` calls the reference makes
(``ai_agent.py:522-523``).  The forward's outputs are produced but, as in the
reference, never read by the search.  Finished games are appended as
(planes, move, player, z) records; slots restart with the next game id.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .boards import RECORD_DTYPE, STATE_DTYPE, words_to_cells
from .device import GNWeights, PVWeights, ptr, require_gpu, search_params, stream

COUNTER_DTYPE = np.dtype([("records", "<i4"), ("leaves", "<i4"), ("records_dropped", "<i4"),
                          ("leaves_dropped", "<i4"), ("moves", "<i8"), ("games", "<i8"),
                          ("mcts_moves", "<i8")])


class SelfPlayEngine:
    def __init__(self, n_slots=4096, num_simulations=200, c_puct=1.6, exploration=0.05, beta=0.2,
                 seed=0, max_depth=100, pv_weights=None, plies_per_step=1, game_id_base=0,
                 game_id_stride=None, planner_steps=0, planner_difficulty="medium", gn_weights=None,
                 pv_mode="full", game_id_end=None):
        """game_id_end: a slot whose next game id would be >= game_id_end goes idle
        instead of restarting (gz_selfplay_set_game_end; default: continuous refill);
        :meth:`compact` then moves the active slots to the front so that only those run.
        planner_steps > 0: BG-planner rollout plies (config 4); gn_weights = the
        planner's GraphNet/DQN blob (gzero.planner_nets) or a GNWeights.
        pv_mode: "full" = one full forward per node (gz_pv_forward); "tree" = the
        incremental forward (gz_pv_forward_tree, f16x3 only): a root's children as the
        root's pre-BN accumulators plus the convolution of their input differences
        (within 2e-5 of the full forward), its grandchildren recomputing the windows
        around their new stone; roots and other nodes bit-identical to "full"."""
        self.lib = require_gpu()
        self.n_slots = int(n_slots)
        self.n_active = self.n_slots  # the slots the launches run (the first n_active)
        self.plies_per_step = int(plies_per_step)
        self.gather = pv_weights is not None
        self.planner_steps = int(planner_steps)
        self.params = search_params(num_simulations, c_puct, exploration, beta, seed, max_depth,
                                    self.planner_steps, self.gather)
        if self.planner_steps:
            if gn_weights is None:
                raise ValueError("planner_steps > 0 needs gn_weights (the planner's GraphNet/DQN)")
            self.gn_weights = gn_weights if isinstance(gn_weights, GNWeights) else GNWeights(gn_weights)
            self.pparams = _lib.planner_params(planner_difficulty)
            self.d_plan_ws = torch.empty(self.lib.gz_selfplay_plan_workspace_bytes(self.n_slots, num_simulations),
                                         dtype=torch.uint8, device="cuda")
            self.gn_stats(reset=True)
        self.pv_weights = pv_weights if (pv_weights is None or isinstance(pv_weights, PVWeights)) \
            else PVWeights(pv_weights)
        if pv_mode not in ("full", "tree"):
            raise ValueError(f"pv_mode must be 'full' or 'tree', not {pv_mode!r}")
        self.tree = pv_mode == "tree" and self.gather
        self.pv_mode = pv_mode if self.gather else "full"
        if self.tree and self.pv_weights.mode != _lib.GZ_PV_F16X3:
            raise ValueError(f"pv_mode={pv_mode!r} needs f16x3 weights")
        S = self.params.num_simulations
        slot_bytes = self.lib.gz_slot_bytes(S)
        self.d_slots = torch.zeros(self.n_slots * slot_bytes, dtype=torch.uint8, device="cuda")
        # a slot can finish one 200-ply game plus any games played inside a step
        self.record_cap = self.n_slots * (_lib.GZ_MAX_GAME_PLIES + self.plies_per_step)
        self.d_records = torch.zeros(self.record_cap * RECORD_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        self.d_counters = torch.zeros(COUNTER_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        self.leaf_cap = self.n_slots * self.plies_per_step * (S + 1) if self.gather else 0
        if self.gather:
            self.d_leaves = torch.zeros(self.leaf_cap * 16, dtype=torch.int32, device="cuda")
            self.d_logits = torch.empty(self.leaf_cap * 225, dtype=torch.float32, device="cuda")
            self.d_value = torch.empty(self.leaf_cap, dtype=torch.float32, device="cuda")
            self.d_probs = torch.empty(self.leaf_cap * 225, dtype=torch.float32, device="cuda")
            # MCTSNode.prior_prob of every node (ai_agent.py:522-523,564-582), dense float64
            self.d_prior = torch.empty(self.leaf_cap * 225, dtype=torch.float64, device="cuda")
        else:
            self.d_leaves = self.d_logits = self.d_value = self.d_probs = self.d_prior = None
        self.d_meta = self.d_tree_ws = None
        if self.tree:
            self.d_meta = torch.empty(self.leaf_cap, dtype=torch.int32, device="cuda")
            self.root_cap = self.n_slots * self.plies_per_step  # one root per slot per ply
            self.d_tree_ws = torch.empty(self.lib.gz_pv_tree_workspace_bytes(self.leaf_cap, self.root_cap),
                                         dtype=torch.uint8, device="cuda")
        base = int(game_id_base)
        stride = self.n_slots if game_id_stride is None else int(game_id_stride)
        _lib.check(self.lib.gz_selfplay_init(ptr(self.d_slots), self.n_slots, S, base, stride, stream()),
                   "gz_selfplay_init")
        self.d_slots_alt = self.d_compact_ws = self.d_n_active = None
        if game_id_end is not None:
            _lib.check(self.lib.gz_selfplay_set_game_end(ptr(self.d_slots), self.n_slots, int(game_id_end), stream()),
                       "gz_selfplay_set_game_end")
            self.d_slots_alt = torch.empty_like(self.d_slots)
            self.d_compact_ws = torch.empty(self.lib.gz_selfplay_compact_workspace_bytes(self.n_slots),
                                            dtype=torch.uint8, device="cuda")
            self.d_n_active = torch.zeros(1, dtype=torch.int32, device="cuda")

    def compact(self):
        """Launch gz_selfplay_compact: the active slots to the front of the slot buffer
        (the two buffers swap).  Returns the device int32 [1] active count; the caller
        sets :attr:`n_active` from it once read (the next launches run that many)."""
        if self.d_slots_alt is None:
            raise ValueError("compact() needs an engine built with game_id_end")
        _lib.check(self.lib.gz_selfplay_compact(ptr(self.d_slots), self.n_slots, ptr(self.d_slots_alt),
                                                ptr(self.d_n_active), ptr(self.d_compact_ws), stream()),
                   "gz_selfplay_compact")
        self.d_slots, self.d_slots_alt = self.d_slots_alt, self.d_slots
        return self.d_n_active

    # ---- launches (asynchronous, current torch stream)
    def launch_search(self, n_plies=None):
        n = self.plies_per_step if n_plies is None else int(n_plies)
        if n > self.plies_per_step and self.gather:
            raise ValueError("n_plies exceeds the leaf buffer sized for plies_per_step")
        self.d_counters.zero_()
        if self.n_active == 0:  # every game is done
            return
        if self.planner_steps:
            _lib.check(self.lib.gz_selfplay_plan_run(ptr(self.d_slots), self.n_active, ctypes.byref(self.params),
                                                     ctypes.byref(self.pparams), ptr(self.gn_weights.tensor),
                                                     ptr(self.d_plan_ws), n, ptr(self.d_records), self.record_cap,
                                                     ptr(self.d_leaves), self.leaf_cap, ptr(self.d_meta),
                                                     ptr(self.d_counters), stream()), "gz_selfplay_plan_run")
            return
        _lib.check(self.lib.gz_selfplay_run(ptr(self.d_slots), self.n_active, ctypes.byref(self.params), n,
                                            ptr(self.d_records), self.record_cap, ptr(self.d_leaves),
                                            self.leaf_cap, ptr(self.d_meta), ptr(self.d_counters), stream()),
                   "gz_selfplay_run")

    def gn_stats(self, reset=False, check=None):
        """Planner-net rows since the last reset: {"full", "incremental", "checked",
        "mismatched"} (gz_selfplay_plan_gn_stats; synchronises).  check=True/False
        turns GZ_FLAG_GN_CHECK (every incremental row re-run by the full forward and
        compared bitwise) on/off for the following searches."""
        if getattr(self, "d_slots_alt", None) is not None:
            # a compacting engine carves the planner workspace for n_active slots, so the
            # counters' place moves with it: they cannot be read at n_slots
            raise ValueError("gn_stats() is not available on an engine built with game_id_end (compaction)")
        if check is not None:
            f = self.params.flags & ~_lib.GZ_FLAG_GN_CHECK
            self.params.flags = f | (_lib.GZ_FLAG_GN_CHECK if check else 0)
        out = (ctypes.c_int64 * 4)()
        _lib.check(self.lib.gz_selfplay_plan_gn_stats(ptr(self.d_plan_ws), self.n_slots, self.params.num_simulations,
                                                      out, 1 if reset else 0, stream()), "gz_selfplay_plan_gn_stats")
        return {"full": out[0], "incremental": out[1], "checked": out[2], "mismatched": out[3]}

    def advance(self, n_plies):
        """Play n_plies plies on every slot without gathering leaves for the PV forward
        (the moves are the same either way: the search never reads the priors,
        ai_agent.py:523).  Used to bring the slots to a steady-state mix of game plies
        (continuous refill) before a measurement; records of games finished here are
        not kept.  On a planner engine (config 4) the burn-in plies are searched without
        planner plies (the planner pipeline needs the GN forward per ply): the slots
        reach a steady-state mix of positions, and the measured plies are planner plies."""
        p = _lib.SearchParams.from_buffer_copy(self.params)
        p.flags = 0
        p.planner_steps = 0
        for _ in range(int(n_plies)):
            self.d_counters.zero_()
            _lib.check(self.lib.gz_selfplay_run(ptr(self.d_slots), self.n_slots, ctypes.byref(p), 1,
                                                ptr(self.d_records), self.record_cap, None, 0, None,
                                                ptr(self.d_counters), stream()), "gz_selfplay_run")

    def launch_pv(self):
        if not self.gather or self.n_active == 0:
            return
        d_count = self.d_counters[4:8]  # counters.leaves
        if self.tree:
            _lib.check(self.lib.gz_pv_forward_tree(ptr(self.pv_weights.tensor), ptr(self.d_leaves),
                                                   ptr(self.d_meta), self.leaf_cap, ptr(d_count), self.root_cap,
                                                   ptr(self.d_logits), ptr(self.d_value), ptr(self.d_probs),
                                                   ptr(self.d_prior), ptr(self.d_tree_ws), stream()),
                       "gz_pv_forward_tree")
            return
        _lib.check(self.lib.gz_pv_forward(ptr(self.pv_weights.tensor), ptr(self.d_leaves), self.leaf_cap,
                                          ptr(d_count), ptr(self.d_logits), ptr(self.d_value),
                                          ptr(self.d_probs), ptr(self.d_prior),
                                          ptr(self.pv_weights.workspace_for(self.leaf_cap)),
                                          self.pv_weights.mode, stream()), "gz_pv_forward")

    def step(self, n_plies=None):
        self.launch_search(n_plies)
        self.launch_pv()

    def tree_stats(self):
        """List sizes of the last tree forward: roots seen, roots with maps,
        incremental root children, full-forward boards, incremental grandchildren,
        patch slots claimed (synchronising)."""
        out = torch.zeros(6, dtype=torch.int32, device="cuda")
        _lib.check(self.lib.gz_pv_tree_stats(ptr(self.d_tree_ws), self.leaf_cap, ptr(out), stream()),
                   "gz_pv_tree_stats")
        return [int(x) for x in out.cpu()]

    def tree_exec_flops(self):
        """(executed MFMA FLOP of the last tree forward, its node count): roots and
        deeper nodes run the full forward, a root child or grandchild the row tiles
        of its windows (csrc/gz_pvinc.hip).  Reads the leaves and tags (synchronising)."""
        n = min(int(self.counters()["leaves"]), self.leaf_cap)
        rows = self.d_leaves[: n * 16].cpu().numpy().view(np.uint32).reshape(n, 16)
        meta = self.d_meta[:n].cpu().numpy()
        return tree_exec_flops(rows, meta), n

    # ---- host views (synchronising)
    def counters(self):
        return np.frombuffer(self.d_counters.cpu().numpy().tobytes(), COUNTER_DTYPE)[0]

    def records(self):
        """Records of the games that finished during the last step."""
        c = self.counters()
        n = min(int(c["records"]), self.record_cap)
        raw = self.d_records[: n * RECORD_DTYPE.itemsize].cpu().numpy()
        return np.frombuffer(raw.tobytes(), RECORD_DTYPE)

    def records_device(self):
        """(device uint8 tensor of records, count) without copying to the host."""
        n = min(int(self.counters()["records"]), self.record_cap)
        return self.d_records[: n * RECORD_DTYPE.itemsize], n

    def boards(self):
        out = torch.zeros(self.n_slots * STATE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        gids = torch.zeros(self.n_slots, dtype=torch.int64, device="cuda")
        _lib.check(self.lib.gz_selfplay_boards(ptr(self.d_slots), self.n_slots, self.params.num_simulations,
                                               ptr(out), ptr(gids), stream()), "gz_selfplay_boards")
        return np.frombuffer(out.cpu().numpy().tobytes(), STATE_DTYPE), gids.cpu().numpy()


    def draws(self):
        """int64 [n_slots, 3]: (predict calls, main-stream RNG draws, simulation-stream
        RNG draws) summed over every search each slot ran since the engine was created
        (gz_selfplay_draws)."""
        out = torch.zeros(self.n_slots * 3, dtype=torch.int64, device="cuda")
        _lib.check(self.lib.gz_selfplay_draws(ptr(self.d_slots), self.n_slots, ptr(out), stream()),
                   "gz_selfplay_draws")
        return out.cpu().numpy().reshape(self.n_slots, 3)


def records_to_games(recs):
    """Group records by game id -> {game_id: dict(moves, players, z, cells)} (ply order)."""
    out = {}
    for gid in np.unique(recs["game_id"]):
        r = recs[recs["game_id"] == gid]
        r = r[np.argsort(r["ply"])]
        out[int(gid)] = {"moves": [int(x) for x in r["move"]], "players": [int(x) for x in r["player"]],
                         "z": [int(x) for x in r["z"]], "cells": words_to_cells(r["black"], r["white"])}
    return out


def records_to_replay(recs):
    """SimpleReplay fields (training.py:77-97): states float32 [n,3,15,15], move
    indices, players, outcomes."""
    cells = words_to_cells(recs["black"], recs["white"]).reshape(-1, 15, 15)
    planes = np.stack([(cells == 1), (cells == 2), (cells == 0)], axis=1).astype(np.float32)
    return planes, recs["move"].astype(np.int64), recs["player"].astype(np.int64), recs["z"].astype(np.int64)


PV_FLOP_FULL = 2 * 133690114  # one full forward (gzero.weights.PV_MACS)


def _window_rows(rc, r):
    lo = np.maximum(rc - r, 0)
    hi = np.minimum(rc + r, 14)
    return hi - lo + 1


def tree_exec_flops(rows, meta):
    """MFMA FLOP the tree forward executes for leaves `rows` ([n,16] uint32) tagged
    `meta`: 2 x (MACs of every 16-row tile it runs), fp32-equivalent like the full
    forward's 267.38 MFLOP.  A tagged node (meta >= 0: a root child or a child of
    one; assumes no map / patch slot ran out) whose stone is at (r, c) runs, per residual conv L = 1..4
    (window radius L + 1), ceil(rows_L / 16) tiles of 16 positions x 128 channels x
    1152, one conv0 tile, the 1x1 heads at radius 5 and the FC heads."""
    meta = np.asarray(meta)
    kids = np.flatnonzero(meta >= 0)
    full = len(meta) - len(kids)
    if len(kids) == 0:
        return float(full * PV_FLOP_FULL)
    diff = rows[kids] ^ rows[meta[kids]]
    both = diff[:, :8] | diff[:, 8:]
    word = np.argmax(both != 0, axis=1)
    bitv = both[np.arange(len(kids)), word]
    bit = word * 32 + np.log2(bitv.astype(np.float64)).astype(np.int64)
    r, c = bit // 16, bit % 16
    macs = np.zeros(len(kids), np.float64)
    for L in range(1, 5):
        n_rows = _window_rows(r, L + 1) * _window_rows(c, L + 1)
        macs += np.ceil(n_rows / 16.0) * 16 * 128 * 1152
    n4 = _window_rows(r, 5) * _window_rows(c, 5)
    macs += 16 * 128 * 27 + n4 * 128 * 3 + 450 * 225 + 225 * 64 + 64
    return float(full * PV_FLOP_FULL + 2.0 * macs.sum())
