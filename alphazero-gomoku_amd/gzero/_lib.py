"""ctypes binding of libgzero.so (include/gzero.h).

The shared library is built in-tree by ``csrc/Makefile`` (``gzero.build()``).
There is no CPU fallback: if the library or a GPU is missing, every entry point
raises ``GzeroUnavailable``.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# GZ_LIBRARY: an alternative build of the same library (A/B kernel experiments, tools/Makefile)
LIB_PATH = os.environ.get("GZ_LIBRARY") or os.path.join(HERE, "libgzero.so")

GZ_OK = 0
GZ_FLAG_GATHER_LEAVES = 1
GZ_FLAG_GN_CHECK = 2  # planner searches: check every incremental GraphNet row against the full forward
GZ_MAX_SIMULATIONS = 4095
GZ_MAX_GAME_PLIES = 200
GZ_PV_FP32 = 0
GZ_PV_F16X3 = 1
GZ_AUG_FIX_LABELS = 1


class GzeroUnavailable(RuntimeError):
    pass


class GzeroError(RuntimeError):
    pass


class BoardState(ctypes.Structure):  # gz_board_state, 80 bytes
    _fields_ = [("black", ctypes.c_uint32 * 8), ("white", ctypes.c_uint32 * 8),
                ("n_moves", ctypes.c_int32), ("player", ctypes.c_int32),
                ("over", ctypes.c_int32), ("winner", ctypes.c_int32)]


class SearchParams(ctypes.Structure):  # gz_search_params
    _fields_ = [("num_simulations", ctypes.c_int32), ("max_depth", ctypes.c_int32),
                ("c_puct", ctypes.c_double), ("exploration", ctypes.c_double),
                ("beta", ctypes.c_double), ("seed", ctypes.c_uint64),
                ("planner_steps", ctypes.c_int32), ("flags", ctypes.c_int32)]


class PlannerParams(ctypes.Structure):  # gz_planner_params
    _fields_ = [("k", ctypes.c_int32), ("pad", ctypes.c_int32), ("alpha", ctypes.c_double),
                ("explore", ctypes.c_double)]


# BGPlannerAI.params (bg_planner.py:215-219)
PLANNER = {"easy": (8, 0.5, 0.2), "medium": (12, 0.65, 0.1), "hard": (16, 0.75, 0.05)}


def planner_params(difficulty):
    k, a, e = PLANNER.get(difficulty, PLANNER["medium"])
    return PlannerParams(k, 0, a, e)


class Record(ctypes.Structure):  # gz_record, 80 bytes
    _fields_ = [("black", ctypes.c_uint32 * 8), ("white", ctypes.c_uint32 * 8),
                ("game_id", ctypes.c_int64), ("ply", ctypes.c_int16), ("move", ctypes.c_int16),
                ("player", ctypes.c_int8), ("z", ctypes.c_int8), ("pad", ctypes.c_int8 * 2)]


class SearchStats(ctypes.Structure):
    _fields_ = [("n_nodes", ctypes.c_int32), ("predicts", ctypes.c_int32),
                ("main_draws", ctypes.c_int32), ("pad", ctypes.c_int32), ("sim_draws", ctypes.c_int64)]


class SelfplayCounters(ctypes.Structure):
    _fields_ = [("records", ctypes.c_int32), ("leaves", ctypes.c_int32),
                ("records_dropped", ctypes.c_int32), ("leaves_dropped", ctypes.c_int32),
                ("moves", ctypes.c_int64), ("games", ctypes.c_int64), ("mcts_moves", ctypes.c_int64)]


assert ctypes.sizeof(BoardState) == 80 and ctypes.sizeof(Record) == 80
assert ctypes.sizeof(SearchStats) == 24 and ctypes.sizeof(SelfplayCounters) == 40

class SgdNet(ctypes.Structure):  # gz_sgd_net
    _fields_ = [("bn_weight", ctypes.c_void_p * 5), ("bn_bias", ctypes.c_void_p * 5),
                ("bn_running_mean", ctypes.c_void_p * 5), ("bn_running_var", ctypes.c_void_p * 5),
                ("conv_weight", ctypes.c_void_p * 4), ("conv_bias", ctypes.c_void_p * 4),
                ("momentum", ctypes.c_float), ("eps", ctypes.c_float),
                ("conv0_weight", ctypes.c_void_p), ("conv0_bias", ctypes.c_void_p),
                ("policy_weight", ctypes.c_void_p), ("policy_bias", ctypes.c_void_p),
                ("value_weight", ctypes.c_void_p), ("value_bias", ctypes.c_void_p)]


class SgdGrads(ctypes.Structure):  # gz_sgd_grads
    _fields_ = [("bn_weight", ctypes.c_void_p * 5), ("bn_bias", ctypes.c_void_p * 5),
                ("conv_weight", ctypes.c_void_p * 4), ("conv_bias", ctypes.c_void_p * 4),
                ("conv0_weight", ctypes.c_void_p), ("conv0_bias", ctypes.c_void_p),
                ("policy_weight", ctypes.c_void_p), ("policy_bias", ctypes.c_void_p),
                ("value_weight", ctypes.c_void_p), ("value_bias", ctypes.c_void_p)]


class SgdFc(ctypes.Structure):  # gz_sgd_fc / gz_sgd_fc_grads
    _fields_ = [("policy_weight", ctypes.c_void_p), ("policy_bias", ctypes.c_void_p),
                ("value1_weight", ctypes.c_void_p), ("value1_bias", ctypes.c_void_p),
                ("value2_weight", ctypes.c_void_p), ("value2_bias", ctypes.c_void_p)]


GZ_SGD_MAX_BOARDS = 65535
GZ_ADAM_MAX_TENSORS = 48


class AdamTensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("numel", ctypes.c_int64)]

_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_SZ = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/gzero.h
SIGNATURES = {
    "gz_last_error": (ctypes.c_char_p, []),
    "gz_version": (ctypes.c_int, []),
    "gz_board_step": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P]),
    "gz_policy_move": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P]),
    "gz_rollout": (ctypes.c_int, [_P, _P, _P, _I32, _I32, _P, _P, _P, _P]),
    "gz_pattern_score": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P]),
    "gz_tree_bytes": (_SZ, [_I32]),
    "gz_search": (ctypes.c_int, [_P, _P, _I32, ctypes.POINTER(SearchParams), _P, _P, _P, _P, _I32, _P, _P]),
    "gz_slot_bytes": (_SZ, [_I32]),
    "gz_selfplay_init": (ctypes.c_int, [_P, _I32, _I32, _I64, _I64, _P]),
    "gz_selfplay_run": (ctypes.c_int, [_P, _I32, ctypes.POINTER(SearchParams), _I32, _P, _I32, _P, _I32, _P, _P, _P]),
    "gz_selfplay_boards": (ctypes.c_int, [_P, _I32, _I32, _P, _P, _P]),
    "gz_selfplay_draws": (ctypes.c_int, [_P, _I32, _P, _P]),
    "gz_selfplay_set_game_end": (ctypes.c_int, [_P, _I32, _I64, _P]),
    "gz_adam_workspace_bytes": (_SZ, []),
    "gz_adam_step": (ctypes.c_int, [_P, _I32, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                    ctypes.c_float, _I64, ctypes.c_float, _P, _P, _P]),
    "gz_selfplay_compact_workspace_bytes": (_SZ, [_I32]),
    "gz_selfplay_compact": (ctypes.c_int, [_P, _I32, _P, _P, _P, _P]),
    "gz_pv_weight_floats": (_SZ, []),
    "gz_pv_workspace_bytes": (_SZ, [_I32]),
    "gz_pv_forward": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P, _P, _I32, _P]),
    "gz_pv_tree_workspace_bytes": (_SZ, [_I32, _I32]),
    "gz_pv_forward_tree": (ctypes.c_int, [_P, _P, _P, _I32, _P, _I32, _P, _P, _P, _P, _P, _P]),
    "gz_pv_tree_stats": (ctypes.c_int, [_P, _I32, _P, _P]),
    "gz_pv_tree_exec_tiles": (ctypes.c_int, [_P, _I32, _P, _P]),
    "gz_gn_weight_floats": (_SZ, []),
    "gz_gn_workspace_bytes": (_SZ, [_I32]),
    "gz_gn_forward": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P, _P]),
    "gz_plan_workspace_bytes": (_SZ, [_I32, _I32]),
    "gz_plan_search": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _I32, _P, _P]),
    "gz_planner_move_workspace_bytes": (_SZ, [_I32]),
    "gz_selfplay_plan_workspace_bytes": (_SZ, [_I32, _I32]),
    "gz_selfplay_plan_run": (ctypes.c_int, [_P, _I32, _P, _P, _P, _P, _I32, _P, _I32, _P, _I32, _P, _P, _P]),
    "gz_planner_move": (ctypes.c_int, [_P, _P, _P, _I32, _P, _P, _P, _P, _P, _P]),
    "gz_plan_gn_stats": (ctypes.c_int, [_P, _I32, _I32, _P, _I32, _P]),
    "gz_gn_slot_bytes": (_SZ, []),
    "gz_gn_chain_workspace_bytes": (_SZ, [_I32]),
    "gz_gn_forward_chain": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _P, _P]),
    "gz_selfplay_plan_gn_stats": (ctypes.c_int, [_P, _I32, _I32, _P, _I32, _P]),
    "gz_knowledge_scores": (ctypes.c_int, [_P, _P, _I32, _P, _P]),
    "gz_dataset_build": (ctypes.c_int, [_P, _I32, _P, _I32, _I32, _P, _P, _P, _P]),
    "gz_dataset_gather": (ctypes.c_int, [_P, _I32, _P, _I32, _P, _I64, _I32, _P, _P, _P, _P]),
    "gz_sgd_workspace_bytes": (_SZ, [_I32]),
    "gz_sgd_forward": (ctypes.c_int, [ctypes.POINTER(SgdNet), _I32, _P, _P, _P, _P, _P]),
    "gz_sgd_backward": (ctypes.c_int, [ctypes.POINTER(SgdNet), _I32, _P, _P, _P, ctypes.POINTER(SgdGrads), _P, _P]),
    "gz_sgd_saved": (ctypes.c_int, [_P, _I32, _I32, _P, _P]),
    "gz_sgd_fc_workspace_bytes": (_SZ, [_I32]),
    "gz_sgd_fc_loss": (ctypes.c_int, [ctypes.POINTER(SgdFc), _I32, _P, _P, _P, _P, ctypes.c_float, _P, _P,
                                      ctypes.POINTER(SgdFc), _P, _P, _P]),
}

_lib = None


def load(path=LIB_PATH):
    """Load libgzero.so (no GPU needed to load it); raises GzeroUnavailable if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GzeroUnavailable(
            f"{path} is missing: build the HIP extension first (python -c 'import __graft_entry__ as g; g.build()')")
    L = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc, what):
    if rc != GZ_OK:
        msg = load().gz_last_error()
        raise GzeroError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")
