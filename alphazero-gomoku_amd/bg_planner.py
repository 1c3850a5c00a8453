"""Drop-in ``bg_planner`` module (reference: bg_planner.py:22-269) -- partial.

``KnowledgeSearch._pattern_score`` runs on the GPU pattern kernel
(``gz_pattern_score``, the same LUT the search uses for the UCB's BG term).
The planner itself (``BGPlannerAI.get_move``: knowledge-scored top-k +
GraphNet/OpponentDQN composition, bg_planner.py:232-269) is not on the device
yet; constructing ``BGPlannerAI`` raises ``GzeroError`` rather than silently
running a CPU version.
"""
import numpy as np

from gzero import _lib


class KnowledgeSearch:
    def __init__(self, board_size: int = 15):
        self.n = board_size

    def _pattern_score(self, board, player: int) -> float:
        from gzero import device
        st = board.to_state()
        s, _ = device.pattern_score(st, [player])
        return float(s[0])

    def _center_bias(self, move) -> float:
        c = self.n // 2
        return max(0.0, (6 - (abs(move[0] - c) + abs(move[1] - c))) * 0.5)


class BGPlannerAI:
    def __init__(self, player: int, difficulty: str = "medium", device: str = "cpu"):
        raise _lib.GzeroError("BGPlannerAI (GraphNet + OpponentDQN + knowledge search) is not implemented on the "
                              "device yet")
