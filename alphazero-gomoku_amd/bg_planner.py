"""Drop-in ``bg_planner`` module (reference: bg_planner.py:22-269).

* ``GraphNet`` / ``OpponentDQN`` -- the reference's torch modules (same parameter
  names, gzero/planner_nets.py); they are the weights' home and training side.
* ``KnowledgeSearch._pattern_score`` runs on the GPU pattern kernel.
* ``BGPlannerAI.get_move`` runs on the GPU (``gz_planner_move``): both nets in one
  batched MFMA kernel (gz_gnet.hip), then the knowledge-search top-k, the
  alpha-mix with the opponent DQN and the exploration draw in one wavefront.

Randomness: the reference draws from the global ``random`` module.  Here each
call draws from the counter-based stream (``seed``, ``game_id``, ply, call index).
"""
import random
from typing import List, Optional, Tuple

import numpy as np
import torch

from gzero import _lib
from gzero.planner_nets import GraphNet, OpponentDQN, pack_planner_weights  # noqa: F401  (re-exported)


class KnowledgeSearch:
    """bg_planner.py:81-196.  ``score_move`` / ``top_k_moves`` score every cell of
    the board in one wavefront on the GPU (``gz_knowledge_scores``); the stable
    descending sort of ``top_k_moves`` is the reference's own (Python's sort)."""

    def __init__(self, board_size: int = 15):
        self.n = board_size

    def scores(self, board, player: int) -> np.ndarray:
        """score_move(board, (r, c), player) of all 225 cells, float64 (-1e9 at stones)."""
        from gzero import device
        if not board.game_over:
            return device.knowledge_scores(board.to_state(), [player])[0]
        # finished board: make_move fails on the copy, which keeps its winner
        # (bg_planner.py:94-106) -- the same score for every empty cell but the bias
        empty = board.board.reshape(-1) == 0
        opp = 2 if player == 1 else 1
        out = np.full(225, -1e9)
        if board.winner == player:
            out[empty] = 1e6
        elif board.winner == opp and empty.any():
            out[empty] = -1e5
        else:
            base = self._pattern_score(board, player)
            for cell in np.flatnonzero(empty):
                out[cell] = base + self._center_bias(divmod(int(cell), self.n))
        return out

    def score_move(self, board, move: Tuple[int, int], player: int) -> float:
        r, c = int(move[0]), int(move[1])
        if not board.is_valid_move(r, c):  # off-board or occupied (bg_planner.py:92-93)
            return -1e9
        return float(self.scores(board, player)[r * self.n + c])

    def top_k_moves(self, board, player: int, k: int = 10) -> List[Tuple[int, int]]:
        moves = board.get_valid_moves()
        if not moves:
            return []
        sc = self.scores(board, player)
        scored = [(float(sc[r * self.n + c]), (r, c)) for r, c in moves]
        scored.sort(reverse=True, key=lambda x: x[0])
        return [m for _, m in scored[:k]]

    def _opponent_can_win_next(self, board, opponent: int) -> bool:
        """bg_planner.py:116-125: some valid cell where ``opponent``, moving next,
        ends the game as the winner (make_move fails on a finished board, whose
        winner then stands)."""
        if not board.get_valid_moves():
            return False
        if board.game_over:
            return board.winner == opponent
        from gzero import device
        st = board.to_state()
        st["player"] = opponent
        new, ok, _ = device.board_step(np.repeat(st, 225), np.arange(225))
        return bool(((new["over"] == 1) & (new["winner"] == opponent) & (ok == 1)).any())

    def _pattern_score(self, board, player: int) -> float:
        from gzero import device
        st = board.to_state()
        s, _ = device.pattern_score(st, [player])
        return float(s[0])

    def _center_bias(self, move) -> float:
        c = self.n // 2
        return max(0.0, (6 - (abs(move[0] - c) + abs(move[1] - c))) * 0.5)


class BGPlannerAI:
    """BG-Planner AI (bg_planner.py:199-269) on the GPU."""

    def __init__(self, player: int, difficulty: str = "medium", device: str = "cpu", seed: Optional[int] = None,
                 game_id: int = 0):
        self.player = player
        self.difficulty = difficulty
        self.device = torch.device(device)
        self.board_size = 15
        self.graph_net = GraphNet(self.board_size).to(self.device)
        self.opp_dqn = OpponentDQN(self.board_size).to(self.device)
        self.k_search = KnowledgeSearch(self.board_size)
        self.params = {
            'easy': {'k': 8, 'mix_alpha': 0.5, 'explore': 0.2},
            'medium': {'k': 12, 'mix_alpha': 0.65, 'explore': 0.1},
            'hard': {'k': 16, 'mix_alpha': 0.75, 'explore': 0.05},
        }[difficulty if difficulty in ['easy', 'medium', 'hard'] else 'medium']
        self.graph_net.eval()
        self.opp_dqn.eval()
        self.seed = random.getrandbits(64) if seed is None else int(seed)
        self.game_id = int(game_id)
        self._calls = 0
        self._packed = None
        self._packed_key = None

    def _param_key(self):
        return tuple((p.data_ptr(), p._version) for m in (self.graph_net, self.opp_dqn)
                     for p in m.state_dict().values())

    def device_weights(self):
        """Both nets packed on the GPU, repacked after any parameter change."""
        from gzero.device import GNWeights
        key = self._param_key()
        if self._packed is None or key != self._packed_key:
            self._packed = GNWeights(pack_planner_weights(self.graph_net.state_dict(), self.opp_dqn.state_dict()))
            self._packed_key = key
        return self._packed

    def planner_params(self):
        return _lib.PlannerParams(int(self.params['k']), 0, float(self.params['mix_alpha']),
                                  float(self.params['explore']))

    def _board_to_planes(self, board_state: np.ndarray) -> np.ndarray:
        planes = np.zeros((3, self.board_size, self.board_size), dtype=np.float32)
        planes[0] = (board_state == 1).astype(np.float32)
        planes[1] = (board_state == 2).astype(np.float32)
        planes[2] = (board_state == 0).astype(np.float32)
        return planes

    def get_move(self, board) -> Optional[Tuple[int, int]]:
        from gzero import device, rng
        if not board.get_valid_moves():
            return None
        self._calls += 1
        key = rng.stream_key(self.seed, self.game_id, board.get_move_count(), self._calls)
        mv, _ = device.planner_move(board.to_state(), [self.player], [key], self.planner_params(),
                                    self.device_weights())
        m = int(mv[0])
        return None if m < 0 else (m // 15, m % 15)
