"""Drop-in ``gomoku_board`` module (reference: gomoku_board.py:17-327).

``GomokuBoard`` is the host-side game object the reference's callers hold and
mutate (UI, ``play_one_game``, ``AlphaZeroGomokuAI.get_move``): same public
attributes (``board`` int array, ``move_history``, ``current_player``,
``game_over``, ``winner``) and methods.  Single-board bookkeeping stays on the
host as in the reference; every batched board step, legal-mask and
five-in-a-row evaluation of the engine runs on the GPU (``gz_board_step`` and
the search kernels), and ``to_state()`` hands a board to them.
"""
from typing import List, Optional, Tuple

import numpy as np


class GomokuBoard:
    BOARD_SIZE = 15
    EMPTY = 0
    BLACK = 1
    WHITE = 2
    DIRECTIONS = [(0, 1), (1, 0), (1, 1), (1, -1)]  # gomoku_board.py:33-38

    def __init__(self):
        self.board = np.zeros((self.BOARD_SIZE, self.BOARD_SIZE), dtype=int)
        self.move_history: List[Tuple[int, int, int]] = []
        self.current_player = self.BLACK
        self.game_over = False
        self.winner: Optional[int] = None

    def reset(self):
        self.board.fill(self.EMPTY)
        self.move_history.clear()
        self.current_player = self.BLACK
        self.game_over = False
        self.winner = None

    def _on_board(self, row, col):
        return 0 <= row < self.BOARD_SIZE and 0 <= col < self.BOARD_SIZE

    def is_valid_move(self, row: int, col: int) -> bool:
        return self._on_board(row, col) and self.board[row, col] == self.EMPTY

    def make_move(self, row: int, col: int) -> bool:
        """gomoku_board.py:84-113: place, win check (>=5, overlines win), draw on a
        full board or at 200 moves, then hand the turn over (also after the end)."""
        if self.game_over or not self.is_valid_move(row, col):
            return False
        mover = self.current_player
        self.board[row, col] = mover
        self.move_history.append((row, col, mover))
        if self.check_win(row, col):
            self.game_over, self.winner = True, mover
        elif self.is_board_full() or self.get_move_count() >= 200:
            self.game_over, self.winner = True, None
        self.current_player = self.WHITE if mover == self.BLACK else self.BLACK
        return True

    def undo_move(self) -> bool:
        if not self.move_history:
            return False
        row, col, player = self.move_history.pop()
        self.board[row, col] = self.EMPTY
        self.game_over = False
        self.winner = None
        self.current_player = player
        return True

    def _count_consecutive(self, row: int, col: int, direction: Tuple[int, int], player: int) -> int:
        dr, dc = direction
        n = 0
        r, c = row + dr, col + dc
        while self._on_board(r, c) and self.board[r, c] == player:
            n += 1
            r, c = r + dr, c + dc
        return n

    def check_win(self, row: int, col: int) -> bool:
        p = self.board[row, col]
        return any(1 + self._count_consecutive(row, col, d, p) + self._count_consecutive(row, col, (-d[0], -d[1]), p) >= 5
                   for d in self.DIRECTIONS)

    def is_board_full(self) -> bool:
        return bool(np.all(self.board != self.EMPTY))

    def get_valid_moves(self) -> List[Tuple[int, int]]:
        rows, cols = np.nonzero(self.board == self.EMPTY)  # row-major, ignores game_over
        return [(int(r), int(c)) for r, c in zip(rows, cols)]

    def get_board_state(self) -> np.ndarray:
        return self.board.copy()

    def copy_board(self) -> "GomokuBoard":
        b = GomokuBoard()
        b.board = self.board.copy()
        b.move_history = list(self.move_history)
        b.current_player = self.current_player
        b.game_over = self.game_over
        b.winner = self.winner
        return b

    def get_board_tensor(self) -> np.ndarray:
        """[black, white, empty] float32 planes (gomoku_board.py:239-260)."""
        return np.stack([self.board == self.BLACK, self.board == self.WHITE, self.board == self.EMPTY]).astype(np.float32)

    def get_last_move(self) -> Optional[Tuple[int, int]]:
        return self.move_history[-1][:2] if self.move_history else None

    def get_move_count(self) -> int:
        return len(self.move_history)

    def get_game_status(self) -> dict:
        return {"current_player": self.current_player, "game_over": self.game_over, "winner": self.winner,
                "move_count": self.get_move_count(), "board_full": self.is_board_full()}

    def __str__(self) -> str:
        sym = {self.EMPTY: ".", self.BLACK: "●", self.WHITE: "○"}
        head = "   " + " ".join(f"{i:2d}" for i in range(self.BOARD_SIZE))
        rows = [f"{i:2d} " + " ".join(sym[int(v)] for v in row) for i, row in enumerate(self.board)]
        return "\n".join([head] + rows)

    def __eq__(self, other) -> bool:
        return (isinstance(other, GomokuBoard) and np.array_equal(self.board, other.board)
                and self.current_player == other.current_player)

    # ---- device hand-off -------------------------------------------------
    def to_state(self):
        """gz_board_state record (gzero.boards.STATE_DTYPE) of this board."""
        from gzero.boards import make_states
        return make_states(self.board.reshape(1, -1), n_moves=self.get_move_count(),
                           player=self.current_player, over=int(self.game_over), winner=self.winner or 0)


def test_gomoku_board():
    """Module smoke check, as the reference's (gomoku_board.py:330-373): prints a
    board, plays the centre, five alternating stones along a row, and an undo."""
    b = GomokuBoard()
    print(b)
    print("current player", b.current_player, "| valid moves", len(b.get_valid_moves()))
    print("make_move(7, 7):", b.make_move(7, 7))
    five = GomokuBoard()
    for c in range(5):
        five.make_move(7, 7 + c)  # the colours alternate along row 7, so no five forms (as in the reference)
    print(five)
    print("game over", five.game_over, "| winner", five.winner)
    b.make_move(6, 6)
    b.undo_move()
    print(b)
    print("GomokuBoard smoke check done")


if __name__ == "__main__":
    test_gomoku_board()
