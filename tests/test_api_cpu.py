"""Drop-in API pieces that need no GPU: the host GomokuBoard against the
reference's board fixture, the augmentation map, SimpleReplay, and the
"fail loudly" contract of the device entry points."""
import zlib

import numpy as np
import pytest

from conftest import golden


def test_gomoku_board_matches_reference():
    from gomoku_board import GomokuBoard
    g = golden("board")
    for game in g["games"]:
        b = GomokuBoard()
        masks = []
        for i, mv in enumerate(game["moves"]):
            ok = b.make_move(mv // 15, mv % 15)
            assert ok == game["ok"][i]
            assert b.game_over == game["over"][i]
            assert (b.winner or 0) == game["winner"][i]
            assert b.current_player == game["player"][i]
            x = 0
            for r, c in b.get_valid_moves():
                x |= 1 << (r * 15 + c)
            masks.append(format(x, "057x"))
        assert zlib.crc32("".join(masks).encode()) == game["mask_crc32"]
        assert b.get_move_count() == game["n_history"]
    for r, c, ok in g["offboard"]:
        assert GomokuBoard().make_move(r, c) == ok
    for case in g["crafted"]:
        b = GomokuBoard()
        for mv in case["moves"]:
            b.make_move(mv // 15, mv % 15)
        assert b.game_over == case["over"] and (b.winner or 0) == case["winner"], case["name"]


def test_board_copy_undo_tensor():
    from gomoku_board import GomokuBoard
    b = GomokuBoard()
    b.make_move(7, 7)
    b.make_move(7, 8)
    c = b.copy_board()
    assert c == b and c.move_history == b.move_history
    assert b.undo_move() and b.current_player == 2 and b.board[7, 8] == 0
    t = c.get_board_tensor()
    assert t.shape == (3, 15, 15) and t[0, 7, 7] == 1 and t[1, 7, 8] == 1 and t[2].sum() == 223
    st = c.to_state()
    from gzero.boards import words_to_cells
    assert (words_to_cells(st["black"], st["white"])[0] == c.board.reshape(-1)).all()
    assert st["n_moves"][0] == 2 and st["player"][0] == 1


def test_augment_sample_matches_reference():
    from training import augment_sample
    cases = golden("augment")["cases"]
    for idx in range(225):
        planes = np.zeros((3, 15, 15), np.float32)
        planes[0].flat[idx] = 1.0
        planes[2] = 1.0 - planes[0]
        got = [[int(y), int(np.argmax(x[0]))] for x, y in augment_sample(planes, idx)]
        assert got == cases[idx]
        # fixed mode: label follows the stone
        fixed = augment_sample(planes, idx, fix_labels=True)
        assert all(int(y) == int(np.argmax(x[0])) for x, y in fixed)


def test_simple_replay_finalize():
    from training import SimpleReplay
    r = SimpleReplay()
    for i in range(5):
        r.add(np.zeros((3, 15, 15)), i, 1 + i % 2)
    r.finalize_with_winner(2)
    assert r.outcomes == [-1, 1, -1, 1, -1]
    r2 = SimpleReplay()
    r2.add(np.zeros((3, 15, 15)), 0, 1)
    r2.finalize_with_winner(None)
    assert r2.outcomes == [0]


def test_device_paths_fail_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from gzero import _lib, device
    with pytest.raises(_lib.GzeroUnavailable):
        device.require_gpu()
    from ai_agent import AlphaZeroGomokuAI
    from gomoku_board import GomokuBoard
    ai = AlphaZeroGomokuAI(1, planner_steps=0, seed=1)
    with pytest.raises(_lib.GzeroUnavailable):
        ai.get_move(GomokuBoard())
