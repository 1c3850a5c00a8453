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


def test_device_failure_matches_whole_words_only():
    """play_one_game re-raises device errors but, like the reference
    (training.py:191-198), plays a random move after any other AI error."""
    from training import _is_device_failure
    from gzero._lib import GzeroError
    assert _is_device_failure(RuntimeError("HIP error: an illegal memory access was encountered"))
    assert _is_device_failure(RuntimeError("hipErrorOutOfMemory in hipMalloc"))
    assert _is_device_failure(RuntimeError("CUDA error: device-side assert triggered"))
    assert _is_device_failure(GzeroError("gz_selfplay_step failed"))
    assert not _is_device_failure(RuntimeError("bad relationship between ownership and chips"))
    assert not _is_device_failure(ValueError("HIP error"))


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


def test_tree_exec_flops_counts_window_tiles():
    """bench.py's executed-FLOP count of the tree forward (gzero.selfplay.tree_exec_flops):
    a root costs a full forward; a tagged node whose stone is at (r, c) runs, per
    residual conv L = 1..4, ceil(rows / 16) tiles over the radius-(L+1) square clipped
    to the board, plus conv0, the 1x1 heads at radius 5 and the FC heads -- counted
    here by brute force over the squares."""
    from gzero import boards
    from gzero.selfplay import PV_FLOP_FULL, tree_exec_flops

    def macs(r, c):
        m = 0
        for L in range(1, 5):
            rows = sum(1 for pr in range(15) for pc in range(15) if abs(pr - r) <= L + 1 and abs(pc - c) <= L + 1)
            m += -(-rows // 16) * 16 * 128 * 1152
        n5 = sum(1 for pr in range(15) for pc in range(15) if abs(pr - r) <= 5 and abs(pc - c) <= 5)
        return m + 16 * 128 * 27 + n5 * 128 * 3 + 450 * 225 + 225 * 64 + 64

    root = np.zeros(225, np.int8)
    root[[112, 113]] = [1, 2]
    cells, meta, want = [root], [-1], float(PV_FLOP_FULL)
    for cell in (0, 7, 14, 100, 112 - 15, 224):
        if root[cell]:
            continue
        k = root.copy()
        k[cell] = 1
        cells.append(k)
        meta.append(0)
        want += 2.0 * macs(cell // 15, cell % 15)
    cells.append(root.copy())
    meta.append(-2)  # an untagged node: a full forward
    want += PV_FLOP_FULL
    bl, wh = boards.cells_to_words(np.asarray(cells, np.int8))
    rows = boards.leaf_words(bl, wh)
    assert tree_exec_flops(rows, np.asarray(meta)) == pytest.approx(want, rel=1e-12)
