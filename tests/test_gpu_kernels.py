"""HIP kernels (through the C-ABI) against the oracle and the reference's golden vectors."""
import numpy as np
import pytest

from conftest import SEED, golden
from gzero import boards, device, rng

pytestmark = pytest.mark.gpu


def _states_from_moves(oracle, move_lists):
    st = np.zeros(len(move_lists), boards.STATE_DTYPE)
    for i, mv in enumerate(move_lists):
        b = oracle.new_board(mv)
        s = boards.make_states(b.cells()[None], n_moves=b.n_moves, player=b.player, over=b.over, winner=b.winner)
        st[i] = s[0]
    return st


def test_board_step_golden_games(oracle):
    """K1: make_move / legal mask / five-in-a-row, bit-exact on every ply of 240 games."""
    games = golden("board")["games"]
    n = len(games)
    st = boards.make_states(np.zeros((n, 225), np.int8))
    longest = max(len(g["moves"]) for g in games)
    masks = [[] for _ in range(n)]
    for i in range(longest):
        mv = np.array([g["moves"][i] if i < len(g["moves"]) else -1 for g in games], np.int32)
        new, ok, legal = device.board_step(st, mv)
        for k, g in enumerate(games):
            if i >= len(g["moves"]):
                continue
            assert bool(ok[k]) == g["ok"][i]
            assert bool(new["over"][k]) == g["over"][i]
            assert new["winner"][k] == g["winner"][i]
            assert new["player"][k] == g["player"][i]
            masks[k].append(format(boards.legal_int(legal[k]), "057x"))
        st = new
    import zlib
    for k, g in enumerate(games):
        assert zlib.crc32("".join(masks[k]).encode()) == g["mask_crc32"]
        if g["masks"] is not None:
            assert masks[k] == g["masks"]


def test_board_step_crafted(oracle):
    for case in golden("board")["crafted"]:
        st = boards.make_states(np.zeros((1, 225), np.int8))
        for mv in case["moves"]:
            st, ok, _ = device.board_step(st, [mv])
        assert bool(st["over"][0]) == case["over"], case["name"]
        assert st["winner"][0] == case["winner"], case["name"]
    st = boards.make_states(np.zeros((4, 225), np.int8))
    _, ok, _ = device.board_step(st, [-1, 225, 1000, 3])
    assert list(ok) == [0, 0, 0, 1]


def test_policy_step_golden(oracle):
    cases = golden("policy")["cases"]
    st = _states_from_moves(oracle, [c["moves"] for c in cases])
    keys = [rng.stream_key(SEED, i, len(c["moves"]), 1) for i, c in enumerate(cases)]
    mv, dr = device.policy_move(st, keys)
    assert list(mv) == [c["move"] for c in cases]
    assert list(dr) == [c["draws"] for c in cases]


def test_rollouts_golden(oracle):
    cases = golden("rollout")["cases"]
    st = _states_from_moves(oracle, [c["moves"] for c in cases])
    keys = [rng.stream_key(SEED, i, len(c["moves"]), 1) for i, c in enumerate(cases)]
    vals, fin, dr = device.rollout(st, [c["player"] for c in cases], keys)
    cells = boards.words_to_cells(fin["black"], fin["white"])
    for i, c in enumerate(cases):
        assert vals[i] == c["value"], i
        assert dr[i] == c["draws"], i
        assert "".join(str(int(x)) for x in cells[i]) == c["final"], i
        assert fin["n_moves"][i] == c["final_n"]


def test_rollouts_vs_oracle_random(oracle):
    """Larger sample against the oracle: random positions, several depth caps."""
    r = np.random.default_rng(1)
    moves = []
    for i in range(512):
        L = int(r.integers(0, 120))
        b = oracle.new_board()
        mv = []
        while len(mv) < L:
            c = int(r.integers(0, 225))
            if b.cell[c] == 0:
                oracle.lib().or_make_move(b, c // 15, c % 15)
                mv.append(c)
                if b.over:
                    mv.pop()
                    b = oracle.new_board(mv)
        moves.append(mv)
    st = _states_from_moves(oracle, moves)
    for depth in (100, 7):
        keys = [rng.stream_key(77, i, depth, 3) for i in range(len(moves))]
        ai = [1 + (i % 2) for i in range(len(moves))]
        vals, fin, dr = device.rollout(st, ai, keys, max_depth=depth)
        for i, mv in enumerate(moves):
            b = oracle.new_board(mv)
            v, d, fb = oracle.rollout(b, ai[i], keys[i], max_depth=depth)
            assert vals[i] == v and dr[i] == d, (i, depth)
            assert fin["n_moves"][i] == fb.n_moves


def test_pattern_scores_golden(oracle):
    pos = golden("pattern")["positions"]
    st = _states_from_moves(oracle, [c["moves"] for c in pos])
    for pl, key, bgkey in ((1, "s1", "bg1"), (2, "s2", "bg2")):
        s, bg = device.pattern_score(st, [pl] * len(pos))
        assert list(s) == [c[key] for c in pos]
        assert list(bg) == [c[bgkey] for c in pos]
