"""MCTS get_move on the GPU (one wavefront per position) against the reference's
golden vectors and the oracle: chosen move, full root statistics (fp64 values
compared exactly), grandchildren, PV-forward count and RNG draw counts."""
import numpy as np
import pytest

from conftest import SEED, golden
from gzero import boards, device

pytestmark = pytest.mark.gpu

DIFF = {"easy": (1.4, 0.2), "medium": (1.6, 0.05), "hard": (1.8, 0.01)}


def _state(oracle, moves):
    b = oracle.new_board(moves)
    return boards.make_states(b.cells()[None], n_moves=b.n_moves, player=b.player, over=b.over, winner=b.winner)


def _run_case(oracle, c):
    cp, ex = DIFF[c["difficulty"]]
    p = device.search_params(c["sims"], cp, ex, c["beta"], SEED)
    st = _state(oracle, c["moves"])
    mv, stats, trees, _ = device.search(st, [c["game_id"]], p, want_trees=True)
    return int(mv[0]), stats[0], trees[0]


def _compare_golden(c, mv, stats, t):
    assert mv == c["move"], c["game_id"]
    assert stats["predicts"] == c["predicts"]
    assert stats["main_draws"] == c["main_draws"]
    assert stats["sim_draws"] == sum(c["sim_draws"])
    if "children" in c:
        kids = [i for i in range(len(t["move"])) if t["parent"][i] == 0]
        got = [[int(t["move"][i]), int(t["visits"][i]), float(t["value"][i])] for i in kids]
        assert got == c["children"], c["game_id"]
        assert (int(t["visits"][0]), float(t["value"][0])) == (c["root_visits"], c["root_value"])
        pos = {i: k for k, i in enumerate(kids)}
        grand = [[pos[int(t["parent"][i])], int(t["move"][i]), int(t["visits"][i]), float(t["value"][i])]
                 for i in range(len(t["move"])) if int(t["parent"][i]) in pos and t["parent"][i] > 0]
        assert sorted(grand) == sorted(c["grand"])


@pytest.mark.parametrize("fixture", ["mcts", "mcts2"])
def test_search_golden(oracle, fixture):
    try:
        cases = golden(fixture)["cases"]
    except FileNotFoundError:
        pytest.skip(f"{fixture} fixture not generated")
    for c in cases:
        mv, stats, t = _run_case(oracle, c)
        _compare_golden(c, mv, stats, t)


def test_search_vs_oracle_full_tree(oracle):
    """Whole trees (every node's parent/move/visits/value) vs the oracle on
    positions at the metric's 200 simulations and in the sequential phase."""
    r = np.random.default_rng(5)
    cases = []
    for k in range(24):
        L = [6, 8, 10, 20, 30, 40, 90, 130][k % 8]
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
        sims = 200 if L < 90 else (225 - L) + 1 + int(r.integers(5, 60))
        cases.append((mv, sims, [0.0, 0.2][k % 2], 1000 + k))
    for mv, sims, beta, gid in cases:
        p = device.search_params(sims, 1.6, 0.05, beta, SEED)
        st = _state(oracle, mv)
        m, stats, trees, _ = device.search(st, [gid], p, want_trees=True)
        b = oracle.new_board(mv)
        om, ot = oracle.get_move(b, b.player, oracle.make_params("medium", sims=sims, beta=beta, seed=SEED), gid)
        t = trees[0]
        assert int(m[0]) == om
        assert stats[0]["n_nodes"] == len(ot["move"])
        assert stats[0]["predicts"] == ot["predicts"] and stats[0]["sim_draws"] == ot["sim_draws"]
        assert list(t["parent"]) == ot["parent"]
        assert [int(x) if i else -1 for i, x in enumerate(t["move"])] == ot["move"]
        assert list(t["visits"]) == ot["visits"]
        assert list(t["value"]) == ot["value"]


def test_search_batch_and_leaves(oracle):
    """Many positions in one launch; gathered leaf boards = the reference's predict calls."""
    cases = golden("mcts")["cases"][12:]
    st = np.concatenate([_state(oracle, c["moves"]) for c in cases])
    by_params = {}
    for i, c in enumerate(cases):
        by_params.setdefault((c["sims"], c["beta"], c["difficulty"]), []).append(i)
    for (sims, beta, diff), idx in by_params.items():
        cp, ex = DIFF[diff]
        p = device.search_params(sims, cp, ex, beta, SEED, gather_leaves=True)
        cap = sum(cases[i]["predicts"] for i in idx) + 8
        mv, stats, _, leaves = device.search(st[idx], [cases[i]["game_id"] for i in idx], p, leaf_cap=cap)
        assert list(mv) == [cases[i]["move"] for i in idx]
        assert len(leaves) == sum(cases[i]["predicts"] for i in idx)
        # every leaf is a legal successor position of one of the searched roots
        stones = (boards.words_to_cells(leaves[:, :8], leaves[:, 8:]) != 0).sum(axis=1)
        root_stones = {len(cases[i]["moves"]) for i in idx}
        assert all(any(s >= r for r in root_stones) for s in stones)
