"""The C restatement of the BG planner (oracle/gz_oracle.c) against the reference's
own outputs (tests/golden/{gnet,planner,planner_mcts}.json.gz, made by
tests/golden/make_golden.py from bg_planner.py / ai_agent.py).

Integer / fp64 parts (knowledge-search scores, top-k order, the composed
argmax, RNG draws, the search tree) are compared exactly; the nets' fp32 outputs
within tolerance.  Where the planner's move depends on the nets, the reference's
recorded p / q (at the top-k cells) are injected, so that the rest of the search
is compared bit for bit.
"""
import base64

import numpy as np
import pytest

from conftest import golden
import oracle as O
from gzero import planner_nets

N = 15


def _dec(s, shape):
    return np.frombuffer(base64.b64decode(s), dtype=np.float32).reshape(shape)


def _hexf(hs):
    return np.array([int(h, 16) for h in hs], dtype=np.uint32).view(np.float32)


@pytest.fixture(scope="module")
def gn():
    g = golden("gnet")
    gsd = planner_nets.init_graphnet_state(g["gn_seed"])
    dsd = planner_nets.init_dqn_state(g["dqn_seed"])
    return g, gsd, dsd, planner_nets.pack_planner_weights(gsd, dsd)


def test_layout_matches_packer():
    lay = O.gnet_layout()
    P = planner_nets
    want = [P.GE_W, P.GE_B] + [P._layer_off(i) for i in range(8)] + [
        P.GP_W, P.GP_B, P.GF_WT, P.GF_B, P.D0_WT, P.D0_B, P.D1_WT, P.D1_B, P.D2_WT, P.D2_B]
    assert lay == want


def test_torch_modules_match_reference(gn):
    """gzero.planner_nets.GraphNet/OpponentDQN (same names, same init) reproduce the reference modules."""
    g, gsd, dsd, _ = gn
    n = len(g["cases"])
    planes = np.zeros((n, 3, N, N), np.float32)
    for i, c in enumerate(g["cases"]):
        cells = np.zeros(225, np.int8)
        p = 1
        for m in c["moves"]:
            cells[m] = p
            p = 3 - p
        planes[i, 0] = (cells == 1).reshape(N, N)
        planes[i, 1] = (cells == 2).reshape(N, N)
        planes[i, 2] = (cells == 0).reshape(N, N)
    lg, p, q = planner_nets.reference_forward(gsd, dsd, planes)
    np.testing.assert_allclose(lg, _dec(g["logits_f32_b64"], (n, 225)), rtol=0, atol=1e-5)
    np.testing.assert_allclose(p, _dec(g["p_f32_b64"], (n, 225)), rtol=0, atol=1e-6)
    np.testing.assert_allclose(q, _dec(g["q_f32_b64"], (n, 225)), rtol=0, atol=1e-5)


def test_oracle_nets_vs_reference(gn):
    g, _, _, blob = gn
    n = len(g["cases"])
    lg_ref = _dec(g["logits_f32_b64"], (n, 225))
    p_ref = _dec(g["p_f32_b64"], (n, 225))
    q_ref = _dec(g["q_f32_b64"], (n, 225))
    for i, c in enumerate(g["cases"][:16]):
        b = O.new_board(c["moves"])
        lg, p, q = O.gnet_forward(blob, b)
        np.testing.assert_allclose(lg, lg_ref[i], rtol=0, atol=1e-4)
        np.testing.assert_allclose(p, p_ref[i], rtol=0, atol=1e-6)
        np.testing.assert_allclose(q, q_ref[i], rtol=0, atol=1e-4)


def test_knowledge_scores_and_topk():
    g = golden("planner")
    checked = 0
    for c in g["cases"]:
        b = O.new_board(c["moves"])
        k = O.PLANNER[c["difficulty"]][0]
        assert O.topk(b, c["P"], k) == c["top"], c["moves"]
        if c.get("scores"):
            legal = [i for i in range(225) if b.cell[i] == 0]
            got = [O.ks_score(b, m, c["P"]) for m in legal]
            assert got == c["scores"]
            checked += 1
    assert checked >= 150


def test_planner_move_with_reference_nets():
    g = golden("planner")
    for c in g["cases"]:
        b = O.new_board(c["moves"])
        p = np.zeros(225, np.float32)
        q = np.zeros(225, np.float32)
        p[c["top"]] = _hexf(c["p"])
        q[c["top"]] = _hexf(c["q"])
        key = O.lib().or_stream_key(g["seed"], c["game_id"], len(c["moves"]), 1)
        mv, draws = O.planner_move(b, c["P"], c["difficulty"], p, q, key)
        assert mv == c["move"] and draws == c["draws"], (c["game_id"], mv, c["move"])


def _board_str(b):
    return "".join(str(int(v)) for v in b.cells())


@pytest.mark.parametrize("idx", range(20))
def test_planner_search_vs_reference(idx):
    g = golden("planner_mcts")
    c = g["cases"][idx]
    steps = {}
    seen = {}
    for call in c["calls"]:
        s = call["sim"]
        t = seen.get(s, 0)
        seen[s] = t + 1
        steps[(s, t)] = call

    def pq(board, game_id, sim, step):
        call = steps[(sim, step)]
        assert _board_str(board) == call["board"], (sim, step)
        p = np.zeros(225, np.float32)
        q = np.zeros(225, np.float32)
        p[call["top"]] = _hexf(call["p"])
        q[call["top"]] = _hexf(call["q"])
        return p, q

    b = O.new_board(c["moves"])
    prm = O.make_params(c["difficulty"], sims=c["sims"], beta=c["beta"], seed=g["seed"],
                        planner_steps=c["planner_steps"], pq=pq)
    mv, tree = O.get_move(b, b.player, prm, c["game_id"])
    assert mv == c["move"]
    assert tree["main_draws"] == c["main_draws"]
    assert tree["sim_draws"] == sum(c["sim_draws"])
    if "children" in c:
        assert tree["visits"][0] == c["root_visits"]
        assert tree["value"][0] == c["root_value"]
        kids = [[tree["move"][i], tree["visits"][i], tree["value"][i]]
                for i in range(len(tree["parent"])) if tree["parent"][i] == 0]
        assert kids == c["children"]


@pytest.mark.parametrize("idx", range(4))
def test_planner_search_200_sims_vs_reference(idx):
    """Config 4's own settings (tests/golden planner_mcts200.json.gz, make_golden.py
    part_planner_mcts200): reference searches at 200 simulations with 5 planner plies
    (medium, beta 0.2 and 0.0) from positions with 32-39 stones, so the parallel
    phase (every root child) is followed by sequential UCB simulations.  With the
    reference's recorded net outputs injected, in call order, the oracle makes the
    same ~1,000 planner calls on the same boards and returns the reference's move,
    draw counts, predict count and every root child's (move, visits, fp64 value)."""
    g = golden("planner_mcts200")
    c = g["cases"][idx]
    calls = c["calls"]
    pos = [0]

    def pq(board, game_id, sim, step):
        i = pos[0]
        assert i < len(calls)
        call = calls[i]
        assert call["sim"] == sim and _board_str(board) == call["board"], (i, sim, step)
        pos[0] += 1
        p = np.zeros(225, np.float32)
        q = np.zeros(225, np.float32)
        p[call["top"]] = _hexf(call["p"])
        q[call["top"]] = _hexf(call["q"])
        return p, q

    b = O.new_board(c["moves"])
    prm = O.make_params(c["difficulty"], sims=c["sims"], beta=c["beta"], seed=g["seed"],
                        planner_steps=c["planner_steps"], pq=pq)
    with O.Trace() as tr:
        mv, tree = O.get_move(b, b.player, prm, c["game_id"])
    assert pos[0] == len(calls)
    assert tr.planner_moves == [call["move"] for call in calls]
    assert mv == c["move"]
    assert tree["main_draws"] == c["main_draws"] and tree["sim_draws"] == sum(c["sim_draws"])
    assert tree["predicts"] == c["predicts"]
    assert tree["visits"][0] == c["root_visits"] and tree["value"][0] == c["root_value"]
    kids = [[tree["move"][i], tree["visits"][i], tree["value"][i]]
            for i in range(len(tree["parent"])) if tree["parent"][i] == 0]
    assert kids == c["children"]
    assert len(kids) < c["sims"] - 1  # the sequential phase ran


def _replay_arena_case(g, c, perturb=None):
    """Replay one arena_plans case in the oracle, every planner call fed the
    reference's recorded net outputs IN ORDER, and check what the games' moves
    alone cannot show (at 3-4 simulations every root child gets one visit, so the
    move is the highest empty cell unless exploration fires -- SURVEY §0.4):
    the i-th planner call sees the reference's i-th board (which pins every earlier
    planner move, including the first ply's choice inside each rollout), every
    planner move equals the reference's recorded move, and the call count matches.
    ``perturb(p, q) -> (p, q)`` alters the injected outputs (sensitivity check).
    Raises AssertionError (or oracle.CallbackError) on the first difference."""
    calls = c["calls"]
    pos = [0]

    def pq(board, game_id, sim, step):
        i = pos[0]
        assert i < len(calls), f"planner call {i} beyond the reference's {len(calls)}"
        call = calls[i]
        assert _board_str(board) == call["board"], f"planner call {i}: board differs"
        pos[0] += 1
        p = np.zeros(225, np.float32)
        q = np.zeros(225, np.float32)
        p[call["top"]] = _hexf(call["p"])
        q[call["top"]] = _hexf(call["q"])
        return perturb(p, q) if perturb else (p, q)

    cur = O.make_params("easy", sims=c["easy_sims"], beta=0.2, seed=g["seed"], planner_steps=2, pq=pq)
    base = O.make_params("easy", sims=c["eval_num_sim"], beta=0.2, seed=g["seed"], planner_steps=2, pq=pq)
    with O.Trace() as tr:
        games = []
        for k in range(len(c["boards"])):
            black, white = (cur, base) if k % 2 == 0 else (base, cur)
            games.append(O.play_game(black, white, c["game_id_base"] + k))
    for k, (got, ref) in enumerate(zip(games, c["boards"])):
        assert got["moves"] == ref["moves"], (c["game_id_base"], k)
        assert (got["winner"] or None) == ref["winner"]
    assert pos[0] == len(calls), (pos[0], len(calls))
    assert tr.planner_moves == [call["move"] for call in calls]
    return games


def test_arena_with_planner_exact_on_reference_outputs():
    """evaluate_model with the planner ON (eval_plans 2, the reference default,
    training.py:223; tests/golden arena_plans.json.gz, make_golden.py
    part_arena_plans): with every planner call fed the reference's own recorded net
    outputs, the oracle plays each game (the evaluated AI on black in even games,
    easy difficulty with the fixture's simulation counts, beta 0.2, 2 planner plies,
    the fixture's seed on both sides, game id = base + g) move for move and to the
    same winner as the reference's evaluate_model -- and makes the reference's
    planner calls, in order, on the same boards and with the same moves
    (_replay_arena_case), so the planner's decisions are compared, not only the
    games' moves."""
    g = golden("arena_plans")
    for c in g["cases"]:
        _replay_arena_case(g, c)
        # the evaluated AI plays black in even games: its wins / losses are the result's
        won = [b["winner"] == (1 if k % 2 == 0 else 2) for k, b in enumerate(c["boards"])]
        lost = [b["winner"] == (2 if k % 2 == 0 else 1) for k, b in enumerate(c["boards"])]
        assert (sum(won), sum(lost)) == (c["result"]["wins"], c["result"]["losses"])


@pytest.mark.parametrize("how", ["q+1e-4", "raise"])
def test_arena_planner_check_detects_a_perturbed_net(how):
    """The check above must be able to fail: with the injected DQN values moved by
    1e-4 (the nets' own tolerance) times a fixed pattern over the cells, some
    planner choice flips (a different board at a later call, or a different
    recorded move), and a callback that raises is re-raised by the oracle wrapper
    instead of being printed and swallowed by ctypes.
    (Scaling p or q by 1.01 flips nothing in this fixture: the random-init
    GraphNet's softmax is ~1/225 everywhere, so composed = a*p - (1-a)*q is ordered
    like -q and a uniform scale keeps that order; an additive 1e-4 pattern flips 5
    of the 4,006 recorded choices, 1e-3 flips 58.)"""
    g = golden("arena_plans")

    pattern = (np.float32(1e-4) * np.sin(np.arange(225) * 1.7)).astype(np.float32)

    def scaled(p, q):
        return p, q + pattern

    def broken(p, q):
        raise KeyError("no such board")

    failed = 0
    for c in g["cases"]:
        try:
            _replay_arena_case(g, c, perturb=scaled if how == "q+1e-4" else broken)
        except (AssertionError, O.CallbackError):
            failed += 1
    assert failed == len(g["cases"]) if how == "raise" else failed >= 1
