"""Batched arena (training.evaluate_model, training.py:221-270).

evaluate_model plays all games at once, one batched search per (agent, colour)
per ply.  Each game must equal the same game played alone through the
one-board API (AlphaZeroGomokuAI.get_move, pinned to the oracle and the
reference's fixtures by test_gpu_api / test_gpu_plan) with per-game AIs of the
same seeds and ``game_id = g`` -- which pins the batching: grouping, stream
keys, colours, simulation counts and the draw / stop rules.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 77


def _play_alone(current, baseline, g, seeds, sims_a, sims_b, plans=2):
    from ai_agent import AlphaZeroGomokuAI
    from gomoku_board import GomokuBoard
    from training import RandomAgent
    color_a = GomokuBoard.BLACK if g % 2 == 0 else GomokuBoard.WHITE
    other = GomokuBoard.WHITE if color_a == GomokuBoard.BLACK else GomokuBoard.BLACK
    a = AlphaZeroGomokuAI(color_a, "easy", planner_steps=plans, seed=seeds[0], game_id=g)
    a.model = current
    a.params = dict(a.params, num_simulations=sims_a)
    if baseline is None:
        b = RandomAgent(seeds[1], g)
    else:
        b = AlphaZeroGomokuAI(other, "easy", planner_steps=plans, seed=seeds[1], game_id=g)
        b.model = baseline
        b.params = dict(b.params, num_simulations=sims_b)
    board = GomokuBoard()
    moves = []
    while not board.game_over:
        agent = a if board.current_player == color_a else b
        m = agent.get_move(board)
        if m is None:
            break
        board.make_move(*m)
        moves.append(m[0] * 15 + m[1])
    return moves, board.winner


def test_arena_vs_random_equals_games_alone():
    from neural_network import GomokuModel
    from training import evaluate_model
    cur = GomokuModel(device="cpu")
    res = evaluate_model(cur, None, games=4, eval_num_sim=12, seed=SEED, return_games=True)
    for g, rec in enumerate(res["games"]):
        mv, w = _play_alone(cur, None, g, res["seeds"], 12, None)
        assert rec["moves"] == mv and rec["winner"] == w, g
        assert len(mv) >= 9 and w is not None  # five in a row needs 9 plies; random play loses
    assert res["wins"] + res["losses"] + res["draws"] == 4


def test_arena_vs_baseline_equals_games_alone():
    """With a baseline the evaluated AI keeps the difficulty's simulation count
    (easy: 100) and only the baseline's AI runs eval_num_sim (training.py:238-247)."""
    from neural_network import GomokuModel
    from training import evaluate_model
    cur, base = GomokuModel(device="cpu"), GomokuModel(device="cpu")
    res = evaluate_model(cur, base, games=2, eval_num_sim=10, seed=SEED + 1, return_games=True)
    for g, rec in enumerate(res["games"]):
        mv, w = _play_alone(cur, base, g, res["seeds"], 100, 10)
        assert rec["moves"] == mv and rec["winner"] == w, g
        assert len(mv) >= 9, g


def test_arena_vs_reference_fixture(monkeypatch):
    """evaluate_model against the reference's own evaluate_model (tests/golden
    arena.json.gz, make_golden.py part_arena): eval_plans 0 (no net output steers a
    move), the easy table's simulations lowered to the fixture's count on every AI
    the arena builds (as the generator does), one seed for both sides (the
    reference's single global stream) and game ids base + g.  Every game's moves and
    winner and the win / loss / draw counts equal the reference's."""
    import ai_agent
    from conftest import golden
    from neural_network import GomokuModel
    from training import evaluate_model
    g = golden("arena")
    orig = ai_agent.AlphaZeroGomokuAI.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        if self.difficulty == "easy":
            self.params["num_simulations"] = g["cases"][0]["easy_sims"]

    monkeypatch.setattr(ai_agent.AlphaZeroGomokuAI, "__init__", init)
    cur, base = GomokuModel(device="cpu"), GomokuModel(device="cpu")
    for c in g["cases"]:
        res = evaluate_model(cur, base if c["baseline"] else None, games=c["games"], eval_difficulty="easy",
                             eval_num_sim=c["eval_num_sim"], eval_plans=0, seeds=(g["seed"], g["seed"]),
                             game_id_base=c["game_id_base"], return_games=True)
        for k in ("wins", "losses", "draws", "win_rate"):
            assert res[k] == c["result"][k], (c["game_id_base"], k)
        for got, ref in zip(res["games"], c["boards"]):
            assert got["moves"] == ref["moves"], c["game_id_base"]
            assert got["winner"] == ref["winner"]


def test_arena_with_planner_vs_oracle(monkeypatch, oracle):
    """evaluate_model with the planner ON (eval_plans 2, the reference default,
    training.py:223) on the fixture's settings (tests/golden arena_plans.json.gz:
    planner nets of the fixture seeds, easy simulations lowered, one seed, game ids
    base + g): every batched GPU game equals the oracle's game driven by the GPU's own
    planner-net outputs (gz_gn_forward), move for move, AND every ply's search
    statistics -- predict count, main-stream draws and the draws summed over the
    simulations' streams -- equal the oracle's.  At 3-4 simulations the moves
    alone cannot see the planner (every root child gets one visit); the rollouts'
    draw counts can: each planner ply draws, and a different planner move changes
    the rollout that follows it.  A pq callback that fails raises (oracle wrapper).
    With
    test_oracle_planner.test_arena_with_planner_exact_on_reference_outputs (the oracle
    on the reference's recorded outputs = the reference's games) this pins the
    planner-steered arena to the reference's evaluate_model; the games whose moves
    differ from the reference's own (a near-tie of the two implementations' fp32 net
    outputs flips a planner choice) are counted, not failed."""
    import ai_agent
    import bg_planner
    from conftest import golden
    from gzero import boards, device, planner_nets
    from neural_network import GomokuModel
    from training import evaluate_model
    g = golden("arena_plans")
    gsd, dsd = planner_nets.init_graphnet_state(g["gn_seed"]), planner_nets.init_dqn_state(g["dqn_seed"])
    orig_p = bg_planner.BGPlannerAI.__init__

    def pinit(self, *a, **k):
        orig_p(self, *a, **k)
        self.graph_net.load_state_dict(gsd)
        self.opp_dqn.load_state_dict(dsd)

    orig_a = ai_agent.AlphaZeroGomokuAI.__init__

    def ainit(self, *a, **k):
        orig_a(self, *a, **k)
        if self.difficulty == "easy":
            self.params["num_simulations"] = g["cases"][0]["easy_sims"]

    monkeypatch.setattr(bg_planner.BGPlannerAI, "__init__", pinit)
    monkeypatch.setattr(ai_agent.AlphaZeroGomokuAI, "__init__", ainit)
    gnw = device.GNWeights(planner_nets.pack_planner_weights(gsd, dsd))

    def pq(board, game_id, sim, step):
        cells = np.frombuffer(bytes(board.cell), dtype=np.int8).reshape(1, 225)
        bl, wh = boards.cells_to_words(cells)
        p, q, _ = device.gn_forward(gnw, boards.leaf_words(bl, wh))
        return p[0], q[0]

    cur, base = GomokuModel(device="cpu"), GomokuModel(device="cpu")
    differ = planner_draws = 0
    for c in g["cases"]:
        res = evaluate_model(cur, base, games=c["games"], eval_difficulty="easy", eval_num_sim=c["eval_num_sim"],
                             eval_plans=2, seeds=(g["seed"], g["seed"]), game_id_base=c["game_id_base"],
                             return_games=True)
        cp = oracle.make_params("easy", sims=c["easy_sims"], beta=0.2, seed=g["seed"], planner_steps=2, pq=pq)
        bp = oracle.make_params("easy", sims=c["eval_num_sim"], beta=0.2, seed=g["seed"], planner_steps=2, pq=pq)
        for k, got in enumerate(res["games"]):
            black, white = (cp, bp) if k % 2 == 0 else (bp, cp)
            with oracle.Trace() as tr:
                ref = oracle.play_game(black, white, c["game_id_base"] + k)
            assert got["moves"] == ref["moves"], (c["game_id_base"], k)
            assert got["winner"] == (ref["winner"] or None)
            assert len(got["plies"]) == len(tr.plies)
            for ply, (a, b) in enumerate(zip(got["plies"], tr.plies)):
                assert a == b, (c["game_id_base"], k, ply, a, b)
            planner_draws += sum(b[2] for b in tr.plies)
            differ += got["moves"] != c["boards"][k]["moves"]
    assert planner_draws > 0
    print(f"planner-on arena: {differ} of {sum(c['games'] for c in g['cases'])} games differ from the "
          f"reference's own (net near-ties); {planner_draws} simulation-stream draws compared")
