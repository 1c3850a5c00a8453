"""BG planner on the GPU: gz_planner_move (BGPlannerAI.get_move) and
gz_plan_search (MCTS with planner rollout plies).

Exact checks use the GPU's own net outputs: the C oracle is driven with p / q
computed by gz_gn_forward for the same boards (the nets are fp32 and only
tolerance-equal to torch's), so everything else -- knowledge-search scores, top-k,
compose, RNG draws, trees -- must agree bit for bit.  Against the reference's
fixtures the moves must agree except where the reference's own composed scores
are a near-tie (|gap| <= 1e-6) that the nets' rounding can flip.
"""
import numpy as np
import pytest

from conftest import SEED, golden, oracle_slot_draws, planner_net_flips
from gzero import _lib, boards, planner_nets

pytestmark = pytest.mark.gpu

DIFF = {"easy": (1.4, 0.2), "medium": (1.6, 0.05), "hard": (1.8, 0.01)}


def _hexf(hs):
    return np.array([int(h, 16) for h in hs], dtype=np.uint32).view(np.float32)


@pytest.fixture(scope="module")
def gnw():
    from gzero import device
    g = golden("planner")
    gsd = planner_nets.init_graphnet_state(g["gn_seed"])
    dsd = planner_nets.init_dqn_state(g["dqn_seed"])
    return device.GNWeights(planner_nets.pack_planner_weights(gsd, dsd))


def _state(oracle, moves):
    b = oracle.new_board(moves)
    return b, boards.make_states(b.cells()[None], n_moves=b.n_moves, player=b.player, over=b.over, winner=b.winner)


def _rows(cells):
    bl, wh = boards.cells_to_words(np.asarray(cells, np.int8).reshape(-1, 225))
    return boards.leaf_words(bl, wh)


def test_planner_move_exact_vs_oracle(oracle, gnw):
    from gzero import device
    g = golden("planner")
    cases = g["cases"]
    sts, ais, keys, obs = [], [], [], []
    for c in cases:
        b, st = _state(oracle, c["moves"])
        obs.append(b)
        sts.append(st[0])
        ais.append(c["P"])
        keys.append(oracle.lib().or_stream_key(g["seed"], c["game_id"], len(c["moves"]), 1))
    sts = np.array(sts)
    by_diff = {}
    for i, c in enumerate(cases):
        by_diff.setdefault(c["difficulty"], []).append(i)
    p, q, _ = device.gn_forward(gnw, _rows([b.cells() for b in obs]))
    for diff, idx in by_diff.items():
        mv, dr = device.planner_move(sts[idx], [ais[i] for i in idx], [keys[i] for i in idx],
                                     _lib.planner_params(diff), gnw)
        for k, i in enumerate(idx):
            om, od = oracle.planner_move(obs[i], ais[i], diff, p[i], q[i], keys[i])
            assert (int(mv[k]), int(dr[k])) == (om, od), cases[i]["game_id"]


def test_planner_move_vs_reference(oracle, gnw):
    from gzero import device
    g = golden("planner")
    mism = 0
    for diff in ("easy", "medium", "hard"):
        cs = [c for c in g["cases"] if c["difficulty"] == diff]
        sts = np.array([_state(oracle, c["moves"])[1][0] for c in cs])
        keys = [oracle.lib().or_stream_key(g["seed"], c["game_id"], len(c["moves"]), 1) for c in cs]
        mv, dr = device.planner_move(sts, [c["P"] for c in cs], keys, _lib.planner_params(diff), gnw)
        a = _lib.PLANNER[diff][1]
        for k, c in enumerate(cs):
            assert int(dr[k]) == c["draws"]
            if int(mv[k]) == c["move"]:
                continue
            mism += 1
            top = c["top"]
            comp = {cell: a * float(pp) - (1 - a) * float(qq)
                    for cell, pp, qq in zip(top, _hexf(c["p"]), _hexf(c["q"]))}
            assert int(mv[k]) in comp and abs(comp[int(mv[k])] - comp[c["move"]]) <= 1e-6, c["game_id"]
    assert mism <= 3


def _pq_from_gpu(gnw):
    from gzero import device

    def pq(board, game_id, sim, step):
        cells = np.frombuffer(bytes(board.cell), dtype=np.int8)
        p, q, _ = device.gn_forward(gnw, _rows(cells))
        return p[0], q[0]
    return pq


@pytest.mark.parametrize("idx", range(20))
def test_plan_search_exact_vs_oracle(oracle, gnw, idx):
    from gzero import device
    g = golden("planner_mcts")
    c = g["cases"][idx]
    b, st = _state(oracle, c["moves"])
    cp, ex = DIFF[c["difficulty"]]
    p = device.search_params(c["sims"], cp, ex, c["beta"], SEED)
    p.planner_steps = c["planner_steps"]
    mv, stats, trees, _ = device.plan_search(st, [c["game_id"]], p, _lib.planner_params(c["difficulty"]), gnw,
                                             want_trees=True)
    prm = oracle.make_params(c["difficulty"], sims=c["sims"], beta=c["beta"], seed=SEED,
                             planner_steps=c["planner_steps"], pq=_pq_from_gpu(gnw))
    om, ot = oracle.get_move(b, b.player, prm, c["game_id"])
    assert int(mv[0]) == om
    assert stats[0]["main_draws"] == ot["main_draws"]
    assert stats[0]["sim_draws"] == ot["sim_draws"]
    assert stats[0]["predicts"] == ot["predicts"]
    t = trees[0]
    n = len(ot["parent"])
    assert [int(x) for x in t["parent"][:n]] == ot["parent"]
    assert [int(x) for x in t["move"][1:n]] == ot["move"][1:n]
    assert [int(x) for x in t["visits"][:n]] == ot["visits"]
    assert [float(x) for x in t["value"][:n]] == ot["value"]


@pytest.mark.parametrize("idx", range(4))
def test_plan_search_200_sims_exact_vs_oracle(oracle, gnw, idx):
    """Config 4's settings at full depth (tests/golden planner_mcts200: 200
    simulations, planner_steps 5, medium, 32-39 stones -- parallel then sequential
    phase): the GPU search equals the oracle driven by the GPU's net outputs -- move,
    draws, predicts and the whole tree, fp64 values bit for bit."""
    from gzero import device
    g = golden("planner_mcts200")
    c = g["cases"][idx]
    b, st = _state(oracle, c["moves"])
    cp, ex = DIFF[c["difficulty"]]
    p = device.search_params(c["sims"], cp, ex, c["beta"], SEED)
    p.planner_steps = c["planner_steps"]
    mv, stats, trees, _ = device.plan_search(st, [c["game_id"]], p, _lib.planner_params(c["difficulty"]), gnw,
                                             want_trees=True)
    prm = oracle.make_params(c["difficulty"], sims=c["sims"], beta=c["beta"], seed=SEED,
                             planner_steps=c["planner_steps"], pq=_pq_from_gpu(gnw))
    om, ot = oracle.get_move(b, b.player, prm, c["game_id"])
    assert int(mv[0]) == om
    assert stats[0]["main_draws"] == ot["main_draws"] and stats[0]["sim_draws"] == ot["sim_draws"]
    assert stats[0]["predicts"] == ot["predicts"]
    t = trees[0]
    n = len(ot["parent"])
    assert [int(x) for x in t["parent"][:n]] == ot["parent"]
    assert [int(x) for x in t["visits"][:n]] == ot["visits"]
    assert [float(x) for x in t["value"][:n]] == ot["value"]


def test_plan_search_200_sims_vs_reference(oracle, gnw):
    """The 4 reference searches at 200 simulations / planner_steps 5: same move and
    root children as the reference, or -- where one differs -- a recorded planner
    decision inside it that the nets' rounding flips at a near-tie (<= 1e-6)."""
    from gzero import device
    g = golden("planner_mcts200")
    for c in g["cases"]:
        _, st = _state(oracle, c["moves"])
        cp, ex = DIFF[c["difficulty"]]
        p = device.search_params(c["sims"], cp, ex, c["beta"], SEED)
        p.planner_steps = c["planner_steps"]
        mv, stats, trees, _ = device.plan_search(st, [c["game_id"]], p, _lib.planner_params(c["difficulty"]), gnw,
                                                 want_trees=True)
        t = trees[0]
        kids = [i for i in range(len(t["move"])) if t["parent"][i] == 0]
        got = [[int(t["move"][i]), int(t["visits"][i]), float(t["value"][i])] for i in kids]
        if not (int(mv[0]) == c["move"] and got == c["children"]):
            gaps = planner_net_flips(c["calls"], gnw, _lib.PLANNER[c["difficulty"]][1])
            assert gaps and max(gaps) <= 1e-6, (c["game_id"], gaps)


def test_plan_search_vs_reference(oracle, gnw):
    """All 20 reference searches: same move / root statistics, or -- for each
    search that differs -- a recorded planner decision inside it that the nets'
    rounding flips, at a near-tie (<= 1e-6) of the reference's composed scores."""
    from gzero import device
    g = golden("planner_mcts")
    same = 0
    for c in g["cases"]:
        _, st = _state(oracle, c["moves"])
        cp, ex = DIFF[c["difficulty"]]
        p = device.search_params(c["sims"], cp, ex, c["beta"], SEED)
        p.planner_steps = c["planner_steps"]
        mv, stats, trees, _ = device.plan_search(st, [c["game_id"]], p, _lib.planner_params(c["difficulty"]), gnw,
                                                 want_trees=True)
        ok = int(mv[0]) == c["move"] and stats[0]["sim_draws"] == sum(c["sim_draws"])
        if ok and "children" in c:
            t = trees[0]
            kids = [i for i in range(len(t["move"])) if t["parent"][i] == 0]
            got = [[int(t["move"][i]), int(t["visits"][i]), float(t["value"][i])] for i in kids]
            ok = got == c["children"]
        same += ok
        if not ok:
            gaps = planner_net_flips(c["calls"], gnw, _lib.PLANNER[c["difficulty"]][1])
            assert gaps and max(gaps) <= 1e-6, (c["game_id"], gaps)
    assert same >= 15, same


def test_selfplay_planner_games_vs_oracle(oracle, gnw):
    """gz_selfplay_plan_run: whole games (planner_steps 2, 3 sims) equal the oracle's
    play_one_game driven by the GPU's net outputs -- moves, z, and every slot's RNG
    draw counts over all the games it played (gz_selfplay_draws): at 3 simulations
    the moves never depend on a rollout's value, the draw counts depend on every
    planner and rollout decision."""
    from gzero.selfplay import SelfPlayEngine, records_to_games
    n_slots = 3
    eng = SelfPlayEngine(n_slots=n_slots, num_simulations=3, c_puct=1.6, exploration=0.05, beta=0.2, seed=SEED,
                         plies_per_step=16, planner_steps=2, planner_difficulty="medium", gn_weights=gnw)
    games = {}
    for _ in range(40):
        eng.step()
        for gid, g in records_to_games(eng.records()).items():
            if gid < n_slots:
                games[gid] = g
        if len(games) == n_slots:
            break
    assert len(games) == n_slots
    prm = oracle.make_params("medium", sims=3, beta=0.2, seed=SEED, planner_steps=2, pq=_pq_from_gpu(gnw))
    for gid, g in games.items():
        ref = oracle.play_game(prm, prm, gid)
        assert g["moves"] == ref["moves"], gid
        assert g["z"] == ref["z"], gid
    st, cur = eng.boards()
    got = eng.draws()
    for s in range(n_slots):
        done = list(range(s, int(cur[s]), n_slots))  # slot s plays ids s, s + n, s + 2n, ...
        want = oracle_slot_draws(oracle, prm, prm, done, int(cur[s]), int(st["n_moves"][s]))
        assert list(got[s]) == want, (s, list(got[s]), want)
        assert want[2] > 0


def test_config1_game_vs_oracle(oracle, gnw):
    """BASELINE config 1 (1 game, 50 sims, beta 0.2, planner_steps 5, medium), played to
    the end by the self-play engine: moves, players and z equal the oracle's
    play_one_game driven by the GPU's net outputs (injected p / q), and so do the
    slot's RNG draw counts (every planner ply and rollout ply of the game's 50-sim
    searches, gz_selfplay_draws)."""
    from gzero.selfplay import SelfPlayEngine, records_to_games
    eng = SelfPlayEngine(n_slots=1, num_simulations=50, c_puct=1.6, exploration=0.05, beta=0.2, seed=SEED,
                         plies_per_step=16, planner_steps=5, planner_difficulty="medium", gn_weights=gnw)
    game = None
    for _ in range(13):  # <= 200 plies
        eng.step()
        got = records_to_games(eng.records())
        if 0 in got:
            game = got[0]
            break
    assert game is not None
    prm = oracle.make_params("medium", sims=50, beta=0.2, seed=SEED, planner_steps=5, pq=_pq_from_gpu(gnw))
    ref = oracle.play_game(prm, prm, 0)
    assert game["moves"] == ref["moves"]
    assert game["players"] == ref["players"] and game["z"] == ref["z"]
    st, cur = eng.boards()
    want = oracle_slot_draws(oracle, prm, prm, [0], int(cur[0]), int(st["n_moves"][0]))
    assert list(eng.draws()[0]) == want and want[2] > 0


def test_incremental_graphnet_bitwise_on_planner_plies(gnw):
    """Config-4 plies (200 sims, beta 0.2, planner_steps 5, medium) from mid-game
    positions: every planner-net row the incremental GraphNet (gn_inc_kernel) ran
    -- rollout boards one stone from the root, and each later planner ply's board --
    has policy-conv outputs, p and q bitwise equal to the full forward's
    (GZ_FLAG_GN_CHECK re-runs gz_gn_forward on every row of every planner step)."""
    from gzero.selfplay import SelfPlayEngine
    eng = SelfPlayEngine(n_slots=96, num_simulations=200, c_puct=1.6, exploration=0.05, beta=0.2, seed=SEED + 7,
                         plies_per_step=1, planner_steps=5, planner_difficulty="medium", gn_weights=gnw)
    eng.advance(24)
    eng.gn_stats(reset=True, check=True)
    for _ in range(2):
        eng.step()
    st = eng.gn_stats()
    assert st["incremental"] > 0.8 * (st["incremental"] + st["full"]), st
    assert st["checked"] == st["incremental"] + st["full"], st
    assert st["mismatched"] == 0, st


def test_incremental_graphnet_same_games(gnw, monkeypatch):
    """The same planner self-play with the incremental GraphNet on and off
    (GZ_GN_INC=0): identical boards and records after every step."""
    from gzero.selfplay import SelfPlayEngine

    def run(flag):
        monkeypatch.setenv("GZ_GN_INC", flag)
        eng = SelfPlayEngine(n_slots=32, num_simulations=40, c_puct=1.6, exploration=0.05, beta=0.2, seed=SEED + 9,
                             plies_per_step=4, planner_steps=5, planner_difficulty="medium", gn_weights=gnw)
        eng.advance(8)
        out = []
        for _ in range(4):
            eng.step()
            b, g = eng.boards()
            out.append((np.asarray(b).tobytes(), np.asarray(g).tobytes(), eng.records().tobytes()))
        return out, eng.gn_stats()

    on, st_on = run("1")
    off, st_off = run("0")
    assert st_on["incremental"] > 0 and st_off["incremental"] == 0
    assert on == off


def test_incremental_graphnet_long_chains_fall_back_bitwise(gnw):
    """planner_steps 8: chains pass the 6 stones a job can keep squares for, so later
    plies fall back to the full forward (which then becomes the chain's base); every
    row still equals the full forward bit for bit."""
    from gzero.selfplay import SelfPlayEngine
    eng = SelfPlayEngine(n_slots=32, num_simulations=60, c_puct=1.6, exploration=0.05, beta=0.2, seed=SEED + 11,
                         plies_per_step=1, planner_steps=8, planner_difficulty="medium", gn_weights=gnw)
    eng.advance(12)
    eng.gn_stats(reset=True, check=True)
    for _ in range(2):
        eng.step()
    st = eng.gn_stats()
    assert st["incremental"] > 0 and st["full"] > 0, st
    assert st["checked"] == st["incremental"] + st["full"] and st["mismatched"] == 0, st


def _oracle_board(oracle, cells, n_moves, player):
    b = oracle.Board()
    for i in range(225):
        b.cell[i] = int(cells[i])
    b.n_moves, b.player, b.over, b.winner = int(n_moves), int(player), 0, 0
    return b


def test_config4_full_size_step_vs_oracle(oracle, gnw):
    """BASELINE config 4 at its benchmarked size: 4096 slots,
    200 simulations, beta 0.2, planner_steps 5 (medium), the PV tree forward on
    every node, after a 300-ply burn-in (continuous refill: a mix of game plies,
    many past 26 stones, where the searches run sequential-phase simulations).
    One planner ply-step with GZ_FLAG_GN_CHECK: every GraphNet row of the step --
    round 0's 819 k rollouts in 13 chunks of 65,536 jobs (map slots reused from
    chunk to chunk), then the sequential rounds -- is re-run by the full forward
    and bitwise equal; nothing is dropped; and for 12 slots with distinct positions
    (half of them with >= 27 stones) the move, the predict count and the RNG draws
    of the step's search equal the oracle's get_move driven by the GPU's p / q
    (ai_agent.py:168-304, bg_planner.py:232-269)."""
    from gzero.selfplay import SelfPlayEngine
    from test_gpu_selfplay import _pv_weights
    _, w = _pv_weights()
    n_slots, S = 4096, 200
    eng = SelfPlayEngine(n_slots=n_slots, num_simulations=S, c_puct=1.6, exploration=0.05, beta=0.2, seed=SEED + 11,
                         plies_per_step=1, planner_steps=5, planner_difficulty="medium", gn_weights=gnw,
                         pv_weights=w, pv_mode="tree")
    eng.advance(300)
    st0, gid0 = eng.boards()
    d0 = eng.draws()
    eng.gn_stats(reset=True, check=True)
    eng.step()
    gs = eng.gn_stats()
    c = eng.counters()
    assert c["records_dropped"] == 0 and c["leaves_dropped"] == 0 and c["moves"] == n_slots
    assert gs["full"] + gs["incremental"] > n_slots * S  # round 0 alone: one row per rollout ply
    assert gs["checked"] == gs["full"] + gs["incremental"] and gs["mismatched"] == 0, gs
    st1, gid1 = eng.boards()
    d1 = eng.draws()
    assert int(c["leaves"]) == int((d1 - d0)[:, 0].sum())  # every predict() became a PV row
    # sampled slots: a search ran (>= 6 stones), the game went on, distinct positions
    cells0 = boards.words_to_cells(st0["black"], st0["white"])
    cells1 = boards.words_to_cells(st1["black"], st1["white"])
    live = [s for s in range(n_slots) if st0["n_moves"][s] >= 6 and gid1[s] == gid0[s]]
    late = [s for s in live if st0["n_moves"][s] >= 27]
    early = [s for s in live if st0["n_moves"][s] < 27]
    assert len(late) >= 6 and len(early) >= 6
    rng = np.random.default_rng(3)
    pick, seen = [], set()
    for pool in (late, early):
        k = 0
        for s in rng.permutation(pool):
            key = cells0[s].tobytes()
            if key not in seen:
                seen.add(key)
                pick.append(int(s))
                k += 1
                if k == 6:
                    break
    prm = oracle.make_params("medium", sims=S, beta=0.2, seed=SEED + 11, planner_steps=5, pq=_pq_from_gpu(gnw))
    seq = 0
    for s in pick:
        diff = np.flatnonzero(cells1[s] != cells0[s])
        assert len(diff) == 1, s
        b = _oracle_board(oracle, cells0[s], st0["n_moves"][s], st0["player"][s])
        mv, tree = oracle.get_move(b, int(st0["player"][s]), prm, int(gid0[s]), cap=S + 2)
        assert int(diff[0]) == mv, (s, int(diff[0]), mv)
        got = list(d1[s] - d0[s])
        assert got == [tree["predicts"], tree["main_draws"], tree["sim_draws"]], (s, got, tree["predicts"])
        seq += tree["visits"][0] > 0 and len([p for p in tree["parent"] if p == 0]) < S - 1
    assert seq >= 1  # some sampled search ran sequential-phase simulations
