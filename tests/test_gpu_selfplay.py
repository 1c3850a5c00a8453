"""Self-play collector on the GPU (training.play_one_game batched over slots):
finished games' (s, pi, z) records against the reference's golden games and
the oracle, plus the PV leaf count against the reference's predict() calls."""
import numpy as np
import pytest
import torch

from conftest import SEED, golden
from gzero import boards
from gzero.selfplay import SelfPlayEngine, records_to_games, records_to_replay

pytestmark = pytest.mark.gpu


def _play(engine, total_plies, chunk=25):
    recs = []
    done = 0
    while done < total_plies:
        n = min(chunk, total_plies - done)
        engine.step(n)
        recs.append(engine.records())
        c = engine.counters()
        assert c["records_dropped"] == 0
        done += n
    return np.concatenate(recs) if recs else np.zeros(0, boards.RECORD_DTYPE)


def test_selfplay_matches_reference_golden_games():
    games = {g["game_id"]: g for g in golden("games")["games"]}
    for beta, first in ((0.0, 100), (0.2, 101)):
        eng = SelfPlayEngine(n_slots=6, num_simulations=2, c_puct=1.6, exploration=0.05, beta=beta, seed=SEED,
                             plies_per_step=50, game_id_base=100, game_id_stride=6)
        got = records_to_games(_play(eng, 100, chunk=50))
        for gid in range(first, 106, 2):
            g = games[gid]
            assert gid in got, gid
            assert got[gid]["moves"] == g["moves"]
            assert got[gid]["players"] == g["players"]
            assert got[gid]["z"] == g["outcomes"]


def test_selfplay_vs_oracle_many_slots(oracle):
    n_slots = 32
    eng = SelfPlayEngine(n_slots=n_slots, num_simulations=16, beta=0.2, seed=SEED, plies_per_step=40,
                         game_id_base=500)
    got = records_to_games(_play(eng, 160, chunk=40))
    checked = 0
    for gid in range(500, 500 + n_slots):
        if gid not in got:
            continue
        p = oracle.make_params("medium", sims=16, beta=0.2, seed=SEED)
        ref = oracle.play_game(p, p, gid, want_cells=True)
        assert got[gid]["moves"] == ref["moves"], gid
        assert got[gid]["z"] == ref["z"]
        assert (got[gid]["cells"] == ref["cells"]).all()
        checked += 1
    assert checked >= n_slots // 2
    planes, mv, pl, z = records_to_replay(eng.records() if len(eng.records()) else _play(eng, 40))
    assert planes.shape[1:] == (3, 15, 15)


def test_selfplay_leaf_count_equals_reference_predicts(oracle):
    """Reference-work mode: the engine evaluates exactly as many PV forwards as
    the reference's GomokuModel.predict calls (one per non-terminal node)."""
    from gzero import weights
    from gzero.device import PVWeights
    w = PVWeights(weights.pack_pv_weights(weights.init_state_dict(0)), precision="f16x3")
    for gid in (900, 901):
        p = oracle.make_params("medium", sims=24, beta=0.0, seed=SEED)
        ref = oracle.play_game(p, p, gid)
        eng = SelfPlayEngine(n_slots=1, num_simulations=24, beta=0.0, seed=SEED, pv_weights=w,
                             plies_per_step=ref["n"], game_id_base=gid)
        eng.step(ref["n"])
        c = eng.counters()
        assert c["moves"] == ref["n"] and c["games"] == 1
        assert c["leaves"] == ref["predicts"]
        assert c["leaves_dropped"] == 0


def test_sharded_ranks_play_the_single_gpu_games():
    """Config 3's sharding (gzero.dist.shard_ids): rank r of W plays game ids
    r*S + s + g*W*S.  Two 'ranks' of 8 slots each produce exactly the games that one
    16-slot engine plays for the same ids (a game's RNG streams depend only on its id),
    so an N-GPU run is the 1-GPU run's games, partitioned."""
    from gzero import dist as gdist
    S, W = 8, 2
    one = SelfPlayEngine(n_slots=S * W, num_simulations=6, beta=0.2, seed=SEED, plies_per_step=40)
    ref = records_to_games(_play(one, 120, chunk=40))
    shard = {}
    for r in range(W):
        base, stride = gdist.shard_ids(r, W, S)
        eng = SelfPlayEngine(n_slots=S, num_simulations=6, beta=0.2, seed=SEED, plies_per_step=40,
                             game_id_base=base, game_id_stride=stride)
        for gid, g in records_to_games(_play(eng, 120, chunk=40)).items():
            assert gid % (W * S) // S == r  # disjoint by construction
            shard[gid] = g
    common = sorted(set(ref) & set(shard))
    assert len(common) >= S
    for gid in common:
        assert shard[gid]["moves"] == ref[gid]["moves"], gid
        assert shard[gid]["z"] == ref[gid]["z"], gid


def _pv_weights():
    from gzero import weights
    from gzero.device import PVWeights
    sd = weights.init_state_dict(0)
    return sd, PVWeights(weights.pack_pv_weights(sd), precision="f16x3")


def _leaf_rows(eng, n):
    return eng.d_leaves[: n * 16].cpu().numpy().view(np.uint32).reshape(n, 16)


def test_config2_200_sims_vs_oracle(oracle):
    """BASELINE config 2 per slot (200 sims, medium, beta 0, planner_steps 0, the
    PV forward on every node the searches create): 16 slots x 12 plies equal the
    oracle's games and RNG draw counts (every rollout ply), the forwards per step
    equal its predict() count, and the PV
    outputs of the last step's nodes match torch fp32 (1e-4) and the oracle's
    masked prior (exact)."""
    from gzero import weights
    sd, w = _pv_weights()
    n_slots, K, base = 16, 12, 700
    eng = SelfPlayEngine(n_slots=n_slots, num_simulations=200, c_puct=1.6, exploration=0.05, beta=0.0, seed=SEED,
                         pv_weights=w, plies_per_step=1, game_id_base=base)
    leaves = 0
    for _ in range(K):
        eng.step()
        c = eng.counters()
        assert c["leaves_dropped"] == 0 and c["records_dropped"] == 0 and c["moves"] == n_slots
        assert c["games"] == 0  # no game ends in 12 plies: the slots keep their ids
        leaves += int(c["leaves"])
    st, gids = eng.boards()
    p = oracle.make_params("medium", sims=200, beta=0.0, seed=SEED)
    pred = 0
    draws = eng.draws()
    for s in range(n_slots):
        assert int(gids[s]) == base + s
        with oracle.Trace() as tr:
            ref = oracle.play_game(p, p, base + s, max_plies=K)
        assert ref["n"] == K
        cells = boards.words_to_cells(st["black"][s], st["white"][s])
        assert (cells == oracle.new_board(ref["moves"]).cells()).all(), s
        pred += ref["predicts"]
        # the rollouts' draw counts: at 200 sims from the opening every root child
        # gets one visit, so the moves alone never see a rollout
        want = [sum(x[i] for x in tr.plies) for i in range(3)]
        assert list(draws[s]) == want and want[2] > 0, (s, list(draws[s]), want)
    assert leaves == pred
    # the last step's forwards: logits / value vs torch fp32, prior vs the oracle
    n = int(eng.counters()["leaves"])
    rows = _leaf_rows(eng, n)
    sel = np.random.default_rng(1).choice(n, size=min(n, 384), replace=False)
    cells = boards.words_to_cells(rows[sel, :8], rows[sel, 8:])
    ref_lg, ref_v = weights.reference_forward(sd, boards.planes_from_cells(cells))
    lg = eng.d_logits[: n * 225].cpu().numpy().reshape(n, 225)[sel]
    v = eng.d_value[:n].cpu().numpy()[sel]
    assert np.abs(lg - ref_lg).max() < 1e-4 and np.abs(v - ref_v).max() < 1e-4
    probs = eng.d_probs[: n * 225].cpu().numpy().reshape(n, 225)[sel]
    prior = eng.d_prior[: n * 225].cpu().numpy().reshape(n, 225)[sel]
    for k in range(32):  # the reference's vector is the dense prior at the empty cells (row-major)
        assert np.array_equal(prior[k][cells[k] == 0], oracle.prior(probs[k], cells[k])), k
        assert (prior[k][cells[k] != 0] == 0).all()


def test_config2_4096_slot_step_properties(oracle):
    """One timed-size step of the bench workload (4096 slots, 200 sims, PV forward on
    every node) after a burn-in: no drops; for sampled slots the number of
    forwards over boards containing the slot's root equals the oracle's predict()
    count and the move played equals the oracle's; every finished game's records
    are plies 0..n-1 with z = +1 for the winner's plies, -1 for the loser's, 0 on a
    draw; probabilities sum to 1 and priors renormalise over the empty cells."""
    sd, w = _pv_weights()
    eng = SelfPlayEngine(n_slots=4096, num_simulations=200, c_puct=1.6, exploration=0.05, beta=0.0, seed=SEED,
                         pv_weights=w, plies_per_step=1)
    eng.advance(70)
    st0, gid0 = eng.boards()
    eng.step()
    c = eng.counters()
    assert c["leaves_dropped"] == 0 and c["records_dropped"] == 0 and c["moves"] == 4096
    n = int(c["leaves"])
    assert 0 < n <= eng.leaf_cap
    rows = _leaf_rows(eng, n)
    st1, gid1 = eng.boards()
    p = oracle.make_params("medium", sims=200, beta=0.0, seed=SEED)
    nm = st0["n_moves"]
    blk = np.unpackbits(np.ascontiguousarray(st0["black"]).view(np.uint8), axis=1).astype(bool)
    wht = np.unpackbits(np.ascontiguousarray(st0["white"]).view(np.uint8), axis=1).astype(bool)
    cand = [s for s in range(4096) if nm[s] >= 12]
    checked = 0
    for s in np.random.default_rng(3).permutation(cand):
        if checked == 12:
            break
        # a leaf of slot s' holds s's root only if s's stones missing from s' root fit on
        # a search path: skip roots within 8 stones of another slot's (same opening line)
        miss = (blk[s] & ~blk).sum(axis=1) + (wht[s] & ~wht).sum(axis=1)
        miss[s] = 1 << 20
        if miss.min() <= 8:
            continue
        cells0 = boards.words_to_cells(st0["black"][s], st0["white"][s])
        b = oracle.new_board([])
        for i in range(225):
            b.cell[i] = int(cells0[i])
        b.n_moves, b.player = int(st0["n_moves"][s]), int(st0["player"][s])
        mv, tree = oracle.get_move(b, b.player, p, int(gid0[s]))
        par = tree["parent"]
        depth = [0] * len(par)
        for i in range(1, len(par)):
            depth[i] = depth[par[i]] + 1
        assert max(depth) <= 8
        rb, rw = st0["black"][s], st0["white"][s]
        inside = np.all((rows[:, :8] & rb) == rb, axis=1) & np.all((rows[:, 8:] & rw) == rw, axis=1)
        assert int(inside.sum()) == tree["predicts"], (s, int(inside.sum()), tree["predicts"])
        if gid1[s] == gid0[s]:  # the game goes on: the board is the root plus the oracle's move
            cells1 = boards.words_to_cells(st1["black"][s], st1["white"][s])
            exp = cells0.copy()
            exp[mv] = st0["player"][s]
            assert (cells1 == exp).all(), s
        checked += 1
    assert checked == 12
    recs = eng.records()
    for gid in np.unique(recs["game_id"]):
        r = recs[recs["game_id"] == gid]
        r = r[np.argsort(r["ply"])]
        assert list(r["ply"]) == list(range(len(r)))
        assert list(r["player"]) == [1 + (i % 2) for i in range(len(r))]
        z = r["z"]
        if (z == 0).all():
            continue
        winner = int(r["player"][np.argmax(z)])
        assert all(zz == (1 if pl == winner else -1) for zz, pl in zip(z, r["player"]))
    probs = eng.d_probs[: n * 225].view(n, 225)
    assert torch.allclose(probs.sum(dim=1), torch.ones(n, device="cuda"), atol=1e-5)
    ps = eng.d_prior[: n * 225].view(n, 225).sum(dim=1)
    assert torch.allclose(ps, torch.ones_like(ps), rtol=0, atol=1e-12)


@pytest.mark.parametrize("planner_steps", [0, 2])
def test_selfplay_device_bounded_games_compaction(planner_steps):
    """training.selfplay_device with a bounded game range (game_id_end: a slot whose
    games are done goes idle) and the active slots compacted after every step
    (gz_selfplay_compact) against continuous refill: the same rows bit for bit, every
    game once, fewer plies played.  40 games on 16 slots (each slot plays 2-3 games,
    then idles), 12 simulations, with the PV tree forward; planner_steps 2 runs the
    planner pipeline (gz_selfplay_plan_run: idle slots are searched within a step
    and must record nothing)."""
    import training
    from bg_planner import BGPlannerAI
    from gzero import planner_nets, weights
    from neural_network import GomokuModel
    model = GomokuModel(device="cpu")
    model.model.load_state_dict(weights.init_state_dict(seed=3))
    planner = None
    if planner_steps:
        planner = BGPlannerAI(1, "medium", seed=0)
        planner.graph_net.load_state_dict(planner_nets.init_graphnet_state(21))
        planner.opp_dqn.load_state_dict(planner_nets.init_dqn_state(22))
    out = {}
    for compact in (False, True):
        rows, n, st = training.selfplay_device(40, 0, 40, num_simulations=12, beta=0.2, seed=SEED, n_slots=16,
                                               model=model, plies_per_step=4, planner_steps=planner_steps,
                                               planner=planner, compact=compact)
        out[compact] = (rows[:n].cpu().numpy().copy(), st)
    (a, sa), (b, sb) = out[False], out[True]
    assert a.shape == b.shape and np.array_equal(a, b)
    recs = np.frombuffer(b.tobytes(), boards.RECORD_DTYPE)
    assert sorted(set(int(g) for g in recs["game_id"])) == list(range(40))
    assert sb["moves_played"] == len(recs) < sa["moves_played"]


def test_selfplay_device_two_ranks_on_one_gpu(tmp_path):
    """training.selfplay_device under torchrun with 2 ranks (gloo, both on GPU 0:
    GZ_DIST_SAME_DEVICE) through the record exchange, each rank playing its own 24
    game ids with the bounded game range and slot compaction, planner on: every rank
    ends with all 48 games' rows, bit for bit those of one process playing the 48
    (tools/dist_selfplay_check.py)."""
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tool = os.path.join(root, "tools", "dist_selfplay_check.py")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, GZ_DIST_BACKEND="gloo", GZ_DIST_SAME_DEVICE="1")
    subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                    "--master-addr", "127.0.0.1", "--master-port", str(port), tool, str(tmp_path)],
                   env=env, check=True, timeout=240)
    out = subprocess.run([sys.executable, tool, str(tmp_path)], check=True, timeout=180, capture_output=True,
                         text=True).stdout
    assert "every rank's rows == the single-process rows" in out
