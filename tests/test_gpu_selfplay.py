"""Self-play collector on the GPU (training.play_one_game batched over slots):
finished games' (s, pi, z) records against the reference's golden games and
the oracle, plus the PV leaf count against the reference's predict() calls."""
import numpy as np
import pytest

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
