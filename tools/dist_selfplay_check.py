#!/usr/bin/env python3
"""Multi-rank rehearsal of training.selfplay_device (the bounded self-play of
run_iteration) on one GPU: under torchrun (GZ_DIST_BACKEND=gloo, GZ_DIST_SAME_DEVICE=1)
each of the ranks plays its G game ids and saves the collected rows (which must be
every rank's games); run without torchrun it plays all ws * G games in one process
and checks that every rank's rows equal them bit for bit.
Usage: torchrun --nproc-per-node 2 tools/dist_selfplay_check.py OUT; then
       python tools/dist_selfplay_check.py OUT"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gomoku_amd"))
import numpy as np  # noqa: E402

G, WS, SLOTS, SIMS, SEED = 24, 2, 16, 12, 5


def play(n_games, id_lo, id_hi, base):
    import training
    from bg_planner import BGPlannerAI
    from gzero import planner_nets, weights
    from neural_network import GomokuModel
    model = GomokuModel(device="cpu")
    model.model.load_state_dict(weights.init_state_dict(seed=3))
    planner = BGPlannerAI(1, "medium", seed=0)
    planner.graph_net.load_state_dict(planner_nets.init_graphnet_state(21))
    planner.opp_dqn.load_state_dict(planner_nets.init_dqn_state(22))
    rows, n, st = training.selfplay_device(n_games, id_lo, id_hi, num_simulations=SIMS, beta=0.2, seed=SEED,
                                           n_slots=SLOTS, game_id_base=base, model=model, plies_per_step=4,
                                           planner_steps=2, planner=planner)
    return rows[:n].cpu().numpy(), st


def main():
    out = sys.argv[1]
    os.makedirs(out, exist_ok=True)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from gzero import dist as gdist
        r, ws = gdist.init_from_env()
        assert ws == WS
        rows, st = play(G, 0, WS * G, r * G)
        np.save(os.path.join(out, f"rank{r}.npy"), rows)
        print(f"rank {r}: {len(rows)} rows, {st['moves_played']} plies played, {st['steps']} steps", flush=True)
        return
    rows, st = play(WS * G, 0, WS * G, 0)
    print(f"single: {len(rows)} rows, {st['moves_played']} plies played, {st['steps']} steps", flush=True)
    for r in range(WS):
        got = np.load(os.path.join(out, f"rank{r}.npy"))
        assert got.shape == rows.shape and np.array_equal(got, rows), f"rank {r} differs"
    print(f"every rank's rows == the single-process rows ({len(rows)} rows, {WS * G} games)", flush=True)


if __name__ == "__main__":
    main()
