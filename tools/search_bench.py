#!/usr/bin/env python3
"""Self-play search kernel alone (prior-elided mode: no leaf gather, no PV forward):
4096 games, 200 sims, medium, beta 0; warm up to ply --warmup, then time --plies plies
in launches of 10.  Prints moves/s and the kernel time (HIP events on the launch stream)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "alphazero-gomoku_amd"))
import torch  # noqa: E402

from gzero.selfplay import SelfPlayEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--slots", type=int, default=4096)
ap.add_argument("--warmup", type=int, default=40)
ap.add_argument("--plies", type=int, default=20)
ap.add_argument("--beta", type=float, default=0.0)
a = ap.parse_args()
eng = SelfPlayEngine(n_slots=a.slots, num_simulations=200, c_puct=1.6, exploration=0.05, beta=a.beta, seed=1234,
                     pv_weights=None, plies_per_step=10)
done = 0
while done < a.warmup:
    n = min(10, a.warmup - done)
    eng.launch_search(n)
    done += n
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
moves = 0
done = 0
while done < a.plies:
    n = min(10, a.plies - done)
    eng.launch_search(n)
    moves += int(eng.counters()["moves"])
    done += n
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1)
print(f"search (prior-elided) {a.slots} games, plies {a.warmup}..{a.warmup + a.plies}: {moves} moves in {ms:.1f} ms "
      f"= {moves / ms * 1e3:.0f} moves/s")
