#!/usr/bin/env python3
"""Probe: does a search ply (selfplay_kernel, VALU-bound, ~6 KB LDS per game)
hide behind the tree forward (one 152-KB-LDS workgroup per CU) when both run on
separate streams?  Prints the tree forward alone, the search alone and both
launched together (engine A's forward on the current stream, engine B's search
on a second one)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "alphazero-gomoku_amd"))

import torch  # noqa: E402

from gzero import weights  # noqa: E402
from gzero.device import PVWeights  # noqa: E402
from gzero.selfplay import SelfPlayEngine  # noqa: E402


def main():
    torch.cuda.set_device(0)
    w = PVWeights(weights.pack_pv_weights(weights.init_state_dict(0)), precision="f16x3")
    a = SelfPlayEngine(n_slots=4096, num_simulations=200, beta=0.0, seed=1, pv_weights=w, pv_mode="tree")
    b = SelfPlayEngine(n_slots=4096, num_simulations=200, beta=0.0, seed=2, pv_weights=None)
    a.advance(300)
    b.advance(300)
    a.step()
    torch.cuda.synchronize()
    s2 = torch.cuda.Stream()

    def timed(fn, label, reps=3):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        fn()
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(reps):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        print(f"{label}: {ev[0].elapsed_time(ev[1]) / reps:.2f} ms", flush=True)

    def both():
        cur = torch.cuda.current_stream()
        s2.wait_stream(cur)
        with torch.cuda.stream(s2):
            b.launch_search(1)
        a.launch_pv()
        cur.wait_stream(s2)

    timed(a.launch_pv, "tree forward alone")
    timed(lambda: b.launch_search(1), "search ply alone")
    timed(both, "both, two streams")


if __name__ == "__main__":
    main()
