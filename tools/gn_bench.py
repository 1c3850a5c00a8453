#!/usr/bin/env python3
"""Microbenchmark of the BG planner nets kernel (gz_gn_forward): random boards,
random-init weights; prints boards/s and TFLOP/s (GraphNet + DQN MACs x 2)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "alphazero-gomoku_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gzero import boards, device, planner_nets  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--check", type=int, default=256, help="boards checked against the torch fp32 nets")
a = ap.parse_args()
w = device.GNWeights(planner_nets.pack_planner_weights(planner_nets.init_graphnet_state(0),
                                                       planner_nets.init_dqn_state(1)))
rng = np.random.default_rng(0)
cells = rng.choice(3, size=(a.n, 225), p=[0.5, 0.25, 0.25]).astype(np.int8)
bl, wh = boards.cells_to_words(cells)
d_b = torch.from_numpy(boards.leaf_words(bl, wh).view(np.int32).copy()).cuda()
p = torch.empty(a.n * 225, device="cuda")
q = torch.empty(a.n * 225, device="cuda")
device.gn_forward_dev(w, d_b, a.n, d_p=p, d_q=q)
torch.cuda.synchronize()
ts = []
for _ in range(a.iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    device.gn_forward_dev(w, d_b, a.n, d_p=p, d_q=q)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 1e3)
t = float(np.median(ts))
fl = 2 * (planner_nets.GN_MACS + planner_nets.DQN_MACS)
print(f"gn_kernel n={a.n}: {t*1e3:.2f} ms, {a.n/t:.0f} boards/s, {a.n*fl/t/1e12:.1f} TFLOP/s (fp32-equivalent)")
if a.check:
    ref_lg, ref_p, ref_q = planner_nets.reference_forward(
        planner_nets.init_graphnet_state(0), planner_nets.init_dqn_state(1), boards.planes_from_cells(cells[: a.check]))
    dp = np.abs(p.view(a.n, 225)[: a.check].cpu().numpy() - ref_p).max()
    dq = np.abs(q.view(a.n, 225)[: a.check].cpu().numpy() - ref_q).max()
    print(f"  check {a.check} boards vs torch fp32: max |dp| {dp:.2e}, max |dq| {dq:.2e}",
          "OK" if dp < 1e-6 and dq < 1e-4 else "FAIL")
