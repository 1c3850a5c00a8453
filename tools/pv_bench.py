#!/usr/bin/env python3
"""Microbenchmark of the policy-value forward kernel alone: random boards,
random-init weights; prints boards/s and TFLOP/s (267.38 MFLOP per board)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "alphazero-gomoku_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gzero import boards, device, weights  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=65536)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--precision", default="f16x3")
ap.add_argument("--check", type=int, default=256, help="boards checked against the torch fp32 forward")
a = ap.parse_args()
w = device.PVWeights(weights.pack_pv_weights(weights.init_state_dict(0)), precision=a.precision)
rng = np.random.default_rng(0)
cells = rng.choice(3, size=(a.n, 225), p=[0.5, 0.25, 0.25]).astype(np.int8)
bl, wh = boards.cells_to_words(cells)
rows = boards.leaf_words(bl, wh)
d_b = torch.from_numpy(rows.view(np.int32).copy()).cuda()
lg = torch.empty(a.n * 225, device="cuda")
v = torch.empty(a.n, device="cuda")
pr = torch.empty(a.n * 225, device="cuda")
device.pv_forward_dev(w, d_b, a.n, d_logits=lg, d_value=v, d_probs=pr)
torch.cuda.synchronize()
ts = []
for _ in range(a.iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    device.pv_forward_dev(w, d_b, a.n, d_logits=lg, d_value=v, d_probs=pr)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 1e3)
t = float(np.median(ts))
print(f"pv_kernel[{a.precision}] n={a.n}: {t*1e3:.1f} ms, {a.n/t:.0f} boards/s, {a.n*weights.PV_FLOPS/t/1e12:.1f} TFLOP/s "
      f"({a.n*weights.PV_FLOPS/t/1e12/157.3*100:.1f}% of fp32 MFMA peak)")
if a.check:
    sd = weights.init_state_dict(0)
    ref_lg, ref_v = weights.reference_forward(sd, boards.planes_from_cells(cells[: a.check]))
    dl = np.abs(lg.view(a.n, 225)[: a.check].cpu().numpy() - ref_lg).max()
    dv = np.abs(v[: a.check].cpu().numpy() - ref_v.reshape(-1)).max()
    print(f"  check {a.check} boards vs torch fp32: max |dlogit| {dl:.2e}, max |dvalue| {dv:.2e}", "OK" if max(dl, dv) < 1e-4 else "FAIL")
