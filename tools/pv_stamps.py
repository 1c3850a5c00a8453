#!/usr/bin/env python3
"""Per-phase cycle split of the PV kernel (workgroup 0, wave 0), from the
-DGZ_PV_STAMPS build in tools/_build/libgzpv_stamps.so (make -C tools)."""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gomoku_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gzero import boards, weights  # noqa: E402

PHASES = ["planes", "conv0+store", "tower conv (k-loop)", "tower wait+skip", "tower epilogue",
          "head 1x1", "head FCs", "value/softmax"]

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--precision", default="f16x3")
ap.add_argument("--lib", default="libgzpv_stamps.so")
a = ap.parse_args()
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", a.lib))
P = ctypes.c_void_p
lib.gz_pv_forward.argtypes = [P, P, ctypes.c_int32, P, P, P, P, P, P, ctypes.c_int32, P]
lib.gz_pv_stamps_read.argtypes = [P, ctypes.c_int]
lib.gz_pv_workspace_bytes.restype = ctypes.c_size_t
blob = torch.from_numpy(weights.pack_pv_weights(weights.init_state_dict(0))).cuda()
rng = np.random.default_rng(0)
cells = rng.choice(3, size=(a.n, 225), p=[0.5, 0.25, 0.25]).astype(np.int8)
bl, wh = boards.cells_to_words(cells)
d_b = torch.from_numpy(boards.leaf_words(bl, wh).view(np.int32).copy()).cuda()
lg = torch.empty(a.n * 225, device="cuda")
v = torch.empty(a.n, device="cuda")
pr = torch.empty(a.n * 225, device="cuda")
ws = torch.empty(lib.gz_pv_workspace_bytes(a.n) // 4 + 1, device="cuda")
mode = weights.PRECISIONS[a.precision]
out = np.zeros(32, np.uint64)
for it in range(2):
    lib.gz_pv_stamps_read(out.ctypes.data, 1)
    rc = lib.gz_pv_forward(blob.data_ptr(), d_b.data_ptr(), a.n, None, lg.data_ptr(), v.data_ptr(), pr.data_ptr(), None,
                           ws.data_ptr(), mode, None)
    assert rc == 0
    torch.cuda.synchronize()
lib.gz_pv_stamps_read(out.ctypes.data, 0)
boards_wg0 = (a.n + 255) // 256
tot = sum(int(x) for x in out[:8])
print(f"pv_kernel[{a.precision}] workgroup 0: {boards_wg0} boards, {tot / boards_wg0:.0f} s_memtime ticks/board")
for i, name in enumerate(PHASES):
    print(f"  {name:24s} {int(out[i]) / boards_wg0:10.0f}  {int(out[i]) / tot * 100:5.1f}%")
print("  per wave (tower, all layers): k-loop / wait at barrier")
for w in range(8):
    print(f"    wave {w}: {int(out[8 + w]) / boards_wg0:10.0f} {int(out[16 + w]) / boards_wg0:10.0f}")
