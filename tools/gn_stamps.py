#!/usr/bin/env python3
"""Per-phase cycle split of the planner-nets kernel (workgroup 0, wave 0), from the
-DGZ_GN_STAMPS build (tools/_build/libgzgn_stamps.so, make -C tools)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gomoku_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gzero import boards, planner_nets  # noqa: E402

PHASES = ["planes + record", "(unused)", "embed", "conv3x3 k-loop", "conv3x3 store", "conv1x1 k-loop",
          "conv1x1 store", "policy conv -> record"]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "_build", "libgzgn_stamps.so"))
P = ctypes.c_void_p
lib.gz_gn_forward.argtypes = [P, P, ctypes.c_int32, P, P, P, P, P, P]
lib.gz_gn_workspace_bytes.restype = ctypes.c_size_t
lib.gz_gn_workspace_bytes.argtypes = [ctypes.c_int32]
lib.gz_gn_stamps_read.argtypes = [P, ctypes.c_int]
blob = torch.from_numpy(planner_nets.pack_planner_weights(planner_nets.init_graphnet_state(0),
                                                          planner_nets.init_dqn_state(1))).cuda()
rng = np.random.default_rng(0)
cells = rng.choice(3, size=(n, 225), p=[0.5, 0.25, 0.25]).astype(np.int8)
bl, wh = boards.cells_to_words(cells)
d_b = torch.from_numpy(boards.leaf_words(bl, wh).view(np.int32).copy()).cuda()
p = torch.empty(n * 225, device="cuda")
q = torch.empty(n * 225, device="cuda")
ws = torch.empty(lib.gz_gn_workspace_bytes(n), dtype=torch.uint8, device="cuda")
out = np.zeros(32, np.uint64)
for it in range(2):
    lib.gz_gn_stamps_read(out.ctypes.data, 1)
    assert lib.gz_gn_forward(blob.data_ptr(), d_b.data_ptr(), n, None, p.data_ptr(), q.data_ptr(), None, ws.data_ptr(), None) == 0
    torch.cuda.synchronize()
lib.gz_gn_stamps_read(out.ctypes.data, 0)
nb = (n + 511) // 512
tot = sum(int(x) for x in out[:8])
print(f"gn_kernel workgroup 0: {nb} boards, {tot / nb:.0f} ticks/board")
for i, name in enumerate(PHASES):
    print(f"  {name:18s} {int(out[i]) / nb:9.0f}  {int(out[i]) / tot * 100:5.1f}%")
