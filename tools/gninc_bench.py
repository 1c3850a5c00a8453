#!/usr/bin/env python3
"""Microbenchmark of the incremental GraphNet (gn_inc_kernel) through
gz_gn_forward_chain: --bases full-forward boards keep their maps, then rows that
add one random stone to each are timed --iters times.  With the -DGZ_GN_STAMPS build
(tools/_build/libgzgn_stamps.so: make -C tools) also the per-phase cycle split of
workgroup 0.  Usage: python tools/gninc_bench.py [--stamps] [--bases 8192]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "alphazero-gomoku_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gzero import boards, planner_nets  # noqa: E402

TAG = np.dtype([("mode", "<i4"), ("base", "<i4"), ("job", "<i4"), ("cell", "<i4"), ("nst", "<i4"),
                ("st", "u1", (6,)), ("pad", "u1", (2,)), ("pad2", "<i4")])
PH = {8: "unit table", 9: "rows + fill 0 + im2col", 10: "embed", 11: "L0 3x3", 12: "L1 1x1 + fill 1",
      13: "L2 3x3", 14: "L3 1x1 + fill 2", 15: "L4 3x3", 16: "L5 1x1 + fill 3", 17: "L6 3x3", 18: "L7 1x1",
      19: "policy conv", 20: "records"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bases", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--lib", default=None, help="a library to time instead (tools/_build/libgzgn_<var>.so)")
    a = ap.parse_args()
    path = a.lib or (os.path.join(ROOT, "tools", "_build", "libgzgn_stamps.so") if a.stamps else
                     os.path.join(ROOT, "alphazero-gomoku_amd", "gzero", "libgzero.so"))
    lib = ctypes.CDLL(path)
    P = ctypes.c_void_p
    lib.gz_gn_forward_chain.argtypes = [P, P, ctypes.c_int32, P, P, P, P, P, P]
    lib.gz_gn_chain_workspace_bytes.restype = lib.gz_gn_slot_bytes.restype = ctypes.c_size_t
    lib.gz_gn_chain_workspace_bytes.argtypes = [ctypes.c_int32]
    if a.stamps:
        lib.gz_gn_stamps_read.argtypes = [P, ctypes.c_int]
    blob = torch.from_numpy(planner_nets.pack_planner_weights(planner_nets.init_graphnet_state(0),
                                                              planner_nets.init_dqn_state(1))).cuda()
    R = a.bases
    rng = np.random.default_rng(0)
    cells = rng.choice(3, size=(R, 225), p=[0.6, 0.2, 0.2]).astype(np.int8)
    slots = torch.empty(2 * R * lib.gz_gn_slot_bytes(), dtype=torch.uint8, device="cuda")
    ws = torch.empty(lib.gz_gn_chain_workspace_bytes(R), dtype=torch.uint8, device="cuda")
    p = torch.empty(R * 225, device="cuda")
    q = torch.empty(R * 225, device="cuda")

    def run(c, tags):
        bl, wh = boards.cells_to_words(c)
        d_b = torch.from_numpy(boards.leaf_words(bl, wh).view(np.int32).copy()).cuda()
        d_t = torch.from_numpy(tags.view(np.uint8).copy()).cuda()
        return d_b, d_t

    tags = np.zeros(R, TAG)
    tags["mode"], tags["job"] = 0, np.arange(R)
    d_b, d_t = run(cells, tags)
    assert lib.gz_gn_forward_chain(blob.data_ptr(), d_b.data_ptr(), R, d_t.data_ptr(), slots.data_ptr(),
                                   p.data_ptr(), q.data_ptr(), ws.data_ptr(), None) == 0
    inc = cells.copy()
    tags = np.zeros(R, TAG)
    for r in range(R):
        c = int(rng.choice(np.flatnonzero(inc[r] == 0)))
        inc[r][c] = 1
        tags[r]["cell"] = c
    tags["mode"], tags["base"], tags["job"] = 1, np.arange(R), R + np.arange(R)
    d_b, d_t = run(inc, tags)
    stamps = np.zeros(32, np.uint64)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for it in range(a.iters + 1):
        if it == 1:
            if a.stamps:
                lib.gz_gn_stamps_read(stamps.ctypes.data, 1)
            ev[0].record()
        assert lib.gz_gn_forward_chain(blob.data_ptr(), d_b.data_ptr(), R, d_t.data_ptr(), slots.data_ptr(),
                                       p.data_ptr(), q.data_ptr(), ws.data_ptr(), None) == 0
    ev[1].record()
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / a.iters
    print(f"{R} incremental rows: {ms:.3f} ms per call (split + inc + heads), {R / ms / 1e3:.2f} M rows/s")
    if a.stamps:
        lib.gz_gn_stamps_read(stamps.ctypes.data, 0)
        tot = sum(int(stamps[i]) for i in PH)
        for i, name in PH.items():
            print(f"  {name:24s} {int(stamps[i]) / max(1, tot) * 100:5.1f}%")


if __name__ == "__main__":
    main()
