#!/usr/bin/env python3
"""Microbenchmark of the incremental policy-value forward (gz_pv_forward_tree).

Plays --burn-in plies on --slots self-play slots (200 sims, no PV), then one
step with the leaves gathered and tagged, and runs the tree forward (and, with
--full, the full forward) --iters times on those same leaves.  Prints the list
sizes, ms per launch and the bitwise check of the last launch against the full
forward (--check: within 2e-5).  Used with rocprofv3 (--kernel-trace / --pmc) to
isolate pv_dg_kernel / pv_sib_kernel.
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "alphazero-gomoku_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gzero import _lib, weights  # noqa: E402
from gzero.device import PVWeights, ptr, stream  # noqa: E402
from gzero.selfplay import SelfPlayEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, default=4096)
    ap.add_argument("--burn-in", type=int, default=600)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--full", action="store_true", help="also time the full forward")
    ap.add_argument("--check", type=int, default=1)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    w = PVWeights(weights.pack_pv_weights(weights.init_state_dict(0)), precision="f16x3")
    eng = SelfPlayEngine(n_slots=a.slots, num_simulations=200, beta=0.0, seed=1234, pv_weights=w, pv_mode="tree")
    eng.advance(a.burn_in)
    eng.step()
    torch.cuda.synchronize()
    n = int(eng.counters()["leaves"])
    st = eng.tree_stats()
    st_kids = st[2]
    print(f"leaves {n}: roots {st[1]}, children {st[2]}, grandchildren {st[4]} ({st[5]} patches), full {st[3]}",
          flush=True)
    lib = eng.lib
    d_count = eng.d_counters[4:8]

    def tree():
        _lib.check(lib.gz_pv_forward_tree(ptr(w.tensor), ptr(eng.d_leaves), ptr(eng.d_meta), eng.leaf_cap,
                                          ptr(d_count), eng.root_cap, ptr(eng.d_logits), ptr(eng.d_value),
                                          ptr(eng.d_probs), ptr(eng.d_prior), ptr(eng.d_tree_ws), stream()), "tree")

    def timed(fn, label):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        fn()
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(a.iters):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / a.iters
        print(f"{label}: {ms:.3f} ms per launch, {ms * 1e3 / n:.4f} us per board", flush=True)

    stamps = hasattr(lib, "gz_pvinc_stamps_read")
    if stamps:  # -DGZ_PVINC_STAMPS build (make -C tools variant VAR=pistamps EXTRA=-DGZ_PVINC_STAMPS)
        import ctypes
        lib.gz_pvinc_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
        st = np.zeros(34, np.uint64)
    dgst = hasattr(lib, "gz_pvdg_stamps_read")
    if dgst:  # -DGZ_PVDG_STAMPS build (make -C tools variant VAR=dgstamps EXTRA=-DGZ_PVDG_STAMPS)
        import ctypes
        lib.gz_pvdg_stamps_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
        dst = np.zeros(17, np.uint64)
    dg_names = ["chunk start (units, conv0, y1 rows)", "rows of the next pass", "y1 k-loop", "x1 k-loop",
                "y2 k-loop", "x2 k-loop", "barrier after the k-loop", "y1 epilogue", "x1 epilogue", "y2 epilogue",
                "x2 epilogue + heads", "drain + barrier (y1 -> x1, x2)", "fill issue (+ record) + wait",
                "barrier (image landed)"]
    tiles = torch.zeros(2, dtype=torch.int32, device="cuda")
    sib_names = ["select nodes", "window fills (not overlapped)", "conv0", "y1 k-loop", "y1 barrier + next fill",
                 "y1 epilogue", "x1 k-loop", "x1 barrier + next fill", "x1 epilogue", "y2 k-loop",
                 "y2 barrier + next fill", "y2 epilogue", "x2 k-loop", "x2 barrier + next fill",
                 "x2 epilogue + heads", "record"]
    run = tree
    if hasattr(lib, "gz_pvdg_chk_read"):  # -DGZ_DG_CHK build: global accesses outside the workspace
        import ctypes
        lib.gz_pvdg_chk_read.argtypes = [ctypes.c_void_p]
        chk = np.zeros(16, np.uint64)
        tree()
        lib.gz_pvdg_chk_read(chk.ctypes.data)
        print("pv_dg_kernel checks (loads / stores / fills / record r / record w outside the workspace, LDS "
              "fragment reads, row node index, x2 partial index, tables bad at chunk start, stale past the count, bad "
              "cells, tables bad before y1/x1 passes, before y2/x2 passes):", chk.tolist(), flush=True)
    timed(run, "tree")
    torch.cuda.synchronize()
    out = [t[: n * k].clone() for t, k in ((eng.d_logits, 225), (eng.d_value, 1), (eng.d_probs, 225),
                                           (eng.d_prior, 225))]
    _lib.check(lib.gz_pv_tree_exec_tiles(ptr(eng.d_tree_ws), eng.leaf_cap, ptr(tiles), stream()), "tiles")
    t2 = [int(x) for x in tiles.cpu()]
    print(f"  executed 16-row tile-taps: children {t2[0]} ({t2[0] / max(1, st_kids):.1f} per child), "
          f"grandchildren {t2[1]}", flush=True)
    if dgst:
        lib.gz_pvdg_stamps_read(dst.ctypes.data, 1)
        run()
        torch.cuda.synchronize()
        lib.gz_pvdg_stamps_read(dst.ctypes.data, 0)
        kids = max(1, int(dst[16]))
        vals = [int(x) for x in dst[: len(dg_names)]]
        tot = sum(vals)
        print(f"  stamps, workgroup 0 children (pv_dg_kernel): {kids} nodes, {tot / kids:.0f} ticks per node")
        for i, x in enumerate(dg_names):
            print(f"    {x:36s} {vals[i] / kids:9.0f}  {vals[i] / max(1, tot) * 100:5.1f}%")
    if stamps:
        lib.gz_pvinc_stamps_read(st.ctypes.data, 1)
        run()
        torch.cuda.synchronize()
        lib.gz_pvinc_stamps_read(st.ctypes.data, 0)
        gk = max(1, int(st[32]))
        vals = [int(x) for x in st[: len(sib_names)]]
        tot = sum(vals)
        print(f"  stamps, workgroup 0 grandchildren (pv_sib_kernel): {gk} nodes, {tot / gk:.0f} ticks per node")
        for i, x in enumerate(sib_names):
            print(f"    {x:30s} {vals[i] / gk:9.0f}  {vals[i] / max(1, tot) * 100:5.1f}%")
    if a.full or a.check:
        ws = w.workspace_for(eng.leaf_cap)

        def full():
            _lib.check(lib.gz_pv_forward(ptr(w.tensor), ptr(eng.d_leaves), eng.leaf_cap, ptr(d_count),
                                         ptr(eng.d_logits), ptr(eng.d_value), ptr(eng.d_probs), ptr(eng.d_prior),
                                         ptr(ws), w.mode, stream()), "full")
        if a.full:
            timed(full, "full")
        else:
            full()
        torch.cuda.synchronize()
        ref = [t[: n * k] for t, k in ((eng.d_logits, 225), (eng.d_value, 1), (eng.d_probs, 225), (eng.d_prior, 225))]
        err = [float((x.double() - y.double()).abs().max()) for x, y in zip(out, ref)]
        good = err[0] < 2e-5 and err[1] < 2e-5 and err[2] < 1e-6 and err[3] < 1e-6
        print(f"tree: max |diff| vs the full forward: logits {err[0]:.2e} value {err[1]:.2e} "
              f"probs {err[2]:.2e} prior {err[3]:.2e} -> {'ok' if good else 'FAIL'}", flush=True)
        if not good:
            sys.exit(1)

if __name__ == "__main__":
    main()
