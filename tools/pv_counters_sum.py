#!/usr/bin/env python3
"""Summarise tools/pv_counters.sh output: per-dispatch counter means of the PV kernel + derived ratios."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else "pv_kernel"  # kernel-name substring
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if name not in r["Kernel_Name"]:
            continue
        k = r["Counter_Name"]
        agg[(os.path.basename(os.path.dirname(f)), k)] += float(r["Counter_Value"])
        disp[os.path.basename(os.path.dirname(f))].add(r["Dispatch_Id"])
c = {}
for (p, k), v in agg.items():
    c[k] = v / max(1, len(disp[p]))
for k in sorted(c):
    print(f"{k:32s} {c[k]:.4g}")
cu, simd = 256, 1024
g = c.get("GRBM_GUI_ACTIVE", 0) / 8  # summed over 8 XCDs
if g:
    print(f"kernel cycles (GRBM/XCD)         {g:.4g}")
    print(f"MFMA util                        {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (g * simd) * 100:.1f}%")
    print(f"LDS util                         {c['SQ_LDS_IDX_ACTIVE'] / (g * cu) * 100:.1f}%")
    print(f"LDS bank-conflict share          {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE'] * 100:.1f}%")
w = c.get("SQ_WAVE_CYCLES", 0)
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
        if k in c:
            print(f"{k:32s} {c[k] / w * 100:.1f}% of wave cycles")
