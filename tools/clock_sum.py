#!/usr/bin/env python3
"""Per-dispatch effective clock and MFMA busy share from tools/clock_probe.sh output."""
import collections
import csv
import glob
import sys

for d in sorted(glob.glob(sys.argv[1] + "/*/")):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(d + "run_counter_collection.csv")):
        k = (r["Dispatch_Id"], r["Kernel_Name"][:40])
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        per[k]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for (i, name), c in sorted(per.items(), key=lambda x: int(x[0][0])):
        if c["dur"] < 1e-3:
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        print(f"{d.split('/')[-2]:28s} {name:40s} {c['dur']*1e3:7.2f} ms  {cyc / c['dur'] / 1e9:.3f} GHz  "
              f"MFMA busy {c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (cyc * 1024) * 100:5.1f}%")
