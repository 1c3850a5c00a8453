#!/usr/bin/env python3
"""Per-dispatch effective clock and MFMA busy share from tools/clock_probe.sh output.

usage: tools/clock_sum.py <outdir> [--json out.json]  (--json: per-kernel medians in
the profiles/rNN/clock.json format bench.py reads)"""
import collections
import csv
import glob
import json
import re
import statistics
import sys


def short(name):
    m = re.search(r"(\w+)(<[^(]*>)?\(", name)
    if m:
        return m.group(1)
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)  # <length><name> after the anonymous namespace
    if m:
        return name[m.end():m.end() + int(m.group(1))]
    return name[:40]


kernels = collections.defaultdict(list)
for d in sorted(glob.glob(sys.argv[1] + "/*/")):
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(d + "run_counter_collection.csv")):
        k = (r["Dispatch_Id"], short(r["Kernel_Name"]))
        per[k][r["Counter_Name"]] = per[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        per[k]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    for (i, name), c in sorted(per.items(), key=lambda x: int(x[0][0])):
        if c["dur"] < 1e-3:
            continue
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        ghz = cyc / c["dur"] / 1e9
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (cyc * 1024)
        print(f"{d.split('/')[-2]:28s} {name:40s} {c['dur']*1e3:7.2f} ms  {ghz:.3f} GHz  MFMA busy {busy * 100:5.1f}%")
        kernels[name].append({"ms": round(c["dur"] * 1e3, 3), "ghz": round(ghz, 3), "mfma_busy": round(busy, 4)})
if "--json" in sys.argv:
    out = {"method": "GRBM_GUI_ACTIVE / 8 XCDs / kernel duration, same rocprofv3 --pmc run (tools/clock_probe.sh, "
                     "tools/clock_sum.py); profiled passes run a few % below unprofiled ones", "nominal_ghz": 2.4,
           "kernels": {k: {"median_ghz": statistics.median(x["ghz"] for x in v),
                           "median_mfma_busy": statistics.median(x["mfma_busy"] for x in v), "dispatches": v}
                       for k, v in kernels.items()}}
    with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
        json.dump(out, f, indent=1)
