#!/usr/bin/env python3
"""Per-kernel duration histogram of a rocprofv3 kernel trace (small vs large launches):
usage: kdur_hist.py <trace dir> [substring ...]"""
import csv
import glob
import json
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
edges = [20, 50, 100, 200, 500, 1000, 5000, 1e12]
out = {}
for r in csv.DictReader(open(f)):
    name = r["Kernel_Name"]
    keys = [k for k in sys.argv[2:] if k in name]
    if not keys:
        continue
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    h = out.setdefault(keys[0], {f"<{e:g}us": [0, 0.0] for e in edges})
    for e in edges:
        if d < e:
            h[f"<{e:g}us"][0] += 1
            h[f"<{e:g}us"][1] += d / 1e3
            break
for k, h in out.items():
    for b in h:
        h[b][1] = round(h[b][1], 1)
print(json.dumps(out, indent=1))
