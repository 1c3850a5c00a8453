#!/usr/bin/env python3
"""GPU idle time per host phase: a rocprofv3 kernel trace + tools/c5_trace.py's phase file.
usage: gap_phases.py <trace dir> <phases.json>"""
import csv
import glob
import json
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f)))
gaps = []
cur = rows[0][1]
prev = rows[0][2]
for s, e, n in rows[1:]:
    if s > cur:
        gaps.append((cur, s, prev[-40:], n[:40]))
    if e > cur:
        cur, prev = e, n
phases = json.load(open(sys.argv[2]))
out = []
for label, t0, t1 in phases:
    g = [(b - a) for a, b, _, _ in gaps if a >= t0 and b <= t1]
    big = sorted(((b - a), p, n) for a, b, p, n in gaps if a >= t0 and b <= t1)[-5:]
    busy = sum(min(e, t1) - max(s, t0) for s, e, _ in rows if e > t0 and s < t1)
    out.append({"phase": label, "wall_ms": (t1 - t0) / 1e6, "kernel_ms": busy / 1e6, "idle_ms": sum(g) / 1e6,
                "gaps": len(g), "gaps_over_20us_ms": sum(x for x in g if x > 20000) / 1e6,
                "largest": [(round(d / 1e6, 2), p, n) for d, p, n in big[::-1]]})
print(json.dumps(out, indent=1))
