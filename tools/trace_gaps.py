#!/usr/bin/env python3
"""Idle time of the GPU in a rocprofv3 kernel trace: the span from the first kernel
start to the last kernel end, the union of kernel intervals, and the gaps between
consecutive kernels -- in total, over 20 us, and after a named kernel (e.g. the
planner search's per-round host synchronisation follows plan_resume_kernel).
usage: trace_gaps.py <trace dir> [kernel substring ...]"""
import csv
import glob
import json
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = []
for r in csv.DictReader(open(f)):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
rows.sort()
span = rows[-1][1] - rows[0][0]
busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
gaps = []
for s, e, name in rows[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, name))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
after = {}
for k in sys.argv[2:]:
    tot, n = 0, 0
    for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
        if k in n0 and s1 > e0:
            tot += s1 - e0
            n += 1
    after[k] = {"gaps": n, "total_ms": round(tot / 1e6, 3), "mean_us": round(tot / max(1, n) / 1e3, 2)}
big = [g for g, _ in gaps if g > 20000]
# the kernels on either side of the gaps over 20 us
pairs = {}
for (s0, e0, n0), (s1, e1, n1) in zip(rows, rows[1:]):
    if s1 - e0 > 20000:
        k = (n0.split("(")[0][-40:], n1.split("(")[0][-40:])
        c = pairs.setdefault(k, [0, 0])
        c[0] += 1
        c[1] += s1 - e0
top_pairs = sorted(pairs.items(), key=lambda kv: -kv[1][1])[:8]
print(json.dumps({"kernels": len(rows), "span_ms": round(span / 1e6, 3), "busy_ms": round(busy / 1e6, 3),
                  "idle_ms": round((span - busy) / 1e6, 3), "gaps": len(gaps),
                  "gaps_over_20us": len(big), "gaps_over_20us_ms": round(sum(big) / 1e6, 3),
                  "after": after,
                  "big_gaps_between": [{"before": k[0], "after": k[1], "count": v[0], "total_ms": round(v[1] / 1e6, 3)}
                                       for k, v in top_pairs]}, indent=1))
