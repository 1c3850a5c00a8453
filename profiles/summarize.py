#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run: per-kernel durations from the
rocprofv3 kernel trace and per-launch HBM-side bytes from the separate
FETCH_SIZE / WRITE_SIZE passes.

Bytes: rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md
(HBM section) FETCH_SIZE reads 1/2 of the bytes of a wide (16 B/lane) coalesced
stream on gfx950 and other widths must be calibrated on a known byte count:
tools/hbm_calib.hip streams 1 GiB through each width the PV forward uses
(profiles/r01/hbm_calib.json): FETCH_SIZE = 0.500 x bytes for 4-B AND 16-B
coalesced loads, WRITE_SIZE = 1.000 x bytes for 4-B and 16-B stores.  So
corrected bytes = 2 x FETCH_SIZE + WRITE_SIZE (the raw sum is kept beside it).

The PV forward (one gz_pv_forward) is two kernels for f16x3: pv_kernel_f16x3
(tower) and pv_heads_kernel (batched FC heads); both are summed as "pv_forward".

Usage: python profiles/summarize.py gpurun_out/prof_r01 profiles/r01
"""
import csv
import json
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
trace = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0].split("<")[0].split("::")[-1]


durs = {}
for r in trace:
    durs.setdefault(short(r["Kernel_Name"]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)

bench = json.load(open(os.path.join(src, "bench_trace.json")))
steps = bench["steps"]
summary = {"bench": {k: bench[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup")}, "kernels": {}}
for k, v in durs.items():
    # the bench's timed window is the LAST `steps` PV launches (warm-up launches
    # include opening plies with no leaves)
    timed = v[-steps:] if k.startswith("pv_") else v
    summary["kernels"][k] = {"calls": len(v), "avg_ms_all": sum(v) / len(v),
                             "avg_ms_timed_window": sum(timed) / len(timed), "max_ms": max(v)}


def pmc(name, counter):
    rows = list(csv.DictReader(open(os.path.join(src, name, "run_counter_collection.csv"))))
    out = {}
    for r in rows:
        if r["Counter_Name"] == counter:
            out.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return out


fetch = pmc("pmc_fetch", "FETCH_SIZE")
write = pmc("pmc_write", "WRITE_SIZE")
PVK = [k for k in durs if k.startswith("pv_")]
for k in PVK + ["selfplay_kernel"]:
    if k in fetch and k in write:
        f = fetch[k][-steps:] if k in PVK else fetch[k]
        w = write[k][-steps:] if k in PVK else write[k]
        summary["kernels"].setdefault(k, {})["hbm_bytes_per_launch"] = {
            "fetch_raw": sum(f) / len(f) * 1024, "write": sum(w) / len(w) * 1024,
            "total_raw": (sum(f) / len(f) + sum(w) / len(w)) * 1024,
            "total": (2 * sum(f) / len(f) + sum(w) / len(w)) * 1024,
            "note": "total = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), calibrated by tools/hbm_calib.hip"}
boards = bench["config"]["pv_boards_per_step"]
pvf = {"kernels": PVK,
       "avg_ms_timed_window": sum(summary["kernels"][k]["avg_ms_timed_window"] for k in PVK)}
if PVK and all("hbm_bytes_per_launch" in summary["kernels"][k] for k in PVK):
    tb = sum(summary["kernels"][k]["hbm_bytes_per_launch"]["total"] for k in PVK)
    pvf["hbm_bytes_per_launch"] = tb
    json.dump({"bytes_per_launch": tb, "boards_per_launch": boards, "bytes_per_board": tb / boards,
               "algorithmic_bytes_per_board": 64 + 225 * 4 * 2 + 4,
               "note": ("2 x FETCH_SIZE + WRITE_SIZE (tools/hbm_calib.hip calibration); f16x3: includes the "
                        "tower -> heads record (2,816 B written and read per board)"),
               "kernels": PVK, "source": src},
              open(os.path.join(os.path.dirname(dst.rstrip("/")), "pv_traffic.json"), "w"), indent=1)
summary["pv_forward"] = pvf
json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
for f in ("trace/run_kernel_stats.csv", "pmc_fetch/run_counter_collection.csv",
          "pmc_write/run_counter_collection.csv", "bench_trace.json"):
    p = os.path.join(src, f)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, f.replace("/", "_")))
print(json.dumps(summary, indent=1))
