#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run: per-kernel durations from the
rocprofv3 kernel trace and per-launch HBM-side bytes from the separate
FETCH_SIZE / WRITE_SIZE passes.

Bytes: rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md
(HBM section) FETCH_SIZE reads 1/2 of the bytes of a WIDE (16 B/lane) coalesced
stream on gfx950; the PV kernel's weight loads are 4 B/lane and the self-play
kernel's accesses are mixed, i.e. uncalibrated widths, so the raw counter is
reported (corrected = raw, flagged) rather than guessing a factor.

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
    timed = v[-steps:] if k.startswith("pv_kernel") else v
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
PV = next((k for k in durs if k.startswith("pv_kernel")), "pv_kernel")
for k in (PV, "selfplay_kernel"):
    if k in fetch and k in write:
        f = fetch[k][-steps:] if k == PV else fetch[k]
        w = write[k][-steps:] if k == PV else write[k]
        summary["kernels"].setdefault(k, {})["hbm_bytes_per_launch"] = {
            "fetch_raw": sum(f) / len(f) * 1024, "write": sum(w) / len(w) * 1024,
            "total_raw": (sum(f) / len(f) + sum(w) / len(w)) * 1024,
            "note": "FETCH_SIZE+WRITE_SIZE KiB x 1024; access widths uncalibrated -> raw"}
pv = summary["kernels"].get(PV, {})
boards = bench["config"]["pv_boards_per_step"]
if "hbm_bytes_per_launch" in pv:
    tb = pv["hbm_bytes_per_launch"]["total_raw"]
    json.dump({"bytes_per_launch": tb, "boards_per_launch": boards, "bytes_per_board": tb / boards,
               "algorithmic_bytes_per_board": 64 + 225 * 4 * 2 + 4,
               "source": src}, open(os.path.join(os.path.dirname(dst.rstrip("/")), "pv_traffic.json"), "w"), indent=1)
json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
for f in ("trace/run_kernel_stats.csv", "pmc_fetch/run_counter_collection.csv",
          "pmc_write/run_counter_collection.csv", "bench_trace.json"):
    p = os.path.join(src, f)
    if os.path.exists(p):
        shutil.copy(p, os.path.join(dst, f.replace("/", "_")))
print(json.dumps(summary, indent=1))
