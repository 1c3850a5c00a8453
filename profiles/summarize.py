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

The PV forward is several kernels: full mode pv_kernel_f16x3 (tower),
pv_heads_kernel (batched FC heads) and pv_prior_kernel; tree mode adds the list
kernels (tree_*), the second pv_kernel_f16x3 launch and pv_child_kernel.  All are
summed per step as "pv_forward".

Usage: python profiles/summarize.py gpurun_out/prof_r01 profiles/r01
"""
import csv
import json
import os
import re
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
trace = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))))


def _demangle(name):
    """The identifier of an Itanium-mangled kernel in an anonymous namespace
    (_ZN12_GLOBAL__N_1<len><name>...; rocprofv3 leaves template kernels mangled)."""
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)
    if not m:
        return name
    n = int(m.group(1))
    return name[m.end():m.end() + n]


def short(name):
    n = _demangle(name).replace("(anonymous namespace)::", "")
    if n.startswith("void "):
        n = n[5:]
    return n.split("(")[0].split("<")[0].split("::")[-1]


durs = {}
for r in trace:
    durs.setdefault(short(r["Kernel_Name"]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)

bench = json.load(open(os.path.join(src, "bench_trace.json")))
steps = bench["steps"]
pv_steps = steps + bench["warmup"]  # PV forwards: warm-up + timed steps (the burn-in runs none)
summary = {"bench": {k: bench[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup")}, "kernels": {}}
PV_PREFIX = ("pv_", "tree_")  # the PV forward's kernels (tree mode: lists, roots / full tower, children, heads, prior)
mult = {}
for k, v in durs.items():
    # the bench's timed window is the LAST `steps` PV forwards; a kernel launched m
    # times per forward (pv_kernel_f16x3: roots + full lists) is summed per step
    m = max(1, len(v) // pv_steps) if k.startswith(PV_PREFIX) else 1
    mult[k] = m
    timed = v[-steps * m:] if k.startswith(PV_PREFIX) else v
    summary["kernels"][k] = {"calls": len(v), "launches_per_step": m, "avg_ms_all": sum(v) / len(v),
                             "avg_ms_timed_window": sum(timed) / len(timed),
                             "ms_per_step_timed_window": sum(timed) / (steps if k.startswith(PV_PREFIX) else len(v)),
                             "max_ms": max(v)}


def pmc(name, counter):
    rows = list(csv.DictReader(open(os.path.join(src, name, "run_counter_collection.csv"))))
    out = {}
    for r in rows:
        if r["Counter_Name"] == counter:
            out.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return out


fetch = pmc("pmc_fetch", "FETCH_SIZE")
write = pmc("pmc_write", "WRITE_SIZE")
PVK = [k for k in durs if k.startswith(PV_PREFIX)]
for k in PVK + ["selfplay_kernel"]:
    if k in fetch and k in write:
        m = mult.get(k, 1)
        f = fetch[k][-steps * m:] if k in PVK else fetch[k]
        w = write[k][-steps * m:] if k in PVK else write[k]
        per = steps if k in PVK else len(f)  # bytes per step (per PV forward) for the PV kernels
        summary["kernels"].setdefault(k, {})["hbm_bytes_per_step"] = {
            "fetch_raw": sum(f) / per * 1024, "write": sum(w) / per * 1024,
            "total_raw": (sum(f) + sum(w)) / per * 1024,
            "total": (2 * sum(f) + sum(w)) / per * 1024,
            "note": "total = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024), calibrated by tools/hbm_calib.hip"}
boards = bench["config"]["pv_boards_per_step"]
pvf = {"kernels": PVK,
       "ms_per_step_timed_window": sum(summary["kernels"][k]["ms_per_step_timed_window"] for k in PVK)}
if PVK and all("hbm_bytes_per_step" in summary["kernels"][k] for k in PVK):
    tb = sum(summary["kernels"][k]["hbm_bytes_per_step"]["total"] for k in PVK)
    pvf["hbm_bytes_per_launch"] = tb
    json.dump({"bytes_per_launch": tb, "boards_per_launch": boards, "bytes_per_board": tb / boards,
               # board in; logits, softmax and value out; the masked float64 prior out
               "algorithmic_bytes_per_board": 64 + 225 * 4 * 2 + 4 + 225 * 8,
               "pv_mode": bench["config"].get("pv_mode", "full"),
               "note": ("2 x FETCH_SIZE + WRITE_SIZE (tools/hbm_calib.hip calibration), every kernel of one PV "
                        "forward; includes the tower -> heads record (2,816 B written and read per board) and, in "
                        "tree mode, the roots' stored maps, the children's and grandchildren's window reads and "
                        "the parents' patches"),
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
