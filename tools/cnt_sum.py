#!/usr/bin/env python3
"""Per-kernel counter sums (median dispatch) from tools/r5_dgcnt.sh output dirs."""
import csv, glob, re, statistics, sys, collections
for d in sys.argv[1:]:
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = (r["Dispatch_Id"], r["Kernel_Name"][:40])
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    byk = collections.defaultdict(list)
    for (i, name), c in per.items():
        if "pv_dg" in name:
            byk[name].append((dur[(i, name)], c))
    for name, lst in byk.items():
        lst.sort(key=lambda x: x[0])
        ms, c = lst[len(lst) // 2]
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        print(f"{d}: {name} {ms:.2f} ms  LDS_IDX_ACTIVE/cyc {c['SQ_LDS_IDX_ACTIVE'] / cyc / 256:.3f} per CU  "
              f"BANK_CONFLICT/IDX {c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_LDS_IDX_ACTIVE']):.3f}  "
              f"MFMA busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f}  "
              f"WAIT_INST_LDS/WAVE {c['SQ_WAIT_INST_LDS'] / c['SQ_WAVE_CYCLES']:.3f}  "
              f"WAIT_ANY/WAVE {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}  "
              f"ACTIVE/WAVE {c['SQ_ACTIVE_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}  INSTS_LDS {c['SQ_INSTS_LDS']:.3g}")
