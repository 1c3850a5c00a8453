#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 --stats csv directory."""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
for r in list(csv.DictReader(open(f)))[:n]:
    print(r["Name"][:64].ljust(64), r["Calls"].rjust(7), "%10.1f ms" % (float(r["TotalDurationNs"]) / 1e6),
          ("%5.1f%%" % float(r["Percentage"])), "avg %.3f ms" % (float(r["AverageNs"]) / 1e6))
