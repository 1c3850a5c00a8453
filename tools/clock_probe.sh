#!/bin/bash
# Effective shader clock of a kernel per library variant:
# GRBM_GUI_ACTIVE (summed over 8 XCDs) / 8 / kernel duration (same profiled run).
# usage: tools/clock_probe.sh <outdir> <bench: pv|gn|tree> lib1 lib2 ...
set -e
export TMPDIR=/tmp
out=$1; shift
which=$1; shift
mkdir -p "$out"
if [ "$which" = gn ]; then cmd="python3 tools/gn_bench.py --n 131072 --iters 5 --check 0"
elif [ "$which" = tree ]; then cmd="python3 tools/pvinc_bench.py --iters 3 --check 0"
else cmd="python3 tools/pv_bench.py --n 131072 --iters 5 --check 0"; fi
for lib in "$@"; do
  v=$(basename $lib .so)
  GZ_LIBRARY=$lib timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d "$out/${which}_$v" -o run -- $cmd > "$out/${which}_$v.txt" 2>&1
done
