#!/bin/bash
# same-box A/B of pv_dg_kernel variants (tools/_build/libgzero_<v>.so), interleaved
# usage: tools/r5_ab.sh <reps> v1 v2 ...
set -o pipefail
reps=$1; shift
mkdir -p gpurun_out/r5ab
for r in $(seq 1 $reps); do
  for v in "$@"; do
    GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 5 --check ${GZ_AB_CHECK:-1} > gpurun_out/r5ab/${v}_$r.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/r5ab/${v}_$r.log; exit 1; }
    echo "$v rep $r: $(grep -h 'ms per launch\|max |diff|' gpurun_out/r5ab/${v}_$r.log | tr '\n' ' ')"
  done
done
