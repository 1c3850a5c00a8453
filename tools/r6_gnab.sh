#!/bin/bash
# same-box A/B of gn_inc_kernel variants (tools/_build/libgzgn_<v>.so) with tools/gninc_bench.py
# usage: tools/r6_gnab.sh <reps> v1 v2 ...
set -o pipefail
reps=$1; shift
out=gpurun_out/r6gn
mkdir -p $out
for r in $(seq 1 $reps); do
  for v in "$@"; do
    for b in 8192 49152; do
      timeout -k 10 120 python -u tools/gninc_bench.py --bases $b --lib tools/_build/libgzgn_$v.so > $out/${v}_${b}_$r.txt 2>&1 || { echo "$v failed"; tail -5 $out/${v}_${b}_$r.txt; exit 1; }
      echo "$v $b rep $r: $(grep -h 'rows/s\|ms' $out/${v}_${b}_$r.txt | tail -2 | tr '\n' ' ')"
    done
  done
done
