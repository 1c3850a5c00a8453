#!/bin/bash
# same-box A/B of search-kernel variants (tools/search_bench.py, 4096 games, 200 sims), interleaved
# usage: tools/r6_spab.sh <reps> v1 v2 ...
set -o pipefail
out=gpurun_out/r6spab
mkdir -p $out
reps=$1; shift
for r in $(seq 1 $reps); do
  for v in "$@"; do
    GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -k 10 200 python -u tools/search_bench.py --warmup 100 --plies 40 > $out/${v}_$r.log 2>&1 || { echo "$v failed"; tail -5 $out/${v}_$r.log; exit 1; }
    echo "$v rep $r: $(grep -v amdgpu $out/${v}_$r.log | tail -1)"
  done
done
