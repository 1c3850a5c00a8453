#!/bin/bash
# same-box A/B of pv_dg_kernel variants (tools/_build/libgzero_<v>.so), interleaved, each
# checked against the full forward (--check 1); then the stamps of the variants named in
# $STAMPS (libgzero_<v>.so built with -DGZ_PVDG_STAMPS) at two and one workgroups per CU
# usage: [STAMPS="v1st ..."] tools/r6_ab.sh <reps> v1 v2 ...
set -o pipefail
reps=$1; shift
out=gpurun_out/r6ab
mkdir -p $out
for r in $(seq 1 $reps); do
  for v in "$@"; do
    GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 5 --check ${GZ_AB_CHECK:-1} > $out/${v}_$r.log 2>&1 || { echo "$v failed"; tail -5 $out/${v}_$r.log; exit 1; }
    echo "$v rep $r: $(grep -h 'ms per launch\|max |diff|' $out/${v}_$r.log | tr '\n' ' ')"
  done
done
for v in $STAMPS; do
  GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 3 --check 0 > $out/${v}_st2.log 2>&1 || exit $?
  GZ_PVDG_WPS=1 GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 3 --check 0 > $out/${v}_st1.log 2>&1 || exit $?
  echo "== $v stamps (2 / 1 workgroups per CU)"; grep -h "ticks per node\|k-loop\|epilogue" $out/${v}_st2.log $out/${v}_st1.log
done
