#!/bin/bash
# same-box A/B of training-step variants: tools/sgd_bench.py native per library
# (tools/_build/libgzero_<v>.so, "prod" = the product library), interleaved.
# usage: tools/r6_sgdab.sh <reps> v1 v2 ...
set -o pipefail
reps=$1; shift
out=gpurun_out/r6sgdab
mkdir -p $out
for r in $(seq 1 $reps); do
  for v in "$@"; do
    lib=tools/_build/libgzero_$v.so; [ "$v" = prod ] && lib=alphazero-gomoku_amd/gzero/libgzero.so
    GZ_LIBRARY=$lib timeout -k 10 300 python -u tools/sgd_bench.py native > $out/${v}_$r.log 2>&1 || { echo "$v failed"; tail -5 $out/${v}_$r.log; exit 1; }
    echo "$v rep $r: $(grep -h 'ms/step' $out/${v}_$r.log | tr '\n' ' ')"
  done
done
