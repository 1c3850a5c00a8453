#!/bin/bash
# config 5 (512 games, 2 iterations) with the gn_inc chunks sized to the launch (0) and fixed at 3 boards
set -o pipefail
mkdir -p gpurun_out/r5hd
for r in 1 2; do
for cap in 1 0; do
  GZ_GN_HEADS_SPLIT=$cap timeout -k 10 300 python -u tools/c5_trace.py 512 2 > gpurun_out/r5hd/split_${cap}_$r.log 2>&1 || { tail -20 gpurun_out/r5hd/split_${cap}_$r.log; exit 1; }
  echo "cap $cap rep $r $(grep '^{' gpurun_out/r5hd/split_${cap}_$r.log)"
done
done
