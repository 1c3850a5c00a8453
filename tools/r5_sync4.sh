#!/bin/bash
# pending count read every 2 rounds: planner / self-play / arena tests, then config 5 A/B (every 1 vs 2)
set -o pipefail
mkdir -p gpurun_out/r5sy4
for r in 1 2; do
  for e in 2 4; do
    GZ_PLAN_SYNC_EVERY=$e timeout -k 10 300 python -u tools/c5_trace.py 512 2 > gpurun_out/r5sy4/c5_${e}_$r.log 2>&1 || { tail -20 gpurun_out/r5sy4/c5_${e}_$r.log; exit 1; }
    echo "every $e rep $r $(grep '^{' gpurun_out/r5sy4/c5_${e}_$r.log)"
  done
done
