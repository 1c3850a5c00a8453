#!/bin/bash
# pending count read every 2 rounds: planner / self-play / arena tests, then config 5 A/B (every 1 vs 2)
set -o pipefail
mkdir -p gpurun_out/r5sy
timeout -k 10 900 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_selfplay.py tests/test_gpu_arena.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5sy/tests.log 2>&1 || { tail -30 gpurun_out/r5sy/tests.log; exit 1; }
tail -1 gpurun_out/r5sy/tests.log
for r in 1 2; do
  for e in 2 1; do
    GZ_PLAN_SYNC_EVERY=$e timeout -k 10 300 python -u tools/c5_trace.py 512 2 > gpurun_out/r5sy/c5_${e}_$r.log 2>&1 || { tail -20 gpurun_out/r5sy/c5_${e}_$r.log; exit 1; }
    echo "every $e rep $r $(grep '^{' gpurun_out/r5sy/c5_${e}_$r.log)"
  done
done
