#!/bin/bash
# alternating planner-step counters: planner / self-play / arena / API / GraphNet tests, then config 5 A/B vs the previous library
set -o pipefail
mkdir -p gpurun_out/r5ct
timeout -k 10 900 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_selfplay.py tests/test_gpu_arena.py tests/test_gpu_api.py tests/test_gpu_gnet.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ct/tests.log 2>&1 || { tail -30 gpurun_out/r5ct/tests.log; exit 1; }
tail -1 gpurun_out/r5ct/tests.log
for r in 1 2; do
  for v in new old; do
    lib=alphazero-gomoku_amd/gzero/libgzero.so; [ $v = old ] && lib=tools/_build/libgzero_planold.so
    GZ_LIBRARY=$lib timeout -k 10 300 python -u tools/c5_trace.py 512 2 > gpurun_out/r5ct/c5_${v}_$r.log 2>&1 || { tail -20 gpurun_out/r5ct/c5_${v}_$r.log; exit 1; }
    echo "$v rep $r $(grep '^{' gpurun_out/r5ct/c5_${v}_$r.log)"
  done
done
