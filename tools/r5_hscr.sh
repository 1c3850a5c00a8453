#!/bin/bash
# heads scratch in the caller's workspace: GraphNet / planner / self-play tests, config 5 (2 iterations)
set -o pipefail
mkdir -p gpurun_out/r5hs
timeout -k 10 900 python -u -m pytest tests/test_gpu_gnet.py tests/test_gpu_plan.py tests/test_gpu_selfplay.py tests/test_gpu_arena.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5hs/tests.log 2>&1 || { tail -30 gpurun_out/r5hs/tests.log; exit 1; }
tail -1 gpurun_out/r5hs/tests.log
timeout -k 10 300 python -u tools/c5_trace.py 512 2 > gpurun_out/r5hs/c5.log 2>&1 || { tail -20 gpurun_out/r5hs/c5.log; exit 1; }
grep '^{' gpurun_out/r5hs/c5.log
