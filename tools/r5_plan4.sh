#!/bin/bash
# plan_step with 4 waves per row for small launches: planner tests, then config 5 A/B
# (new, new with the 1-wave kernel only, the previous library)
set -o pipefail
mkdir -p gpurun_out/r5p4
timeout -k 10 900 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_gnet.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5p4/tests.log 2>&1 || { tail -30 gpurun_out/r5p4/tests.log; exit 1; }
tail -1 gpurun_out/r5p4/tests.log
for r in 1 2; do
  for v in new old; do
    lib=alphazero-gomoku_amd/gzero/libgzero.so; cap=4096
    [ $v = old ] && lib=tools/_build/libgzero_planold.so
    [ $v = one ] && cap=0
    GZ_LIBRARY=$lib GZ_PLAN_STEP4=$cap timeout -k 10 300 python -u tools/c5_trace.py 512 2 > gpurun_out/r5p4/c5_${v}_$r.log 2>&1 || { tail -20 gpurun_out/r5p4/c5_${v}_$r.log; exit 1; }
    echo "$v rep $r $(grep '^{' gpurun_out/r5p4/c5_${v}_$r.log)"
  done
done
