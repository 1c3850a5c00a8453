#!/bin/bash
# after removing the one-kernel small heads: GraphNet / planner tests
set -o pipefail
mkdir -p gpurun_out/r5cl
timeout -k 10 900 python -u -m pytest tests/test_gpu_gnet.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5cl/tests.log 2>&1 || { tail -30 gpurun_out/r5cl/tests.log; exit 1; }
tail -1 gpurun_out/r5cl/tests.log
