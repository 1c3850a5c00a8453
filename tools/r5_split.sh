#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5hd
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnet.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5hd/tests_split.log 2>&1 || { tail -30 gpurun_out/r5hd/tests_split.log; exit 1; }
tail -1 gpurun_out/r5hd/tests_split.log
bash tools/r5_split_ab.sh
