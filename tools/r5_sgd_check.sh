#!/bin/bash
# SGD tests (device FC heads + loss, NetStep) and the training-step bench
set -o pipefail
mkdir -p gpurun_out/r5sgd
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgd.py tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5sgd/tests.log 2>&1 || { echo "tests rc $?"; tail -40 gpurun_out/r5sgd/tests.log; exit 1; }
tail -3 gpurun_out/r5sgd/tests.log
timeout -k 10 300 python -u tools/sgd_bench.py > gpurun_out/r5sgd/sgd_bench.log 2>&1 || { tail -20 gpurun_out/r5sgd/sgd_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5sgd/sgd_bench.log | tail -8
