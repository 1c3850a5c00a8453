#!/bin/bash
# GPU test suite + smoke on the shipped tree mode (round 5)
set -o pipefail
mkdir -p gpurun_out/r5t
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r5t/pytest_gpu.log 2>&1 || { echo "pytest rc $?"; tail -30 gpurun_out/r5t/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r5t/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5t/smoke.log 2>&1 || { echo "smoke rc $?"; tail -20 gpurun_out/r5t/smoke.log; exit 1; }
tail -2 gpurun_out/r5t/smoke.log
