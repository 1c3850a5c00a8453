#!/bin/bash
# kernel trace of the training-step bench (tools/sgd_bench.py trainer part)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r5sgdprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5sgdprof -o run -- python3 tools/sgd_bench.py native > gpurun_out/r5sgdprof/bench.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5sgdprof/bench.log | tail -4
