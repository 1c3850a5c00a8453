#!/bin/bash
# kernel trace of the training-step bench (tools/sgd_bench.py native: the device trainer)
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r6sgd${1:-}
mkdir -p $o
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- python3 tools/sgd_bench.py native > $o/bench.log 2>&1 || exit $?
grep -v amdgpu.ids $o/bench.log | tail -4
