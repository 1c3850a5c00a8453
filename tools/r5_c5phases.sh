#!/bin/bash
# config 5 kernel trace with the host phases: the GPU's idle time per phase
set -o pipefail
mkdir -p gpurun_out/r5c5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GZ_PHASES=gpurun_out/r5c5/phases.json timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5c5/trace -o run -- python3 tools/c5_trace.py 512 2 > gpurun_out/r5c5/run.log 2>&1 || { tail -20 gpurun_out/r5c5/run.log; exit 1; }
grep '^{' gpurun_out/r5c5/run.log
python3 tools/gap_phases.py gpurun_out/r5c5/trace gpurun_out/r5c5/phases.json > gpurun_out/r5c5/gap_phases.json || exit 1
rm -rf gpurun_out/r5c5/trace
