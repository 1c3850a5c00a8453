#!/bin/bash
# config 5 kernel trace: per-kernel totals and the GPU's idle time (the raw trace is deleted)
set -o pipefail
mkdir -p gpurun_out/r6c5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6c5/trace -o run -- python3 tools/c5_trace.py 512 1 > gpurun_out/r6c5/run.log 2>&1 || { tail -20 gpurun_out/r6c5/run.log; exit 1; }
grep '^{' gpurun_out/r6c5/run.log
python3 tools/trace_gaps.py gpurun_out/r6c5/trace plan_resume_kernel gn_inc_kernel > gpurun_out/r6c5/gaps.json || exit 1
python3 tools/kdur_hist.py gpurun_out/r6c5/trace gn_inc_kernel gn_heads_kernel plan_step_kernel plan_collect plan_resume gn_kernel pv_dg_kernel > gpurun_out/r6c5/hist.json && cp $(find gpurun_out/r6c5/trace -name '*kernel_stats.csv' | head -1) gpurun_out/r6c5/kernel_stats.csv
rm -rf gpurun_out/r6c5/trace
head -c 1200 gpurun_out/r6c5/gaps.json
