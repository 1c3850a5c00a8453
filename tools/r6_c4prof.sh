#!/bin/bash
# config 4 kernel trace (3 planner ply-steps after the burn-in): per-kernel totals and idle time; the raw trace is deleted
set -o pipefail
mkdir -p gpurun_out/r6c4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6c4/trace -o run -- python3 bench.py --planner-steps 5 --beta 0.2 --steps 3 --warmup 1 --no-cpu-baseline --config4-steps 0 --fp32-steps 0 --no-elided --config5-games 0 > gpurun_out/r6c4/bench.json 2> gpurun_out/r6c4/bench.err || { tail -20 gpurun_out/r6c4/bench.err; exit 1; }
python3 tools/kdur_hist.py gpurun_out/r6c4/trace gn_inc_kernel gn_heads gn_hn plan_step pv_dg_kernel pv_sib_kernel gn_kernel plan_resume > gpurun_out/r6c4/hist.json || exit 1
cp $(find gpurun_out/r6c4/trace -name '*kernel_stats.csv' | head -1) gpurun_out/r6c4/kernel_stats.csv
rm -rf gpurun_out/r6c4/trace
python3 -c "
import json; d=json.loads(open('gpurun_out/r6c4/bench.json').read().strip().splitlines()[-1]); print('planner bench', d['value'], d['ms_per_step'])"
