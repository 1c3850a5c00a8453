#!/bin/bash
# config 4 with the 4-wave planner ply for every launch size vs the default cap
set -o pipefail
mkdir -p gpurun_out/r5pb
for cap in 4096 100000000 4096; do
  GZ_PLAN_STEP4=$cap timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-elided --config5-games 0 --config4-steps 6 > gpurun_out/r5pb/c4_$cap.json 2> gpurun_out/r5pb/c4_$cap.err || { tail -20 gpurun_out/r5pb/c4_$cap.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r5pb/c4_$cap.json').read().strip().splitlines()[-1]); print('cap $cap config4', d['config4']['value'], d['config4']['ms_per_step'])"
done
