#!/bin/bash
# config 4 with the 4-wave plan_step below 4096 rows (default), below 1024, and the previous library
set -o pipefail
mkdir -p gpurun_out/r5p4
for v in new4096 new1024 old; do
  lib=alphazero-gomoku_amd/gzero/libgzero.so; cap=4096
  [ $v = old ] && lib=tools/_build/libgzero_planold.so
  [ $v = new1024 ] && cap=1024
  GZ_LIBRARY=$lib GZ_PLAN_STEP4=$cap timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-elided --config5-games 0 --config4-steps 6 > gpurun_out/r5p4/c4_$v.json 2> gpurun_out/r5p4/c4_$v.err || { tail -20 gpurun_out/r5p4/c4_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r5p4/c4_$v.json').read().strip().splitlines()[-1]); print('$v config4', d['config4']['value'], d['config4']['ms_per_step'])"
done
