#!/bin/bash
# config 4 with the small-launch heads at the default cap, off, and below 1024 rows only
set -o pipefail
mkdir -p gpurun_out/r5hd
for r in 1; do
for cap in -1 100000000; do
  GZ_GN_SMALL_HEADS=$cap timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-elided --config5-games 0 --config4-steps 6 > gpurun_out/r5hd/ab_${cap}_$r.json 2> gpurun_out/r5hd/ab_${cap}_$r.err || { tail -20 gpurun_out/r5hd/ab_${cap}_$r.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r5hd/ab_${cap}_$r.json').read().strip().splitlines()[-1]); print('cap $cap rep $r config4', d['config4']['value'], d['config4']['ms_per_step'])"
done
done
for cap in -1 100000000; do
  GZ_GN_SMALL_HEADS=$cap timeout -k 10 300 python -u tools/c5_trace.py 512 2 > gpurun_out/r5hd/c5cap_${cap}.log 2>&1 || { tail -20 gpurun_out/r5hd/c5cap_${cap}.log; exit 1; }
  echo "config5 cap $cap $(grep '^{' gpurun_out/r5hd/c5cap_${cap}.log)"
done
