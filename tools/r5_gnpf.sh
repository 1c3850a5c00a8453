#!/bin/bash
# gn_inc_kernel next-chunk prefetch: GraphNet / planner tests, then gninc_bench and config 4 A/B
# against the previous kernel (tools/_build/libgzero_gnold.so)
set -o pipefail
mkdir -p gpurun_out/r5pf
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnet.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r5pf/tests.log 2>&1 || { tail -30 gpurun_out/r5pf/tests.log; exit 1; }
tail -1 gpurun_out/r5pf/tests.log
for r in 1 2; do
  for v in old new; do
    lib=alphazero-gomoku_amd/gzero/libgzero.so; [ $v = old ] && lib=tools/_build/libgzero_gnold.so
    timeout -k 10 200 python -u tools/gninc_bench.py --bases 49152 --lib $lib > gpurun_out/r5pf/gi_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r5pf/gi_${v}_$r.log; exit 1; }
    echo "$v rep $r: $(grep -h 'rows/s' gpurun_out/r5pf/gi_${v}_$r.log)"
  done
done
for v in old new; do
  lib=alphazero-gomoku_amd/gzero/libgzero.so; [ $v = old ] && lib=tools/_build/libgzero_gnold.so
  GZ_LIBRARY=$lib timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-elided --config5-games 0 --config4-steps 6 > gpurun_out/r5pf/c4_$v.json 2> gpurun_out/r5pf/c4_$v.err || { tail -20 gpurun_out/r5pf/c4_$v.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r5pf/c4_$v.json').read().strip().splitlines()[-1]); print('$v config4', d['config4']['value'], d['config4']['ms_per_step'])"
done
