#!/bin/bash
# small-launch heads: gnet / plan tests, then config 5 and config 4 (short)
set -o pipefail
mkdir -p gpurun_out/r5hd
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnet.py tests/test_gpu_plan.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5hd/tests.log 2>&1 || { tail -30 gpurun_out/r5hd/tests.log; exit 1; }
tail -1 gpurun_out/r5hd/tests.log
timeout -k 10 300 python -u tools/c5_trace.py 512 2 > gpurun_out/r5hd/c5.log 2>&1 || { tail -20 gpurun_out/r5hd/c5.log; exit 1; }
grep '^{' gpurun_out/r5hd/c5.log
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-elided --config5-games 0 --config4-steps 8 > gpurun_out/r5hd/bench.json 2> gpurun_out/r5hd/bench.err || { tail -20 gpurun_out/r5hd/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r5hd/bench.json').read().strip().splitlines()[-1]); print('headline', d['value'], 'config4', d['config4']['value'], d['config4']['ms_per_step'])"
