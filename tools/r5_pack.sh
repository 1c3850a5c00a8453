#!/bin/bash
# device weight packer: parity test, then a short bench with config 5 (its self-play repacks per iteration)
set -o pipefail
mkdir -p gpurun_out/r5pk
timeout -k 10 300 python -u -m pytest tests/test_weights_pack.py tests/test_gpu_sgd.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r5pk/tests.log 2>&1 || { tail -30 gpurun_out/r5pk/tests.log; exit 1; }
grep -h "device pack\|passed\|failed" gpurun_out/r5pk/tests.log
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --burn-in 0 --no-cpu-baseline --fp32-steps 0 --no-elided --config4-steps 0 > gpurun_out/r5pk/bench.json 2> gpurun_out/r5pk/bench.err || { tail -20 gpurun_out/r5pk/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r5pk/bench.json').read().strip().splitlines()[-1]); c=d['config5']
print({k: c.get(k) for k in ('value','iteration_s','selfplay_s','sgd_s','sgd_parts_s','first_iteration_s')})"
