#!/bin/bash
# kernel validation: trainer / sgd tests, then a short bench with config 5
set -o pipefail
mkdir -p gpurun_out/r5val
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_weights_pack.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r5val/tests.log 2>&1 || { tail -30 gpurun_out/r5val/tests.log; exit 1; }
tail -1 gpurun_out/r5val/tests.log
timeout -k 10 500 python -u bench.py --steps 2 --warmup 1 --burn-in 0 --no-cpu-baseline --fp32-steps 0 --no-elided --config4-steps 0 > gpurun_out/r5val/bench.json 2> gpurun_out/r5val/bench.err || { tail -20 gpurun_out/r5val/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r5val/bench.json').read().strip().splitlines()[-1]); c=d['config5']
print({k: c.get(k) for k in ('value','iteration_s','selfplay_s','sgd_s','sgd_parts_s','first_iteration_s')})"
