#!/bin/bash
# round-5 closing evidence: GPU test suite + smoke, then the default bench (N = 1)
set -o pipefail
bash tools/r5_gpu_tests.sh || exit $?
mkdir -p gpurun_out/r5f
timeout -k 10 900 python -u bench.py > gpurun_out/r5f/bench.json 2> gpurun_out/r5f/bench.err || { tail -20 gpurun_out/r5f/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r5f/bench.json').read().strip().splitlines()[-1])
print('headline', d['value'], d['ms_per_step'], 'config4', d['config4']['value'], 'config5', d['config5']['value'], d['config5']['selfplay_s'], d['config5']['sgd_s'])"
