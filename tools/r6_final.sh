#!/bin/bash
# Round-6 evidence on the shipped code, one GPU box:
#   1. the GPU test suite (incl. the bench-size tree-forward test) and smoke()
#   2. the default bench line (N = 1)
#   3. the 2-rank rehearsal of the self-launched multi-GPU bench (two ranks on this one
#      GPU, gloo: the code path the driver's 8-GPU run takes, minus RCCL)
# usage: tools/r6_final.sh <tag>
set -o pipefail
tag=${1:-final}
out=gpurun_out/r6_$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $out/pytest_gpu.log 2>&1 || { echo "pytest rc $?"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
grep -h "tree vs full forward\|tree vs torch\|capacity fallbacks" $out/pytest_gpu.log || true
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke rc $?"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
timeout -k 10 900 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench rc $?"; tail -20 $out/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$out/bench.json').read().strip().splitlines()[-1])
print('headline', d['value'], d['ms_per_step'], 'frac', d['roofline']['frac'], 'config4', d['config4']['value'], 'config5', d['config5']['value'], d['config5']['selfplay_s'], d['config5']['sgd_s'])"
GZ_DIST_SAME_DEVICE=1 GZ_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --slots 1024 --steps 6 --warmup 2 \
    --burn-in 200 > $out/dist2.json 2> $out/dist2.err || { echo "dist2 rc $?"; tail -20 $out/dist2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$out/dist2.json').read().strip().splitlines()[-1])
print('dist2', d['value'], d['n_gpus'], d['distributed']['backend'], d['distributed']['world_size'], d.get('record_exchange'))"
