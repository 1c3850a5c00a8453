#!/bin/bash
# (1) the f16x3 FULL forward (no incremental tree) at the bench size beside the exact-fp32 full
#     forward: the like-for-like precision comparison; (2) a 4-rank self-launched rehearsal of
#     bench.py --gpus 4 (gloo, all ranks on this one GPU)
set -o pipefail
o=gpurun_out/r6x
mkdir -p $o
timeout -k 10 600 python -u bench.py --pv-mode full --steps 6 --warmup 2 --no-cpu-baseline --config4-steps 0 --no-elided --config5-games 0 > $o/full_f16x3.json 2> $o/full_f16x3.err || { tail -20 $o/full_f16x3.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$o/full_f16x3.json').read().strip().splitlines()[-1]); print('full f16x3', d['value'], d['ms_per_step'], d['config'].get('pv_mode'), 'fp32', d['fp32']['value'], d['fp32']['ms_per_step'])"
GZ_DIST_SAME_DEVICE=1 GZ_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 4 --slots 512 --steps 6 --warmup 2 --burn-in 200 > $o/dist4.json 2> $o/dist4.err || { echo "dist4 rc $?"; tail -20 $o/dist4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$o/dist4.json').read().strip().splitlines()[-1]); print('dist4', d['value'], d['n_gpus'], d['distributed']['backend'], d['distributed']['world_size'], d.get('record_exchange'))"
