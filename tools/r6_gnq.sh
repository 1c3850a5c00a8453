#!/bin/bash
# gn_inc_kernel's chunk queue: the GraphNet / planner GPU tests (bitwise vs the full forward and
# the oracle) on the product library, then gninc_bench and config-4 bench A/B (gqbase vs gq)
set -o pipefail
o=gpurun_out/gnq
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_gpu_gnet.py tests/test_gpu_plan.py -x -q --timeout 400 --timeout-method thread > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -2 $o/t.log
for r in 1 2; do
  for v in gqbase gq; do
    timeout -k 10 200 python -u tools/gninc_bench.py --lib tools/_build/libgzero_$v.so > $o/gn_${v}_$r.log 2>&1 || { echo "$v gninc failed"; tail -5 $o/gn_${v}_$r.log; exit 1; }
    echo "$v gninc rep $r: $(grep -v amdgpu $o/gn_${v}_$r.log | tail -2 | tr '\n' ' ')"
    GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -k 10 400 python -u bench.py --planner-steps 5 --beta 0.2 --steps 8 --warmup 2 --no-cpu-baseline --config4-steps 0 --fp32-steps 0 --no-elided --config5-games 0 > $o/c4_${v}_$r.json 2> $o/c4_${v}_$r.err || { echo "$v bench failed"; tail -5 $o/c4_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$o/c4_${v}_$r.json').read().strip().splitlines()[-1]); print('$v config4 rep $r:', d['value'], d['ms_per_step'])"
  done
done
