#!/bin/bash
# gn_inc_kernel: timing (product lib) and phase stamps (tools/_build/libgzgn_stamps.so)
set -o pipefail
mkdir -p gpurun_out/r5gn
for b in 8192 49152; do
  timeout -k 10 200 python -u tools/gninc_bench.py --bases $b > gpurun_out/r5gn/t_$b.log 2>&1 || { tail -5 gpurun_out/r5gn/t_$b.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/r5gn/t_$b.log
done
timeout -k 10 200 python -u tools/gninc_bench.py --bases 49152 --stamps > gpurun_out/r5gn/stamps.log 2>&1 || { tail -5 gpurun_out/r5gn/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5gn/stamps.log
