#!/bin/bash
# round 6 baseline: tree forward (product library) with the full-forward check, then the
# stamps build at two and one workgroups per CU
set -o pipefail
mkdir -p gpurun_out/r6base
timeout -k 10 240 python -u tools/pvinc_bench.py --iters 5 --check 1 > gpurun_out/r6base/prod.log 2>&1 || { tail -20 gpurun_out/r6base/prod.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r6base/prod.log
GZ_LIBRARY=tools/_build/libgzero_basest.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 3 --check 0 > gpurun_out/r6base/st2.log 2>&1 || exit $?
GZ_PVDG_WPS=1 GZ_LIBRARY=tools/_build/libgzero_basest.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 3 --check 0 > gpurun_out/r6base/st1.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r6base/st2.log; grep -v amdgpu.ids gpurun_out/r6base/st1.log
