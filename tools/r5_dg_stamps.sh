#!/bin/bash
# phase stamps of pv_dg_kernel (tools/_build/libgzero_dg2x2.so), two and one workgroups per CU
set -o pipefail
mkdir -p gpurun_out/r5s
GZ_LIBRARY=tools/_build/libgzero_dg2x2.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 3 --check 0 > gpurun_out/r5s/stamps.log 2>&1 || exit $?
GZ_PVDG_WPS=1 GZ_LIBRARY=tools/_build/libgzero_dg2x2.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 3 --check 0 > gpurun_out/r5s/stamps_wps1.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5s/stamps.log; grep -v amdgpu.ids gpurun_out/r5s/stamps_wps1.log
