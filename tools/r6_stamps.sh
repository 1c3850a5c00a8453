#!/bin/bash
# phase stamps of pv_dg_kernel (tools/_build/libgzero_<v>.so built with -DGZ_PVDG_STAMPS),
# two and one workgroups per CU.  usage: tools/r6_stamps.sh <v>
set -o pipefail
v=${1:-st}
mkdir -p gpurun_out/r6s
GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 3 --check 0 > gpurun_out/r6s/${v}_wps2.log 2>&1 || exit $?
GZ_PVDG_WPS=1 GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 3 --check 0 > gpurun_out/r6s/${v}_wps1.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r6s/${v}_wps2.log; grep -v amdgpu.ids gpurun_out/r6s/${v}_wps1.log
