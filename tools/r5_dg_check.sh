#!/bin/bash
# tree-forward parity tests + pv_dg_kernel timing (tools/pvinc_bench.py) on the current build,
# then the phase stamps (tools/_build/libgzero_dgstamps.so)
set -o pipefail
mkdir -p gpurun_out/r5c
timeout -k 10 400 python -u -m pytest tests/test_gpu_pvdelta.py tests/test_gpu_pvinc.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5c/tests.log 2>&1 || { echo "tests rc $?"; tail -30 gpurun_out/r5c/tests.log; exit 1; }
tail -2 gpurun_out/r5c/tests.log
timeout -k 10 200 python -u tools/pvinc_bench.py --iters 5 --check 1 > gpurun_out/r5c/pvinc.log 2>&1 || { cat gpurun_out/r5c/pvinc.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r5c/pvinc.log
if [ "$1" = stamps ]; then
  GZ_LIBRARY=tools/_build/libgzero_dgstamps.so timeout -k 10 200 python -u tools/pvinc_bench.py --iters 3 --check 0 > gpurun_out/r5c/stamps.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r5c/stamps.log | tail -n 16
fi
