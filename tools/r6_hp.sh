#!/bin/bash
# the pv_dg_kernel chunk queue: GPU PV-net tests (outputs vs the reference fixtures / the oracle) on the
# product library, then the tree-forward A/B (tools/_build/libgzero_hbase.so vs hnew)
set -o pipefail
mkdir -p gpurun_out/hp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pvnet.py tests/test_gpu_pvinc.py tests/test_gpu_pvdelta.py -x -q --timeout 300 --timeout-method thread > gpurun_out/hp/t.log 2>&1 || { tail -30 gpurun_out/hp/t.log; exit 1; }
tail -2 gpurun_out/hp/t.log
bash tools/r6_ab.sh 3 hpbase hp
