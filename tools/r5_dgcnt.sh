#!/bin/bash
# SQ counters of the tree forward per library variant (one --pmc pass each, kernel trace only)
# usage: tools/r5_dgcnt.sh v1 v2 ...
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r5cnt
mkdir -p $out
for v in "$@"; do
  GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $out/$v -o run -- python3 tools/pvinc_bench.py --iters 2 --check 0 --burn-in 300 > $out/$v.txt 2>&1 || { echo "$v rc $?"; tail -5 $out/$v.txt; exit 1; }
  echo "$v done"
done
