#!/bin/bash
# Counters of the incremental forward's kernels (pv_child_kernel et al.), one --pmc
# pass each, kernel-trace only.  usage: tools/pvinc_counters.sh <outdir> [pvinc_bench args]
set -e
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 tools/pvinc_bench.py "$@" > "$out/trace.txt" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$out/p1" -o run -- python3 tools/pvinc_bench.py "$@" > "$out/p1.txt" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE --output-format csv -d "$out/p4" -o run -- python3 tools/pvinc_bench.py "$@" > "$out/p4.txt" 2>&1
echo collected
