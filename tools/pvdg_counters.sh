#!/bin/bash
# Kernel trace + counters of the delta tree forward's child kernel (pv_dg_kernel), one
# --pmc pass each.  usage: tools/pvdg_counters.sh <outdir>
set -e
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
args="--iters 2 --check 0 --burn-in 300"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 tools/pvinc_bench.py $args > "$out/trace.txt" 2>&1
run() { k=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out/p$k" -o run -- python3 tools/pvinc_bench.py $args > "$out/p$k.txt" 2>&1; }
run 1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run 2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE
run 3 SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE
echo collected
