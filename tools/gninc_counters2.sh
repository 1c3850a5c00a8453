#!/bin/bash
# gn_inc_kernel: gninc_bench rate + three --pmc passes (kernel-trace only), summarised on the
# box (the per-dispatch CSVs are deleted).  usage: tools/gninc_counters2.sh <outdir>
set -e
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
timeout -k 10 240 python3 tools/gninc_bench.py > "$out/bench.txt" 2>&1
run() { k=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out/p$k" -o run -- python3 tools/gninc_bench.py > "$out/p$k.txt" 2>&1; }
run 1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run 2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE
run 3 SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE
python3 tools/pv_counters_sum.py "$out" gn_inc_kernel > "$out/summary.txt"
rm -f "$out"/p*/run_counter_collection.csv
