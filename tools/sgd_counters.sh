#!/bin/bash
# Counters of the device training step's kernels (csrc/gz_sgd.hip), one --pmc pass each,
# kernel-trace only.  usage: tools/sgd_counters.sh <outdir>
set -e
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
run() { k=$1; shift; timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv -d "$out/p$k" -o run -- python3 tools/sgd_bench.py native > "$out/p$k.txt" 2>&1; }
run 1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
run 3 SQ_INSTS_VALU_MFMA_F16 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE
echo collected
for k in sgd_conv_kernel\<0 sgd_conv_kernel\<1 sgd_wgrad16 sgd_conv0_kernel sgd_heads_bwd; do
  echo "== $k"; python3 tools/pv_counters_sum.py "$out" "$k"
done > "$out/summary.txt"
rm -f "$out"/p*/run_counter_collection.csv
