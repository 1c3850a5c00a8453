#!/bin/bash
# SQ / LDS counters of the PV kernel (two --pmc passes, kernel-trace only).
# usage: tools/pv_counters.sh <outdir> [pv_bench args...]
set -e
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d "$out/p1" -o run -- python3 tools/pv_bench.py "$@" > "$out/p1.txt" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d "$out/p2" -o run -- python3 tools/pv_bench.py "$@" > "$out/p2.txt" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d "$out/p3" -o run -- python3 tools/pv_bench.py "$@" > "$out/p3.txt" 2>&1 || true
