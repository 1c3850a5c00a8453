#!/bin/bash
# Instruction mix / occupancy / HBM bytes of the self-play search kernel (prior-elided
# run of tools/search_bench.py), one --pmc pass per counter group, kernel-trace only.
# usage: tools/search_counters.sh <outdir>
set -e
export TMPDIR=/tmp
out=$1
mkdir -p "$out"
cmd="python3 tools/search_bench.py --warmup 40 --plies 20"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- $cmd > "$out/trace.txt" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$out/p1" -o run -- $cmd > "$out/p1.txt" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d "$out/p2" -o run -- $cmd > "$out/p2.txt" 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/p3" -o run -- $cmd > "$out/p3.txt" 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/p4" -o run -- $cmd > "$out/p4.txt" 2>&1
echo done
