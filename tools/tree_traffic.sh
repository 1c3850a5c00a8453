#!/bin/bash
# HBM-side bytes of the tree forward alone (tools/pvinc_bench.py, one timed launch set):
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (kernel-trace only).
# usage: tools/tree_traffic.sh <outdir> [pvinc_bench args]
set -e
export TMPDIR=/tmp
out=$1; shift
mkdir -p "$out"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 tools/pvinc_bench.py --iters 2 --check 0 "$@" > "$out/fetch.txt" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 tools/pvinc_bench.py --iters 2 --check 0 "$@" > "$out/write.txt" 2>&1
echo collected
