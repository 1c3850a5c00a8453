#!/bin/bash
# Round-5 evidence on the shipped code: kernel trace + FETCH / WRITE passes of the
# bench (profiles/collect.sh), then the clock / MFMA-busy pass of the tree forward.
# usage: tools/r5_evidence.sh <tag>
set -o pipefail
tag=${1:-r05}
bash profiles/collect.sh $tag || exit $?
export TMPDIR=/tmp
out=gpurun_out/clock_$tag
mkdir -p $out
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $out/tree_product -o run -- python3 tools/pvinc_bench.py --iters 3 --check 0 > $out/tree_product.txt 2>&1 || exit $?
echo evidence collected
