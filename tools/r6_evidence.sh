#!/bin/bash
# Round-6 rocprof evidence on the shipped code: kernel trace + FETCH / WRITE passes of the
# bench (profiles/collect.sh), the clock / MFMA-busy pass of the tree forward, and the
# bench-size tree-forward test with its printed numbers.  usage: tools/r6_evidence.sh <tag>
set -o pipefail
tag=${1:-r06}
bash profiles/collect.sh $tag || exit $?
export TMPDIR=/tmp
out=gpurun_out/clock_$tag
mkdir -p $out
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d $out/tree_product -o run -- python3 tools/pvinc_bench.py --iters 3 --check 0 > $out/tree_product.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_size.py -m gpu -s -q --timeout 280 -p no:cacheprovider > $out/bench_size_test.log 2>&1 || { tail -20 $out/bench_size_test.log; exit 1; }
grep -h "leaves\|max |diff|\|torch fp32\|passed" $out/bench_size_test.log
echo evidence collected
