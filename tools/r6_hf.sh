#!/bin/bash
# f16x3 PV heads: the whole GPU suite on the product library, then the tree-forward A/B
set -o pipefail
o=gpurun_out/hf
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1 || { tail -40 $o/t.log; exit 1; }
tail -2 $o/t.log
bash tools/r6_ab.sh 3 hfbase hf
