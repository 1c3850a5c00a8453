#!/bin/bash
# training-step convolutions in position halves: the SGD GPU tests on the new library, then the trainer A/B and kernel times
set -o pipefail
o=gpurun_out/sph
mkdir -p $o
GZ_LIBRARY=tools/_build/libgzero_sph.so timeout -k 10 500 python -u -m pytest tests/test_gpu_sgd.py tests/test_gpu_train.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -2 $o/t.log
bash tools/r6_sgdab.sh 2 sphbase sph && bash tools/r6_sgdk.sh sphbase sph
