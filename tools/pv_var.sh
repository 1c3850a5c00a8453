set -o pipefail
# tree-forward variants: tests on each, then a same-box A/B: bash tools/pv_var.sh base.so var1.so var2.so ...
mkdir -p gpurun_out/pvvar
base=$1; shift
for v in "$@"; do
  GZ_LIBRARY=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_gpu_pvinc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pvvar/t_$(basename $v).log 2>&1 || exit 1
done
REPS=3 bash tools/ab.sh "python tools/pvinc_bench.py --check 0" $base "$@" > gpurun_out/pvvar/ab.log 2>&1
