set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 150 python -u -m pytest -x -v --timeout 100 --timeout-method thread tests/test_gpu_pvdelta.py -s -k every_cell > gpurun_out/r5b/tests1.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pvdelta.py -s > gpurun_out/r5b/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/pvinc_bench.py --mode both --full --iters 5 > gpurun_out/r5b/pvinc.log 2>&1
