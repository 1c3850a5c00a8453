set -o pipefail
mkdir -p gpurun_out/r5g
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pvdelta.py -s > gpurun_out/r5g/tests.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/pvinc_bench.py --mode both --iters 5 --check 1 > gpurun_out/r5g/pvinc.log 2>&1 || exit $?
GZ_LIBRARY=tools/_build/libgzero_dgstamps.so timeout -k 10 300 python -u tools/pvinc_bench.py --mode delta --iters 3 --check 0 > gpurun_out/r5g/stamps.log 2>&1
