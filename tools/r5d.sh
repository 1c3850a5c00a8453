set -o pipefail
mkdir -p gpurun_out/r5d
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pvdelta.py -s > gpurun_out/r5d/tests.log 2>&1 || exit $?
for v in 1 0 1 0; do GZ_PVDG_VARIANT=$v timeout -k 10 200 python -u tools/pvinc_bench.py --mode delta --iters 5 --check 1 > gpurun_out/r5d/pvinc_v$v.log 2>&1 || exit $?; cat gpurun_out/r5d/pvinc_v$v.log; done
