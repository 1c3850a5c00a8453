set -o pipefail
mkdir -p gpurun_out/r5e
GZ_LIBRARY=tools/_build/libgzero_dgstamps.so timeout -k 10 300 python -u tools/pvinc_bench.py --mode delta --iters 3 --check 0 > gpurun_out/r5e/stamps_v1.log 2>&1 || exit $?
GZ_PVDG_VARIANT=1 timeout -k 10 900 bash tools/pvdg_counters.sh gpurun_out/r5e/ctr > gpurun_out/r5e/ctr.log 2>&1
