set -o pipefail
mkdir -p gpurun_out/r5k
for v in dgstamps pw pl pm; do GZ_PVDG_WPS=1 GZ_LIBRARY=tools/_build/libgzero_$v.so timeout -k 10 200 python -u tools/pvinc_bench.py --mode delta --iters 3 --check 0 > gpurun_out/r5k/$v.log 2>&1 || exit $?; done
