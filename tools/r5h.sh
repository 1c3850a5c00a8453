set -o pipefail
mkdir -p gpurun_out/r5h
GZ_PVDG_WPS=1 GZ_LIBRARY=tools/_build/libgzero_dgstamps.so timeout -k 10 300 python -u tools/pvinc_bench.py --mode delta --iters 3 --check 0 > gpurun_out/r5h/stamps_wps1.log 2>&1
