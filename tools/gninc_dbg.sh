set -o pipefail
mkdir -p gpurun_out/gninc
timeout -k 10 300 python -u -m pytest tests/test_gpu_gnet.py -x -v --timeout 120 --timeout-method thread -k chains > gpurun_out/gninc/dbg_gnet.log 2>&1
echo done
