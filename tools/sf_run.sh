set -o pipefail
mkdir -p gpurun_out/sibfill
timeout -k 10 500 python -u -m pytest tests/test_gpu_pvinc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sibfill/t.log 2>&1 &&
bash tools/ab.sh "python tools/pvinc_bench.py --check 0" "$@" > gpurun_out/sibfill/ab.log 2>&1
