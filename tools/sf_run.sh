set -o pipefail
mkdir -p gpurun_out/sibfill
timeout -k 10 500 python -u -m pytest tests/test_gpu_pvinc.py tests/test_gpu_gnet.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sibfill/t.log 2>&1 &&
bash tools/ab.sh "python tools/pvinc_bench.py --check 0" $PWD/tools/_build/libgzero_fill0.so $PWD/alphazero-gomoku_amd/gzero/libgzero.so > gpurun_out/sibfill/ab.log 2>&1 &&
timeout -k 10 120 python tools/gninc_bench.py --bases 49152 --iters 5 >> gpurun_out/sibfill/ab.log 2>&1
