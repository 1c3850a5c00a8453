set -o pipefail
mkdir -p gpurun_out/ev3
bash profiles/collect.sh r03b &&
bash tools/ab.sh "python tools/pvinc_bench.py --check 0" $PWD/alphazero-gomoku_amd/gzero/libgzero.so $PWD/tools/_build/libgzero_probe3.so > gpurun_out/ev3/probe3.log 2>&1
