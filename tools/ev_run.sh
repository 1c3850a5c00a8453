set -o pipefail
mkdir -p gpurun_out/ev8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ev8/tests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev8/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/ev8/bench.json 2> gpurun_out/ev8/bench.err
