set -o pipefail
mkdir -p gpurun_out/w4
timeout -k 10 500 python -u -m pytest tests/test_gpu_pvinc.py tests/test_gpu_pvnet.py tests/test_gpu_selfplay.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w4/t2.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/w4/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py --config5-games 0 --fp32-steps 0 > gpurun_out/w4/bench.json 2> gpurun_out/w4/bench.err
