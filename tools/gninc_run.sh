set -o pipefail
mkdir -p gpurun_out/gninc
timeout -k 10 900 python -u -m pytest tests/test_gpu_gnet.py tests/test_gpu_plan.py tests/test_gpu_selfplay.py tests/test_gpu_arena.py -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_arena.py::test_arena_with_planner_vs_oracle > gpurun_out/gninc/tests.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-elided --config5-games 0 --config4-steps 8 > gpurun_out/gninc/bench_inc.json 2> gpurun_out/gninc/bench_inc.err
