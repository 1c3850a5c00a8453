# gn_inc_kernel change check: bitwise GraphNet / planner tests, the microbenchmark at two
# sizes, and a short config-4 bench (run on the GPU box from the repo root)
set -o pipefail
out=gpurun_out/${1:-gnab}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnet.py tests/test_gpu_plan.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 120 python tools/gninc_bench.py --bases 8192 > $out/gninc_8k.txt 2>&1 &&
timeout -k 10 120 python tools/gninc_bench.py --bases 49152 > $out/gninc_48k.txt 2>&1 &&
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-elided --config5-games 0 --config4-steps 8 > $out/bench_c4.json 2> $out/bench_c4.err
