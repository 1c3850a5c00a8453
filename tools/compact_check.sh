# bounded-game self-play with slot compaction: its GPU tests, the config-5 training
# tests and a bench run with config 5 (run on the GPU box from the repo root)
set -o pipefail
out=gpurun_out/${1:-compact}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_selfplay.py tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-elided --config4-steps 0 > $out/bench_c5.json 2> $out/bench_c5.err
