# device clip + Adam: the SGD / training GPU tests, the trainer step time, a kernel trace
# of it and a config-5 bench (run on the GPU box from the repo root)
set -o pipefail
out=gpurun_out/${1:-adam}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sgd.py tests/test_gpu_train.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1 &&
timeout -k 10 300 python tools/sgd_bench.py native > $out/sgd_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 tools/sgd_bench.py native > $out/sgd_trace.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --fp32-steps 0 --no-elided --config4-steps 0 > $out/bench_c5.json 2> $out/bench_c5.err
