set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_sgd.py tests/test_gpu_train.py -s > gpurun_out/r5a/tests.log 2>&1 || exit $?
GZ_DIST_SAME_DEVICE=1 GZ_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --slots 512 --steps 4 --warmup 1 --burn-in 40 --no-cpu-baseline --config4-steps 0 --config5-games 0 --fp32-steps 0 --no-elided > gpurun_out/r5a/dist2.json 2> gpurun_out/r5a/dist2.err
