set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c4prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof/trace -o run -- python3 bench.py --planner-steps 5 --beta 0.2 --steps 3 --warmup 1 --no-cpu-baseline --config4-steps 0 --fp32-steps 0 --no-elided --config5-games 0 > gpurun_out/c4prof/bench.json 2> gpurun_out/c4prof/bench.err
rm -f gpurun_out/c4prof/trace/run_kernel_trace.csv.gz
echo done
