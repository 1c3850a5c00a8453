# config-4 kernel trace (3 timed ply-steps) -> per-kernel stats + GPU idle gaps,
# e.g. after plan_resume_kernel (the planner search's per-round host synchronisation)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${1:-c4gaps}
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --planner-steps 5 --beta 0.2 --steps 3 --warmup 1 --no-cpu-baseline --config4-steps 0 --fp32-steps 0 --no-elided --config5-games 0 > $out/bench.json 2> $out/bench.err &&
python3 tools/trace_gaps.py $out/trace plan_resume_kernel plan_collect_kernel gn_heads_kernel > $out/gaps.json &&
rm -f $out/trace/*/run_kernel_trace.csv $out/trace/run_kernel_trace.csv
