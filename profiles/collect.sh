#!/bin/bash
# Collect the rocprofv3 evidence for one round (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command (per-kernel average durations)
#   2. separate --pmc passes for FETCH_SIZE and WRITE_SIZE (HBM-side bytes)
# Usage: profiles/collect.sh <round-tag> [bench args...]
set -u
tag=${1:-r01}; shift || true
args=${*:-"--steps 8 --warmup 2 --no-cpu-baseline --config4-steps 0 --fp32-steps 0 --no-elided --config5-games 0"}
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args > $out/bench_trace.json 2> $out/bench_trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/pmc_fetch -o run -- python3 bench.py $args > $out/bench_fetch.json 2> $out/bench_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/pmc_write -o run -- python3 bench.py $args > $out/bench_write.json 2> $out/bench_write.err || exit $?
echo collected
