# Round-4 evidence, part 2 (after the GPU tests): smoke, the default bench line, the
# rocprof kernel trace + FETCH/WRITE passes of the bench, the config-4 gap trace
set -o pipefail
out=gpurun_out/ev4
mkdir -p $out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err &&
bash profiles/collect.sh r04 &&
bash tools/c4_gaps.sh c4gaps_r04
