# same-box A/B of planner-net variants on tools/gninc_bench.py: bash tools/ab_gn.sh lib1 lib2 ...
mkdir -p gpurun_out/gninc
for rep in 1 2; do
for lib in "$@"; do
  echo -n "$lib: " >> gpurun_out/gninc/ab.log
  timeout -k 10 120 python tools/gninc_bench.py --bases 49152 --iters 5 --lib $PWD/$lib 2>/dev/null | tail -n 1 >> gpurun_out/gninc/ab.log || exit 1
done
done
