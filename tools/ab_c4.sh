# same-box A/B of config 4 (main bench line with planner plies): bash tools/ab_c4.sh lib1 lib2 ...
mkdir -p gpurun_out/abc4
for rep in 1 2; do
for lib in "$@"; do
  echo -n "$(basename $lib): " >> gpurun_out/abc4/ab.log
  GZ_LIBRARY=$lib timeout -k 10 300 python bench.py --planner-steps 5 --beta 0.2 --steps 4 --warmup 1 --burn-in 300 --no-cpu-baseline --config4-steps 0 --fp32-steps 0 --no-elided --config5-games 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" >> gpurun_out/abc4/ab.log || exit 1
done
done
