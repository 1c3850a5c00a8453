set -o pipefail
# variant check + same-box A/B: bash tools/var_run.sh gn|pv <variant lib> <base lib>
#   gn: planner-net tests on the variant, then config-4 bench A/B (tools/ab_c4.sh)
#   pv: tree-forward tests on the variant, then tools/pvinc_bench.py A/B (tools/ab.sh)
mkdir -p gpurun_out/var
if [ "$1" = gn ]; then
  GZ_LIBRARY=$PWD/$2 timeout -k 10 400 python -u -m pytest tests/test_gpu_gnet.py tests/test_gpu_plan.py -x -q --timeout 200 --timeout-method thread > gpurun_out/var/gn_t.log 2>&1 &&
  bash tools/ab_c4.sh "$3" "$2"
else
  GZ_LIBRARY=$PWD/$2 timeout -k 10 400 python -u -m pytest tests/test_gpu_pvinc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/var/pv_t.log 2>&1 &&
  bash tools/ab.sh "python tools/pvinc_bench.py --check 0" "$3" "$2" > gpurun_out/var/pv_ab.log 2>&1
fi
