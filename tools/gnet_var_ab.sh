# A/B of gn_inc_kernel variants built into tools/_build/var/lib<V>.so (GZ_LIBRARY):
# gninc_bench at 8192 and 49152 rows, 3 interleaved rounds
set -o pipefail
out=gpurun_out/${1:-gnvar}
shift
mkdir -p $out
for r in 1 2 3; do
  for v in "$@"; do
    GZ_LIBRARY=tools/_build/var/lib$v.so timeout -k 10 120 python tools/gninc_bench.py --bases 8192 >> $out/$v.txt 2>&1 || exit 1
    GZ_LIBRARY=tools/_build/var/lib$v.so timeout -k 10 120 python tools/gninc_bench.py --bases 49152 >> $out/$v.txt 2>&1 || exit 1
  done
done
