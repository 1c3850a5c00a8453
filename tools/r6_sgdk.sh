#!/bin/bash
# per-kernel times of the training step (rocprof kernel trace of tools/sgd_bench.py native) per library variant
# usage: tools/r6_sgdk.sh v1 v2 ...   ("prod" = the product library)
set -o pipefail
export TMPDIR=/tmp
for v in "$@"; do
  lib=tools/_build/libgzero_$v.so; [ "$v" = prod ] && lib=alphazero-gomoku_amd/gzero/libgzero.so
  o=gpurun_out/r6sgdk/$v
  mkdir -p $o
  GZ_LIBRARY=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o -o run -- python3 tools/sgd_bench.py native > $o/bench.log 2>&1 || exit $?
  rm -f $o/run_kernel_trace.csv
  echo "$v: $(grep -h 'trainer native-2nd' $o/bench.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('$o/run_kernel_stats.csv')):
    if 'sgd_' in r['Name'] or 'adam' in r['Name']: print('   ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
"
done
