#!/bin/bash
# Same-box A/B: tools/ab.sh "<bench cmd>" lib1 lib2 ...  (each lib run twice, interleaved)
cmd=$1; shift
for rep in $(seq ${REPS:-2}); do
  for lib in "$@"; do
    echo -n "$(basename $lib): "
    GZ_LIBRARY=$lib timeout -k 10 120 $cmd 2>/dev/null | tail -2 | tr "\n" " "; echo || exit 1
  done
done
