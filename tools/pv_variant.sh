#!/bin/bash
# Rebuild only the PV objects of a full-library variant (tools/Makefile `variant`):
#   tools/pv_variant.sh NAME "-DFLAG ..."  -> tools/_build/libgzero_NAME.so
# (the other objects must exist: run `make -C tools variant VAR=NAME EXTRA=...` once)
set -e
cd "$(dirname "$0")"
V=$1; X=$2
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function $X -ffp-contract=off"
C=../alphazero-gomoku_amd/csrc
$H -c $C/gz_pvnet.hip -o _build/$V/b.o &
$H -mllvm -amdgpu-mfma-vgpr-form -c $C/gz_pvinc.hip -o _build/$V/f.o
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o _build/libgzero_$V.so _build/$V/*.o
