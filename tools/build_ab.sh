#!/bin/bash
# Build an A/B variant of libgym_lorenz_amd.so: lz_kernels.hip recompiled with extra
# defines, linked with the product's other objects (make -C gym-lorenz_amd first).
#   tools/build_ab.sh <name> <hipcc defines...>    e.g. tools/build_ab.sh state_nt -DLZ_STATE_NT=1
# -> ablib/libgym_lorenz_amd_<name>.so (git-ignored; travels to the GPU box; load it with
# LZ_LIB_AB=ablib/libgym_lorenz_amd_<name>.so, e.g. through tools/ab_lib.py)
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/gym-lorenz_amd
mkdir -p $ROOT/ablib $PKG/build_ab
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -Wall -I$ROOT/include -I$PKG/csrc"
# AB_SRC=lz_policy recompiles the policy kernels instead (the other objects from build/)
SRC=${AB_SRC:-lz_kernels}
/opt/rocm/bin/hipcc $FLAGS "$@" -c $PKG/csrc/$SRC.hip -o $PKG/build_ab/${SRC}_$NAME.o
OBJS=""
for o in lz_kernels lz_rms lz_policy lz_wrappers lz_api lz_pack; do
  if [ $o = $SRC ]; then OBJS="$OBJS $PKG/build_ab/${SRC}_$NAME.o"; else OBJS="$OBJS $PKG/build/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/ablib/libgym_lorenz_amd_$NAME.so $OBJS
echo $ROOT/ablib/libgym_lorenz_amd_$NAME.so
