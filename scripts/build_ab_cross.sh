#!/bin/bash
# Build-level A/B of a few kernel sources: the product objects
# (recommender_system_amd/build) with $SRCS (default: cross.hip) recompiled
# under each flag set ($1, $2, ...: "-DX -DY", or "-" for none) into
# scripts/ab/librs_ab_cross_<i>.so (diagnostics only; never the product).
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/ab
C=recommender_system_amd/csrc
SRCS=${SRCS:-cross.hip}
EXCL=$(for s in $SRCS; do printf '%s\n' "/${s%.*}.o"; done)
OBJS=$(ls recommender_system_amd/build/*.o | grep -v -F "$EXCL")
i=0
for flags in "$@"; do
  [ "$flags" = "-" ] && flags=""
  (
    objs=""
    for s in $SRCS; do
      o=/tmp/ab_${i}_${s%.*}.o
      hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function $flags -I include -I $C -c $C/$s -o $o
      objs="$objs $o"
    done
    hipcc --offload-arch=gfx950 -shared -fPIC -o scripts/ab/librs_ab_cross_$i.so $OBJS $objs
  ) &
  i=$((i+1))
done
wait
ls -la scripts/ab/librs_ab_cross_*.so
