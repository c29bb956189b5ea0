#!/bin/bash
# A/B(/C) builds of the headline kernel: $1 = source of variant A (default:
# HEAD's embed_fm.hip), the working tree's embed_fm.hip as B (extra hipcc
# flags for B in $BFLAGS, for A in $AFLAGS) and, when $CFLAGS is set, the
# working tree again with those flags as C.  Output: scripts/ab/librs_ab_{A,B,C}.so
# (diagnostics only; never loaded by the product).
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/ab
rm -f scripts/ab/librs_ab_*.so
A=${1:-}
if [ -z "$A" ]; then A=$(mktemp -d)/embed_fm.hip; git show HEAD:recommender_system_amd/csrc/embed_fm.hip > "$A"; fi
C=recommender_system_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include -I $C"
hipcc $F ${AFLAGS:-} "$A" $C/embed_fm_tiles.hip $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_ab_A.so &
hipcc $F ${BFLAGS:-} $C/embed_fm.hip $C/embed_fm_tiles.hip $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_ab_B.so &
if [ -n "${CFLAGS:-}" ]; then
  hipcc $F $CFLAGS $C/embed_fm.hip $C/embed_fm_tiles.hip $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_ab_C.so &
fi
wait
