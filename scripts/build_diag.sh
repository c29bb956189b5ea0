#!/bin/bash
# Diagnostic build of the whole library with the per-wave phase stamps compiled
# in (RS_DIAG_STAMPS: the FM body's s_memrealtime stamps, the towers' and the
# fused DeepFM's MLP_STAMP, DIN / CrossNet / inner-product stamps).  Output:
# recommender_system_amd/librs_hip_diag.so (never loaded by the product path;
# the stamp scripts point _lib at it).  Objects are kept in
# recommender_system_amd/build_diag/ and recompiled only when their source or
# a header is newer.
set -e
cd "$(dirname "$0")/.."
O=recommender_system_amd/build_diag
mkdir -p $O
HDR=$(ls -t recommender_system_amd/csrc/*.hpp include/*.h scripts/build_diag.sh | head -1)
for src in recommender_system_amd/csrc/*.hip recommender_system_amd/csrc/*.cpp; do
  obj=$O/$(basename $src).o
  if [ ! -f $obj ] || [ $src -nt $obj ] || [ $HDR -nt $obj ]; then echo $src; fi
done | xargs -r -P 8 -I{} sh -c \
  'hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -DRS_DIAG_STAMPS -I include -I recommender_system_amd/csrc -c {} -o '"$O"'/$(basename {}).o'
hipcc --offload-arch=gfx950 -shared -fPIC -o recommender_system_amd/librs_hip_diag.so $O/*.o
