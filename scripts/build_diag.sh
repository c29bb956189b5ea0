#!/bin/bash
# Diagnostic build of the whole library with the per-wave phase stamps compiled
# in (RS_DIAG_STAMPS: the FM body's s_memrealtime stamps, the towers' and the
# fused DeepFM's MLP_STAMP).  Output: recommender_system_amd/librs_hip_diag.so
# (never loaded by the product path; the stamp scripts point _lib at it).
set -e
cd "$(dirname "$0")/.."
O=$(mktemp -d)
ls recommender_system_amd/csrc/*.hip recommender_system_amd/csrc/*.cpp | xargs -P 8 -I{} sh -c \
  'hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -DRS_DIAG_STAMPS -I include -I recommender_system_amd/csrc -c {} -o '"$O"'/$(basename {}).o'
hipcc --offload-arch=gfx950 -shared -fPIC -o recommender_system_amd/librs_hip_diag.so "$O"/*.o
rm -rf "$O"
