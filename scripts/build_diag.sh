#!/bin/bash
# Diagnostic build of the fused gather+FM kernel with s_memrealtime phase
# stamps (RS_DIAG_STAMPS).  Output: recommender_system_amd/librs_hip_diag.so
# (never loaded by the product path).
set -e
cd "$(dirname "$0")/.."
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DRS_DIAG_STAMPS -I include -I recommender_system_amd/csrc \
  recommender_system_amd/csrc/embed_fm.hip recommender_system_amd/csrc/embed_fm_tiles.hip recommender_system_amd/csrc/mlp.hip recommender_system_amd/csrc/capi.cpp \
  -o recommender_system_amd/librs_hip_diag.so
