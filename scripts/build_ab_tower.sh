#!/bin/bash
# Tower build variants for scripts/ab_tower.py (diagnostics only): groups of
# the weight ring issued ahead in the 16 / 8 / 4-group layers (MLP_SMALL_D):
# A = 2 (the product), B = 1, C = 4.  rs_mlp_fwd only.
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/ab
rm -f scripts/ab/librs_tower_*.so
C=recommender_system_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include -I $C"
hipcc $F $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_tower_A.so &
hipcc $F -DMLP_SMALL_D=1 $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_tower_B.so &
hipcc $F -DMLP_SMALL_D=4 $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_tower_C.so &
wait
