#!/bin/bash
# Tower build variants for scripts/ab_tower.py (diagnostics only): the weight
# ring depth of the unrolled contraction (A: MLP_RING 4 -> 3 / 2 groups ahead,
# the product; B: MLP_RING 9 -> 9 / 8 / 8 / 4 ahead; C: layers with < 16 output
# tiles split K over the idle waves, MLP_SPLIT_T 16; D: 4 groups ahead in the
# 16 / 8 / 4-group layers, MLP_SMALL_D 4).  rs_mlp_fwd only.
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/ab
rm -f scripts/ab/librs_tower_*.so
C=recommender_system_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include -I $C"
hipcc $F -DMLP_RING=4 $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_tower_A.so &
hipcc $F -DMLP_RING=9 $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_tower_B.so &
hipcc $F -DMLP_SPLIT_T=16 $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_tower_C.so &
hipcc $F -DMLP_SMALL_D=4 $C/mlp.hip $C/capi.cpp -o scripts/ab/librs_tower_D.so &
wait
