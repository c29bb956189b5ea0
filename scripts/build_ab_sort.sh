#!/bin/bash
# Sort variants for scripts/ab_sort.py (diagnostics only): tile = 256 threads x
# RX_ITEMS pairs (A: 8, the product; D: 4; E: 16); H = the hipCUB radix sort.
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/ab
rm -f scripts/ab/librs_sort_*.so
C=recommender_system_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include -I $C"
hipcc $F -DRX_ITEMS=8 $C/radix_sort.hip $C/capi.cpp -o scripts/ab/librs_sort_A.so &
hipcc $F -DRX_ITEMS=4 $C/radix_sort.hip $C/capi.cpp -o scripts/ab/librs_sort_D.so &
hipcc $F -DRX_ITEMS=16 $C/radix_sort.hip $C/capi.cpp -o scripts/ab/librs_sort_E.so &
hipcc $F scripts/diag_hipcub_sort.hip -o scripts/ab/librs_sort_H.so &
wait
