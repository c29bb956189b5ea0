#!/bin/bash
# A/B build of the headline kernel: $1 = source of variant A (default: HEAD's
# embed_fm.hip), the working tree's embed_fm.hip as B (extra hipcc flags for B
# in $BFLAGS, for A in $AFLAGS).  Output: scripts/ab/librs_ab_{A,B}.so
# (diagnostics only; never loaded by the product).
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/ab
A=${1:-}
if [ -z "$A" ]; then A=$(mktemp -d)/embed_fm.hip; git show HEAD:recommender_system_amd/csrc/embed_fm.hip > "$A"; fi
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -I include -I recommender_system_amd/csrc"
hipcc $F ${AFLAGS:-} "$A" recommender_system_amd/csrc/capi.cpp -o scripts/ab/librs_ab_A.so &
hipcc $F ${BFLAGS:-} recommender_system_amd/csrc/embed_fm.hip recommender_system_amd/csrc/capi.cpp -o scripts/ab/librs_ab_B.so &
wait
