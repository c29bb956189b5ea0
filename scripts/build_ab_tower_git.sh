#!/bin/bash
# Tower builds for scripts/ab_tower.py / ab_tower_stamps.py (diagnostics only):
# A = mlp_tower.hpp at git revision $1 (default HEAD), B = the working tree,
# C = the working tree with MLP_SMALL_D 4, D = with MLP_SMALL_D 1.  Each
# compiles mlp.hip beside its copy of the header; outputs scripts/ab/librs_tower_{A..D}.so.
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
mkdir -p scripts/ab
rm -f scripts/ab/librs_tower_*.so
C=recommender_system_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DRS_DIAG_STAMPS -I include"  # (stamps for ab_tower_stamps.py)
T=$(mktemp -d)
for v in A B C D; do mkdir -p $T/$v; cp $C/mlp.hip $C/mlp_tower.hpp $T/$v/; done
git show $REV:$C/mlp_tower.hpp > $T/A/mlp_tower.hpp
sed -i 's/constexpr int MLP_SMALL_D = 2;/constexpr int MLP_SMALL_D = 4;/' $T/C/mlp_tower.hpp
sed -i 's/constexpr int MLP_SMALL_D = 2;/constexpr int MLP_SMALL_D = 1;/' $T/D/mlp_tower.hpp
for v in C D; do ! cmp -s $C/mlp_tower.hpp $T/$v/mlp_tower.hpp || { echo "variant $v: sed matched nothing"; exit 1; }; done
for v in A B C D; do
  hipcc $F -I $T/$v -I $C $T/$v/mlp.hip $C/capi.cpp -o scripts/ab/librs_tower_$v.so &
done
wait
rm -rf $T
