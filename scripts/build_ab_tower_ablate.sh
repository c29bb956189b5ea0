#!/bin/bash
# Ablation builds of rs_mlp_fwd for scripts/ab_tower.py (diagnostics only; the
# product sources are untouched, each variant compiles mlp.hip beside a
# sed-edited copy of mlp_tower.hpp): A = the product; B = every B-fragment load of a
# contraction reads its first k-group (no streaming of the weights); C = no
# MFMA (one VALU FMA keeps the loads live); D = every A-fragment read hits
# the first k-group's LDS address.  Outputs scripts/ab/librs_tower_{A..D}.so.
set -e
cd "$(dirname "$0")/.."
mkdir -p scripts/ab
rm -f scripts/ab/librs_tower_*.so
C=recommender_system_amd/csrc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DRS_DIAG_STAMPS -I include"  # (stamps for ab_tower_stamps.py)
T=$(mktemp -d)
for v in A B C D; do mkdir -p $T/$v; cp $C/mlp_tower.hpp $C/mlp.hip $T/$v/; done
sed -i 's/ring\[u\] = bp\[(int64_t)min(g + u + D, g1 - 1) \* 64\];/ring[u] = bp[(int64_t)g0 * 64];/' $T/B/mlp_tower.hpp
sed -i 's/acc\.mac4(av, ring\[u\]);/acc.c[0][0] = fmaf(av[0], ring[u][0] + ring[u][1] + ring[u][2] + ring[u][3], acc.c[0][0]);/' $T/C/mlp_tower.hpp
sed -i 's/an = \*reinterpret_cast<const floatx4\*>(ap + 16 \* min(g + u + 1, g1 - 1));/an = *reinterpret_cast<const floatx4*>(ap + 16 * g0);/' $T/D/mlp_tower.hpp
for v in B C D; do ! cmp -s $C/mlp_tower.hpp $T/$v/mlp_tower.hpp || { echo "variant $v: sed matched nothing"; exit 1; }; done
for v in A B C D; do
  hipcc $F -I $T/$v -I $C $T/$v/mlp.hip $C/capi.cpp -o scripts/ab/librs_tower_$v.so &
done
wait
rm -rf $T
