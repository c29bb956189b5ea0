#!/bin/bash
# Build-level A/B on one box: scripts/ab_options.py (one process per library,
# libraries alternated, $ROUNDS rounds) for each workload in $WORKLOADS.
# Usage: LIBS="scripts/ab/libA.so scripts/ab/libB.so" WORKLOADS="deepfm mlp" bash scripts/ab_libs.sh > out.jsonl
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
for wl in ${WORKLOADS:-deepfm}; do
  for r in $(seq 1 ${ROUNDS:-3}); do
    for lib in $LIBS; do
      timeout -k 10 120 python3 "$R/scripts/ab_options.py" --option mlp_unroll --values 1 --workload $wl \
        --lib "$R/$lib" --rounds 6 --save "/tmp/ab_$(basename $lib)_$wl.pt"
    done
  done
done
