#!/bin/bash
# A/B(/C/D) timing of the headline kernel builds in scripts/ab (build_ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for B in ${AB_BATCHES:-4096}; do
  DIAG_B=$B timeout -k 10 180 python scripts/ab_embed_fm.py > gpurun_out/ab_$B.json 2> gpurun_out/ab_$B.err || { tail gpurun_out/ab_$B.err; exit 3; }
  echo "B=$B"; cat gpurun_out/ab_$B.json
done
