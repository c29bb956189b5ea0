#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/diag_ablate.py > gpurun_out/ablate.txt 2>&1 || { tail gpurun_out/ablate.txt; exit 3; }
cat gpurun_out/ablate.txt
timeout -k 10 200 python scripts/diag_gather_bw.py > gpurun_out/gbw.txt 2>&1 || { tail gpurun_out/gbw.txt; exit 3; }
cat gpurun_out/gbw.txt
