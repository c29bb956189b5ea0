#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for B in 4096 300; do
DIAG_B=$B timeout -k 10 120 python scripts/diag_stamps_hot.py > gpurun_out/stamps_hot_$B.json 2> gpurun_out/stamps_hot.err || { tail gpurun_out/stamps_hot.err; exit 3; }
python scripts/fmt_diag.py < gpurun_out/stamps_hot_$B.json
done
