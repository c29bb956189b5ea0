#!/bin/bash
# Headline-kernel timeline: stamps (1e7 rows), ablation, launch regime.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DIAG_V=1e7 timeout -k 10 120 python scripts/diag_stamps.py > gpurun_out/stamps.json 2> gpurun_out/stamps.err || { tail gpurun_out/stamps.err; exit 3; }
python scripts/fmt_diag.py < gpurun_out/stamps.json
timeout -k 10 300 python scripts/diag_ablate.py > gpurun_out/ablate.txt 2>&1 || { tail gpurun_out/ablate.txt; exit 3; }
cat gpurun_out/ablate.txt
timeout -k 10 200 python scripts/diag_launch.py > gpurun_out/launch.txt 2>&1 || { tail gpurun_out/launch.txt; exit 3; }
cat gpurun_out/launch.txt
echo DONE
