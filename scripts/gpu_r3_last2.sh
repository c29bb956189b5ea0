#!/bin/bash
# Round 3 last call: smoke + the driver's exact bench command, then the tower
# build variants (scripts/ab_tower.py, B 4096).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r3_last.sh || exit 3
AB_B=4096 timeout -k 10 300 python scripts/ab_tower.py > gpurun_out/ab_tower_last.json 2> gpurun_out/ab_tower_last.err || { tail -5 gpurun_out/ab_tower_last.err; exit 4; }
cat gpurun_out/ab_tower_last.json
echo DONE
