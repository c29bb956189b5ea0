#!/bin/bash
# Round 3: tower ring-depth build variants (scripts/ab_tower.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in 4096 65536; do
  AB_B=$b timeout -k 10 300 python scripts/ab_tower.py > gpurun_out/ab_tower_$b.json 2> gpurun_out/ab_tower_$b.err || { tail -5 gpurun_out/ab_tower_$b.err; exit 3; }
  cat gpurun_out/ab_tower_$b.json
done
echo DONE
