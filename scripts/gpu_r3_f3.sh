#!/bin/bash
# Round 3: host wait-mode A/B (scripts/gpu_r3_sync.sh), then the final
# profiling session's part 2 (scripts/gpu_r3_final2.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r3_sync.sh || exit 3
bash scripts/gpu_r3_final2.sh
