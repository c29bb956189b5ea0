#!/bin/bash
# Round 3: A/B of the headline kernel's flattened loads (A: HEAD, B: every wave
# issues the dense and second-pass id loads unconditionally), then the final
# profiling session (scripts/gpu_r3_final1.sh) on the working tree's library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_BATCHES="4096 2048" bash scripts/gpu_ab.sh || exit 3
bash scripts/gpu_r3_final1.sh
