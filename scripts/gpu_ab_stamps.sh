#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_ab.sh || exit 3
bash scripts/gpu_stamps_hot.sh || exit 3
