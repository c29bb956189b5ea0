#!/bin/bash
# GPU tests (stop on fault) then timeline diagnostics.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc: stop"; exit $rc; }
for v in 1e4 1e7; do
  DIAG_V=$v timeout -k 10 120 python scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids || { echo "diag rc fail"; exit 3; }
done
DIAG_V=1e7 DIAG_B=65536 timeout -k 10 120 python scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids || exit 3
echo DONE
