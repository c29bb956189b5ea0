#!/bin/bash
# GPU parity tests (stop on fault), then the phase timeline at B=4096.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { echo "pytest rc=$rc: stop"; grep -v "^Extension" gpurun_out/pytest_gpu.log | tail -30; exit $rc; }
for v in ${DIAG_VS:-1e4 1e7}; do
  DIAG_V=$v timeout -k 10 120 python scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids || { echo "diag failed"; exit 3; }
done
[ -n "${SWEEP:-}" ] && { SWEEP_ROWS=260000000 timeout -k 10 300 python scripts/sweep_embed_fm.py --quick 2>&1 | grep -v amdgpu.ids || exit 3; }
timeout -k 10 120 python scripts/diag_launch.py 2>&1 | grep -v amdgpu.ids | head -2
echo DONE
