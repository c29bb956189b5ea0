#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -m pytest tests -m gpu -q -x > /tmp/pytest_gpu.log 2>&1
rc=$?; tail -2 /tmp/pytest_gpu.log; [ $rc -eq 0 ] || { grep -v "^Extension" /tmp/pytest_gpu.log | tail -30; exit $rc; }
DIAG_V=1e7 timeout -k 10 120 python scripts/diag_stamps.py 2>&1 | grep -v amdgpu.ids || exit 3
timeout -k 10 300 python scripts/diag_gather_bw.py 2>&1 | grep -v amdgpu.ids || exit 3
echo DONE
