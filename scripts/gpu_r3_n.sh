#!/bin/bash
# Round 3: embed_fm tests after the waves-per-tile schedule, then the whole suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "embed_fm" --timeout 300 --timeout-method thread > gpurun_out/pytest_n1.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_n1.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_n1.log | tail -60; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_n2.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_n2.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_n2.log | tail -60; exit $rc; }
