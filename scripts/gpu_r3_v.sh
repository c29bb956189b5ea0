#!/bin/bash
# Round 3: the sort's parity tests on the product build, then same-box timing
# of the sort variants and hipCUB (scripts/ab_sort.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_v.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_v.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_v.log; exit $rc; }
timeout -k 10 300 python scripts/ab_sort.py > gpurun_out/ab_sort.jsonl 2> gpurun_out/ab_sort.err; rc=$?
cat gpurun_out/ab_sort.jsonl; [ $rc -eq 0 ] || { grep -v "^frame" gpurun_out/ab_sort.err | tail -8; exit $rc; }
echo DONE
