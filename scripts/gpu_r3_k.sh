#!/bin/bash
# Round 3: phase stamps of the dedup route's hash kernel (Zipf / uniform ids).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/diag_dedup_stamps.py > gpurun_out/dd_stamps.jsonl 2> gpurun_out/dd_stamps.err || { tail gpurun_out/dd_stamps.err; exit 3; }
DD_UNIFORM=1 timeout -k 10 120 python scripts/diag_dedup_stamps.py >> gpurun_out/dd_stamps.jsonl 2>> gpurun_out/dd_stamps.err || { tail gpurun_out/dd_stamps.err; exit 3; }
cat gpurun_out/dd_stamps.jsonl
timeout -k 10 400 python -u -m pytest tests/test_sharded_gloo.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_k.log | tail -80; exit $rc; }
timeout -k 10 300 python scripts/prof_dedup.py > gpurun_out/prof_dedup.json 2> gpurun_out/prof_dedup.err || { tail gpurun_out/prof_dedup.err; exit 4; }
cat gpurun_out/prof_dedup.json
