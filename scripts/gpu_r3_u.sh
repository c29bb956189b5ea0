#!/bin/bash
# Round 3: the GPU suite and the training lines after the sort's launch fusion
# (one histogram launch + one scatter launch per 8-bit pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_u.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_u.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_u.log | tail -60; exit $rc; }
timeout -k 10 300 python bench.py --config fm_train --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_fm_train_u.json 2> gpurun_out/bench_fm_train_u.err || { tail gpurun_out/bench_fm_train_u.err; exit 4; }
python scripts/fmt_lines.py gpurun_out/bench_fm_train_u.json
echo DONE
