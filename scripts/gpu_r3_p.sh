#!/bin/bash
# Round 3: host-metadata headline entry: tests, then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "embed_fm or headline or deepfm" --timeout 300 --timeout-method thread > gpurun_out/pytest_p.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_p.log; [ $rc -eq 0 ] || [ $rc -eq 4 ] || [ $rc -eq 5 ] || { grep -v "^Extension" gpurun_out/pytest_p.log | tail -60; exit $rc; }
timeout -k 10 400 python bench.py --no-config5 > gpurun_out/bench_p.json 2> gpurun_out/bench_p.err || { tail gpurun_out/bench_p.err; exit 4; }
python scripts/fmt_lines.py gpurun_out/bench_p.json
