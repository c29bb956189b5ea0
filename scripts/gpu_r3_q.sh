#!/bin/bash
# Round 3: host-metadata fused DeepFM: the whole GPU suite; A/B of the
# embed_fm kernarg variants (scripts/ab A: product, B: + B-fragment prefetch,
# C: kernarg metadata at every grid); the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_q.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_q.log | tail -60; exit $rc; }
AB_BATCHES="4096 16384 65536" bash scripts/gpu_ab.sh || exit 3
timeout -k 10 400 python bench.py > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { tail gpurun_out/bench_q.err; exit 4; }
python scripts/fmt_lines.py gpurun_out/bench_q.json
python -c "
import json; d=json.load(open('gpurun_out/bench_q.json')); c=d['config5_n1']; print('config5_n1', c['ms_per_step'], c['roofline']['kernel_ms'])"
