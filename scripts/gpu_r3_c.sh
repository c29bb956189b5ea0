#!/bin/bash
# Round 3: every GPU test, the rs_embed_fm_fwd variant A/B (B 4096 / 16384), the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_gpu.log | tail -60; exit $rc; }
for B in 4096 16384; do
  timeout -k 10 300 python scripts/ab_options.py --option embed_fm_kernel --values 0,1,2,3 --workload embed_fm --batch $B > gpurun_out/ab_fm_$B.json 2> gpurun_out/ab_fm.err || { tail gpurun_out/ab_fm.err; exit 3; }
  cat gpurun_out/ab_fm_$B.json
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.json
