#!/bin/bash
# Round 3: parity of the rs_embed_fm_fwd kernel variants, then their A/B timing
# at the headline shape (B 4096) and at B 16384.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -k "variant or headline or embed_fm" > gpurun_out/pytest_variants.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_variants.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_variants.log | tail -60; exit $rc; }
for B in 4096 16384; do
  timeout -k 10 300 python scripts/ab_options.py --option embed_fm_kernel --values 0,1,2,3 --workload embed_fm --batch $B > gpurun_out/ab_fm_$B.json 2> gpurun_out/ab_fm.err || { tail gpurun_out/ab_fm.err; exit 3; }
  cat gpurun_out/ab_fm_$B.json
done
