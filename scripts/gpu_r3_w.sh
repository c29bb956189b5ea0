#!/bin/bash
# Round 3: sort parity + the tower tests with both contraction forms, then the
# sort variants vs hipCUB and the unrolled-tower option A/B (DeepFM, DCN).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sort.py tests/test_gpu_kernels.py -x -q -k "sort or sum or tower or deepfm_fused or dcn_fused" --timeout 120 --timeout-method thread > gpurun_out/pytest_w.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_w.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_w.log; exit $rc; }
timeout -k 10 300 python scripts/ab_sort.py > gpurun_out/ab_sort_w.jsonl 2> gpurun_out/ab_sort_w.err; rc=$?
cat gpurun_out/ab_sort_w.jsonl; [ $rc -eq 0 ] || { grep -v "^frame" gpurun_out/ab_sort_w.err | tail -8; exit $rc; }
for wl in deepfm dcn; do
  timeout -k 10 300 python scripts/ab_options.py --option mlp_unroll --workload $wl > gpurun_out/ab_unroll_$wl.json 2> gpurun_out/ab_unroll_$wl.err || { tail -5 gpurun_out/ab_unroll_$wl.err; exit 5; }
  cat gpurun_out/ab_unroll_$wl.json
done
echo DONE
