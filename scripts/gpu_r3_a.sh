#!/bin/bash
# Round 3: GPU parity (all -m gpu tests), MLP dataflow hand-off A/B, headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_gpu.log | tail -40; exit $rc; }
timeout -k 10 300 python scripts/ab_options.py --option mlp_flow --workload deepfm > gpurun_out/ab_flow_deepfm.json 2> gpurun_out/ab_flow.err || { tail gpurun_out/ab_flow.err; exit 3; }
cat gpurun_out/ab_flow_deepfm.json
timeout -k 10 300 python scripts/ab_options.py --option mlp_flow --workload dcn > gpurun_out/ab_flow_dcn.json 2>> gpurun_out/ab_flow.err || { tail gpurun_out/ab_flow.err; exit 3; }
cat gpurun_out/ab_flow_dcn.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 4; }
cat gpurun_out/bench.json
