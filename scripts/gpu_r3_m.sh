#!/bin/bash
# Round 3: the headline kernel timed by the A/B harness (A = the product
# library, B = the A/B build of the same source) beside the default bench,
# then the bench under rocprofv3 --kernel-trace --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_BATCHES="4096" bash scripts/gpu_ab.sh || exit 3
timeout -k 10 400 python bench.py --no-config5 > gpurun_out/bench_m.json 2> gpurun_out/bench_m.err || { tail gpurun_out/bench_m.err; exit 4; }
python -c "
import json; d=json.load(open('gpurun_out/bench_m.json')); print('bench', d['ms_per_step'], d['roofline']['kernel_ms'])"
rm -rf gpurun_out/prof_bench
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench -o run -- python3 bench.py > gpurun_out/prof_bench.log 2>&1 || { tail gpurun_out/prof_bench.log; exit 5; }
