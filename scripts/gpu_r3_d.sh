#!/bin/bash
# Round 3: sharded pipelined forward tests, the config-5 bench at N = 1, the
# default bench line, and the headline kernel's stamp timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sharded_gloo.py tests/test_train.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_d.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_d.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_d.log | tail -60; exit $rc; }
timeout -k 10 400 python bench.py --sharded --steps 64 --warmup 5 --no-cpu-baseline > gpurun_out/bench_sharded.json 2> gpurun_out/bench_sharded.err || { tail gpurun_out/bench_sharded.err; exit 4; }
python -c "
import json; d=json.load(open('gpurun_out/bench_sharded.json'))
print('sharded', d['ms_per_step'], d.get('pipelined'), d.get('per_batch'), d['exchange'].get('exchange_ms_per_step_unpipelined'), d['roofline']['kernel_ms'])"
for B in 4096 16384; do DIAG_B=$B DIAG_POOL=64 timeout -k 10 200 python scripts/diag_stamps.py >> gpurun_out/stamps.jsonl 2>> gpurun_out/stamps.err || exit 5; done
cat gpurun_out/stamps.jsonl
