#!/bin/bash
# Round 3: the whole GPU suite, then the config-5 bench at N = 1 with the Zipf
# dedup line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_f.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_f.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_f.log | tail -60; exit $rc; }
timeout -k 10 400 python bench.py --sharded --steps 64 --warmup 5 --no-cpu-baseline > gpurun_out/bench_sharded.json 2> gpurun_out/bench_sharded.err || { tail gpurun_out/bench_sharded.err; exit 4; }
python -c "
import json; d=json.load(open('gpurun_out/bench_sharded.json'))
print('sharded', d['ms_per_step'], d['value_kind'], d['pipelined']['ms_per_step'], d['per_batch']['ms_per_step'])
print('zipf', json.dumps(d['zipf_ids']))"
