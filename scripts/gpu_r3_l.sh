#!/bin/bash
# Round 3: the whole GPU suite, the default bench line, the config-5 bench at
# N = 1 with the Zipf lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_l.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_l.log | tail -60; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail gpurun_out/bench_default.err; exit 4; }
timeout -k 10 400 python bench.py --sharded --steps 64 --warmup 5 > gpurun_out/bench_sharded.json 2> gpurun_out/bench_sharded.err || { tail gpurun_out/bench_sharded.err; exit 5; }
python -c "
import json
d=json.load(open('gpurun_out/bench_default.json'))
print('default', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])
c=d.get('config5_n1', {}); print('config5_n1', c.get('ms_per_step'), c.get('value_kind'))
d=json.load(open('gpurun_out/bench_sharded.json'))
print('sharded', d['ms_per_step'], d['config']['value_kind'], d['pipelined']['ms_per_step'], d['per_batch']['ms_per_step'])
print('zipf', json.dumps(d['zipf_ids']))
print('train', json.dumps(d['train_step']))"
