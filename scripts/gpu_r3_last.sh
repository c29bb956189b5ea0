#!/bin/bash
# Round 3 last check: the driver's exact bench command and smoke on HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_last.log 2>&1
rc=$?; tail -1 gpurun_out/smoke_last.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_last.json 2> gpurun_out/bench_last.err || { tail gpurun_out/bench_last.err; exit 4; }
python scripts/fmt_lines.py gpurun_out/bench_last.json
python -c "import json; d=json.load(open('gpurun_out/bench_last.json')); print('host_wait', d.get('host_wait'), 'cpu_baseline', d['cpu_baseline']['value'], 'config5_n1', d['config5_n1']['ms_per_step'])"
echo DONE
