#!/bin/bash
# Round 3: the whole GPU suite, smoke, the default bench line and the training
# / DCN lines after the hand-written sort (row-scan form) and the unrolled
# tower contraction.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_x.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_x.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_x.log | tail -60; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_x.log 2>&1
rc=$?; tail -1 gpurun_out/smoke_x.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_x.json 2> gpurun_out/bench_x.err || { tail gpurun_out/bench_x.err; exit 4; }
python scripts/fmt_lines.py gpurun_out/bench_x.json
: > gpurun_out/bench_x_configs.jsonl
for cfg in fm_train dcn; do
  timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline >> gpurun_out/bench_x_configs.jsonl 2> gpurun_out/bench_x_$cfg.err || { tail gpurun_out/bench_x_$cfg.err; exit 5; }
done
python scripts/fmt_lines.py gpurun_out/bench_x_configs.jsonl
echo DONE
