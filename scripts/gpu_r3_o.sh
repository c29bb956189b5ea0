#!/bin/bash
# Round 3: l2-decay streaming (4 loads in flight): training tests, FM / FFM training bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_interactions.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_o.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_o.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_o.log | tail -60; exit $rc; }
for cfg in fm_train ffm; do
  timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_o_$cfg.json 2> gpurun_out/bench_o_$cfg.err || { tail gpurun_out/bench_o_$cfg.err; exit 4; }
done
python scripts/fmt_lines.py gpurun_out/bench_o_fm_train.json
python scripts/fmt_lines.py gpurun_out/bench_o_ffm.json
