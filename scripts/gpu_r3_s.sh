#!/bin/bash
# Round 3 (re-entry): the restored tree's GPU suite, smoke, the default bench
# line and its rocprof kernel-trace summary.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_s.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_s.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_s.log | tail -60; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_s.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err || { tail gpurun_out/bench_s.err; exit 4; }
python scripts/fmt_lines.py gpurun_out/bench_s.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_s" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-cpu-baseline > "$R/gpurun_out/prof_s_bench.json" 2> "$R/gpurun_out/prof_s.err"
rc=$?; [ $rc -eq 0 ] || { tail -5 "$R/gpurun_out/prof_s.err"; exit $rc; }
cd "$R"
timeout -k 10 400 python scripts/diag_mtype.py > gpurun_out/mtype.jsonl 2> gpurun_out/mtype.err; rc=$?; cat gpurun_out/mtype.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/mtype.err; exit $rc; }
echo DONE
