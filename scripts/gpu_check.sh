#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprof kernel trace.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }   # 1 = test failures (no fault)
STEPS=${STEPS:-200}

timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; ok $rc || { echo "pytest rc=$rc: stopping"; exit $rc; }

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || { echo "smoke rc=$rc: stopping"; exit $rc; }

if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python bench.py --steps $STEPS --warmup 20 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || { echo "bench rc=$rc: stopping"; exit $rc; }
fi

if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run \
      --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps $STEPS --warmup 20 --no-cpu-baseline \
      > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err"
  rc=$?; cd "$GRAFT_REPO_ROOT"; tail -2 gpurun_out/prof.err; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; exit $rc; }
  find gpurun_out/prof -name "*stats*" | head
fi
echo DONE
