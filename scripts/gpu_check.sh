#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprof kernel trace -> PMC passes.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-200}

if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest rc=$rc: stopping"; grep -v "^Extension" gpurun_out/pytest_gpu.log | tail -30; exit $rc; }

  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || { echo "smoke rc=$rc: stopping"; exit $rc; }
fi

if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 600 python bench.py --steps $STEPS --warmup 20 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err; [ $rc -eq 0 ] || { echo "bench rc=$rc: stopping"; exit $rc; }
fi

if [ "${SKIP_CONFIGS:-0}" != 1 ]; then
  : > gpurun_out/bench_configs.jsonl
  for cfg in deepfm1e6 dcn din pnn nfm afm ffm fm_train io; do
    timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 10 >> gpurun_out/bench_configs.jsonl 2> gpurun_out/bench_$cfg.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg rc=$rc"; tail -5 gpurun_out/bench_$cfg.err; exit $rc; }
  done
  python scripts/fmt_lines.py gpurun_out/bench_configs.jsonl
  timeout -k 10 300 python bench.py --sharded --steps $STEPS --warmup 20 --no-cpu-baseline > gpurun_out/bench_sharded.json 2> gpurun_out/bench_sharded.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench sharded rc=$rc"; tail -5 gpurun_out/bench_sharded.err; exit $rc; }
  python scripts/fmt_lines.py gpurun_out/bench_sharded.json
fi

if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
      -- python3 "$R/bench.py" --steps $STEPS --warmup 20 --no-cpu-baseline > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err"
  rc=$?; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; tail -5 "$R/gpurun_out/prof.err"; exit $rc; }
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $ctr -d "$R/gpurun_out/pmc$i" -o pmc --output-format csv \
        -- python3 "$R/scripts/pmc_driver.py" > "$R/gpurun_out/pmc$i.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "pmc pass $i rc=$rc"; tail -5 "$R/gpurun_out/pmc$i.log"; exit $rc; }
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_sharded" -o run --output-format csv \
      -- python3 "$R/bench.py" --sharded --steps 100 --warmup 10 --no-cpu-baseline > "$R/gpurun_out/prof_sharded.json" 2> "$R/gpurun_out/prof_sharded.err"
  rc=$?; [ $rc -eq 0 ] || { echo "rocprof sharded rc=$rc"; tail -5 "$R/gpurun_out/prof_sharded.err"; exit $rc; }
  for cfg in dcn din pnn nfm afm ffm fm_train; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$cfg" -o run --output-format csv \
        -- python3 "$R/bench.py" --config $cfg --steps 50 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/prof_$cfg.json" 2> "$R/gpurun_out/prof_$cfg.err"
    rc=$?; [ $rc -eq 0 ] || { echo "rocprof $cfg rc=$rc"; tail -5 "$R/gpurun_out/prof_$cfg.err"; exit $rc; }
  done
  # MFMA utilisation of the MFMA-shaped kernels (CrossNet, DIN attention, DNN tower in the fused DeepFM)
  for cfg in dcn din hotpath; do
    timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        -d "$R/gpurun_out/mfma_$cfg" -o pmc --output-format csv \
        -- python3 "$R/bench.py" --config $cfg --steps 20 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/mfma_$cfg.log" 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "mfma pmc $cfg rc=$rc"; tail -5 "$R/gpurun_out/mfma_$cfg.log"; exit $rc; }
  done
  cd "$R"
fi
echo DONE
