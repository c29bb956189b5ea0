#!/bin/bash
# Round 3 final session, part 1: GPU suite, smoke, the default bench line,
# its rocprofv3 kernel trace, the PMC passes of the headline kernel and the
# MFMA-utilisation passes (summaries: scripts/summarize_profiles.py r3final).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_gpu.log | tail -60; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 4; }
python scripts/fmt_lines.py gpurun_out/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_driver_shape.json 2> gpurun_out/bench_driver_shape.err || { tail gpurun_out/bench_driver_shape.err; exit 4; }
python scripts/fmt_lines.py gpurun_out/bench_driver_shape.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 200 --warmup 20 --no-cpu-baseline > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err"
rc=$?; [ $rc -eq 0 ] || { echo "rocprof rc=$rc"; tail -5 "$R/gpurun_out/prof.err"; exit $rc; }
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d "$R/gpurun_out/pmc$i" -o pmc --output-format csv \
      -- python3 "$R/scripts/pmc_driver.py" > "$R/gpurun_out/pmc$i.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "pmc pass $i rc=$rc"; tail -5 "$R/gpurun_out/pmc$i.log"; exit $rc; }
done
for cfg in dcn din hotpath; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
      -d "$R/gpurun_out/mfma_$cfg" -o pmc --output-format csv \
      -- python3 "$R/bench.py" --config $cfg --steps 20 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/mfma_$cfg.log" 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "mfma pmc $cfg rc=$rc"; tail -5 "$R/gpurun_out/mfma_$cfg.log"; exit $rc; }
done
cd "$R"
echo DONE
