#!/bin/bash
# Round 3 final session, part 2: the config lines, config 5 at N = 1, their
# rocprofv3 kernel traces, and the N = 2 bench path rehearsed with gloo on the
# one device (every rank on cuda:0; a rehearsal, not a result).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/bench_configs.jsonl
for cfg in deepfm1e6 dcn din pnn nfm afm ffm fm_train io; do
  timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 10 >> gpurun_out/bench_configs.jsonl 2> gpurun_out/bench_$cfg.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg rc=$rc"; tail -5 gpurun_out/bench_$cfg.err; exit $rc; }
done
python scripts/fmt_lines.py gpurun_out/bench_configs.jsonl
timeout -k 10 300 python bench.py --sharded --steps 200 --warmup 20 > gpurun_out/bench_sharded.json 2> gpurun_out/bench_sharded.err
rc=$?; [ $rc -eq 0 ] || { echo "bench sharded rc=$rc"; tail -5 gpurun_out/bench_sharded.err; exit $rc; }
python scripts/fmt_lines.py gpurun_out/bench_sharded.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_sharded" -o run --output-format csv \
    -- python3 "$R/bench.py" --sharded --steps 100 --warmup 10 --no-cpu-baseline > "$R/gpurun_out/prof_sharded.json" 2> "$R/gpurun_out/prof_sharded.err"
rc=$?; [ $rc -eq 0 ] || { echo "rocprof sharded rc=$rc"; tail -5 "$R/gpurun_out/prof_sharded.err"; exit $rc; }
for cfg in dcn din pnn fm_train; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$cfg" -o run --output-format csv \
      -- python3 "$R/bench.py" --config $cfg --steps 50 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/prof_$cfg.json" 2> "$R/gpurun_out/prof_$cfg.err"
  rc=$?; [ $rc -eq 0 ] || { echo "rocprof $cfg rc=$rc"; tail -5 "$R/gpurun_out/prof_$cfg.err"; exit $rc; }
done
cd "$R"
RS_BENCH_BACKEND=gloo RS_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/rehearsal_n2.json 2> gpurun_out/rehearsal_n2.err
rc=$?; [ $rc -eq 0 ] || { echo "rehearsal rc=$rc"; tail -8 gpurun_out/rehearsal_n2.err; exit $rc; }
python scripts/fmt_lines.py gpurun_out/rehearsal_n2.json
echo DONE
