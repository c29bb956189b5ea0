#!/bin/bash
# Round 3: the driver's bench shape (--steps 20 --warmup 5) with the runtime's
# default host wait vs busy-wait (RS_BENCH_SYNC=spin), alternated 3 times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/sync_ab.jsonl
for r in 1 2 3; do
  for m in "" spin; do
    RS_BENCH_SYNC=${m:-default} timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config5 > gpurun_out/sync_$r$m.json 2> gpurun_out/sync_$r$m.err || { tail -5 gpurun_out/sync_$r$m.err; exit 3; }
    python -c "
import json,sys; d=json.load(open('gpurun_out/sync_$r$m.json')); print(json.dumps({'mode': '$m' or 'default', 'round': $r, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms']}))" >> gpurun_out/sync_ab.jsonl
  done
done
cat gpurun_out/sync_ab.jsonl; grep -h hipSetDeviceFlags gpurun_out/sync_*spin.err | head -1
echo DONE
