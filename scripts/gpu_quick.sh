#!/bin/bash
# GPU parity tests (stop on fault) then selected bench configs (CONFIGS="hotpath pnn ...").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -v "^Extension" gpurun_out/pytest_gpu.log | tail -40; exit $rc; }
for cfg in ${CONFIGS:-hotpath}; do
  timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 10 --no-cpu-baseline > gpurun_out/q_$cfg.json 2> gpurun_out/q_$cfg.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $cfg rc=$rc"; tail -8 gpurun_out/q_$cfg.err; exit $rc; }
  python -c "
import json,sys
d=json.load(open('gpurun_out/q_$cfg.json'))
r=d['roofline']
print('$cfg', 'value=%.4g'%d['value'], 'ms=%.4f'%d['ms_per_step'], 'roof=%.3f'%r['frac'], 'kern_ms=%.4f'%r.get('kernel_ms',0), {k:v for k,v in d.items() if k in ('concurrent_batches','deepfm_forward')})
"
done
echo DONE
