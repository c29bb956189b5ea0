#!/bin/bash
# HBM traffic (PMC) of each config line's dominant kernel: one rocprofv3 pass
# per config with TCC_EA0_RDREQ (x 128 B: every request is a 128-B fill on
# gfx950, profiles/r2_pmc.json "calibration") and WRITE_SIZE (KB), over
# `bench.py --config $CFG`; summarised by scripts/pmc_configs.py into
# gpurun_out/pmc_configs.json (copied to profiles/).
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
for CFG in ${CFGS:-dcn pnn nfm afm ffm din}; do
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum WRITE_SIZE -d "$R/gpurun_out/cpmc_$CFG" -o pmc \
    --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 20 --warmup 2 --no-cpu-baseline \
    > "$R/gpurun_out/cpmc_$CFG.log" 2>&1 || { echo "pmc pass $CFG failed"; tail -20 "$R/gpurun_out/cpmc_$CFG.log"; exit 1; }
  echo "pmc pass $CFG done"
done
python3 "$R/scripts/pmc_configs.py" "$R/gpurun_out" > "$R/gpurun_out/pmc_configs.json"
cat "$R/gpurun_out/pmc_configs.json"
