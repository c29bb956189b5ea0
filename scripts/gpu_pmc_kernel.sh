#!/bin/bash
# One PMC pass (SQ issue/wait breakdown) over `bench.py --config $CFG`, summarised for kernels matching $KPAT.
set -u
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/kpmc_$CFG" -o pmc --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 20 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/kpmc_$CFG.log" 2>&1 || { tail -20 "$R/gpurun_out/kpmc_$CFG.log"; exit 1; }
python3 - "$R/gpurun_out/kpmc_$CFG/pmc_counter_collection.csv" "$KPAT" <<'PY'
import csv, sys, statistics as st, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print("  ", c, st.median(v))
PY
