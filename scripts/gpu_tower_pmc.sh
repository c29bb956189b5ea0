#!/bin/bash
# PMC passes for the MLP tower (counters per pass kept within the gfx950 slots).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $R/gpurun_out/tpmc1 -o run --output-format csv -- python3 $R/scripts/tower_pmc.py > $R/gpurun_out/tpmc1.log 2>&1 || { tail -20 $R/gpurun_out/tpmc1.log; exit 1; }
timeout -k 10 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d $R/gpurun_out/tpmc2 -o run --output-format csv -- python3 $R/scripts/tower_pmc.py > $R/gpurun_out/tpmc2.log 2>&1 || { tail -20 $R/gpurun_out/tpmc2.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for d in ("tpmc1", "tpmc2"):
    for f in glob.glob(f"/root/repo/gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "mlp_tower" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in sorted(agg.items()):
            v = sorted(v)
            print(d, k, v[len(v) // 2])
PY
