#!/bin/bash
# Round 6: PMC passes on deepfm_ws (scripts/pmc_deepfm_ws.py), one rocprofv3 run per pass, then the
# split-role kernel's stamps (diagnostic library).  Output under gpurun_out/r6pmc_*.
set -eu
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$R/gpurun_out/r6pmc_$name" -o pmc --output-format csv \
    -- python3 "$R/scripts/pmc_deepfm_ws.py" > "$R/gpurun_out/r6pmc_$name.log" 2>&1
  python3 "$R/scripts/pmc_summary.py" "$(ls "$R"/gpurun_out/r6pmc_$name/pmc_counter_collection.csv "$R"/gpurun_out/r6pmc_$name/*/pmc_counter_collection.csv 2>/dev/null | head -1)" deepfm_ws > "$R/gpurun_out/r6pmc_$name.json"
}
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE
pass wait SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_FLAT SQ_LDS_ADDR_CONFLICT SQ_INSTS_FLAT
DIAG_DEEPFM_OPT=0 timeout -k 10 120 python3 "$R/scripts/diag_deepfm_stamps.py" > "$R/gpurun_out/r6_deepfm_ws_stamps.json"
pass icache SQC_ICACHE_MISSES SQC_ICACHE_HITS
