"""Turn a gpu_check.sh session (gpurun_out/) into committed summaries under
profiles/ (tag = round, e.g. r1):

  profiles/<tag>_rocprof_kernel_stats.csv   rocprofv3 --kernel-trace --stats of bench.py
  profiles/<tag>_embed_fm_trace_summary.json  per-dispatch durations of the headline kernel
  profiles/<tag>_pmc.json                   PMC counters per launch + calibrated HBM bytes
  profiles/pmc_embed_fm.json                the numbers bench.py reports as roofline.traffic
  profiles/<tag>_bench.json / _bench_configs.jsonl   the bench lines of the session

HBM bytes calibration (gfx950, ROCm 7.2): the probe kernel in
scripts/pmc_driver.py shows one TCC_EA0_RDREQ per randomly gathered 64-B row
and ONE per 128-B line when both halves are requested, i.e. every request is a
128-B fill, while FETCH_SIZE tallies 64 B per request (TCC_BUBBLE is 0).  So
read bytes = TCC_EA0_RDREQ_sum * 128; writes = WRITE_SIZE * 1024.
"""
import csv
import json
import os
import shutil
import statistics as st
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")
P = os.path.join(ROOT, "profiles")


def pmc(i):
    path = os.path.join(G, f"pmc{i}", "pmc_counter_collection.csv")
    by = defaultdict(list)
    if not os.path.exists(path):
        return by
    for r in csv.DictReader(open(path)):
        by[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return by


def main(tag):
    os.makedirs(P, exist_ok=True)
    src = os.path.join(G, "prof", "run_kernel_stats.csv")
    if os.path.exists(src):
        shutil.copy(src, os.path.join(P, f"{tag}_rocprof_kernel_stats.csv"))
    tr = os.path.join(G, "prof", "run_kernel_trace.csv")
    if os.path.exists(tr):
        rows = [r for r in csv.DictReader(open(tr)) if "embed_fm_mfma" in r["Kernel_Name"]]
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows]
        ts = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
        b2b = [d[i] for i in range(1, len(d)) if ts[i][0] - ts[i - 1][1] < 3000]
        json.dump({"kernel": rows[0]["Kernel_Name"] if rows else None, "dispatches": len(d),
                   "duration_ns_median": st.median(d) if d else None,
                   "duration_ns_mean": st.mean(d) if d else None,
                   "duration_ns_median_back_to_back": st.median(b2b) if b2b else None,
                   "vgpr": rows[0]["VGPR_Count"] if rows else None, "sgpr": rows[0]["SGPR_Count"] if rows else None,
                   "lds_bytes": rows[0]["LDS_Block_Size"] if rows else None,
                   "grid": rows[0]["Grid_Size_X"] if rows else None,
                   "workgroup": rows[0]["Workgroup_Size_X"] if rows else None},
                  open(os.path.join(P, f"{tag}_embed_fm_trace_summary.json"), "w"), indent=1)
    c = {}
    for i in (1, 2, 3, 4):
        for (k, name), v in pmc(i).items():
            key = "embed_fm" if "embed_fm_mfma" in k else ("probe_gather" if "diag_gather" in k else None)
            if key:
                c.setdefault(key, {})[name] = v
    out = {"calibration": __doc__.split("HBM bytes calibration")[1].strip()}
    if "embed_fm" in c:
        e = c["embed_fm"]
        rd = st.median(e["TCC_EA0_RDREQ_sum"]) * 128
        wr = st.median(e["WRITE_SIZE"]) * 1024
        out["embed_fm"] = {"launches": len(e["TCC_EA0_RDREQ_sum"]),
                           "TCC_EA0_RDREQ_sum_median": st.median(e["TCC_EA0_RDREQ_sum"]),
                           "TCC_EA0_RDREQ_DRAM_sum_median": st.median(e.get("TCC_EA0_RDREQ_DRAM_sum", [0])),
                           "FETCH_SIZE_KB_median": st.median(e["FETCH_SIZE"]),
                           "WRITE_SIZE_KB_median": st.median(e["WRITE_SIZE"]),
                           "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                           "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes_per_launch": 4096 * 1824 + 18880,
                           "traffic_over_algorithmic": (rd + wr) / (4096 * 1824 + 18880)}
        json.dump({"hbm_bytes_per_launch": rd + wr, "source": f"profiles/{tag}_pmc.json"},
                  open(os.path.join(P, "pmc_embed_fm.json"), "w"), indent=1)
    if "probe_gather" in c:
        p = c["probe_gather"]
        req = p["TCC_EA0_RDREQ_sum"]
        out["probe_gather"] = {"rows_per_dispatch": 1703936, "index_lines_128B": 1703936 * 8 // 128,
                               "RDREQ_random_rows_dispatches": req[:5], "RDREQ_line_pair_dispatches": req[5:]}
    json.dump(out, open(os.path.join(P, f"{tag}_pmc.json"), "w"), indent=1)
    # per-config kernel stats (rocprofv3 --kernel-trace --stats of bench.py --config X)
    for cfg in ("dcn", "din", "pnn", "nfm", "afm", "ffm", "fm_train", "sharded"):
        src = os.path.join(G, f"prof_{cfg}", "run_kernel_stats.csv")
        if os.path.exists(src):
            shutil.copy(src, os.path.join(P, f"{tag}_rocprof_kernel_stats_{cfg}.csv"))
    # MFMA utilisation: SQ_VALU_MFMA_BUSY_CYCLES summed over the 1024 SIMDs,
    # against the dispatch's wall cycles (GRBM_GUI_ACTIVE is summed over 8 XCDs)
    mf = {}
    for cfg in ("dcn", "din", "hotpath"):
        path = os.path.join(G, f"mfma_{cfg}", "pmc_counter_collection.csv")
        if not os.path.exists(path):
            continue
        per = defaultdict(lambda: defaultdict(list))
        for r in csv.DictReader(open(path)):
            per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for kname, cs in per.items():
            if "SQ_VALU_MFMA_BUSY_CYCLES" not in cs or not any(v > 0 for v in cs["SQ_VALU_MFMA_BUSY_CYCLES"]):
                continue
            busy = st.median(cs["SQ_VALU_MFMA_BUSY_CYCLES"])
            wall = st.median(cs["GRBM_GUI_ACTIVE"]) / 8
            mf[kname[:90]] = {"config": cfg, "dispatches": len(cs["SQ_VALU_MFMA_BUSY_CYCLES"]),
                              "mfma_busy_cycles_median": busy, "wall_cycles_median": wall,
                              "mfma_util": busy / (1024 * wall) if wall else None}
    if mf:
        json.dump({"formula": "mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)",
                   "kernels": mf}, open(os.path.join(P, f"{tag}_mfma_util.json"), "w"), indent=1)
    for n in ("bench.json", "bench_configs.jsonl"):
        s = os.path.join(G, n)
        if os.path.exists(s):
            shutil.copy(s, os.path.join(P, f"{tag}_{n.replace('.json', '') if n.endswith('.json') else n}"
                                        + (".json" if n.endswith(".json") else "")))
    print(json.dumps(out.get("embed_fm", {}), indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r1")
