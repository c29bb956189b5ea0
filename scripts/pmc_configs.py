"""Summarise scripts/gpu_pmc_configs.sh: per config, the dominant kernel's
median per-dispatch HBM bytes = TCC_EA0_RDREQ_sum x 128 + WRITE_SIZE x 1024
(the gfx950 calibration in profiles/r2_pmc.json).  The batch-4096 dispatches
are picked by the kernel name and the most common grid size."""
import collections
import csv
import json
import os
import statistics as st
import sys

# config -> (bench line's roofline "kernel" key, kernel-name substring)
KERNELS = {"dcn": ("embed_cross_ka", "rs::embed_cross_ka<"), "pnn": ("inner_fast_ka", "rs::inner_fast_ka<"),
           "nfm": ("pair_pool_ksplit", "rs::pair_pool_ksplit<"), "afm": ("pair_pool_ksplit", "rs::pair_pool_ksplit<"),
           "ffm": ("ffm4_kernel", "rs::ffm4_kernel<"), "din": ("din_fused", "rs::din_fused<")}


def main():
    root = sys.argv[1]
    out = {"method": "rocprofv3 --pmc TCC_EA0_RDREQ_sum WRITE_SIZE over bench.py --config <cfg> --steps 20; "
                     "bytes = RDREQ x 128 + WRITE_SIZE x 1024 per dispatch, median over the dominant grid"}
    for cfg, (key, pat) in KERNELS.items():
        p = os.path.join(root, f"cpmc_{cfg}", "pmc_counter_collection.csv")
        if not os.path.exists(p):
            continue
        disp = collections.defaultdict(dict)
        grid = {}
        for r in csv.DictReader(open(p)):
            if pat not in r["Kernel_Name"]:
                continue
            d = r.get("Dispatch_Id") or r.get("Correlation_Id") or r.get("Index")
            disp[d][r["Counter_Name"]] = float(r["Counter_Value"])
            grid[d] = r.get("Grid_Size", r.get("Grid_Size_X", ""))
        if not disp:
            continue
        common = collections.Counter(grid.values()).most_common(1)[0][0]
        sel = [c for d, c in disp.items() if grid[d] == common and "TCC_EA0_RDREQ_sum" in c and "WRITE_SIZE" in c]
        rd = [c["TCC_EA0_RDREQ_sum"] * 128 for c in sel]
        wr = [c["WRITE_SIZE"] * 1024 for c in sel]
        out[cfg] = {"kernel": key, "dispatches": len(sel), "grid_size": common,
                    "hbm_read_bytes_per_launch": st.median(rd), "hbm_write_bytes_per_launch": st.median(wr),
                    "hbm_bytes_per_launch": st.median([a + b for a, b in zip(rd, wr)])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
