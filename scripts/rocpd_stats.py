"""Kernel statistics from a rocprofv3 rocpd database (the default output of
`rocprofv3 --kernel-trace --stats` without --output-format csv): one row per
(kernel, grid) with calls, total / average / median / min / max duration in ns,
in the column order of rocprofv3's kernel_stats.csv plus the grid size.

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/x.csv
"""
import collections
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    q = ("select s.kernel_name, d.end - d.start, d.grid_size_x / d.workgroup_size_x from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    agg = collections.defaultdict(list)
    for name, dur, grid in c.execute(q):
        agg[(name, grid)].append(dur)
    rows = []
    for (name, grid), v in agg.items():
        v.sort()
        rows.append({"Name": name, "Grid": grid, "Calls": len(v), "TotalDurationNs": sum(v),
                     "AverageNs": sum(v) / len(v), "MedianNs": v[len(v) // 2], "MinNs": v[0], "MaxNs": v[-1]})
    rows.sort(key=lambda r: -r["TotalDurationNs"])
    return rows


def main():
    rows = stats(sys.argv[1])
    w = csv.DictWriter(sys.stdout, fieldnames=list(rows[0].keys()) if rows else ["Name"])
    w.writeheader()
    for r in rows:
        w.writerow(r)


if __name__ == "__main__":
    main()
