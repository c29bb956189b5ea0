"""Per-kernel totals from a rocprofv3 rocpd database (kernels view):
python scripts/kernel_stats_db.py <results.db> [top] [--csv out.csv]
--csv writes rocprofv3's kernel_stats.csv columns (Name, Calls,
TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev) for every
kernel, so a database-only run can be committed like a --stats run."""
import csv
import math
import sqlite3
import sys


def main():
    args = [a for a in sys.argv[1:]]
    out = None
    if "--csv" in args:
        i = args.index("--csv")
        out = args[i + 1]
        del args[i:i + 2]
    db, top = args[0], int(args[1]) if len(args) > 1 else 25
    c = sqlite3.connect(db)
    if out:
        rows = c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start), "
                         "avg((end-start)*(end-start)) from kernels group by name order by sum(end-start) desc").fetchall()
        total = sum(r[2] for r in rows) or 1
        with open(out, "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_ALL)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
            for name, n, tot, avg, mn, mx, sq in rows:
                sd = math.sqrt(max(sq - avg * avg, 0.0))
                w.writerow([name, n, tot, f"{avg:.6f}", f"{100.0 * tot / total:.4f}", mn, mx, f"{sd:.6f}"])
    q = ("select name, count(*), sum(end-start)/1e3, avg(end-start)/1e3 from kernels group by name "
         "order by sum(end-start) desc limit ?")
    for name, n, tot, avg in c.execute(q, (top,)):
        print(f"{tot:10.1f} us tot {n:4d} x {avg:9.1f} us  {name[:110]}")


if __name__ == "__main__":
    main()
