"""Per-kernel totals from a rocprofv3 rocpd database (kernels view):
python scripts/kernel_stats_db.py <results.db> [top]"""
import sqlite3
import sys


def main():
    db, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25
    c = sqlite3.connect(db)
    q = ("select name, count(*), sum(end-start)/1e3, avg(end-start)/1e3 from kernels group by name "
         "order by sum(end-start) desc limit ?")
    for name, n, tot, avg in c.execute(q, (top,)):
        print(f"{tot:10.1f} us tot {n:4d} x {avg:9.1f} us  {name[:110]}")


if __name__ == "__main__":
    main()
