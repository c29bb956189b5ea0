"""Overlap of the RCCL all-to-all and rs_shard_fm_pipe kernels in a
rocprofv3 kernel trace (sharded.PipeLanes check).
usage: python scripts/trace_overlap.py <kernel_trace.csv> [last_n]"""
import csv
import sys


def main():
    path = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            kind = "rccl" if "nccl" in name.lower() else ("pipe" if "shard_fm_pipe" in name else None)
            if kind:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
    rows.sort()
    rows = rows[-last:]
    busy = {"rccl": 0, "pipe": 0}
    over = 0
    for i, (s, e, k) in enumerate(rows):
        busy[k] += e - s
        for s2, e2, k2 in rows[i + 1:i + 6]:
            if k2 != k and s2 < e:
                over += min(e, e2) - s2
    span = rows[-1][1] - rows[0][0]
    print(f"{len(rows)} kernels over {span / 1e3:.1f} us: rccl busy {busy['rccl'] / 1e3:.1f} us, "
          f"pipe busy {busy['pipe'] / 1e3:.1f} us, overlapped {over / 1e3:.1f} us")
    for s, e, k in rows[-10:]:
        print(f"  {k:5s} {(s - rows[0][0]) / 1e3:9.2f} .. {(e - rows[0][0]) / 1e3:9.2f} us")


if __name__ == "__main__":
    main()
