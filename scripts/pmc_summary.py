"""Median per-dispatch value of every counter in a rocprofv3 --pmc CSV
(pmc_counter_collection.csv) for kernels whose name contains a pattern:
    python scripts/pmc_summary.py <csv> <pattern> > out.json"""
import collections
import csv
import json
import statistics
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(sys.argv[1])):
        if sys.argv[2] in r["Kernel_Name"]:
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: {c: statistics.median(v) for c, v in sorted(cs.items())} | {"dispatches": max(len(v) for v in cs.values())}
           for k, cs in agg.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
