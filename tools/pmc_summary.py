"""Summarise rocprofv3 --pmc counter CSVs per kernel (mean over dispatches)."""
import csv
import sys
from collections import defaultdict


def load(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].split("(")[0]
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


if __name__ == "__main__":
    acc = load(sys.argv[1:])
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} mean {sum(v)/len(v):16.1f}  (n={len(v)})")
