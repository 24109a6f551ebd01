"""Summarise rocprofv3 --pmc CSVs (one directory per pass) into per-kernel averages per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(root):
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for (d, c), v in per.items():
            acc[names[d]][c].append(v)
    return acc


if __name__ == "__main__":
    acc = load(sys.argv[1])
    for k, cs in sorted(acc.items()):
        print(k[:70])
        for c, vs in sorted(cs.items()):
            print(f"    {c:28s} {sum(vs)/len(vs):16.1f}  (n={len(vs)})")
