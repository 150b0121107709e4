#!/usr/bin/env python3
"""Per-kernel mean of every counter over rocprofv3 --pmc output directories."""
import csv
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    base = m.group(1) if m else name[:40]
    for tag in ("PackSizes", "ArrayVals"):
        if tag in name:
            base += f"<{tag}>"
    return base


def main(dirs):
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    for d in dirs:
        path = os.path.join(d, "run_counter_collection.csv")
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(path)):
            key = (r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (disp, cn), v in per.items():
            vals[names[disp]][cn].append(v)
    for k, cs in vals.items():
        print(k)
        for cn in sorted(cs):
            v = cs[cn]
            print(f"   {cn:26s} mean {sum(v) / len(v):16.1f}  n={len(v)}")


if __name__ == "__main__":
    main(sys.argv[1:])
