#!/usr/bin/env python3
"""Median duration per (kernel, grid) from a rocprofv3 kernel_trace.csv."""
import csv
import re
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    base = m.group(1) if m else name[:40]
    for tag in ("PackSizes", "ArrayVals", "FirstAndChars"):
        if tag in name:
            base += f"<{tag}>"
    return base


def main(path: str) -> None:
    d = defaultdict(list)
    order = []
    for r in csv.DictReader(open(path)):
        key = (short(r["Kernel_Name"]), int(r["Grid_Size_X"]), int(r.get("LDS_Block_Size", 0) or 0))
        if key not in d:
            order.append(key)
        d[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for key in order:
        v = d[key]
        print(f"{key[0]:34s} grid {key[1]:>10d} lds {key[2]:>6d}  calls {len(v):4d}  "
              f"median {statistics.median(v) / 1e3:9.2f} us  min {min(v) / 1e3:9.2f} us")


if __name__ == "__main__":
    main(sys.argv[1])
