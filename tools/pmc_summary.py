#!/usr/bin/env python3
"""Summarise rocprofv3 kernel-trace / PMC CSVs into per-kernel numbers.

    python tools/pmc_summary.py --stats DIR --fetch DIR --write DIR --records N --out profiles/x.json

HBM bytes per launch follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts exactly half
of a wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024;
write bytes = WRITE_SIZE * 1024.  FETCH_SIZE and WRITE_SIZE are collected in
separate passes (they do not fit one TCC pass).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics


def kname(full: str) -> str:
    for k in ("k_pack_dword_x4", "k_unpack_dword_x4", "k_pack_dword", "k_unpack_dword", "k_pack_tile",
              "k_unpack_tile", "k_pack_var", "k_unpack_var", "k_fill_splitmix", "k_set_status"):
        if k in full:
            return k
    return full[:40]


def role(k: str) -> str | None:
    if k.startswith("k_pack"):
        return "pack"
    if k.startswith("k_unpack"):
        return "unpack"
    return None


def load(dirname, pattern):
    f = glob.glob(os.path.join(dirname, "**", pattern), recursive=True)
    if not f:
        raise FileNotFoundError(f"{pattern} under {dirname}")
    return list(csv.DictReader(open(f[0])))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--records", type=int, required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    out = {"records": a.records, "source": "rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE",
           "correction": "read_bytes = 2 * FETCH_SIZE * 1024 (gfx950 half-count of wide streaming reads); "
                         "write_bytes = WRITE_SIZE * 1024",
           "kernels": {}}
    for r in load(a.stats, "*kernel_stats.csv"):
        k = kname(r["Name"])
        rl = role(k)
        if rl:
            out["kernels"].setdefault(rl, {})
            out["kernels"][rl].update({"kernel": k, "calls": int(r["Calls"]),
                                       "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                                       "max_ns": float(r["MaxNs"])})
    for tag, d, ctr in (("fetch", a.fetch, "FETCH_SIZE"), ("write", a.write, "WRITE_SIZE")):
        vals = {}
        for r in load(d, "*counter_collection.csv"):
            if r["Counter_Name"] != ctr:
                continue
            rl = role(kname(r["Kernel_Name"]))
            if rl:
                vals.setdefault(rl, []).append(float(r["Counter_Value"]))
        for rl, v in vals.items():
            out["kernels"].setdefault(rl, {})[ctr] = statistics.median(v)
    for rl, e in out["kernels"].items():
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            rd = 2 * e["FETCH_SIZE"] * 1024
            wr = e["WRITE_SIZE"] * 1024
            e["hbm_read_bytes_per_launch"] = int(rd)
            e["hbm_write_bytes_per_launch"] = int(wr)
            e["hbm_bytes_per_launch"] = int(rd + wr)
            e["alg_bytes_per_launch"] = 32 * a.records
            e["traffic_over_alg"] = round((rd + wr) / (32 * a.records), 4)
            if "avg_ns" in e:
                e["achieved_GBps_alg"] = round(32 * a.records / e["avg_ns"], 1)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
