#!/usr/bin/env python3
"""Per-kernel table from tools/pmc_paths.sh output: calls, median duration
(--kernel-trace pass, no counters), HBM bytes per call (read = 2 x FETCH_SIZE
x 1024 with the gfx950 half-count of wide streaming reads; write = WRITE_SIZE
x 1024; both calibrated only for 16-B-per-lane streaming access, so for
other shapes they are upper/lower hints, see MI355X_MICROARCH.md HBM), and
the SQ counters per call with derived ratios: VALU-active and LDS-active
share of the wave cycles, stalled share (WAIT_ANY + WAIT_INST_ANY), mean
resident waves per SIMD, LDS bank-conflict share of LDS-array cycles.

    python tools/pmc_paths_table.py gpurun_out/pmc_<tag>_<filter>
"""
import csv
import glob
import os
import re
import statistics
import sys
from collections import defaultdict

SIMDS = 256 * 4
CLOCK_GHZ = 2.4


def short(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    base = m.group(1) if m else name[:40]
    for tag in ("PackSizes", "ArrayValsY", "ArrayVals", "SingleStrLen"):
        if tag in name:
            base += f"<{tag}>"
            break
    t = re.search(r"<(true|false|\d+)>", name)
    if t and "<" not in base:
        base += f"<{t.group(1)}>"
    return base


def main(d: str) -> None:
    dur = defaultdict(list)
    order = []
    for path in glob.glob(os.path.join(d, "stats", "*kernel_trace.csv")):
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if k not in dur:
                order.append(k)
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    cnt = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(d, "p*", "*counter_collection.csv"))):
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(path)):
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = short(r["Kernel_Name"])
        for (disp, cn), v in per.items():
            cnt[names[disp]][cn].append(v)

    def m(k, c):
        v = cnt[k].get(c)
        return statistics.mean(v) if v else None

    print(f"# {d}")
    print(f"{'kernel':34s} {'calls':>5s} {'med_us':>8s} {'rd_MB':>8s} {'wr_MB':>8s} {'VALU%':>6s} "
          f"{'LDS%':>6s} {'stall%':>7s} {'waves/SIMD':>10s} {'ldsconf%':>8s} {'VALUi/wave':>10s} "
          f"{'LDSi/wave':>9s} {'VMRDi/wave':>10s} {'VMWRi/wave':>10s}")
    for k in order:
        if k.startswith("__amd") or k not in cnt:
            continue
        med = statistics.median(dur[k]) / 1e3
        fs, ws = m(k, "FETCH_SIZE"), m(k, "WRITE_SIZE")
        rd = 2 * fs * 1024 / 1e6 if fs is not None else float("nan")
        wr = ws * 1024 / 1e6 if ws is not None else float("nan")
        wc, waves = m(k, "SQ_WAVE_CYCLES"), m(k, "SQ_WAVES")
        valu = m(k, "SQ_ACTIVE_INST_VALU")
        ldsa = m(k, "SQ_ACTIVE_INST_LDS")
        stall = (m(k, "SQ_WAIT_ANY") or 0) + (m(k, "SQ_WAIT_INST_ANY") or 0)
        # SQ_WAVE_CYCLES counts quad-cycles
        occ = wc * 4 / (med * 1e3 * CLOCK_GHZ * SIMDS) if wc and med else float("nan")
        conf, idx = m(k, "SQ_LDS_BANK_CONFLICT"), m(k, "SQ_LDS_IDX_ACTIVE")

        def pct(a, b):
            return 100 * a / b if a is not None and b else float("nan")

        def per_wave(c):
            v = m(k, c)
            return v / waves if v is not None and waves else float("nan")

        print(f"{k:34s} {len(dur[k]):5d} {med:8.1f} {rd:8.1f} {wr:8.1f} {pct(valu, wc):6.1f} {pct(ldsa, wc):6.1f} "
              f"{pct(stall, wc):7.1f} {occ:10.2f} {pct(conf, idx):8.1f} {per_wave('SQ_INSTS_VALU'):10.1f} "
              f"{per_wave('SQ_INSTS_LDS'):9.1f} {per_wave('SQ_INSTS_VMEM_RD'):10.1f} {per_wave('SQ_INSTS_VMEM_WR'):10.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
