#!/usr/bin/env python3
"""A/B sweep of DWORD-path variants on the bench workload (16M Quad records).

Interleaved rounds in ONE process (cdna_hip_programming.md §5.4 rule 24):
every variant is timed once per round, rounds repeat, and the median and min
per variant are reported.  Each pack/unpack is timed on the kernel clock of
srpc_time_next_call (dispatch begin/end); the torch copy by events around it.  "cold" rounds write a 1 GiB scratch buffer before each
timed kernel so the 256 MiB Infinity Cache holds none of its inputs.

Known-good reference on the same device: torch's device-to-device copy of the
same 512 MiB (256 MiB read + 256 MiB write), i.e. the chip's copy ceiling for
this byte count.

    python tools/sweep.py [--records N] [--rounds R] [--out gpurun_out/sweep.json]
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--schema", default="quad", choices=["quad", "number", "two"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--grids", default="", help="comma list of workgroup caps to sweep (0 = full grid)")
    ap.add_argument("--base", default="1,1,3", help="rpl,iter,nt for the --grids sweep")
    args = ap.parse_args()

    import torch

    import srpc_amd
    from srpc_amd import NUMBER, QUAD, TWO_NUMBERS, GpuPacker

    sch = {"quad": QUAD, "number": NUMBER, "two": TWO_NUMBERS}[args.schema]
    F = len(sch.kinds)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    n = args.records
    cols = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(F)]
    back = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(F)]
    wire = torch.empty(n * 4 * F, dtype=torch.uint8, device=dev)
    srpc_amd.fill_splitmix_i32(cols, n, 0x5EED, 0, s)
    flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
    copy_src = torch.empty(n * 4 * F, dtype=torch.uint8, device=dev)
    copy_dst = torch.empty_like(copy_src)
    p = GpuPacker(sch)

    if args.grids:
        base = [int(x) for x in args.base.split(",")]
        variants = [("dword", base[0], base[1], base[2], g) for g in [int(x) for x in args.grids.split(",")]]
    else:
        variants = [("dword", rpl, it, nt, 0)
                    for rpl, it, nt in itertools.product((1, 4), (1, 2, 4, 8), (0, 1, 2, 3))]
        variants.append(("tile", 0, 0, 0, 0))
    alg = 2 * 4 * F * n  # bytes per kernel: read F*4 + write F*4 per record

    def timed(fn, cold, hook=True):
        if cold:
            flush.fill_(1)
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        if hook:  # kernel clock (srpc_time_next_call) restamps a and b
            b.record(s)
            srpc_amd.time_next_call(a, b)
        fn()
        if not hook:
            b.record(s)
        return a, b

    res = {}
    for _ in range(2):  # warm-up every variant
        for v in variants:
            set_variant(p, v, srpc_amd)
            p.pack(cols, n, wire, stream=s)
            p.unpack(wire, wire.numel(), n, back, stream=s)
    torch.cuda.synchronize()
    ok = all(torch.equal(x, y) for x, y in zip(cols, back))
    for rnd in range(args.rounds):
        for cold in (False, True):
            evs = []
            for v in variants:
                set_variant(p, v, srpc_amd)
                evs.append((v, "pack", timed(lambda: p.pack(cols, n, wire, stream=s), cold)))
                evs.append((v, "unpack", timed(lambda: p.unpack(wire, wire.numel(), n, back, stream=s), cold)))
            evs.append((("copy",), "d2d", timed(lambda: copy_dst.copy_(copy_src), cold, hook=False)))
            torch.cuda.synchronize()
            for v, k, (a, b) in evs:
                res.setdefault((v, k, cold), []).append(a.elapsed_time(b))
    out = {"records": n, "schema": sch.name, "alg_bytes_per_kernel": alg, "roundtrip_ok": ok,
           "rows": []}
    for (v, k, cold), ts in sorted(res.items(), key=lambda kv: (kv[0][2], kv[0][1], statistics.median(kv[1]))):
        med, mn = statistics.median(ts), min(ts)
        out["rows"].append({"variant": "/".join(map(str, v)), "kernel": k, "cold": cold,
                            "median_us": round(med * 1e3, 2), "min_us": round(mn * 1e3, 2),
                            "GBps_median": round(alg / (med / 1e3) / 1e9, 1),
                            "frac_of_8TBps": round(alg / (med / 1e3) / 8e12, 4)})
    txt = json.dumps(out, indent=1)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(txt)
    for r in out["rows"]:
        print(f'{"cold" if r["cold"] else "warm"} {r["kernel"]:6s} {r["variant"]:16s} '
              f'med {r["median_us"]:8.2f} us  min {r["min_us"]:8.2f} us  {r["GBps_median"]:8.1f} GB/s  '
              f'{r["frac_of_8TBps"]:.3f}')


def set_variant(p, v, srpc_amd):
    if v[0] == "tile":
        p.force_path(srpc_amd.SRPC_PATH_TILE)
    else:
        p.force_path(srpc_amd.SRPC_PATH_DWORD)
        p.tune(v[1], v[2], v[3], grid=v[4])


if __name__ == "__main__":
    main()
