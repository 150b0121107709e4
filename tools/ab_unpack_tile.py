#!/usr/bin/env python3
"""Interleaved A/B of TILE unpack image sizes (SRPC_TUNE_TILE_BYTES; the pack
tile is held at its own setting) on fixed schemas, kernel clock, 16M records.

    python tools/ab_unpack_tile.py [--cases all_kinds17] [--sizes 8192,...] [--reps 8] [--rounds 2]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--sizes", default="8192,16384,24576,32768,49152")
    ap.add_argument("--cases", default="all_kinds17,request53,response19")
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle
    import srpc_amd
    from srpc_amd import NUMBER, SQUARE_METHOD, GpuPacker, Schema

    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    n = 1 << 24
    cases = {
        "all_kinds17": (Schema.of("all_kinds", ("a", "bool"), ("b", "int8"), ("c", "char"), ("d", "int16"),
                                  ("e", "int32"), ("f", "int64")), b""),
        "request53": (NUMBER, srpc_amd.request_prefix(SQUARE_METHOD, "Number")),
        "response19": (NUMBER, srpc_amd.response_prefix(0, "Number")),
    }
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(s)
    b.record(s)
    sizes = [int(x) for x in args.sizes.split(",")]
    for name in args.cases.split(","):
        sch, pre = cases[name]
        p = GpuPacker(sch, pre)
        rng = np.random.default_rng(1)
        cols = [torch.from_numpy(rng.integers(0, 2 if k == oracle.BOOL else 256, n * oracle.KIND_SIZE[k],
                                              dtype=np.uint8)).to(dev) for k in sch.kinds]
        wire = torch.empty(n * p.record_bytes + 16, dtype=torch.uint8, device=dev)
        back = [torch.empty_like(c) for c in cols]
        p.pack(cols, n, wire, stream=s)
        res = {}
        for _ in range(args.rounds):
            for ts in sizes:
                p.tune(tile_bytes=ts)
                for _ in range(2):
                    p.unpack(wire, n * p.record_bytes, n, back, stream=s)
                for _ in range(args.reps):
                    srpc_amd.time_next_call(a, b)
                    p.unpack(wire, n * p.record_bytes, n, back, stream=s)
                    torch.cuda.synchronize()
                    res.setdefault(ts, []).append(a.elapsed_time(b) * 1e3)
        ok = all(torch.equal(x, y) for x, y in zip(cols, back))
        for ts, t in sorted(res.items()):
            print(f"{name:12s} unpack tile {ts:6d} {statistics.median(t):8.1f} us  parity={ok}", flush=True)
        del cols, wire, back
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
