#!/usr/bin/env python3
"""A/B of TILE-path image sizes (SRPC_TUNE_TILE_BYTES) on the envelope and
mixed-width schemas, interleaved rounds in one process; median kernel time
per setting from HIP events.

    python tools/sweep_tile.py [--records N] [--rounds R]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import numpy as np
    import torch

    import srpc_amd
    from srpc_amd import NUMBER, QUAD, SQUARE_METHOD, GpuPacker, Schema

    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    n = args.records
    cases = {
        "request53": (NUMBER, srpc_amd.request_prefix(SQUARE_METHOD, "Number")),
        "response19": (NUMBER, srpc_amd.response_prefix(0, "Number")),
        "all_kinds17": (Schema.of("k", ("a", "bool"), ("b", "int8"), ("c", "char"), ("d", "int16"),
                                  ("e", "int32"), ("f", "int64")), b""),
        "quad16_tile": (QUAD, b""),
    }
    sizes = [4096, 6144, 8192, 12288, 16384, 24576, 32768]
    res = {}
    for name, (sch, pre) in cases.items():
        p = GpuPacker(sch, pre)
        p.force_path(srpc_amd.SRPC_PATH_TILE)
        rng = np.random.default_rng(3)
        cols = []
        for k in sch.kinds:
            nb = n * srpc_amd.packer.KIND_SIZE[k]
            c = torch.from_numpy(rng.integers(0, 2, nb, dtype=np.uint8)).to(dev)
            cols.append(c)
        wire = torch.empty(n * p.record_bytes + 16, dtype=torch.uint8, device=dev)
        back = [torch.empty_like(c) for c in cols]
        ref = None
        for _ in range(args.rounds):
            for tb in sizes:
                p.tune(tile_bytes=tb)
                for kern in ("pack", "unpack"):
                    fn = (lambda: p.pack(cols, n, wire, stream=s)) if kern == "pack" else (
                        lambda: p.unpack(wire, n * p.record_bytes, n, back, stream=s))
                    fn()
                    a = torch.cuda.Event(enable_timing=True)
                    b = torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    fn()
                    b.record(s)
                    torch.cuda.synchronize()
                    res.setdefault((name, tb, kern), []).append(a.elapsed_time(b))
                if ref is None:
                    ref = wire.clone()
                assert torch.equal(ref, wire), (name, tb)
                assert all(torch.equal(x, y) for x, y in zip(cols, back)), (name, tb)
        del wire, back, cols, ref
        torch.cuda.empty_cache()
    rows = []
    for (name, tb, kern), ts in sorted(res.items()):
        sch, pre = cases[name]
        rb = len(pre) + sch.body_bytes
        alg = n * (rb + sch.body_bytes)
        med = statistics.median(ts) / 1e3
        rows.append({"case": name, "tile_bytes": tb, "kernel": kern, "median_us": round(med * 1e6, 1),
                     "GBps": round(alg / med / 1e9, 1), "frac": round(alg / med / 8e12, 4)})
        print(f"{name:12s} {tb:6d} {kern:6s} {med*1e6:9.1f} us {alg/med/1e9:8.1f} GB/s {alg/med/8e12:.3f}")
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
