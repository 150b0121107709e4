#!/usr/bin/env python3
"""Interleaved A/B of TILE pack image sizes (SRPC_TUNE_PACK_TILE_BYTES) in two
loop shapes: pack after pack (tools/bench_paths.py's loop) and pack after
unpack (a round trip, bench.py's loop).  Kernel clock (srpc_time_next_call),
median of R reps per setting and shape, 16M records.

    python tools/ab_pack_tile.py [--reps 10] [--rounds 3]
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
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--sizes", default="8192,12288,16384,24576,32768")
    ap.add_argument("--cases", default="request53,response19,quad16_tile")
    args = ap.parse_args()
    import torch

    import oracle
    import srpc_amd
    from srpc_amd import NUMBER, QUAD, SQUARE_METHOD, GpuPacker

    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    n = 1 << 24
    cases = {
        "request53": (NUMBER, srpc_amd.request_prefix(SQUARE_METHOD, "Number")),
        "response19": (NUMBER, srpc_amd.response_prefix(0, "Number")),
        "quad16_tile": (QUAD, b""),
        "all_kinds17": (srpc_amd.Schema.of("all_kinds", ("a", "bool"), ("b", "int8"), ("c", "char"),
                                           ("d", "int16"), ("e", "int32"), ("f", "int64")), b""),
    }
    cases = {k: v for k, v in cases.items() if k in args.cases.split(",")}
    sizes = [int(x) for x in args.sizes.split(",")]
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(s)
    b.record(s)
    for name, (sch, pre) in cases.items():
        p = GpuPacker(sch, pre)
        p.force_path(srpc_amd.SRPC_PATH_TILE)
        import numpy as np
        rng = np.random.default_rng(1)
        cols = [torch.from_numpy(rng.integers(0, 2 if k == oracle.BOOL else 256, n * oracle.KIND_SIZE[k],
                                              dtype=np.uint8)).to(dev) for k in sch.kinds]
        wire = torch.empty(n * p.record_bytes + 16, dtype=torch.uint8, device=dev)
        back = [torch.empty_like(c) for c in cols]
        res = {}
        for _ in range(args.rounds):
            for tb in sizes:
                p.tune(pack_tile_bytes=tb)
                for shape in ("after_pack", "after_unpack"):
                    for _ in range(2):
                        p.pack(cols, n, wire, stream=s)
                    for _ in range(args.reps):
                        if shape == "after_unpack":
                            p.unpack(wire, n * p.record_bytes, n, back, stream=s)
                        srpc_amd.time_next_call(a, b)
                        p.pack(cols, n, wire, stream=s)
                        torch.cuda.synchronize()
                        res.setdefault((tb, shape), []).append(a.elapsed_time(b) * 1e3)
        for (tb, shape), ts in sorted(res.items()):
            print(f"{name:12s} pack tile {tb:6d} {shape:13s} {statistics.median(ts):8.1f} us", flush=True)
        del cols, wire, back
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
