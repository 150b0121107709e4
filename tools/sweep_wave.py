#!/usr/bin/env python3
"""Interleaved sweep of TILE wave-tile sizes (SRPC_TUNE_WAVE_PACK_BYTES /
SRPC_TUNE_WAVE_UNPACK_BYTES; 0 = workgroup tiles) per schema and direction,
in two loop shapes: the same call back to back (`same`) and alternating with
the other direction (`trip`, bench.py's round trip).  Kernel clock
(srpc_time_next_call), median of R reps, 16M records.  Each setting's output
is checked against the workgroup-tile kernels' bytes / the input columns.

    python tools/sweep_wave.py [--reps 10] [--rounds 2] [--sizes 0,2048,4096,8192]
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
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--sizes", default="0,1024,2048,3072,4096,6144,8192")
    ap.add_argument("--cases", default="quad16,all_kinds17,request53,response19")
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle
    import srpc_amd
    from srpc_amd import NUMBER, QUAD, SQUARE_METHOD, GpuPacker

    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    n = 1 << 24
    cases = {
        "quad16": (QUAD, b""),
        "all_kinds17": (srpc_amd.Schema.of("all_kinds", ("a", "bool"), ("b", "int8"), ("c", "char"),
                                           ("d", "int16"), ("e", "int32"), ("f", "int64")), b""),
        "request53": (NUMBER, srpc_amd.request_prefix(SQUARE_METHOD, "Number")),
        "response19": (NUMBER, srpc_amd.response_prefix(0, "Number")),
        "two_i16_i8": (srpc_amd.Schema.of("t", ("a", "int16"), ("b", "int8")), b""),
        "i8": (srpc_amd.Schema.of("t", ("a", "int8")), b""),
        "i16": (srpc_amd.Schema.of("t", ("a", "int16")), b""),
        "bool_i32": (srpc_amd.Schema.of("t", ("a", "bool"), ("b", "int32")), b""),
        "i32_i16": (srpc_amd.Schema.of("t", ("a", "int32"), ("b", "int16")), b""),
        "i64_i8": (srpc_amd.Schema.of("t", ("a", "int64"), ("b", "int8")), b""),
        "i64_i32_i16_i8": (srpc_amd.Schema.of("t", ("a", "int64"), ("b", "int32"), ("c", "int16"),
                                              ("d", "int8")), b""),
    }
    sizes = [int(x) for x in args.sizes.split(",")]
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(s)
    b.record(s)
    for name in args.cases.split(","):
        sch, pre = cases[name]
        p = GpuPacker(sch, pre)
        p.force_path(srpc_amd.SRPC_PATH_TILE)
        rng = np.random.default_rng(1)
        cols = [torch.from_numpy(rng.integers(0, 2 if k == oracle.BOOL else 256, n * oracle.KIND_SIZE[k],
                                              dtype=np.uint8)).to(dev) for k in sch.kinds]
        W = n * p.record_bytes
        wire = torch.empty(W + 16, dtype=torch.uint8, device=dev)
        ref = torch.empty(W + 16, dtype=torch.uint8, device=dev)
        back = [torch.empty_like(c) for c in cols]
        p.tune(wave_pack_bytes=0, wave_unpack_bytes=0)
        p.pack(cols, n, ref, stream=s)
        torch.cuda.synchronize()
        res = {}
        ok = {}
        for _ in range(args.rounds):
            for tb in sizes:
                p.tune(wave_pack_bytes=tb, wave_unpack_bytes=tb)
                wire.zero_()
                for c in back:
                    c.zero_()
                p.pack(cols, n, wire, stream=s)
                p.unpack(wire, W, n, back, stream=s)
                torch.cuda.synchronize()
                ok[tb] = bool(torch.equal(wire[:W], ref[:W]) and all(torch.equal(x, y) for x, y in zip(cols, back)))
                for d in ("pack", "unpack"):
                    for shape in ("same", "trip"):
                        for _ in range(2):
                            p.pack(cols, n, wire, stream=s)
                        for _ in range(args.reps):
                            if shape == "trip":
                                if d == "pack":
                                    p.unpack(wire, W, n, back, stream=s)
                                else:
                                    p.pack(cols, n, wire, stream=s)
                            srpc_amd.time_next_call(a, b)
                            if d == "pack":
                                p.pack(cols, n, wire, stream=s)
                            else:
                                p.unpack(wire, W, n, back, stream=s)
                            torch.cuda.synchronize()
                            res.setdefault((d, shape, tb), []).append(a.elapsed_time(b) * 1e3)
        alg = sum(c.numel() for c in cols) + W
        for (d, shape, tb), ts in sorted(res.items()):
            us = statistics.median(ts)
            print(f"{name:12s} {d:6s} {shape:4s} wave {tb:6d} {us:8.1f} us ({alg / us / 8e6:.3f})  ok={ok[tb]}",
                  flush=True)
        del cols, wire, back, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
