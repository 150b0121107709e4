#!/usr/bin/env python3
"""Per-phase clock of the VAR record-tile unpack kernel (a library built with
-DSRPC_PHASES, given by SRPC_GPU_LIB): thread 0 of every workgroup adds the
clock64() cycles between its phase markers; printed per workgroup.

    SRPC_GPU_LIB=build_ab/p.so python tools/var_phases.py [--case two_str|multiple]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="two_str")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--tiled", action="store_true", help="time srpc_gpu_unpack_var_tiled (the tile table) instead")
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle
    import srpc_amd
    from srpc_amd import Schema, _lib
    from tests.test_gpu_parity import _random_string_batch, dev, empty, _dev_u64

    L = _lib.lib()
    fn = L.srpc_debug_phases
    fn.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    if args.case == "two_str":
        kinds, n, maxlen = [oracle.STRING, oracle.INT32, oracle.STRING], 1 << 21, 32
        prefix = srpc_amd.request_prefix("Svc_servicer::two", "Two")
    else:
        kinds, n, maxlen = [oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING], 1 << 21, 64
        prefix = b""
    rng = np.random.default_rng(5)
    cols, offs = _random_string_batch(kinds, n, rng, maxlen)
    p = srpc_amd.GpuPacker(Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds))), prefix)
    wire = oracle.pack(kinds, cols, n, p.prefix, list(offs))
    fixed = len(p.prefix) + sum(8 if k == oracle.STRING else oracle.KIND_SIZE[k] for k in kinds)
    sizes = np.full(n, fixed, np.uint64)
    for k, o in zip(kinds, offs):
        if k == oracle.STRING:
            sizes += np.diff(o.astype(np.uint64))
    rec = np.zeros(n + 1, np.uint64)
    rec[1:] = np.cumsum(sizes)
    w = dev(np.frombuffer(wire, np.uint8))
    W = len(wire)
    outs, soffs = [], []
    for k in kinds:
        if k == oracle.STRING:
            outs.append(empty(W + 16))
            soffs.append(empty(8 * (n + 1)))
        else:
            outs.append(empty(n * oracle.KIND_SIZE[k] + 16))
            soffs.append(None)
    sb = p.var_scratch_bytes(n, W)
    scratch = empty(sb + 16)
    drec = _dev_u64(rec)
    h = (ctypes.c_uint64 * 8)()
    for _ in range(2):
        p.unpack_var(w, W, n, drec, outs, soffs, scratch, sb, None)
    torch.cuda.synchronize()
    if args.tiled:
        table = empty(8 * p.var_tile_table_words(n) + 16)
        p.var_tile_table(soffs, n, table)
        torch.cuda.synchronize()

        def call():
            p.unpack_var_tiled(w, W, n, drec, table, outs, soffs, scratch, sb, None)
    else:
        def call():
            p.unpack_var(w, W, n, drec, outs, soffs, scratch, sb, None)
    call()
    torch.cuda.synchronize()
    fn(h, 1)
    for _ in range(args.reps):
        call()
    torch.cuda.synchronize()
    fn(h, 1)
    wgs = h[6] or 1
    names = ["table", "dma", "parse", "scan+base", "build", "store"]
    tot = sum(h[i] for i in range(6))
    print(f"{args.case}{' tiled' if args.tiled else ''}: {wgs} workgroups over {args.reps} calls, cycles per workgroup:")
    for i, nm in enumerate(names):
        print(f"  {nm:10s} {h[i] / wgs:10.0f}  ({100 * h[i] / max(tot, 1):5.1f} %)")
    print(f"  {'total':10s} {tot / wgs:10.0f}")


if __name__ == "__main__":
    main()
