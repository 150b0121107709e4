#!/usr/bin/env python3
"""Per-phase clock of the single-pass stream decode (a library built with
-DSRPC_STREAM_PHASES, given by SRPC_GPU_LIB): thread 0 of every block adds the
clock64() cycles between its phase marks, plus look-back counters; printed
per block (cycles and us at 2.4 GHz).

    python tools/ab_build.py ph=WORKTREE:SRPC_STREAM_PHASES
    SRPC_GPU_LIB=build_ab/ph.so python tools/stream_phases.py [--only NAME]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PHASES = ["stage", "speculate", "segments", "cand+AGG", "lookback(a)", "lookback(b)", "own+INC",
          "record walk+table", "fixed out", "chars out"]
SD_PHASES = ["stage", "speculate+walk", "segments+scans", "AGG chain", "look-back", "own+INC", "table",
             "fixed out", "chars out", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--sdec", action="store_true", help="the speculative decode (sdec.hip, -DSRPC_SDEC_PHASES)")
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle
    import srpc_amd
    from srpc_amd import GpuPacker, Schema, _lib
    from tools.stream_bench import gen_random, gen_zero_heavy

    fn = _lib.lib().srpc_debug_sdec_phases if args.sdec else _lib.lib().srpc_debug_stream_phases
    hook = _lib.lib().srpc_debug_stream_force_single
    hook.argtypes, hook.restype = [ctypes.c_int], ctypes.c_int
    hook(4 if args.sdec else 2)  # the speculative decode never giving up / the bounded pass alone
    names = SD_PHASES if args.sdec else PHASES
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
    dev = torch.device("cuda:0")
    S, I8, C8, I16, I32, I64 = oracle.STRING, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64
    cases = [("multiple_primitives_str0-64_4M", [I8, C8, I64, S], 1 << 22, lambda k, n, r: gen_random(k, n, r, 64)),
             ("string_0-16_8M", [S], 1 << 23, lambda k, n, r: gen_random(k, n, r, 16)),
             ("two_str_0-32_4M", [S, I32, S], 1 << 22, lambda k, n, r: gen_random(k, n, r, 32)),
             ("zh4_zero_heavy_4M", [I8, S, I16, S], 1 << 22, gen_zero_heavy),
             ("multiple_primitives_zeros_4M", [I8, C8, I64, S], 1 << 22,
              lambda k, n, r: gen_zero_heavy(k, n, r, maxlen=1, p_empty=1.0, p_nonzero=0.0))]
    for name, kinds, n, gen in cases:
        if args.only not in name:
            continue
        cols, offs = gen(kinds, n, np.random.default_rng(7))
        p = GpuPacker(Schema("V", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
        wire_h = oracle.pack(kinds, cols, n, b"", list(offs))
        W = len(wire_h)
        wire = torch.frombuffer(bytearray(wire_h), dtype=torch.uint8).to(dev)
        outs = [torch.empty(W + 16 if k == S else n * oracle.KIND_SIZE[k] + 16, dtype=torch.uint8, device=dev)
                for k in kinds]
        ooffs = [torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev) if k == S else None for k in kinds]
        rec = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
        sb = p.var_stream_scratch_bytes(n, W)
        scr = torch.empty(sb + 256, dtype=torch.uint8, device=dev)
        base = scr.data_ptr() + (-scr.data_ptr()) % 256
        p.unpack_var_stream(wire, W, n, rec, outs, ooffs, base, sb)
        torch.cuda.synchronize()
        nb = (W + 8191) // 8192
        buf = torch.zeros(16 * nb, dtype=torch.int64, device=dev)
        fn(buf.data_ptr(), nb)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            p.unpack_var_stream(wire, W, n, rec, outs, ooffs, base, sb)
        e1.record()
        torch.cuda.synchronize()
        call_us = e0.elapsed_time(e1) * 1e3 / args.reps
        fn(None, 0)
        per = buf.view(nb, 16).cpu().numpy().astype(np.float64)
        h = per.sum(axis=0)
        h[10] = per[:, 10].sum()
        blocks = max(1, h[10])
        print(f"{name}: {int(blocks) // args.reps} blocks per call, {h[15] / blocks:.3f} write outputs; "
              f"look-back(a)+(b) us per block: p50 {np.median(per[:, 4] + per[:, 5]) / args.reps / 2400:.1f} "
              f"p90 {np.percentile(per[:, 4] + per[:, 5], 90) / args.reps / 2400:.1f}")
        tot = sum(h[i] for i in range(10))
        life = tot / blocks / 2400
        print(f"  call {call_us:.1f} us; mean block lifetime {life:.1f} us -> {life * blocks / args.reps / call_us:.0f} "
              f"blocks resident on average")
        for i, nm in enumerate(names):
            cyc = h[i] / blocks
            print(f"  {nm:20s} {cyc:10.0f} cycles/block {cyc / 2400:8.2f} us  {100 * h[i] / max(tot, 1):5.1f} %")
        if args.sdec:
            print(f"  misses {h[12] / args.reps:.0f} per call; look-back depth {h[13] / blocks:.1f} blocks, "
                  f"windows past the first {h[11] / blocks:.2f}, INC waits {h[14] / blocks:.3f} per block", flush=True)
            continue
        print(f"  look-back: depth {h[13] / blocks:.1f} blocks, windows {h[11] / blocks:.2f}, "
              f"fast windows {h[14] / max(h[11], 1):.3f}, slow steps {h[12] / blocks:.2f} per block", flush=True)


if __name__ == "__main__":
    main()
