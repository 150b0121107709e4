#!/usr/bin/env python3
"""Per-phase clock of the stream decoder's per-block kernels (sdx.hip built
with -DSRPC_SX_PHASES: build_ab/sx_phases.so, `python tools/ab_build.py
sx_phases=WORKTREE:SRPC_SX_PHASES`): thread 0 of every block adds the clock64()
cycles between its phase marks.  Prints, per stream_bench case, the mean
cycles per block of each phase of k_sx_spec (stage, speculate + walk, link,
table) and k_sx_decode (stage, chunk walk, link, chain + record list, fixed
fields, strings), and the kernel's resident blocks implied by its duration.

    SRPC_GPU_LIB=build_ab/sx_phases.so python tools/sx_phases.py [--only NAME]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SPEC = ["stage", "speculate+walk", "link", "chains+header"]
DEC = ["stage+state", "chunk walk", "link", "chain+list", "fixed fields", "strings"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import numpy as np
    import torch

    import oracle
    import srpc_amd
    from srpc_amd import GpuPacker, Schema
    from tests.streams import straddler_stream
    from tools.stream_bench import gen_random, gen_zero_heavy

    lib = srpc_amd._lib.lib()
    hook = lib.srpc_debug_sx_phases
    hook.argtypes, hook.restype = [ctypes.c_void_p, ctypes.c_uint64], ctypes.c_int
    dev = torch.device("cuda:0")
    S, I8, C8, I32 = oracle.STRING, oracle.INT8, oracle.CHAR, oracle.INT32
    cases = [("multiple_primitives_str0-64_4M", [I8, C8, oracle.INT64, S], 1 << 22, lambda k, n, r: gen_random(k, n, r, 64), b""),
             ("two_str_request_0-32_4M", [S, I32, S], 1 << 22, lambda k, n, r: gen_random(k, n, r, 32),
              srpc_amd.request_prefix("Svc_servicer::method", "TwoStr")),
             ("string_0-16_8M", [S], 1 << 23, lambda k, n, r: gen_random(k, n, r, 16), b""),
             ("string_0-1024_1M", [S], 1 << 20, lambda k, n, r: gen_random(k, n, r, 1024), b""),
             ("zh4_zero_heavy_4M", [I8, S, oracle.INT16, S], 1 << 22, gen_zero_heavy, b""),
             ("zh4_random_4M", [I8, S, oracle.INT16, S], 1 << 22, lambda k, n, r: gen_random(k, n, r, 24), b""),
             ("zh4_straddle_zero_long_1M", [I8, S, oracle.INT16, S], 1 << 20,
              lambda k, n, r: straddler_stream(n, r, (1, 6000), (65, 6000), "zero"), b""),
             ("zh4_straddle_heavy_long_1M", [I8, S, oracle.INT16, S], 1 << 20,
              lambda k, n, r: straddler_stream(n, r, (1100, 6000), (65, 6000), "heavy"), b"")]
    for name, kinds, n, gen, prefix in cases:
        if args.only not in name:
            continue
        rng = np.random.default_rng(7)
        cols, offs = gen(kinds, n, rng)
        p = GpuPacker(Schema("V", tuple((f"f{i}", k) for i, k in enumerate(kinds))), prefix)
        wire_h = oracle.pack(kinds, cols, n, prefix, list(offs))
        W = len(wire_h)
        wire = torch.empty(W + 16, dtype=torch.uint8, device=dev)
        wire[:W].copy_(torch.frombuffer(bytearray(wire_h), dtype=torch.uint8))
        outs = [torch.empty(W + 16 if k == S else n * oracle.KIND_SIZE[k] + 16, dtype=torch.uint8, device=dev)
                for k in kinds]
        ooffs = [torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev) if k == S else None for k in kinds]
        rec = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
        sb = p.var_stream_scratch_bytes(n, W)
        scr = torch.empty(sb + 256, dtype=torch.uint8, device=dev)
        sbase = scr.data_ptr() + (-scr.data_ptr()) % 256
        nb = (W + 8191) // 8192
        buf = torch.zeros(nb * 16, dtype=torch.int64, device=dev)
        for _ in range(2):
            p.unpack_var_stream(wire, W, n, rec, outs, ooffs, sbase, sb)
        torch.cuda.synchronize()
        assert hook(buf.data_ptr(), nb) == 0
        p.unpack_var_stream(wire, W, n, rec, outs, ooffs, sbase, sb)
        torch.cuda.synchronize()
        assert hook(None, 0) == 0
        b = buf.cpu().numpy().reshape(nb, 16).astype(np.float64)
        spec = b[:, 0:4]
        dec = b[:, 8:14]
        ran = dec.sum(1) > 0
        print(f"{name}: {nb} blocks, {int(ran.sum())} decoded")
        print("  k_sx_spec   " + "  ".join(f"{k} {v:8.0f}" for k, v in zip(SPEC, spec.mean(0))) +
              f"   total {spec.sum(1).mean():8.0f} cycles/block")
        print(f"  chunks whose first pick failed (plausible() loop): {b[:, 4].mean():.1f} per block")
        print(f"  landing scan per block: candidates {b[:, 5].mean():.1f}, ends past the window {b[:, 6].mean():.1f}, "
              f"slots {b[:, 7].mean():.2f} (blocks with any {np.mean(b[:, 7] > 0):.3f}, max {b[:, 7].max():.0f})")
        print("  k_sx_decode " + "  ".join(f"{k} {v:8.0f}" for k, v in zip(DEC, dec[ran].mean(0))) +
              f"   total {dec[ran].sum(1).mean():8.0f} cycles/block", flush=True)
        print(f"  decode fast path (entered at sF, one segment): {b[ran, 15].mean():.3f} of the blocks decoded",
              flush=True)
        nt = b[:, 14]
        print(f"  speculation segments per block: mean {nt.mean():.2f}, one {np.mean(nt == 1):.3f}, "
              f"two {np.mean(nt == 2):.3f}, more {np.mean(nt > 2):.3f}", flush=True)


if __name__ == "__main__":
    main()
