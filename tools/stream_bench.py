#!/usr/bin/env python3
"""Index-free stream decode (srpc_gpu_unpack_var_stream) on one MI355X: the
whole call on the kernel clock (srpc_time_next_call: dispatch begin of the
call's first kernel to the end of its last), median of --reps, for random
string streams (the bench_paths VAR rows) and adversarial ones (zero-heavy
strings, records of zeros only: every phase parses), each checked first
against the oracle's cursor (rec_offs, columns, str_offs, chars).

Algorithmic bytes per call = wire read + every output written once: fixed
columns, chars, str_offs (8 B per record per string field) and rec_offs
(8 B per record).

    python tools/stream_bench.py [--reps 10] [--only NAME] [--out FILE.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def gen_random(kinds, n, rng, maxlen):
    import numpy as np

    import oracle
    cols, offs = [], []
    for k in kinds:
        if k == oracle.STRING:
            lens = rng.integers(0, maxlen + 1, n).astype(np.uint64)
            o = np.zeros(n + 1, np.uint64)
            o[1:] = np.cumsum(lens)
            cols.append(rng.integers(0, 256, int(o[-1]) + 1, dtype=np.uint8))
            offs.append(o)
        else:
            dt = np.dtype(oracle.KIND_DTYPE[k])
            cols.append(rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt))
            offs.append(None)
    return cols, offs


def gen_zero_heavy(kinds, n, rng, maxlen=24, p_empty=0.5, p_nonzero=0.05):
    import numpy as np

    import oracle
    cols, offs = [], []
    for k in kinds:
        if k == oracle.STRING:
            lens = rng.integers(0, maxlen, n).astype(np.uint64)
            lens[rng.random(n) < p_empty] = 0
            o = np.zeros(n + 1, np.uint64)
            o[1:] = np.cumsum(lens)
            c = np.zeros(max(1, int(o[-1])), np.uint8)
            c[rng.random(c.size) < p_nonzero] = 7
            cols.append(c)
            offs.append(o)
        else:
            cols.append(np.zeros(n, np.dtype(oracle.KIND_DTYPE[k])))
            offs.append(None)
    return cols, offs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default=None)
    ap.add_argument("--tables", type=int, default=0,
                    help="srpc_debug_stream_tables bits (sdx.hip): 1 sF-only tables, 2 empty tables, "
                         "4 the exact speculation filter, 8 no repair pass")
    args = ap.parse_args()

    import numpy as np
    import torch

    import oracle
    import srpc_amd
    from srpc_amd import GpuPacker, Schema

    if args.tables:
        import ctypes
        th = srpc_amd._lib.lib().srpc_debug_stream_tables
        th.argtypes, th.restype = [ctypes.c_int], ctypes.c_int
        th(args.tables)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    rows = []

    def timeit(fn):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
        for a, b in ev:
            a.record(s)
            b.record(s)
        fn()
        torch.cuda.synchronize()
        for a, b in ev:
            srpc_amd.time_next_call(a, b)
            fn()
        torch.cuda.synchronize()
        t = sorted(a.elapsed_time(b) for a, b in ev)
        return t[len(t) // 2] / 1e3

    def u8(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)

    def case(name, kinds, n, gen, prefix=b""):
        if args.only not in name:
            return
        rng = np.random.default_rng(7)
        cols, offs = gen(kinds, n, rng)
        p = GpuPacker(Schema("V", tuple((f"f{i}", k) for i, k in enumerate(kinds))), prefix)
        wire_h = oracle.pack(kinds, cols, n, prefix, list(offs))
        W = len(wire_h)
        wire = torch.empty(W + 16, dtype=torch.uint8, device=dev)
        wire[:W].copy_(torch.frombuffer(bytearray(wire_h), dtype=torch.uint8))
        outs = [torch.empty(W + 16 if k == oracle.STRING else n * oracle.KIND_SIZE[k] + 16, dtype=torch.uint8,
                            device=dev) for k in kinds]
        ooffs = [torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev) if k == oracle.STRING else None
                 for k in kinds]
        rec = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
        sb = p.var_stream_scratch_bytes(n, W)
        scr = torch.empty(sb + 256, dtype=torch.uint8, device=dev)
        sbase = scr.data_ptr() + (-scr.data_ptr()) % 256
        st = torch.zeros(16, dtype=torch.uint8, device=dev)
        p.unpack_var_stream(wire, W, n, rec, outs, ooffs, sbase, sb, st, stream=s)
        torch.cuda.synchronize()
        rc, ocols, ooffs_h, _, _ = oracle.unpack(kinds, wire_h, n, prefix)
        ok = rc == oracle.ORC_OK
        fixed = len(prefix) + sum(8 if k == oracle.STRING else oracle.KIND_SIZE[k] for k in kinds)
        want_rec = np.full(n + 1, 0, np.uint64)
        sizes = np.full(n, fixed, np.uint64)
        for k, o in zip(kinds, offs):
            if k == oracle.STRING:
                sizes += np.diff(o)
        want_rec[1:] = np.cumsum(sizes)
        ok = ok and np.array_equal(rec.cpu().numpy().view(np.uint64), want_rec)
        for k, o, so, oc, oo in zip(kinds, outs, ooffs, ocols, ooffs_h):
            if k == oracle.STRING:
                got_o = so.cpu().numpy().view(np.uint64)
                ok = ok and np.array_equal(got_o, oo)
                ok = ok and o[:int(got_o[n])].cpu().numpy().tobytes() == oc.tobytes()
            else:
                ok = ok and o[:n * oracle.KIND_SIZE[k]].cpu().numpy().tobytes() == oc.tobytes()
        st_h = st.cpu().numpy()
        reserved = int(st_h[4:8].view(np.uint32)[0])
        t = timeit(lambda: p.unpack_var_stream(wire, W, n, rec, outs, ooffs, sbase, sb, stream=s))
        col_bytes = sum(c.nbytes for c, k in zip(cols, kinds) if k != oracle.STRING)
        str_bytes = W - n * fixed
        nstr = sum(k == oracle.STRING for k in kinds)
        alg = W + col_bytes + str_bytes + 8 * (n + 1) * nstr + 8 * (n + 1)
        row = {"case": name, "records": n, "wire_bytes": W, "alg_bytes": alg, "us": round(t * 1e6, 2),
               "GBps": round(alg / t / 1e9, 1), "frac": round(alg / t / 8e12, 4), "parity_ok": bool(ok),
               "blocks": (W + 8191) // 8192, "walk_waves": reserved >> 8, "diag_bits": reserved & 15,
               "off_primary": bool(reserved & 1), "walked_miss": bool(reserved & 2), "repaired": bool(reserved & 4), "exit_overflow": bool(reserved & 8)}
        rows.append(row)
        print(f'{name:36s} {n:9d} rec {W / 2**20:8.1f} MiB  {row["us"]:9.1f} us  {row["GBps"]:7.1f} GB/s '
              f'({row["frac"]:.3f})  parity={ok}  off_primary={row["off_primary"]} walked={row["walked_miss"]} '
              f'repaired={row["repaired"]} overflow={row["exit_overflow"]} '
              f'walk_waves {row["walk_waves"]}/{row["blocks"]} blocks',
              flush=True)

    S, I8, C8, I16, I32, I64 = oracle.STRING, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64
    mp = [I8, C8, I64, S]
    case("multiple_primitives_str0-64_4M", mp, 1 << 22, lambda k, n, r: gen_random(k, n, r, 64))
    case("string_0-1024_1M", [S], 1 << 20, lambda k, n, r: gen_random(k, n, r, 1024))
    case("string_0-16_8M", [S], 1 << 23, lambda k, n, r: gen_random(k, n, r, 16))
    case("string_0-32_4M", [S], 1 << 22, lambda k, n, r: gen_random(k, n, r, 32))
    case("two_str_request_0-32_4M", [S, I32, S], 1 << 22, lambda k, n, r: gen_random(k, n, r, 32),
         srpc_amd.request_prefix("Svc_servicer::method", "TwoStr"))
    zh = [I8, S, I16, S]
    case("zh4_random_1M", zh, 1 << 20, lambda k, n, r: gen_random(k, n, r, 24))
    case("zh4_zero_heavy_1M", zh, 1 << 20, gen_zero_heavy)
    case("zh4_random_4M", zh, 1 << 22, lambda k, n, r: gen_random(k, n, r, 24))
    case("zh4_zero_heavy_4M", zh, 1 << 22, gen_zero_heavy)
    case("multiple_primitives_zeros_4M", mp, 1 << 22,
         lambda k, n, r: gen_zero_heavy(k, n, r, maxlen=1, p_empty=1.0, p_nonzero=0.0))
    # a record straddling EVERY 8 KiB boundary, ending
    # past the block's window (tests/streams.py)
    from tests.streams import straddler_stream
    case("zh4_straddle_zero_4M", zh, 1 << 22, lambda k, n, r: straddler_stream(n, r, (1, 960), (65, 1000), "zero"))
    case("zh4_straddle_zero_long_4M", zh, 1 << 22,
         lambda k, n, r: straddler_stream(n, r, (1, 6000), (65, 6000), "zero"))
    case("zh4_straddle_heavy_4M", zh, 1 << 22, lambda k, n, r: straddler_stream(n, r, (1, 900), (65, 100), "heavy"))
    # the residual: zero-heavy straddlers that start more than kPre before the boundary
    case("zh4_straddle_heavy_long_256K", zh, 1 << 18,
         lambda k, n, r: straddler_stream(n, r, (1100, 4000), (65, 1000), "heavy"))
    # (its random counterpart: the same schema and record count)
    case("zh4_random_256K", zh, 1 << 18, lambda k, n, r: gen_random(k, n, r, 24))
    case("zh4_straddle_heavy_long_4M", zh, 1 << 22,
         lambda k, n, r: straddler_stream(n, r, (1100, 6000), (65, 6000), "heavy"))
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
