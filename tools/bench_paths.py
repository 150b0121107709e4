#!/usr/bin/env python3
"""Throughput of every kernel family on representative schemas (one MI355X).

For each case: pack and unpack of N records through the C ABI, timed on the
kernel clock of srpc_time_next_call (dispatch begin of the call's first
kernel to end of its last; median of R reps after warm-up), reported
as algorithmic GB/s (columns + wire bytes moved once) and fraction of the
8 TB/s HBM3E peak.  Every case is first checked bit-exact against the CPU
oracle on a 4096-record prefix of the same inputs.

    python tools/bench_paths.py [--reps 20] [--out gpurun_out/paths.json]
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="", help="substring filter on case names")
    ap.add_argument("--var-kernel", default="", help="VAR cases: comma list of pack kernels to time "
                    "(1 record tiles, 0 scan + walk; default: the plan's default)")
    ap.add_argument("--var-caps", default="", help="VAR record tiles: IMAGE:CHARS bytes (default: the plan's)")
    ap.add_argument("--rec-ab", action="store_true",
                    help="fixed cases: also time the generic TILE kernels (rec_kernel=0) beside the default")
    ap.add_argument("--no-stream", dest="stream", action="store_false",
                    help="VAR cases: skip the index-free stream decode timing")
    args = ap.parse_args()

    import numpy as np
    import torch

    import oracle
    import srpc_amd
    from srpc_amd import NUMBER, QUAD, SQUARE_METHOD, GpuPacker, Schema

    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    rows = []

    def timeit(fn):
        for _ in range(3):
            fn()
        ts = []
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(s)
        b.record(s)
        for _ in range(args.reps):
            # kernel clock: the call's first kernel begin -> last kernel end
            srpc_amd.time_next_call(a, b)
            fn()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) / 1e3)
        return statistics.median(ts)

    def t_u8(a):
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(dev)

    def fixed_case(name, sch, n, prefix=b"", path=None):
        if args.only not in name:
            return
        p = GpuPacker(sch, prefix)
        if path:
            p.force_path(path)
        rng = np.random.default_rng(1)
        cols = []
        for k in sch.kinds:
            dt = np.dtype(oracle.KIND_DTYPE[k])
            c = rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt)
            cols.append((c & 1).astype(np.uint8) if k == oracle.BOOL else c)
        dcols = [t_u8(c) for c in cols]
        wire = torch.empty(n * p.record_bytes + 16, dtype=torch.uint8, device=dev)
        back = [torch.empty_like(c) for c in dcols]
        p.pack(dcols, n, wire, stream=s)
        torch.cuda.synchronize()
        m = 4096
        ok = wire[: m * p.record_bytes].cpu().numpy().tobytes() == oracle.pack(
            sch.kinds, [c[:m] for c in cols], m, prefix)
        col_bytes = sum(c.nbytes for c in cols)
        alg = col_bytes + n * p.record_bytes
        tp = timeit(lambda: p.pack(dcols, n, wire, stream=s))
        tu = timeit(lambda: p.unpack(wire, n * p.record_bytes, n, back, stream=s))
        ok = ok and all(torch.equal(a, b) for a, b in zip(dcols, back))
        generic = {}
        if args.rec_ab and p.path == 2:
            p.tune(rec_kernel=0)
            gp = timeit(lambda: p.pack(dcols, n, wire, stream=s))
            gu = timeit(lambda: p.unpack(wire, n * p.record_bytes, n, back, stream=s))
            p.tune(rec_kernel=2)
            rp = timeit(lambda: p.pack(dcols, n, wire, stream=s))
            ru = timeit(lambda: p.unpack(wire, n * p.record_bytes, n, back, stream=s))
            p.tune(rec_kernel=1)
            generic = {"generic_pack_frac": round(alg / gp / 8e12, 4), "generic_unpack_frac": round(alg / gu / 8e12, 4),
                       "rec_pack_frac": round(alg / rp / 8e12, 4), "rec_unpack_frac": round(alg / ru / 8e12, 4)}
        rows.append({"case": name, "path": {1: "dword", 2: "tile", 3: "var"}[p.path], "records": n,
                     "record_bytes": p.record_bytes, "alg_bytes": alg, "pack_us": round(tp * 1e6, 2),
                     "unpack_us": round(tu * 1e6, 2), "pack_GBps": round(alg / tp / 1e9, 1),
                     "unpack_GBps": round(alg / tu / 1e9, 1), "pack_frac": round(alg / tp / 8e12, 4),
                     "unpack_frac": round(alg / tu / 8e12, 4), "parity_ok": bool(ok), **generic})

    def aos_case(name, sch, n, vptr=True):
        """Records as C-aligned structs behind an 8-byte vtable slot (a C++
        std::vector<T> of srpc messages copied to the device; vptr=False: a
        plain struct): srpc_gpu_pack_aos / unpack_aos.  Algorithmic bytes: the
        whole struct array (read by pack, written by unpack) + the wire."""
        if args.only not in name:
            return
        p = GpuPacker(sch)
        fmts = ([np.uint64] if vptr else []) + [np.dtype(oracle.KIND_DTYPE[k]) for k in sch.kinds]
        dt = np.dtype({"names": (["_v"] if vptr else []) + [f"f{i}" for i in range(len(sch.kinds))], "formats": fmts},
                      align=True)
        rng = np.random.default_rng(3)
        recs = rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt)
        for i, k in enumerate(sch.kinds):
            if k == oracle.BOOL:
                recs[f"f{i}"] &= 1
        offs = [dt.fields[f"f{i}"][1] for i in range(len(sch.kinds))]
        drecs = t_u8(recs)
        back = torch.empty_like(drecs)
        wire = torch.empty(n * p.record_bytes + 16, dtype=torch.uint8, device=dev)
        p.pack_aos(drecs, dt.itemsize, offs, n, wire, stream=s)
        torch.cuda.synchronize()
        m = 4096
        ok = wire[: m * p.record_bytes].cpu().numpy().tobytes() == oracle.pack(
            sch.kinds, [np.ascontiguousarray(recs[f"f{i}"][:m]) for i in range(len(sch.kinds))], m)
        alg = n * dt.itemsize + n * p.record_bytes
        tp = timeit(lambda: p.pack_aos(drecs, dt.itemsize, offs, n, wire, stream=s))
        back.copy_(drecs)
        tu = timeit(lambda: p.unpack_aos(wire, n * p.record_bytes, n, back, dt.itemsize, offs, stream=s))
        ok = ok and torch.equal(back, drecs)
        fill_row = {}
        if hasattr(p, "unpack_aos_fill"):
            # into fresh objects (srpc_gpu_unpack_aos_fill): non-field bytes from
            # record 0's image; the fields must equal the source's
            fill = recs[:1].view(np.uint8).tobytes()
            back.zero_()
            tf = timeit(lambda: p.unpack_aos_fill(wire, n * p.record_bytes, n, back, dt.itemsize, offs, fill, stream=s))
            got = back[: m * dt.itemsize].cpu().numpy().view(dt)
            ok = ok and all(np.array_equal(got[f"f{i}"], recs[f"f{i}"][:m]) for i in range(len(sch.kinds)))
            if vptr:
                ok = ok and bool(np.all(got["_v"] == recs["_v"][0]))
            fill_row = {"unpack_fill_us": round(tf * 1e6, 2), "unpack_fill_frac": round(alg / tf / 8e12, 4)}
        rows.append({"case": name, "path": "aos", "records": n, "record_bytes": p.record_bytes,
                     "struct_bytes": dt.itemsize, "alg_bytes": alg, "pack_us": round(tp * 1e6, 2),
                     "unpack_us": round(tu * 1e6, 2), "pack_GBps": round(alg / tp / 1e9, 1),
                     "unpack_GBps": round(alg / tu / 1e9, 1), "pack_frac": round(alg / tp / 8e12, 4),
                     "unpack_frac": round(alg / tu / 8e12, 4), "parity_ok": bool(ok), **fill_row})

    def var_case(name, kinds, n, maxlen, prefix=b""):
        if args.only not in name:
            return
        sch = Schema("V", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
        p = GpuPacker(sch, prefix)
        rng = np.random.default_rng(2)
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
        fixed = len(prefix) + sum(8 if k == oracle.STRING else oracle.KIND_SIZE[k] for k in kinds)
        total = n * fixed + int(sum(int(o[-1]) for o in offs if o is not None))
        dcols = [t_u8(c) for c in cols]
        doffs = [t_u8(o) if o is not None else None for o in offs]
        wire = torch.empty(total + 16, dtype=torch.uint8, device=dev)
        rec = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
        sb = p.var_scratch_bytes(n, total)
        scratch = torch.empty(sb + 16, dtype=torch.uint8, device=dev)
        outs = [torch.empty(total + 16 if k == oracle.STRING else n * oracle.KIND_SIZE[k] + 16,
                            dtype=torch.uint8, device=dev) for k in kinds]
        ooffs = [torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev) if k == oracle.STRING else None
                 for k in kinds]
        want = oracle.pack(kinds, cols, n, prefix, list(offs))
        col_bytes = sum(c.nbytes for c, k in zip(cols, kinds) if k != oracle.STRING)
        str_bytes = total - n * fixed
        alg = col_bytes + str_bytes + 8 * (n + 1) * sum(k == oracle.STRING for k in kinds) + total
        if args.var_caps:
            ib, cb = (int(x) for x in args.var_caps.split(":"))
            p.tune(var_image_bytes=ib, var_chars_bytes=cb)
        kernels = [int(k) for k in args.var_kernel.split(",") if k] or [None]
        for vk in kernels:
            label = name if vk is None else f"{name}_k{vk}"
            if vk is not None:
                p.tune(var_kernel=vk)
            wire.fill_(0)
            p.pack_var(dcols, doffs, n, wire, total, rec, scratch, sb, stream=s)
            torch.cuda.synchronize()
            ok = wire[:total].cpu().numpy().tobytes() == want
            tp = timeit(lambda: p.pack_var(dcols, doffs, n, wire, total, rec, scratch, sb, stream=s))
            tu = timeit(lambda: p.unpack_var(wire, total, n, rec, outs, ooffs, scratch, sb, stream=s))
            row = {"case": label, "path": "var", "records": n, "wire_bytes": total, "alg_bytes": alg,
                   "pack_us": round(tp * 1e6, 2), "unpack_us": round(tu * 1e6, 2),
                   "pack_GBps": round(alg / tp / 1e9, 1), "unpack_GBps": round(alg / tu / 1e9, 1),
                   "pack_frac": round(alg / tp / 8e12, 4), "unpack_frac": round(alg / tu / 8e12, 4),
                   "parity_ok": bool(ok)}
            if sum(k == oracle.STRING for k in kinds) > 1:
                # several string fields: the unpack with the batch's tile table
                # (srpc_gpu_unpack_var_tiled, ABI 6; the table from the pack's
                # own input offsets), checked against the look-back unpack
                tw = p.var_tile_table_words(n)
                table = torch.empty(8 * tw + 16, dtype=torch.uint8, device=dev)
                p.var_tile_table(doffs, n, table, stream=s)
                p.unpack_var(wire, total, n, rec, outs, ooffs, scratch, sb, stream=s)
                torch.cuda.synchronize()
                ref = [o.clone() for o in outs], [o.clone() if o is not None else None for o in ooffs]
                for o in outs:
                    o.fill_(0)
                tt = timeit(lambda: p.unpack_var_tiled(wire, total, n, rec, table, outs, ooffs, scratch, sb,
                                                       stream=s))
                torch.cuda.synchronize()
                # the bytes the batch owns (the columns' slack is nobody's)
                same = True
                for k, a_, b_, oa, ob in zip(kinds, outs, ref[0], ooffs, ref[1]):
                    if k == oracle.STRING:
                        same = same and torch.equal(oa, ob)
                        used = int(ob[-8:].cpu().numpy().view(np.uint64)[0]) if n else 0
                    else:
                        used = n * oracle.KIND_SIZE[k]
                    same = same and torch.equal(a_[:used], b_[:used])
                row["tiled_ok"] = bool(same)
                row["parity_ok"] = row["parity_ok"] and same
                row.update({"unpack_tiled_us": round(tt * 1e6, 2), "unpack_tiled_frac": round(alg / tt / 8e12, 4)})
            if args.stream:
                # the same wire decoded with NO record index (srpc_gpu_unpack_var_stream),
                # the index rebuilt on the device and written out (8 B per record more)
                ssb = p.var_stream_scratch_bytes(n, total)
                sscr = torch.empty(ssb + 256, dtype=torch.uint8, device=dev)
                sbase = sscr.data_ptr() + (-sscr.data_ptr()) % 256
                rec2 = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
                ts = timeit(lambda: p.unpack_var_stream(wire, total, n, rec2, outs, ooffs, sbase, ssb, stream=s))
                torch.cuda.synchronize()
                row["stream_ok"] = bool(torch.equal(rec2, rec))
                row["parity_ok"] = row["parity_ok"] and row["stream_ok"]
                salg = alg + 8 * (n + 1)
                row.update({"stream_us": round(ts * 1e6, 2), "stream_frac": round(salg / ts / 8e12, 4)})
            rows.append(row)

    N = 1 << 24
    fixed_case("quad_dword_16M", QUAD, N)
    fixed_case("quad_tile_16M", QUAD, N, path=srpc_amd.SRPC_PATH_TILE)
    fixed_case("number_body_16M", NUMBER, N)
    fixed_case("all_kinds_17B_16M", Schema.of("all_kinds", ("a", "bool"), ("b", "int8"), ("c", "char"),
                                              ("d", "int16"), ("e", "int32"), ("f", "int64")), N)
    fixed_case("square_request_53B_16M", NUMBER, N, srpc_amd.request_prefix(SQUARE_METHOD, "Number"))
    fixed_case("square_response_19B_16M", NUMBER, N, srpc_amd.response_prefix(0, "Number"))
    two = Schema.of("TwoNumbers", ("left", "int32"), ("right", "int32"))
    fixed_case("add_request_58B_16M", two, N, srpc_amd.request_prefix("Calculator_servicer::add", "TwoNumbers"))
    fixed_case("subtract_request_63B_16M", two, N,
               srpc_amd.request_prefix("Calculator_servicer::subtract", "TwoNumbers"))
    fixed_case("two_numbers_response_23B_16M", two, N, srpc_amd.response_prefix(0, "TwoNumbers"))
    aos_case("quad_aos_16M", QUAD, N)
    aos_case("quad_aos_plain_16M", QUAD, N, vptr=False)
    aos_case("all_kinds_aos_16M", Schema.of("all_kinds", ("a", "bool"), ("b", "int8"), ("c", "char"),
                                            ("d", "int16"), ("e", "int32"), ("f", "int64")), N)
    var_case("multiple_primitives_str0-64_4M", [oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING],
             1 << 22, 64)
    var_case("string_0-1024_1M", [oracle.STRING], 1 << 20, 1024)
    var_case("string_0-16_8M", [oracle.STRING], 1 << 23, 16)
    var_case("string_0-32_4M", [oracle.STRING], 1 << 22, 32)
    var_case("two_str_request_0-32_4M", [oracle.STRING, oracle.INT32, oracle.STRING], 1 << 22, 32,
             srpc_amd.request_prefix("Svc_servicer::method", "TwoStr"))
    txt = json.dumps(rows, indent=1)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(txt)
    for r in rows:
        extra = f'  stream {r["stream_us"]:8.1f} us ({r["stream_frac"]:.3f})' if "stream_us" in r else ""
        for k in ("tiled_ok", "stream_ok"):
            if k in r and not r[k]:
                extra += f"  {k}=False"
        if "unpack_tiled_us" in r:
            extra += f'  unpack_tiled {r["unpack_tiled_us"]:8.1f} us ({r["unpack_tiled_frac"]:.3f})'
        if "unpack_fill_us" in r:
            extra += f'  unpack_fill {r["unpack_fill_us"]:8.1f} us ({r["unpack_fill_frac"]:.3f})'
        if "generic_pack_frac" in r:
            extra += (f'  generic ({r["generic_pack_frac"]:.3f} / {r["generic_unpack_frac"]:.3f})'
                      f'  rec ({r["rec_pack_frac"]:.3f} / {r["rec_unpack_frac"]:.3f})')
        print(f'{r["case"]:34s} {r["path"]:5s} pack {r["pack_us"]:9.1f} us {r["pack_GBps"]:7.1f} GB/s '
              f'({r["pack_frac"]:.3f})  unpack {r["unpack_us"]:9.1f} us {r["unpack_GBps"]:7.1f} GB/s '
              f'({r["unpack_frac"]:.3f})  parity={r["parity_ok"]}{extra}')


if __name__ == "__main__":
    main()
