#!/usr/bin/env python3
"""Phase cycles of k_pack_var from a -DSRPC_PHASES build (tools/ab_build.py
name=REV:SRPC_PHASES, then SRPC_GPU_LIB=build_ab/name.so python tools/phases.py).
Thread 0 of each workgroup adds its clock64() deltas per phase; printed per tile."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
NAMES = ["tile_first load", "window load + barrier", "find_record", "segment walk", "store", "end barrier"]
STAGED = ["region table (lane 0)", "barrier 1", "staging loads", "barrier 2", "chunk table + barrier 3",
          "assemble + store", "-", "end barrier"]


def main():
    import numpy as np
    import torch

    import oracle
    from srpc_amd import GpuPacker, Schema, _lib

    dev = torch.device("cuda:0")
    kinds, n, maxlen = [oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING], 1 << 22, 64
    if len(sys.argv) > 1 and sys.argv[1] == "str1k":
        kinds, n, maxlen = [oracle.STRING], 1 << 20, 1024
    rng = np.random.default_rng(2)
    cols, offs = [], []
    for k in kinds:
        if k == oracle.STRING:
            lens = rng.integers(0, maxlen + 1, n).astype(np.uint64)
            o = np.zeros(n + 1, np.uint64)
            o[1:] = np.cumsum(lens)
            cols.append(torch.from_numpy(rng.integers(0, 256, int(o[-1]) + 1, dtype=np.uint8)).to(dev))
            offs.append(torch.from_numpy(o.view(np.uint8)).to(dev))
        else:
            dt = np.dtype(oracle.KIND_DTYPE[k])
            cols.append(torch.from_numpy(rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8)).to(dev))
            offs.append(None)
    fixed = sum(8 if k == oracle.STRING else oracle.KIND_SIZE[k] for k in kinds)
    total = n * fixed + sum(int(o.view(torch.int64)[-1].item()) for o in offs if o is not None)
    p = GpuPacker(Schema("V", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
    if os.environ.get("SRPC_PHASES_STAGED"):
        p.tune(var_kernel=1, var_tile=int(os.environ["SRPC_PHASES_STAGED"]))
    wire = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    rec = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
    sb = p.var_scratch_bytes(n, total)
    scratch = torch.empty(sb + 16, dtype=torch.uint8, device=dev)
    L = _lib.lib()
    fn = L.srpc_debug_phases
    fn.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    h = (C.c_uint64 * 8)()
    p.pack_var(cols, offs, n, wire, total, rec, scratch, sb)
    torch.cuda.synchronize()
    fn(h, 1)
    reps = 5
    for _ in range(reps):
        p.pack_var(cols, offs, n, wire, total, rec, scratch, sb)
    torch.cuda.synchronize()
    fn(h, 1)
    v = list(h)
    tiles = v[6]
    names = STAGED if os.environ.get("SRPC_PHASES_STAGED") else NAMES
    idx = [i for i, nm in enumerate(names) if nm != "-"]
    tot = sum(v[i] for i in idx)
    print(f"tiles {tiles / reps:.0f} per call, {tot / tiles:.0f} cycles per tile (thread 0 of each workgroup)")
    for i in idx:
        print(f"   {names[i]:24s} {v[i] / tiles:8.0f} cyc/tile  {100 * v[i] / tot:5.1f} %")


if __name__ == "__main__":
    main()
