#!/usr/bin/env python3
"""Host-terminated legs (bench.py pcie_inclusive) over chunk counts and ring
depths, one MI355X: prints one JSON line per setting (pipelined ms per
direction, the link's one-way and duplex rates)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    from srpc_amd import QUAD, GpuPacker

    dev = torch.device("cuda:0")
    p = GpuPacker(QUAD)
    for chunks, depth in [(16, 3), (32, 3), (32, 4), (64, 4), (64, 6), (128, 6)]:
        r = bench.pcie_inclusive(p, 1 << 24, dev, reps=3, chunks=chunks, depth=depth)
        print(json.dumps({"chunks": chunks, "depth": depth, "pack_ms": r["pipelined"]["pack"]["ms"],
                          "unpack_ms": r["pipelined"]["unpack"]["ms"], "serial_pack_ms": r["serial"]["pack"]["ms"],
                          "link": r["link"], "verified": r["verified"]}), flush=True)


if __name__ == "__main__":
    main()
