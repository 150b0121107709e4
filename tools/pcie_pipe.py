#!/usr/bin/env python3
"""Host-terminated Quad pack (pinned host columns -> H2D -> pack -> D2H wire):
one stream vs chunked pipelines over several streams.  Prints ms and wire GiB/s
per (chunks, streams); chunk i's three steps stay ordered on stream i % S."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from srpc_amd import QUAD, GpuPacker

    dev = torch.device("cuda:0")
    n = 1 << 24
    rb = 16
    p = GpuPacker(QUAD)
    cols = [torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev) for _ in range(4)]
    wire = torch.empty(n * rb, dtype=torch.uint8, device=dev)
    hcols = [c.cpu().pin_memory() for c in cols]
    hwire = torch.empty(n * rb, dtype=torch.uint8).pin_memory()
    main_s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def run(chunks, nstreams, reps=3):
        streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
        per = n // chunks
        torch.cuda.synchronize()
        e0.record(main_s)
        for st in streams:
            st.wait_event(e0)
        for _ in range(reps):
            for i in range(chunks):
                st = streams[i % nstreams]
                lo, hi = i * per, (i + 1) * per
                with torch.cuda.stream(st):
                    dc = [c[lo:hi] for c in cols]
                    for h, c in zip(hcols, dc):
                        c.copy_(h[lo:hi], non_blocking=True)
                    p.pack(dc, per, wire[lo * rb:hi * rb], stream=st)
                    hwire[lo * rb:hi * rb].copy_(wire[lo * rb:hi * rb], non_blocking=True)
        for st in streams:
            ev = torch.cuda.Event()
            ev.record(st)
            main_s.wait_event(ev)
        e1.record(main_s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"chunks {chunks:3d} streams {nstreams}: {ms:7.3f} ms  {n * rb / 2**30 / (ms / 1e3):6.2f} GiB/s wire",
              flush=True)

    # H2D alone and D2H alone, for the link's one-way rates
    torch.cuda.synchronize()
    e0.record(main_s)
    for h, c in zip(hcols, cols):
        c.copy_(h, non_blocking=True)
    e1.record(main_s)
    torch.cuda.synchronize()
    print(f"H2D 256 MiB alone: {e0.elapsed_time(e1):.3f} ms")
    e0.record(main_s)
    hwire.copy_(wire, non_blocking=True)
    e1.record(main_s)
    torch.cuda.synchronize()
    print(f"D2H 256 MiB alone: {e0.elapsed_time(e1):.3f} ms")
    for chunks, ns in [(1, 1), (2, 2), (4, 2), (8, 2), (4, 4), (16, 3), (16, 2)]:
        run(chunks, ns)


if __name__ == "__main__":
    main()
