#!/usr/bin/env python3
"""Which call in a hipGraph capture of bench.py's PCIe pipeline crashes the
process?  Round 4 captured the whole pipelined leg
(bench.py pcie_inclusive: pinned H2D copies on one stream, the library's
kernels on a second, D2H copies on a third, events between them, streams
created before the capture) with torch.cuda.graph and the process dumped core
during the capture.  Here the capture is rebuilt piece by piece, each piece
in its own child process, in order of how much of the pipeline it holds; the
first child that dies by a signal ends the probe (nothing more runs on the
GPU after a crash) and names the piece.

    python tools/capture_probe.py [--only NAME] [--out FILE.json]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N = 1 << 20  # Quads per leg (16 MiB of wire)
CHUNKS, DEPTH = 4, 2

CASES = [
    # name, what is captured
    ("kernels", "srpc_gpu_pack + srpc_gpu_unpack on device buffers (the library's claim: capturable)"),
    ("d2d_copy", "a device-to-device copy_ and srpc_gpu_pack"),
    ("events_side_streams", "kernels on two side streams created before the capture, joined by events "
                            "(the pipeline's event pattern, no host memory)"),
    ("pinned_h2d", "one pinned host -> device copy_ (non_blocking)"),
    ("pinned_d2h", "one device -> pinned host copy_ (non_blocking)"),
    ("host_direct", "srpc_gpu_pack_host in direct mode (hipPointerGetAttributes on pinned memory)"),
    ("host_chunked", "srpc_gpu_pack_host chunked (the library's internal streams): must be refused"),
    ("pinned_slice_h2d", "pinned -> device copies of SLICES of a pinned tensor (h[lo:hi], offset views)"),
    ("pinned_side_stream", "a whole pinned tensor copied on a side stream joined to the capture by events"),
    ("pinned_slice_side_stream", "pinned slices copied on a side stream joined by events (the pipeline's H2D)"),
    ("pinned_slice_d2h_side", "device -> pinned SLICE copies on a side stream joined by events (the pipeline's D2H)"),
    # round 5, second pass: pipeline_device died (rc -11) with no host memory
    # in the graph at all; take it apart
    ("pd_1chunk", "pipeline_device with ONE chunk (fork to three streams, copy, pack, copy, join)"),
    ("pd_noring", "pipeline_device with a slot per chunk (no waits on an earlier chunk's events)"),
    # third pass: pd_nocopy died (rc -11) and pd_noring did not -- the ring's
    # waits on events an earlier chunk recorded on another stream
    ("ring_in_only", "pd_nocopy with only s_in's waits on the kernel stream's earlier events"),
    ("ring_k_only", "pd_nocopy with only the kernel stream's waits on s_out's earlier events"),
    ("ring_torch", "the ring of pd_nocopy with torch elementwise kernels in place of the library's packs"),
    ("pd_nocopy", "pipeline_device's streams, events and ring waits with only the packs (no copies)"),
    ("pd_nostart", "pipeline_device without the start-event fork of s_in / s_out (each joins at its first wait)"),
    ("pipeline_device", "the pipeline's streams, events and ring waits with device buffers in place of pinned ones"),
    ("pipeline_no_ring", "the pipeline with a slot per chunk (no waits on an earlier chunk's events)"),
    ("pipeline", "bench.py's whole pipelined pack leg: pinned copies + kernels on three streams"),
]


def child(name: str) -> dict:
    import numpy as np
    import torch

    import srpc_amd
    from srpc_amd import QUAD, GpuPacker

    dev = torch.device("cuda:0")
    p = GpuPacker(QUAD)
    rb = 16
    cols = [torch.randint(-2**31, 2**31 - 1, (N,), dtype=torch.int32, device=dev) for _ in range(4)]
    back = [torch.empty(N, dtype=torch.int32, device=dev) for _ in range(4)]
    wire = torch.empty(N * rb, dtype=torch.uint8, device=dev)
    hcols = [c.cpu().pin_memory() for c in cols]
    hwire = torch.empty(N * rb, dtype=torch.uint8).pin_memory()
    torch.cuda.synchronize()
    side = torch.cuda.Stream(dev)
    s_in, s_k, s_out = (torch.cuda.Stream(dev) for _ in range(3))
    g = torch.cuda.CUDAGraph()
    out = {"case": name}

    def body():
        cur = torch.cuda.current_stream(dev)
        if name == "kernels":
            p.pack(cols, N, wire, stream=cur)
            p.unpack(wire, N * rb, N, back, stream=cur)
        elif name == "d2d_copy":
            back[0].copy_(cols[0])
            p.pack(cols, N, wire, stream=cur)
        elif name == "events_side_streams":
            e0 = torch.cuda.Event()
            e0.record(cur)
            s_k.wait_event(e0)
            p.pack(cols, N, wire, stream=s_k)
            e1 = torch.cuda.Event()
            e1.record(s_k)
            s_out.wait_event(e1)
            p.unpack(wire, N * rb, N, back, stream=s_out)
            e2 = torch.cuda.Event()
            e2.record(s_out)
            cur.wait_event(e2)
        elif name == "pinned_h2d":
            cols[0].copy_(hcols[0], non_blocking=True)
        elif name == "pinned_d2h":
            hwire.copy_(wire, non_blocking=True)
        elif name == "pinned_slice_h2d":
            per = N // CHUNKS
            for i in range(CHUNKS):
                cols[0][i * per:(i + 1) * per].copy_(hcols[0][i * per:(i + 1) * per], non_blocking=True)
        elif name in ("pinned_side_stream", "pinned_slice_side_stream"):
            e0 = torch.cuda.Event()
            e0.record(cur)
            s_in.wait_event(e0)
            with torch.cuda.stream(s_in):
                if name == "pinned_side_stream":
                    cols[0].copy_(hcols[0], non_blocking=True)
                else:
                    per = N // CHUNKS
                    for i in range(CHUNKS):
                        cols[0][i * per:(i + 1) * per].copy_(hcols[0][i * per:(i + 1) * per], non_blocking=True)
                e1 = torch.cuda.Event()
                e1.record(s_in)
            cur.wait_event(e1)
        elif name == "pinned_slice_d2h_side":
            e0 = torch.cuda.Event()
            e0.record(cur)
            s_out.wait_event(e0)
            with torch.cuda.stream(s_out):
                per = N // CHUNKS
                for i in range(CHUNKS):
                    hwire[i * per * rb:(i + 1) * per * rb].copy_(wire[i * per * rb:(i + 1) * per * rb],
                                                                 non_blocking=True)
                e1 = torch.cuda.Event()
                e1.record(s_out)
            cur.wait_event(e1)
        elif name.startswith("pipeline") or name.startswith("pd_") or name.startswith("ring_"):
            chunks = 1 if name == "pd_1chunk" else CHUNKS
            per = N // chunks
            rcols = body.rcols
            rwire = body.rwire
            depth = chunks if name in ("pipeline_no_ring", "pd_noring", "pd_1chunk") else DEPTH
            dev_bufs = name == "pipeline_device" or name.startswith("pd_") or name.startswith("ring_")
            copies = name != "pd_nocopy" and not name.startswith("ring_")
            src_cols, dst_wire = (body.dcols, body.dwire) if dev_bufs else (hcols, hwire)
            start = torch.cuda.Event()
            start.record(cur)
            for st in ((s_k,) if name == "pd_nostart" else (s_in, s_k, s_out)):
                st.wait_event(start)
            ev_k, ev_out = [None] * chunks, [None] * chunks
            for i in range(chunks):
                sl = i % depth
                lo, hi = i * per, (i + 1) * per
                if i >= depth:
                    if name != "ring_k_only":
                        s_in.wait_event(ev_k[i - depth])
                    if name != "ring_in_only":
                        s_k.wait_event(ev_out[i - depth])
                if name == "pd_nostart" and i == 0:
                    e_k0 = torch.cuda.Event()
                    e_k0.record(s_k)
                    s_in.wait_event(e_k0)
                with torch.cuda.stream(s_in):
                    if copies:
                        for h, c in zip(src_cols, rcols[sl]):
                            c.copy_(h[lo:hi], non_blocking=True)
                    ev_in = torch.cuda.Event()
                    ev_in.record(s_in)
                s_k.wait_event(ev_in)
                if name == "ring_torch":
                    with torch.cuda.stream(s_k):
                        rwire[sl].add_(1)
                else:
                    p.pack(rcols[sl] if copies else [c[lo:hi] for c in body.dcols], per, rwire[sl], stream=s_k)
                ev_k[i] = torch.cuda.Event()
                ev_k[i].record(s_k)
                s_out.wait_event(ev_k[i])
                with torch.cuda.stream(s_out):
                    if copies:
                        dst_wire[lo * rb:hi * rb].copy_(rwire[sl], non_blocking=True)
                    ev_out[i] = torch.cuda.Event()
                    ev_out[i].record(s_out)
            cur.wait_event(ev_out[-1])
        elif name == "host_direct":
            p.pack_host([h.data_ptr() for h in hcols], N, hwire, 0, 0, 0, depth=1, stream=cur)
        elif name == "host_chunked":
            per = N // CHUNKS
            sb = p.host_scratch_bytes(per, DEPTH)
            try:
                p.pack_host([h.data_ptr() for h in hcols], N, hwire, per, body.sp, sb, depth=DEPTH, stream=cur)
                out["refused"] = False
            except srpc_amd.SrpcError as e:
                out["refused"] = str(e)

    if name.startswith("pipeline") or name.startswith("pd_") or name.startswith("ring_"):
        per = N // CHUNKS
        big = N if name == "pd_1chunk" else per
        body.rcols = [[torch.empty(big, dtype=torch.int32, device=dev) for _ in range(4)] for _ in range(CHUNKS)]
        body.rwire = [torch.empty(big * rb, dtype=torch.uint8, device=dev) for _ in range(CHUNKS)]
        body.dcols = [c.clone() for c in cols]
        body.dwire = torch.empty(N * rb, dtype=torch.uint8, device=dev)
    if name == "host_chunked":
        sb = p.host_scratch_bytes(N // CHUNKS, DEPTH)
        body.scr = torch.empty(sb + 256, dtype=torch.uint8, device=dev)
        body.sp = body.scr.data_ptr() + (-body.scr.data_ptr()) % 256
    torch.cuda.synchronize()
    print(f"capturing {name}", flush=True)
    with torch.cuda.graph(g, stream=side):
        body()
    print(f"captured {name}", flush=True)
    hwire.zero_()
    for b in back:
        b.zero_()
    g.replay()
    torch.cuda.synchronize()
    want = None
    if name in ("kernels", "events_side_streams"):
        out["ok"] = all(torch.equal(a, b) for a, b in zip(cols, back))
    elif name == "pipeline_device" or name in ("pd_1chunk", "pd_noring", "pd_nostart"):
        ref = torch.empty(N * rb, dtype=torch.uint8, device=dev)
        p.pack(cols, N, ref)
        torch.cuda.synchronize()
        out["ok"] = bool(torch.equal(body.dwire, ref))
    elif name in ("pipeline", "pipeline_no_ring", "host_direct", "pinned_d2h", "pinned_slice_d2h_side") or (
            name == "host_chunked" and not out.get("refused")):
        ref = torch.empty(N * rb, dtype=torch.uint8, device=dev)
        p.pack(cols, N, ref)
        torch.cuda.synchronize()
        want = wire.cpu() if name in ("pinned_d2h", "pinned_slice_d2h_side") else ref.cpu()
        out["ok"] = bool(torch.equal(hwire, want))
    else:
        out["ok"] = True
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", default=None)
    ap.add_argument("--only", default="", help="comma-separated case names, run in that order")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.child:
        r = child(args.child)
        print("RESULT " + json.dumps(r), flush=True)
        return
    rows = []
    want = [c for c in args.only.split(",") if c]
    cases = [(n, dict(CASES)[n]) for n in want] if want else CASES
    for name, what in cases:
        pr = subprocess.run([sys.executable, __file__, "--child", name], capture_output=True, text=True, timeout=300)
        res = [l for l in pr.stdout.splitlines() if l.startswith("RESULT ")]
        row = {"case": name, "what": what, "rc": pr.returncode,
               "result": json.loads(res[-1][7:]) if res else None,
               "tail": (pr.stdout + pr.stderr).strip().splitlines()[-6:]}
        rows.append(row)
        print(json.dumps(row), flush=True)
        if pr.returncode < 0 or pr.returncode >= 128:  # killed by a signal: the crashing piece; stop here
            print(f"STOP: {name} died with rc={pr.returncode}", flush=True)
            break
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
