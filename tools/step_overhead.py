#!/usr/bin/env python3
"""Where the step time goes beyond the two kernels (16M Quad, one MI355X).

bench.py's ms_per_step is ~15 us longer than pack + unpack kernel time.  This
tool separates the candidates, each over K back-to-back steps:
  host   - host-side enqueue cost of one step (no sync inside the loop);
  null   - launches on the legacy null stream (torch's default);
  stream - launches on a dedicated torch stream;
  hook   - as `stream`, with srpc_time_next_call armed for every call;
  graph  - the K steps captured once into a hipGraph and replayed.

    python tools/step_overhead.py [--steps 50] [--out gpurun_out/step_overhead.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 24)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    import torch

    import srpc_amd
    from srpc_amd import QUAD, GpuPacker

    dev = torch.device("cuda:0")
    n, K = args.records, args.steps
    cols = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(4)]
    back = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(4)]
    wire = torch.empty(n * 16, dtype=torch.uint8, device=dev)
    srpc_amd.fill_splitmix_i32(cols, n, 0x5EED, 0, torch.cuda.current_stream())
    p = GpuPacker(QUAD)
    side = torch.cuda.Stream(dev)
    kev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for e in kev:
        e.record(side)

    def steps(s, hook=False):
        for _ in range(K):
            if hook:
                srpc_amd.time_next_call(kev[0], kev[1])
            p.pack(cols, n, wire, stream=s)
            if hook:
                srpc_amd.time_next_call(kev[0], kev[1])
            p.unpack(wire, n * 16, n, back, stream=s)

    def run(name, s, body):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        a.record(s)
        body()
        b.record(s)
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        return {"gpu_us_per_step": a.elapsed_time(b) * 1e3 / K, "host_enqueue_us_per_step": t_host * 1e6 / K,
                "wall_us_per_step": t_all * 1e6 / K}

    null = torch.cuda.default_stream(dev)
    with torch.cuda.stream(side):
        steps(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            steps(side)
        torch.cuda.synchronize()

    res = {}
    for _ in range(args.rounds):
        for name, s, body in [("null", null, lambda: steps(null)),
                              ("stream", side, lambda: steps(side)),
                              ("hook", side, lambda: steps(side, hook=True)),
                              ("graph", side, lambda: g.replay())]:
            with torch.cuda.stream(s):
                r = run(name, s, body)
            for k, v in r.items():
                res.setdefault(name, {}).setdefault(k, []).append(v)
    ok = all(torch.equal(a, b) for a, b in zip(cols, back))
    out = {"records": n, "steps": K, "roundtrip_ok": ok,
           "median": {m: {k: round(statistics.median(v), 2) for k, v in d.items()} for m, d in res.items()}}
    txt = json.dumps(out, indent=1)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()
