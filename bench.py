#!/usr/bin/env python3
"""Benchmark: device-resident pack + unpack of Quad{4 x int32} records.

BASELINE.json metric: "packer GiB/s + Mrecords/s device-resident, 1/2/4/8 MI355X".
One step = one pass of the hot path over one batch of synthetic records
already resident in HBM: srpc_gpu_pack (4 int32 columns -> 16-byte wire
records) followed by srpc_gpu_unpack (wire -> 4 columns), both through the
C ABI of srpc_amd/libsrpc_gpu.so.  Weak scaling: every rank owns 16M records
(configs[2] of BASELINE.json per GPU; at 4 GPUs that is configs[3]'s 64M).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Prints ONE JSON line on rank 0.  `value` = wire GiB/s through a full
pack+unpack round trip summed over all ranks (records * 16 B / 2^30 / step
time, the max over ranks).  The roofline object prices the dominant kernel
against HBM3E (8.0 TB/s spec) with algorithmic bytes (32 B per record per
kernel); the cpu_baseline object times the reference packer (compiled from
/root/reference into oracle/_ref, or the C restatement if that is absent) on
this host.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
HBM_MEASURED_COPY_GBPS = 6290.0  # measured float4 copy ceiling (same table)
REC_BYTES = 16                  # Quad body
ALG_BYTES_PER_REC = 32          # per kernel: pack reads 4x4 B + writes 16 B; unpack the reverse


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE, else 1); without torchrun N > 1 spawns "
                         "N rank processes itself")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--records", type=int, default=1 << 24, help="records per GPU")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU-baseline work (rank 0, N=1 only); 0 disables")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-pcie", action="store_true")
    ap.add_argument("--no-cold", action="store_true", help="skip the cold-cache kernel clock")
    ap.add_argument("--path", choices=["auto", "dword", "tile"], default="auto")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (production); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--tune", default=None,
                    help="DWORD-path variant rpl,iter,nt (default: the library's tuned default)")
    ap.add_argument("--strong-records", type=int, default=1 << 26,
                    help="strong-scaling line beside the weak one: this many records in all, "
                         "split over the ranks (configs[3]: 64M); 0 disables")
    return ap.parse_args()


XGMI_LINK_GBPS = 153.0  # per xGMI link and direction (the task's MI355X figure: 7 links x ~153 GB/s)


def free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_plan(gpus, env: dict, device_count: int, backend: str) -> dict:
    """What `bench.py --gpus N` does, decided without touching a GPU.

    - Under a launcher (WORLD_SIZE set, as torch.distributed.run does): run as
      that rank; --gpus, when given, must equal WORLD_SIZE.
    - No launcher and N > 1: spawn N rank processes (children of this one,
      never an exec) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rank
      r on device r; rank 0 prints the line.
    - N = 1: run in this process.
    With the NCCL backend every rank needs its own GPU: fewer visible devices
    than ranks is an error (gloo may share one GPU: a rehearsal only).
    Returns {"mode": "rank"|"spawn"|"single", "world": N, "envs": [...]} or
    {"error": message}."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        try:
            world = int(ws)
        except ValueError:
            return {"error": f"WORLD_SIZE={ws!r} is not an integer"}
        if world < 1:
            return {"error": f"WORLD_SIZE={world}"}
        if gpus is not None and gpus != world:
            return {"error": f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks"}
        mode = "rank" if world > 1 else "single"
    else:
        world = 1 if gpus is None else gpus
        if world < 1:
            return {"error": f"--gpus {world}: need at least one GPU"}
        mode = "spawn" if world > 1 else "single"
    if world > 1 and backend == "nccl" and device_count < world:
        return {"error": f"{world} ranks over RCCL need {world} GPUs, {device_count} visible "
                         f"(one rank per GPU; --dist-backend gloo rehearses N > 1 on fewer)"}
    if world == 1 and device_count < 1:
        return {"error": "no GPU visible"}
    out = {"mode": mode, "world": world, "envs": []}
    if mode == "spawn":
        port = env.get("MASTER_PORT") or str(free_port())
        for r in range(world):
            e = dict(env)
            e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                     GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
            out["envs"].append(e)
    return out


def spawn_ranks(envs: list, argv: list) -> int:
    """Runs one child per rank (this script, same arguments) and waits; when
    one fails the others are stopped (their PIDs only) and its code returned."""
    import signal
    import subprocess

    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=e) for e in envs]
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc:
        print(f"bench.py: a rank failed with exit code {rc}; stopped the others", file=sys.stderr, flush=True)
    return rc


def committed_profiles(dom_name: str, n: int) -> dict:
    """The newest round's committed rocprof evidence for the dominant kernel:
    profiles/rNN_kernel_stats.csv (rocprofv3 --kernel-trace --stats of this
    bench) and profiles/rNN_pmc_traffic.json (FETCH_SIZE / WRITE_SIZE passes),
    NN the highest round that has each file; the file names go into the line."""
    import csv
    import glob
    import re

    out = {"traffic": None, "committed_rocprof_avg_us": None, "kernel_stats_file": None, "pmc_file": None}
    kname = {"pack": "k_pack_dword", "unpack": "k_unpack_dword"}[dom_name]

    def newest(pattern):
        files = [f for f in glob.glob(os.path.join(ROOT, "profiles", pattern))
                 if re.match(r"r\d\d_", os.path.basename(f))]
        return max(files, key=os.path.basename) if files else None

    stats = newest("r??_kernel_stats.csv")
    if stats:
        with open(stats) as f:
            for row in csv.DictReader(f):
                if kname in row["Name"]:
                    out["committed_rocprof_avg_us"] = round(float(row["AverageNs"]) / 1e3, 2)
                    out["kernel_stats_file"] = os.path.relpath(stats, ROOT)
                    break
    pmc = newest("r??_pmc_traffic.json")
    if pmc:
        with open(pmc) as f:
            pm = json.load(f)
        ent = pm.get("kernels", {}).get(dom_name)
        if ent and pm.get("records") == n:
            out["traffic"] = ent.get("hbm_bytes_per_launch")
            out["pmc_file"] = os.path.relpath(pmc, ROOT)
    return out


def pcie_inclusive(p, n: int, dev, reps: int = 3, chunks: int = 16, depth: int = 3) -> dict:
    """The host-terminated path (north_star: it "starts and ends in host
    memory", the socket buffers of the reference's transport.hpp:94-123), in
    both directions, pinned host buffers:
      pack:   host columns -> H2D -> srpc_gpu_pack -> D2H wire;
      unpack: host wire -> H2D -> srpc_gpu_unpack -> D2H columns.
    `serial` runs the three steps on one stream; `pipelined` cuts the batch
    into `chunks` pieces over three streams (H2D / kernels / D2H) and a ring of
    `depth` device buffers, so H2D of chunk k+1, the kernel of chunk k and D2H
    of chunk k-1 overlap (PCIe Gen5 is full duplex).  `link` is the copy
    engines alone: one direction at a time, then both at once (the duplex
    ceiling a pipelined leg can reach).  Every leg's output is checked."""
    import torch

    rb = REC_BYTES
    cols = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(4)]
    import srpc_amd
    main = torch.cuda.current_stream(dev)
    srpc_amd.fill_splitmix_i32(cols, n, 0x5EED, 0, main)
    hcols = [torch.empty(n, dtype=torch.int32).pin_memory() for _ in range(4)]
    hwire = torch.empty(n * rb, dtype=torch.uint8).pin_memory()
    hback = [torch.empty(n, dtype=torch.int32).pin_memory() for _ in range(4)]
    for h, c in zip(hcols, cols):
        h.copy_(c)
    wire = torch.empty(n * rb, dtype=torch.uint8, device=dev)
    back = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(4)]
    p.pack(cols, n, wire, stream=main)
    want_wire = wire.cpu()
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(fn):
        fn()  # first use of this leg's copies
        torch.cuda.synchronize(dev)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2] * 1e3

    def leg(ms, moved):
        return {"ms": round(ms, 3), "wire_GiBps": round(n * rb / 2**30 / (ms / 1e3), 3),
                "mrecords_per_s": round(n / (ms / 1e3) / 1e6, 1),
                "pcie_GBps_both_directions": round(moved / (ms / 1e3) / 1e9, 1)}

    moved = 2 * n * rb  # 256 MiB in + 256 MiB out per 16M Quads, either direction

    # -- serial, one stream
    def serial_pack():
        with torch.cuda.stream(main):
            for h, c in zip(hcols, cols):
                c.copy_(h, non_blocking=True)
            p.pack(cols, n, wire, stream=main)
            hwire.copy_(wire, non_blocking=True)

    def serial_unpack():
        with torch.cuda.stream(main):
            wire.copy_(hwire, non_blocking=True)
            p.unpack(wire, n * rb, n, back, stream=main)
            for h, c in zip(hback, back):
                h.copy_(c, non_blocking=True)

    out = {"what": "pinned host buffers at both ends; 16M Quads per leg; median of %d" % reps}
    ms = timed(serial_pack)
    ok_pack = torch.equal(hwire, want_wire)
    out["serial"] = {"pack": leg(ms, moved)}
    ms = timed(serial_unpack)
    ok_unpack = all(torch.equal(a, b) for a, b in zip(hback, hcols))
    out["serial"]["unpack"] = leg(ms, moved)

    # -- pipelined: three streams, a ring of `depth` chunk buffers
    per = n // chunks
    assert per * chunks == n and per % 16 == 0
    s_in, s_k, s_out = (torch.cuda.Stream(dev) for _ in range(3))
    rcols = [[torch.empty(per, dtype=torch.int32, device=dev) for _ in range(4)] for _ in range(depth)]
    rwire = [torch.empty(per * rb, dtype=torch.uint8, device=dev) for _ in range(depth)]

    def pipelined(direction):
        start = torch.cuda.Event()
        start.record(main)
        for st in (s_in, s_k, s_out):
            st.wait_event(start)
        ev_k, ev_out = [None] * chunks, [None] * chunks
        for i in range(chunks):
            sl = i % depth
            lo, hi = i * per, (i + 1) * per
            src_cols, dst_cols = rcols[sl], rcols[sl]
            if i >= depth:  # the slot's previous chunk: its kernel has read it, its D2H has drained it
                s_in.wait_event(ev_k[i - depth])
                s_k.wait_event(ev_out[i - depth])
            with torch.cuda.stream(s_in):
                if direction == "pack":
                    for h, c in zip(hcols, src_cols):
                        c.copy_(h[lo:hi], non_blocking=True)
                else:
                    rwire[sl].copy_(hwire[lo * rb:hi * rb], non_blocking=True)
                ev_in = torch.cuda.Event()
                ev_in.record(s_in)
            s_k.wait_event(ev_in)
            if direction == "pack":
                p.pack(src_cols, per, rwire[sl], stream=s_k)
            else:
                p.unpack(rwire[sl], per * rb, per, dst_cols, stream=s_k)
            ev_k[i] = torch.cuda.Event()
            ev_k[i].record(s_k)
            s_out.wait_event(ev_k[i])
            with torch.cuda.stream(s_out):
                if direction == "pack":
                    hwire[lo * rb:hi * rb].copy_(rwire[sl], non_blocking=True)
                else:
                    for h, c in zip(hback, dst_cols):
                        h[lo:hi].copy_(c, non_blocking=True)
                ev_out[i] = torch.cuda.Event()
                ev_out[i].record(s_out)
        main.wait_event(ev_out[-1])

    hwire.zero_()
    ms = timed(lambda: pipelined("pack"))
    ok_pack = ok_pack and torch.equal(hwire, want_wire)
    out["pipelined"] = {"pack": leg(ms, moved)}
    for h in hback:
        h.zero_()
    ms = timed(lambda: pipelined("unpack"))
    ok_unpack = ok_unpack and all(torch.equal(a, b) for a, b in zip(hback, hcols))
    out["pipelined"]["unpack"] = leg(ms, moved)
    out["pipelined"].update({"chunks": chunks, "records_per_chunk": per, "ring_depth": depth,
                             "streams": "H2D / kernels / D2H"})

    # -- native pipeline (ABI 7: srpc_gpu_pack_host / srpc_gpu_unpack_host): the
    # same chunked ring enqueued by the library, a few HIP calls per chunk
    h_cols_p = [h.data_ptr() for h in hcols]
    h_back_p = [h.data_ptr() for h in hback]
    native = {}
    for nchunks, ndepth, nstreams in ((16, 3, 3), (16, 3, 2), (0, 1, 3)):
        os.environ["SRPC_HOST_STREAMS"] = str(nstreams)  # host.hip A/B: kernels on their own stream or the H2D one
        per_n = n // nchunks if nchunks else 0  # 0: direct, the kernels on the mapped pinned buffers
        sb = p.host_scratch_bytes(per_n, ndepth)
        scr = torch.empty(sb + 256, dtype=torch.uint8, device=dev)
        sp = scr.data_ptr() + (-scr.data_ptr()) % 256
        name = f"{nchunks}x{ndepth}_{nstreams}streams" if nchunks else "direct"
        hwire.zero_()
        try:  # direct mode needs device-mapped pinned memory: a box without it reports the refusal
            ms_p = timed(lambda: p.pack_host(h_cols_p, n, hwire, per_n, sp, sb, depth=ndepth, stream=main))
        except srpc_amd.SrpcError as e:
            native[name] = {"refused": str(e)}
            del scr
            continue
        okp = torch.equal(hwire, want_wire)
        for h in hback:
            h.zero_()
        ms_u = timed(lambda: p.unpack_host(hwire, n * rb, n, h_back_p, per_n, sp, sb, depth=ndepth, stream=main))
        oku = all(torch.equal(a, b) for a, b in zip(hback, hcols))
        ok_pack, ok_unpack = ok_pack and okp, ok_unpack and oku
        native[name] = {"pack": leg(ms_p, moved), "unpack": leg(ms_u, moved)}
        del scr
    os.environ.pop("SRPC_HOST_STREAMS", None)
    ran = [k for k in native if "pack" in native[k]]
    best = {d: min(ran, key=lambda k: native[k][d]["ms"]) for d in ("pack", "unpack")}
    out["pipelined_native"] = {"configs": native, "best": best,
                               "what": "chunks x ring depth, enqueued by srpc_gpu_pack_host / _unpack_host"}

    # -- the link alone: H2D 256 MiB, D2H 256 MiB, then both at once on two streams
    def h2d():
        with torch.cuda.stream(s_in):
            wire.copy_(hwire, non_blocking=True)
        main.wait_stream(s_in)

    def d2h():
        with torch.cuda.stream(s_out):
            hwire.copy_(wire, non_blocking=True)
        main.wait_stream(s_out)

    wire.copy_(want_wire.to(dev))
    hw2 = torch.empty(n * rb, dtype=torch.uint8).pin_memory()
    w2 = torch.empty(n * rb, dtype=torch.uint8, device=dev)

    def both():  # the same 256 MiB each way, in `chunks` pieces per direction, the two streams interleaved
        cb = n * rb // chunks
        for i in range(chunks):
            with torch.cuda.stream(s_in):
                w2[i * cb:(i + 1) * cb].copy_(hwire[i * cb:(i + 1) * cb], non_blocking=True)
            with torch.cuda.stream(s_out):
                hw2[i * cb:(i + 1) * cb].copy_(wire[i * cb:(i + 1) * cb], non_blocking=True)
        main.wait_stream(s_in)
        main.wait_stream(s_out)

    t_h2d, t_d2h, t_both = timed(h2d), timed(d2h), timed(both)
    out["link"] = {"h2d_GBps": round(n * rb / (t_h2d / 1e3) / 1e9, 1),
                   "d2h_GBps": round(n * rb / (t_d2h / 1e3) / 1e9, 1),
                   "duplex_GBps_both_directions": round(moved / (t_both / 1e3) / 1e9, 1),
                   "duplex_ms_for_one_leg": round(t_both, 3),
                   "note": "a pipelined leg moves 256 MiB each way: duplex_ms_for_one_leg is its copy floor"}
    out["pipelined_over_serial"] = {d: round(out["serial"][d]["ms"] / out["pipelined"][d]["ms"], 3)
                                    for d in ("pack", "unpack")}
    out["pipelined_over_duplex_floor"] = {d: round(t_both / out["pipelined"][d]["ms"], 3)
                                          for d in ("pack", "unpack")}
    nat = {d: out["pipelined_native"]["configs"][best[d]][d]["ms"] for d in ("pack", "unpack")}
    out["native_over_serial"] = {d: round(out["serial"][d]["ms"] / nat[d], 3) for d in ("pack", "unpack")}
    out["native_over_duplex_floor"] = {d: round(t_both / nat[d], 3) for d in ("pack", "unpack")}
    out["verified"] = bool(ok_pack and ok_unpack)
    del cols, back, wire, w2, rcols, rwire
    return out


def cpu_info() -> dict:
    """CPU model and core counts of this host (hardware_concurrency = os.cpu_count())."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover - non-Linux
        allowed = os.cpu_count() or 1
    return {"model": model, "hardware_concurrency": os.cpu_count(), "affinity": allowed}


def baseline_threads(info: dict) -> tuple[int, str]:
    """Threads for the multi-threaded CPU baseline: every core this process may
    use -- the affinity mask, capped by OMP_NUM_THREADS where the host sets it
    (the GPU box shares its host: it sets 16 per GPU and asks jobs to stay within)."""
    nt = info["affinity"] or 1
    why = "all cores in this process's affinity mask"
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and 0 < int(omp) < nt:
        nt = int(omp)
        why = f"OMP_NUM_THREADS={omp}: this host's CPU share per job (hardware_concurrency {info['hardware_concurrency']})"
    return nt, why


def cpu_baseline(n: int, target_s: float) -> dict | None:
    """The reference CPU packer on this host: pack (`p << r` per record) +
    unpack (`r.unpack(bp)` per record) of the same Quad workload.  Timed at
    1 thread and at T threads (one independent packer per contiguous shard,
    T = baseline_threads), each as the median of >= 5 passes over a 4M-record
    slice; the headline `value` is the T-thread median.  Rank 0, N=1 only."""
    import ctypes as C
    import statistics

    import numpy as np

    import oracle

    m = min(n, 1 << 22)  # 4M-record slices of the same splitmix stream
    cols = oracle.splitmix_columns_i32(4, m)
    wire = np.zeros(m * 16, np.uint8)
    back = [np.zeros(m, np.int32) for _ in range(4)]
    info = cpu_info()
    nt, why = baseline_threads(info)
    gib = m * REC_BYTES / 2**30
    if oracle.ref_available():
        ref = oracle.ref_lib()
        kind = "reference"
        tp, tu = C.c_double(0), C.c_double(0)

        def one():
            ref.ref_pack_quad(*[c.ctypes.data for c in cols], m, wire.ctypes.data, wire.size, C.byref(tp))
            ref.ref_unpack_quad(wire.ctypes.data, wire.size, m, *[b.ctypes.data for b in back], C.byref(tu))
            return tp.value + tu.value

        def one_mt():
            ref.ref_pack_quad_mt(*[c.ctypes.data for c in cols], m, wire.ctypes.data, nt, C.byref(tp))
            ref.ref_unpack_quad_mt(wire.ctypes.data, m, *[b.ctypes.data for b in back], nt, C.byref(tu))
            return tp.value + tu.value
    else:
        kind = "port"

        def one():
            t0 = time.perf_counter()
            w = oracle.pack([oracle.INT32] * 4, cols, m)
            oracle.unpack([oracle.INT32] * 4, w, m)
            return time.perf_counter() - t0
        one_mt = None

    def passes(fn, budget):
        ts = []
        while len(ts) < 5 or (sum(ts) < budget and len(ts) < 64):
            ts.append(fn())
        return ts

    t1 = passes(one, target_s * 0.75)
    single = {"value": round(gib / statistics.median(t1), 4), "threads": 1, "passes": len(t1),
              "mrecords_per_s": round(m / statistics.median(t1) / 1e6, 2),
              "min_max_GiBps": [round(gib / max(t1), 4), round(gib / min(t1), 4)]}
    out = {"value": single["value"], "unit": "GiB/s", "cores": 1, "kind": kind,
           "sample": f"median of {len(t1)} pack+unpack passes over a {m}-record slice of the same splitmix "
                     f"stream, 1 thread, {sum(t1):.1f} s",
           "cpu": info, "single_thread": single}
    if one_mt is not None:
        tm = passes(one_mt, target_s * 0.25)
        multi = {"value": round(gib / statistics.median(tm), 4), "threads": nt, "passes": len(tm),
                 "threads_rule": why, "mrecords_per_s": round(m / statistics.median(tm) / 1e6, 2),
                 "min_max_GiBps": [round(gib / max(tm), 4), round(gib / min(tm), 4)]}
        out.update({"value": multi["value"], "cores": nt,
                    "sample": f"median of {len(tm)} pack+unpack passes over a {m}-record slice of the same "
                              f"splitmix stream, {nt} threads (one reference packer per contiguous shard), "
                              f"{sum(tm):.1f} s; single-thread median beside it",
                    "multithread": multi})
        # every hardware thread of the host as well (T =
        # hardware_concurrency) -- beyond this job's CPU share on a shared GPU
        # box, so reported beside the headline, not as it
        hw = int(info.get("affinity") or info.get("hardware_concurrency") or 0)
        if hw > nt:
            def one_hw():
                ref.ref_pack_quad_mt(*[c.ctypes.data for c in cols], m, wire.ctypes.data, hw, C.byref(tp))
                ref.ref_unpack_quad_mt(wire.ctypes.data, m, *[b.ctypes.data for b in back], hw, C.byref(tu))
                return tp.value + tu.value
            th = passes(one_hw, 0)
            out["hardware_concurrency_leg"] = {
                "value": round(gib / statistics.median(th), 4), "threads": hw, "passes": len(th),
                "mrecords_per_s": round(m / statistics.median(th) / 1e6, 2),
                "min_max_GiBps": [round(gib / max(th), 4), round(gib / min(th), 4)],
                "note": f"{hw} threads on a host where this job's CPU share is {nt}: oversubscribed"}
    return out


def main() -> None:
    args = parse()
    import torch

    # torch.cuda.device_count() does not initialise the GPU on this image: the
    # plan is made, and ranks spawned, before any HIP call in this process
    plan = launch_plan(args.gpus, dict(os.environ), torch.cuda.device_count(), args.dist_backend)
    if "error" in plan:
        print(f"bench.py: {plan['error']}", file=sys.stderr, flush=True)
        sys.exit(2)
    if plan["mode"] == "spawn":
        sys.exit(spawn_ranks(plan["envs"], sys.argv[1:]))
    import torch.distributed as dist

    world = plan["world"]
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import srpc_amd
    from srpc_amd import QUAD, GpuPacker, _lib
    from srpc_amd.shard import NativeComm, gather_packed, shard_range

    # the exchange step: the library's own RCCL gather (srpc_gather_wire) on a
    # communicator it owns; the id travels over torch's process group
    comm, comm_note = None, None
    if world > 1 and args.dist_backend == "nccl":
        try:
            comm = NativeComm.from_process_group(local)
        except Exception as e:  # keep the measurement; say which gather ran
            comm_note = f"libsrpc_gpu RCCL comm failed ({e}); torch.distributed gather used"

    n = args.records
    first = rank * n  # the global batch is one splitmix stream sharded contiguously
    p = GpuPacker(QUAD, device=local)
    if args.path != "auto":
        p.force_path({"dword": srpc_amd.SRPC_PATH_DWORD, "tile": srpc_amd.SRPC_PATH_TILE}[args.path])
    if args.tune:
        rpl, it, nt = (int(x) for x in args.tune.split(","))
        p.tune(rpl, it, nt)
    stream = torch.cuda.current_stream(dev)
    cols = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(4)]
    back = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(4)]
    wire = torch.empty(n * REC_BYTES, dtype=torch.uint8, device=dev)
    srpc_amd.fill_splitmix_i32(cols, n, 0x5EED, first, stream)
    torch.cuda.synchronize(dev)

    def step():
        p.pack(cols, n, wire, stream=stream)
        p.unpack(wire, n * REC_BYTES, n, back, stream=stream)

    # correctness of the exact bytes being timed: round trip + reference digest
    verify = {}
    if not args.no_verify:
        step()
        torch.cuda.synchronize(dev)
        ok = all(torch.equal(a, b) for a, b in zip(cols, back))
        verify["roundtrip"] = bool(ok)
        full = gather_packed(wire, REC_BYTES, n * world, comm=comm) if world > 1 else wire
        if rank == 0:
            digest = hashlib.sha256(full.cpu().numpy().tobytes()).hexdigest()
            with open(os.path.join(ROOT, "tests", "golden", "manifest.json")) as f:
                streams = json.load(f)["streams"]
            want = {st["records"]: st["sha256"] for k, st in streams.items()
                    if k.startswith("quad_body_")}.get(n * world)
            verify["sha256"] = digest
            verify["matches_reference"] = (digest == want) if want else None
        if world > 1:
            flag = torch.tensor([int(ok)], device=dev if args.dist_backend == "nccl" else "cpu")
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            verify["roundtrip"] = bool(flag.item())
        del full

    K = args.steps
    step0 = torch.cuda.Event(enable_timing=True)
    step1 = torch.cuda.Event(enable_timing=True)
    kev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(K)]
    for e in [step0, step1] + [e for row in kev for e in row]:
        e.record(stream)  # torch creates the HIP event on its first record

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)

    # Step clock (`value`, ms_per_step): K uninstrumented steps.
    t0 = time.perf_counter()
    step0.record(stream)
    for _ in range(K):
        step()
    step1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0

    # Kernel clock (roofline): K further steps with every pack / unpack call
    # armed by srpc_time_next_call, so its kernel stamps its own dispatch
    # begin/end into a per-call event pair -- the interval rocprofv3
    # --kernel-trace reports.  Arming costs ~5 us of GPU time per call
    # (profiles/r01_step_overhead.json), so it stays out of the step clock.
    for i in range(K):
        srpc_amd.time_next_call(kev[i][0], kev[i][1])
        p.pack(cols, n, wire, stream=stream)
        srpc_amd.time_next_call(kev[i][2], kev[i][3])
        p.unpack(wire, n * REC_BYTES, n, back, stream=stream)
    torch.cuda.synchronize(dev)

    pack_ms = [kev[i][0].elapsed_time(kev[i][1]) for i in range(K)]
    unpack_ms = [kev[i][2].elapsed_time(kev[i][3]) for i in range(K)]

    # Cold-cache kernel clock (SURVEY.md §8d's second regime): 512 MiB written
    # before every armed call evicts the 256 MiB Infinity Cache (and L2).
    cold = None
    if not args.no_cold:
        flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
        kc = min(K, 10)
        for i in range(kc):
            flush.fill_(i & 0xFF)
            srpc_amd.time_next_call(kev[i][0], kev[i][1])
            p.pack(cols, n, wire, stream=stream)
            flush.fill_((i + 1) & 0xFF)
            srpc_amd.time_next_call(kev[i][2], kev[i][3])
            p.unpack(wire, n * REC_BYTES, n, back, stream=stream)
        torch.cuda.synchronize(dev)
        cp = sorted(kev[i][0].elapsed_time(kev[i][1]) for i in range(kc))[kc // 2]
        cu = sorted(kev[i][2].elapsed_time(kev[i][3]) for i in range(kc))[kc // 2]
        cold = {"pack": round(cp, 4), "unpack": round(cu, 4), "reps": kc, "stat": "median",
                "flush": "512 MiB written before each call (Infinity Cache is 256 MiB)"}
        del flush
    gpu_ms = step0.elapsed_time(step1)
    t_rank = max(elapsed, gpu_ms / 1e3)
    t = torch.tensor([t_rank, sum(pack_ms) / K, sum(unpack_ms) / K], dtype=torch.float64,
                     device=dev if args.dist_backend == "nccl" else "cpu")
    # per-rank view before the max: each rank's own kernel clock and what its
    # RCCL communicator says it is (srpc_comm_rank), so a multi-GPU line shows
    # that RCCL saw every rank
    mine = {"rank": rank, "device": local, "pack_ms": round(sum(pack_ms) / K, 4),
            "unpack_ms": round(sum(unpack_ms) / K, 4),
            "frac": round(ALG_BYTES_PER_REC * n / (max(sum(pack_ms), sum(unpack_ms)) / K / 1e3) / 1e9
                          / HBM_PEAK_GBPS, 4),
            "rccl": comm.info() if comm is not None else None}
    per_rank = [mine]
    if world > 1:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max, pack_avg, unpack_avg = t.tolist()
    ms_step = t_max * 1e3 / K

    # gather of the packed shards to rank 0 over RCCL (reported separately)
    gather = None
    if world > 1:
        for _ in range(2):
            gather_packed(wire, REC_BYTES, n * world, comm=comm)
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        reps = 5
        for _ in range(reps):
            gather_packed(wire, REC_BYTES, n * world, comm=comm)
        torch.cuda.synchronize(dev)
        dist.barrier()
        g_ms = (time.perf_counter() - g0) * 1e3 / reps
        moved = n * (world - 1) * REC_BYTES
        # every sender has its own link into the root: the floor is one shard
        # over one link, (G - 1) links in parallel
        floor_ms = n * REC_BYTES / (XGMI_LINK_GBPS * 1e9) * 1e3
        gather = {"ms": round(g_ms, 3), "bytes_to_root": moved,
                  "root_ingress_GBps": round(moved / g_ms / 1e6, 1),
                  "expected_ms_at_link_peak": round(floor_ms, 3),
                  "expected_root_ingress_GBps": round((world - 1) * XGMI_LINK_GBPS, 1),
                  "frac_of_link_floor": round(floor_ms / g_ms, 3),
                  "collective": ("libsrpc_gpu srpc_gather_wire: RCCL ncclSend/ncclRecv to rank 0 in one group"
                                 if comm is not None else
                                 "torch.distributed RCCL gather" if args.dist_backend == "nccl"
                                 else "gloo gather through host memory (rehearsal only)")}
        if comm_note:
            gather["note"] = comm_note

    # Strong scaling (configs[3]): args.strong_records in all, split over the
    # ranks with the library's shard rule; same step, same clock, max over ranks
    strong = None
    if args.strong_records > 0:
        NS = args.strong_records
        lo, hi = shard_range(NS, rank, world)
        m = hi - lo
        scols = [torch.empty(max(m, 1), dtype=torch.int32, device=dev) for _ in range(4)]
        sback = [torch.empty(max(m, 1), dtype=torch.int32, device=dev) for _ in range(4)]
        swire = torch.empty(max(m, 1) * REC_BYTES, dtype=torch.uint8, device=dev)
        srpc_amd.fill_splitmix_i32(scols, m, 0x5EED, lo, stream)

        def sstep():
            p.pack(scols, m, swire, stream=stream)
            p.unpack(swire, m * REC_BYTES, m, sback, stream=stream)

        for _ in range(args.warmup):
            sstep()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        step0.record(stream)
        for _ in range(K):
            sstep()
        step1.record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        ts = torch.tensor([max(time.perf_counter() - t0, step0.elapsed_time(step1) / 1e3)], dtype=torch.float64,
                          device=dev if args.dist_backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(ts, op=dist.ReduceOp.MAX)
        st_max = ts.item()
        sok = all(torch.equal(a[:m], b[:m]) for a, b in zip(scols, sback))
        full = gather_packed(swire[:m * REC_BYTES], REC_BYTES, NS, comm=comm) if world > 1 else swire[:m * REC_BYTES]
        sdig = None
        if rank == 0:
            sdig = hashlib.sha256(full.cpu().numpy().tobytes()).hexdigest()
        del full
        strong = {"records_total": NS, "records_per_gpu_max": max(h - l for l, h in
                                                                  (shard_range(NS, r, world) for r in range(world))),
                  "value": round(NS * K * REC_BYTES / 2**30 / st_max, 3), "unit": "GiB/s",
                  "ms_per_step": round(st_max * 1e3 / K, 4),
                  "mrecords_per_s": round(NS * K / st_max / 1e6, 1), "roundtrip_rank": bool(sok),
                  "sha256": sdig, "scaling": "strong"}
        del scols, sback, swire

    # PCIe-inclusive legs (host buffers at both ends), rank 0 only
    pcie = None
    if rank == 0 and world == 1 and not args.no_pcie:
        pcie = pcie_inclusive(p, n, dev)

    if rank == 0:
        total_recs = n * world
        value = total_recs * K * REC_BYTES / 2**30 / t_max  # wire GiB/s, all ranks
        dom_name, dom_ms = ("pack", pack_avg) if pack_avg >= unpack_avg else ("unpack", unpack_avg)
        achieved = ALG_BYTES_PER_REC * n / (dom_ms / 1e3) / 1e9
        # the same kernel from a cold Infinity Cache (512 MiB written before each
        # call): the warm figure above is partly served on-die, cold is not
        frac_cold = None
        if cold:
            frac_cold = round(ALG_BYTES_PER_REC * n / (cold[dom_name] / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)
        prof = committed_profiles(dom_name, n)
        line = {
            "metric": "packer GiB/s + Mrecords/s device-resident, 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": K,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (splitmix64 stream of SURVEY.md §8c, generated in HBM)",
            "config": {"workload": "Quad{4 x int32} pack+unpack, 16-byte records, device-resident",
                       "records_per_gpu": n, "global_records": total_recs,
                       "record_bytes": REC_BYTES, "parallelism": f"shard{world}",
                       "kernel_path": {1: "dword", 2: "tile"}[p.path],
                       "tune": args.tune or "default"},
            "mrecords_per_s": round(total_recs * K / t_max / 1e6, 1),
            "hbm_algorithmic_GBps": round(2 * ALG_BYTES_PER_REC * total_recs * K / t_max / 1e9, 1),
            "kernels_ms": {"pack": round(pack_avg, 4), "unpack": round(unpack_avg, 4),
                           "clock": "dispatch begin/end stamped by hipExtLaunchKernel (srpc_time_next_call), K armed steps after the step clock"},
            "kernels_ms_cold": cold,
            "roofline": {"bound": "hbm", "kernel": dom_name, "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "frac_of_measured_copy": round(achieved / HBM_MEASURED_COPY_GBPS, 4),
                         "frac_cold": frac_cold,
                         "regime": "frac: warm steps (back to back; the 256 MiB Infinity Cache holds part "
                                   "of the previous call's output); frac_cold: the same kernel after a "
                                   "512 MiB flush",
                         "alg_bytes_per_launch": ALG_BYTES_PER_REC * n,
                         "traffic": prof["traffic"],
                         "traffic_over_alg": (round(prof["traffic"] / (ALG_BYTES_PER_REC * n), 4)
                                              if prof["traffic"] else None),
                         "committed_rocprof_avg_us": prof["committed_rocprof_avg_us"],
                         "kernel_stats_file": prof["kernel_stats_file"],
                         "pmc_file": prof["pmc_file"]},
            "verify": verify,
        }
        if gather:
            line["gather"] = gather
        if world > 1:
            seen = [r["rccl"] for r in per_rank]
            line["rccl"] = {"ranks_seen": [r["rank"] for r in seen] if all(seen) else None,
                            "nranks_seen": sorted({r["nranks"] for r in seen}) if all(seen) else None,
                            "collective": gather["collective"] if gather else None,
                            "note": None if all(seen) else (comm_note or "no libsrpc_gpu communicator "
                                                            f"(--dist-backend {args.dist_backend})")}
        line["per_rank"] = per_rank
        if strong:
            with open(os.path.join(ROOT, "tests", "golden", "manifest.json")) as f:
                streams = json.load(f)["streams"]
            want = {st["records"]: st["sha256"] for k, st in streams.items()
                    if k.startswith("quad_body_")}.get(strong["records_total"])
            strong["matches_reference"] = (strong["sha256"] == want) if want else None
            line["strong_scaling"] = strong
        if pcie:
            line["pcie_inclusive"] = pcie
        if world == 1 and args.cpu_seconds > 0:
            line["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds)
        line["native_lib"] = _lib.so_path()
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
