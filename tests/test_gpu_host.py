"""Host-terminated batches (ABI 7: srpc_gpu_pack_host / srpc_gpu_unpack_host):
columns and wire bytes in pinned host memory, pipelined through a ring of
device chunk buffers.  Every case against the oracle's wire and the host
columns it came from; chunk sizes from 1 record to more than the batch,
rings of 1-3 slots, the direct mode (chunk 0: the kernels on the mapped
pinned buffers, no copies), the DWORD and TILE kernel families, an envelope prefix,
and the unpack's statuses (a bad prefix deep in a later chunk, a short wire)
reported batch-relative as srpc_gpu_unpack reports them."""
import numpy as np
import pytest

import oracle
import srpc_amd
from srpc_amd import (QUAD, GpuPacker, Schema, SRPC_ERR_BOUNDS, SRPC_STATUS_BOUNDS, SRPC_STATUS_PREFIX)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

from tests.test_gpu_parity import read_status, status_buf  # noqa: E402

ALL = [oracle.BOOL, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64]
NP = {oracle.BOOL: np.uint8, oracle.INT8: np.int8, oracle.CHAR: np.uint8, oracle.INT16: np.int16,
      oracle.INT32: np.int32, oracle.INT64: np.int64}


def host_cols(kinds, n, rng):
    cols = []
    for k in kinds:
        a = rng.integers(0, 256, n * oracle.KIND_SIZE[k], dtype=np.uint8).view(NP[k]).copy()
        if k == oracle.BOOL:
            a &= 1
        cols.append(a)
    return cols


def pinned(a: np.ndarray):
    t = torch.empty(max(a.nbytes, 1), dtype=torch.uint8).pin_memory()
    if a.nbytes:
        t[:a.nbytes].copy_(torch.from_numpy(a.view(np.uint8).reshape(-1).copy()))
    return t


def scratch_for(p, chunk, depth):
    sb = p.host_scratch_bytes(chunk, depth)
    t = torch.empty(sb + 256, dtype=torch.uint8, device="cuda:0")
    return t, t.data_ptr() + (-t.data_ptr()) % 256, sb


def plan(kind):
    if kind == "quad":
        return QUAD.kinds, GpuPacker(QUAD)
    sch = Schema("S", tuple((f"f{i}", k) for i, k in enumerate(ALL)))
    return ALL, GpuPacker.for_request(sch, "Svc_servicer::m")


@pytest.mark.parametrize("kind", ["quad", "all_request"])
@pytest.mark.parametrize("n,chunk,depth", [(1, 1, 1), (1000, 1, 3), (1000, 16, 2), (100_003, 4096, 3),
                                           (100_003, 65_536, 1), (100_003, 200_000, 3), (262_144, 32_768, 3),
                                           # chunk 0: direct, the kernels on the mapped host buffers
                                           (1, 0, 1), (100_003, 0, 1), (262_144, 0, 3)])
def test_host_round_trip_vs_oracle(kind, n, chunk, depth):
    kinds, p = plan(kind)
    rng = np.random.default_rng(n + chunk + depth)
    cols = host_cols(kinds, n, rng)
    want = bytes(oracle.pack(kinds, cols, n, p.prefix))
    h_cols = [pinned(c) for c in cols]
    h_wire = torch.full((len(want) + 16,), 0xA5, dtype=torch.uint8).pin_memory()
    keep, sp, sb = scratch_for(p, chunk, depth)
    if chunk == 0:
        assert sb == 0
    s = torch.cuda.current_stream()
    p.pack_host(h_cols, n, h_wire, chunk, sp, sb, depth=depth, stream=s)
    torch.cuda.synchronize()
    assert h_wire[:len(want)].numpy().tobytes() == want
    assert (h_wire[len(want):].numpy() == 0xA5).all()  # nothing past the batch
    back = [pinned(np.full(c.nbytes, 0x5A, np.uint8)) for c in cols]
    st = status_buf()
    assert p.unpack_host(h_wire, len(want), n, back, chunk, sp, sb, depth=depth, status=st, stream=s) == 0
    torch.cuda.synchronize()
    assert read_status(st) == (0, 2**64 - 1)
    for b, c in zip(back, cols):
        assert b[:c.nbytes].numpy().tobytes() == c.tobytes()


@pytest.mark.parametrize("n,chunk,depth", [(1000, 1, 3), (100_003, 4096, 2), (262_144, 32_768, 3)])
def test_host_round_trip_two_streams(monkeypatch, n, chunk, depth):
    """The pipeline with the kernels on the H2D stream (SRPC_HOST_STREAMS=2)."""
    monkeypatch.setenv("SRPC_HOST_STREAMS", "2")
    test_host_round_trip_vs_oracle("all_request", n, chunk, depth)
    test_host_round_trip_vs_oracle("quad", n, chunk, depth)


def test_host_unpack_reports_batch_relative_statuses():
    kinds, p = plan("all_request")
    n, chunk = 50_000, 4096
    cols = host_cols(kinds, n, np.random.default_rng(5))
    wire = bytearray(oracle.pack(kinds, cols, n, p.prefix))
    rb = p.record_bytes
    for bad in (30_001, 41_000):  # two bad prefixes in later chunks: the first is reported
        wire[bad * rb + 3] ^= 0x40
    h_wire = pinned(np.frombuffer(bytes(wire), np.uint8))
    back = [pinned(np.zeros(c.nbytes, np.uint8)) for c in cols]
    keep, sp, sb = scratch_for(p, chunk, 3)
    st = status_buf()
    p.unpack_host(h_wire, len(wire), n, back, chunk, sp, sb, status=st)
    torch.cuda.synchronize()
    assert read_status(st) == (SRPC_STATUS_PREFIX, 30_001)
    # a wire short of the batch: the records that fit, BOUNDS at the first that does not
    short = (n - 777) * rb + 5
    back2 = [pinned(np.zeros(c.nbytes, np.uint8)) for c in cols]
    st2 = status_buf()
    assert p.unpack_host(pinned(np.frombuffer(bytes(oracle.pack(kinds, cols, n, p.prefix)), np.uint8)), short, n,
                         back2, chunk, sp, sb, status=st2) == SRPC_ERR_BOUNDS
    torch.cuda.synchronize()
    assert read_status(st2) == (SRPC_STATUS_BOUNDS, n - 777)
    for b, c in zip(back2, cols):
        k = (n - 777) * c.itemsize
        assert b[:k].numpy().tobytes() == c.tobytes()[:k]


def test_host_argument_errors():
    kinds, p = plan("quad")
    keep, sp, sb = scratch_for(p, 1024, 2)
    cols = [pinned(np.zeros(4096, np.uint8)) for _ in kinds]
    h_wire = pinned(np.zeros(16 * 1024, np.uint8))
    with pytest.raises(srpc_amd.SrpcError):  # scratch too small for the ring
        p.pack_host(cols, 1024, h_wire, 1024, sp, sb - 256, depth=2)
    with pytest.raises(srpc_amd.SrpcError):  # scratch not 256-byte aligned
        p.pack_host(cols, 1024, h_wire, 1024, sp + 16, sb, depth=2)
    with pytest.raises(srpc_amd.SrpcError):  # wire capacity short of the batch
        p.pack_host(cols, 1024, h_wire, 1024, sp, sb, depth=2, wire_cap=16 * 1023)
    with pytest.raises(srpc_amd.SrpcError):  # direct mode on pageable host memory (not device-mapped)
        import numpy as _np
        pageable = [_np.zeros(1024, _np.int32) for _ in kinds]
        p.pack_host([a.ctypes.data for a in pageable], 1024, h_wire, 0, 0, 0, depth=1)
    with pytest.raises(srpc_amd.SrpcError):  # ring of 0 slots
        p.host_scratch_bytes(1024, 0)
    strs = GpuPacker(Schema("T", (("s", oracle.STRING),)))
    with pytest.raises(srpc_amd.SrpcError):  # string schemas have no fixed chunk
        strs.host_scratch_bytes(1024, 2)


def _hip():
    import ctypes
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    lib.hipHostFree.argtypes = [ctypes.c_void_p]
    return lib


def test_host_direct_refuses_short_pinned_allocations():
    """Direct mode checks each pinned allocation's extent (the runtime's own
    record of it), not only that its base is mapped: a wire or column buffer
    shorter than the batch is refused before anything runs."""
    import ctypes
    hip = _hip()
    kinds, p = plan("quad")
    n = 65_536                     # 1 MiB of wire, 256 KiB per column: four times the 64 KiB allocation
    small = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(small), 64 * 1024, 0) == 0
    try:
        cols = host_cols(kinds, n, np.random.default_rng(1))
        h_cols = [pinned(c) for c in cols]
        h_wire = pinned(np.zeros(16 * n, np.uint8))
        with pytest.raises(srpc_amd.SrpcError):   # a wire allocation short of the batch
            p.pack_host(h_cols, n, small.value, 0, 0, 0, depth=1, wire_cap=16 * n)
        with pytest.raises(srpc_amd.SrpcError):   # one column's allocation short of the batch
            p.pack_host(h_cols[:3] + [small.value], n, h_wire, 0, 0, 0, depth=1)
        with pytest.raises(srpc_amd.SrpcError):   # unpack into a short column
            p.unpack_host(h_wire, 16 * n, n, h_cols[:3] + [small.value], 0, 0, 0, depth=1)
        # the same allocation is accepted for a batch it covers
        p.pack_host(h_cols, 4096, small.value, 0, 0, 0, depth=1, wire_cap=16 * 4096)
        torch.cuda.synchronize()
        want = bytes(oracle.pack(kinds, [c[:4096] for c in cols], 4096))
        assert ctypes.string_at(small.value, len(want)) == want
    finally:
        torch.cuda.synchronize()
        hip.hipHostFree(small)


def test_host_direct_short_wire_reports_bounds():
    """Direct mode, a wire shorter than the batch: the records that fit, then
    (SRPC_ERR_BOUNDS, first bad = the first record that does not fit)."""
    kinds, p = plan("all_request")
    n = 30_000
    cols = host_cols(kinds, n, np.random.default_rng(9))
    wire = bytes(oracle.pack(kinds, cols, n, p.prefix))
    rb = p.record_bytes
    short = (n - 321) * rb + 7
    back = [pinned(np.zeros(c.nbytes, np.uint8)) for c in cols]
    st = status_buf()
    assert p.unpack_host(pinned(np.frombuffer(wire, np.uint8)), short, n, back, 0, 0, 0, depth=1,
                         status=st) == SRPC_ERR_BOUNDS
    torch.cuda.synchronize()
    assert read_status(st) == (SRPC_STATUS_BOUNDS, n - 321)
    for b, c in zip(back, cols):
        k = (n - 321) * c.itemsize
        assert b[:k].numpy().tobytes() == c.tobytes()[:k]
    # no record fits: BOUNDS at 0, nothing decoded
    st0 = status_buf()
    assert p.unpack_host(pinned(np.frombuffer(wire, np.uint8)), rb - 1, n, back, 0, 0, 0, depth=1,
                         status=st0) == SRPC_ERR_BOUNDS
    torch.cuda.synchronize()
    assert read_status(st0) == (SRPC_STATUS_BOUNDS, 0)


def test_host_pipe_pool_grows_with_concurrency_not_threads():
    """the chunked calls borrow their streams from a per-device
    pool.  64 short-lived threads, one after another, add at most one pipe;
    4 threads at once add at most 4."""
    import ctypes
    import threading
    hook = srpc_amd._lib.lib().srpc_debug_host_pipes
    hook.argtypes, hook.restype = [ctypes.c_int], ctypes.c_uint64
    kinds, p = plan("quad")
    n, chunk = 20_000, 4096
    cols = host_cols(kinds, n, np.random.default_rng(2))
    want = bytes(oracle.pack(kinds, cols, n))
    h_cols = [pinned(c) for c in cols]
    keep = [scratch_for(p, chunk, 3) for _ in range(4)]
    wires = [pinned(np.zeros(len(want), np.uint8)) for _ in range(4)]
    errs = []

    def one(i):
        try:
            _, sp, sb = keep[i]
            s = torch.cuda.Stream()
            p.pack_host(h_cols, n, wires[i], chunk, sp, sb, depth=3, stream=s)
            s.synchronize()
            assert wires[i].numpy().tobytes() == want
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    one(0)
    base = hook(0)
    for _ in range(64):
        t = threading.Thread(target=one, args=(0,))
        t.start()
        t.join()
    assert not errs and hook(0) - base <= 1, (errs, hook(0) - base)
    ts = [threading.Thread(target=one, args=(i,)) for i in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs and hook(0) - base <= 4, (errs, hook(0) - base)


def _hook(name, res, args):
    import ctypes
    fn = getattr(srpc_amd._lib.lib(), name)
    fn.restype, fn.argtypes = res, args
    return fn


def test_host_pipes_not_shared_across_streams_while_busy():
    """a pipe goes back to the pool when its call has been
    enqueued, long before its copies finish.  A call on ANOTHER caller stream
    must not take that busy pipe (its copies would queue behind the first
    call's on the same internal streams); a call on the SAME stream may (its
    work is ordered behind the first call's anyway); once the calls have
    drained, a call on any stream reuses an idle pipe (one of these or an
    earlier test's) instead of making one."""
    import ctypes
    last = _hook("srpc_debug_host_last_pipe", ctypes.c_uint64, [])
    kinds, p = plan("quad")
    n, chunk = 1 << 22, 1 << 18            # 64 MiB each way: milliseconds of PCIe, microseconds to enqueue
    cols = host_cols(kinds, n, np.random.default_rng(4))
    want = bytes(oracle.pack(kinds, cols, n))
    h_cols = [pinned(c) for c in cols]
    wires = [pinned(np.zeros(len(want), np.uint8)) for _ in range(3)]
    keep = [scratch_for(p, chunk, 3) for _ in range(3)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    p.pack_host(h_cols, n, wires[0], chunk, keep[0][1], keep[0][2], depth=3, stream=s1)
    a = last()
    p.pack_host(h_cols, n, wires[1], chunk, keep[1][1], keep[1][2], depth=3, stream=s2)
    b = last()
    busy = not (s1.query())  # the first call was still moving bytes when the second borrowed
    p.pack_host(h_cols, n, wires[2], chunk, keep[2][1], keep[2][2], depth=3, stream=s1)
    c = last()
    torch.cuda.synchronize()
    for w in wires:
        assert w.numpy().tobytes() == want
    if busy:
        assert a != b, "a busy pipe was lent to a call on another stream"
    assert c == a, "a call on the same stream should reuse that stream's pipe"
    made = _hook("srpc_debug_host_pipes_made", ctypes.c_uint64, [])
    before = made()
    p.pack_host(h_cols, n, wires[1], chunk, keep[1][1], keep[1][2], depth=3, stream=torch.cuda.Stream())
    assert made() == before, "an idle pipe should be reused, not a new one made"
    torch.cuda.synchronize()


def test_host_direct_accepts_host_registered_memory():
    """direct mode on buffers pinned by hipHostRegister (mapped)
    -- numpy memory the runtime did not allocate: the batch that fits is
    accepted and exact, a batch longer than the registered range is refused."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    kinds, p = plan("quad")
    n = 65_536
    cols = host_cols(kinds, n, np.random.default_rng(6))
    want = bytes(oracle.pack(kinds, cols, n))
    page = 4096
    raw = np.zeros(len(want) + 2 * page, np.uint8)
    off = (-raw.ctypes.data) % page
    wire = raw[off:off + len(want)]                       # page-aligned, exactly the batch
    raw_cols = [np.zeros(c.nbytes + 2 * page, np.uint8) for c in cols]
    reg_cols = []
    for r, c in zip(raw_cols, cols):
        o = (-r.ctypes.data) % page
        v = r[o:o + c.nbytes]
        v[:] = c.view(np.uint8)
        reg_cols.append(v)
    regs = [wire] + reg_cols
    for a in regs:
        assert hip.hipHostRegister(a.ctypes.data, a.nbytes, 2) == 0  # hipHostRegisterMapped
    try:
        p.pack_host([c.ctypes.data for c in reg_cols], n, wire.ctypes.data, 0, 0, 0, depth=1,
                    wire_cap=len(want))
        torch.cuda.synchronize()
        assert wire.tobytes() == want
        with pytest.raises(srpc_amd.SrpcError):   # one record more than the registered wire holds
            p.pack_host([c.ctypes.data for c in reg_cols], n + 1, wire.ctypes.data, 0, 0, 0, depth=1,
                        wire_cap=len(want) + 16)
    finally:
        torch.cuda.synchronize()
        for a in regs:
            hip.hipHostUnregister(a.ctypes.data)


@pytest.mark.parametrize("direction", ["pack", "unpack"])
def test_host_ring_error_drains_into_callers_stream(direction):
    """An error part way through the chunked ring (injected at chunk 14 of 16
    through the test hook srpc_debug_host_fail_at) returns it, and the caller's
    stream is ordered after every copy the call already enqueued: once that
    stream is synchronized, chunks 0..13 are complete in the host buffers."""
    import ctypes
    fail_at = _hook("srpc_debug_host_fail_at", None, [ctypes.c_uint64])
    kinds, p = plan("quad")
    n, chunk = 16 * 65_536, 65_536
    cols = host_cols(kinds, n, np.random.default_rng(3))
    want = bytes(oracle.pack(kinds, cols, n))
    keep, sp, sb = scratch_for(p, chunk, 3)
    s = torch.cuda.Stream()
    fail_at(14)
    done = 14 * chunk
    try:
        if direction == "pack":
            h_cols = [pinned(c) for c in cols]
            h_wire = pinned(np.zeros(len(want), np.uint8))
            with pytest.raises(srpc_amd.SrpcError):
                p.pack_host(h_cols, n, h_wire, chunk, sp, sb, depth=3, stream=s)
            s.synchronize()
            assert h_wire[:done * 16].numpy().tobytes() == want[:done * 16]
        else:
            h_wire = pinned(np.frombuffer(want, np.uint8))
            back = [pinned(np.zeros(c.nbytes, np.uint8)) for c in cols]
            with pytest.raises(srpc_amd.SrpcError):
                p.unpack_host(h_wire, len(want), n, back, chunk, sp, sb, depth=3, stream=s)
            s.synchronize()
            for b, c in zip(back, cols):
                assert b[:done * c.itemsize].numpy().tobytes() == c.tobytes()[:done * c.itemsize]
    finally:
        fail_at(2**64 - 1)
        torch.cuda.synchronize()
    # disarmed: the same call succeeds
    if direction == "pack":
        p.pack_host(h_cols, n, h_wire, chunk, sp, sb, depth=3, stream=s)
        s.synchronize()
        assert h_wire.numpy().tobytes() == want
