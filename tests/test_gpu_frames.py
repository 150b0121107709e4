"""Batches of socket frames of several methods bucketed on the device
(srpc_frames_classify / _gather / _scatter, include/srpc_gpu.h), the kernels
under srpc::gpu::batch_server.  The reference server dispatches one frame at
a time by the method name it starts with (server.hpp:58-69); here a batch of
frames is classified at once and each class is gathered into one plan's
contiguous records.  Checked against a host model of that dispatch:
- frames of three registered methods (two body sizes) in random order;
- foreign frames: another method of the same length, a corrupt BE32 length,
  the right method with a longer body, random garbage, empty payloads;
- response offsets (exclusive scan of the per-frame response bytes), the
  gathered records and the scattered responses byte for byte."""
import struct

import numpy as np
import pytest

import srpc_amd
from srpc_amd import FrameClassifier, GpuPacker, Schema, framed_request_prefix

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

from tests.test_gpu_parity import dev, empty, host  # noqa: E402

UNKNOWN = 0xFF
METHODS = [(srpc_amd.NUMBER, "Calculator_servicer::square", 23),
           (srpc_amd.TWO_NUMBERS, "Calculator_servicer::add", 23),
           (srpc_amd.QUAD, "Svc_servicer::quad", 40)]


def _frames(n, rng, foreign_frac):
    """n frames; returns (buffer bytes, offsets, expected classes)."""
    pres = [framed_request_prefix(s, m) for s, m, _ in METHODS]
    parts, cls = [], []
    for i in range(n):
        if rng.random() < foreign_frac:
            kind = int(rng.integers(0, 5))
            if kind == 0:  # same length as square, one byte of the name changed
                f = bytearray(pres[0] + rng.bytes(4))
                f[20] ^= 0x01
            elif kind == 1:  # corrupt BE32 length: the frame ends elsewhere
                body = rng.bytes(int(rng.integers(0, 40)))
                f = struct.pack(">I", len(body)) + body
            elif kind == 2:  # the right method with a longer body
                body = pres[1][4:] + rng.bytes(12)
                f = struct.pack(">I", len(body)) + body
            elif kind == 3:  # an empty payload
                f = struct.pack(">I", 0)
            else:  # a string-bodied method: not a fixed-size plan
                name = b"Calculator_servicer::echo"
                msg = rng.bytes(int(rng.integers(0, 30)))
                body = (struct.pack("<Q", len(name)) + name + struct.pack("<Q", 6) + b"String"
                        + struct.pack("<Q", len(msg)) + msg)
                f = struct.pack(">I", len(body)) + body
            parts.append(bytes(f))
            cls.append(UNKNOWN)
        else:
            k = int(rng.integers(0, len(METHODS)))
            parts.append(pres[k] + rng.bytes(METHODS[k][0].body_bytes))
            cls.append(k)
    offs = np.zeros(n, np.uint32)
    if n:
        offs[1:] = np.cumsum([len(p) for p in parts[:-1]])
    return b"".join(parts), offs, np.array(cls, np.uint8)


@pytest.fixture(scope="module")
def classifier():
    plans = [GpuPacker(s, framed_request_prefix(s, m)) for s, m, _ in METHODS]
    return FrameClassifier([(p, rb) for p, (_, _, rb) in zip(plans, METHODS)])


@pytest.mark.parametrize("n,foreign", [(0, 0.0), (1, 0.0), (1, 1.0), (63, 0.3), (4097, 0.0), (4097, 0.1),
                                       (200_003, 0.01), (50_000, 0.9)])
def test_classify_gather_scatter(classifier, n, foreign):
    rng = np.random.default_rng(n + int(foreign * 100))
    buf, offs, want = _frames(n, rng, foreign)
    K = len(METHODS)
    d_buf = dev(np.frombuffer(buf, np.uint8)) if buf else empty(16)
    d_offs = dev(offs) if n else empty(16)
    d_cls, d_idx = empty(n + 16), empty(4 * K * n + 16)
    d_counts, d_out_off = empty(8 * (K + 2)), empty(8 * (n + 1))
    sb = classifier.scratch_bytes(n)
    scratch = torch.empty(sb, dtype=torch.uint8, device="cuda:0")
    classifier.classify(d_buf, len(buf), d_offs, n, d_cls, d_idx, d_counts, d_out_off, scratch, sb)
    counts = host(d_counts, 8 * (K + 2), np.uint64)
    rb = np.array([m[2] for m in METHODS] + [0], np.uint64)
    per = rb[np.where(want == UNKNOWN, K, want)] if n else np.zeros(0, np.uint64)
    assert [int(counts[k]) for k in range(K)] == [int((want == k).sum()) for k in range(K)]
    assert int(counts[K]) == int(per.sum()) and int(counts[K + 1]) == int((want == UNKNOWN).sum())
    out_off = host(d_out_off, 8 * (n + 1), np.uint64)
    exp_off = np.zeros(n + 1, np.uint64)
    exp_off[1:] = np.cumsum(per)
    assert np.array_equal(out_off, exp_off)
    if not n:
        return
    assert np.array_equal(host(d_cls, n), want)
    idx = host(d_idx, 4 * K * n, np.uint32).reshape(K, n)
    out = empty(int(counts[K]) + 16)
    expect_out = np.zeros(int(counts[K]), np.uint8)
    for k, (schema, _, rbk) in enumerate(METHODS):
        nk = int(counts[k])
        if not nk:
            continue
        got = idx[k, :nk]
        assert np.array_equal(np.sort(got), np.flatnonzero(want == k).astype(np.uint32)), k
        fin = len(framed_request_prefix(schema, METHODS[k][1])) + schema.body_bytes
        g = empty(nk * fin + 16)
        d_ik = d_idx[4 * k * n: 4 * (k * n + nk)] if nk else empty(16)
        classifier.gather(d_buf, d_offs, d_ik, nk, fin, g)
        bnp = np.frombuffer(buf, np.uint8)
        exp_g = np.concatenate([bnp[offs[j]: offs[j] + fin] for j in got])
        assert host(g, nk * fin).tobytes() == exp_g.tobytes(), k
        resp = rng.integers(0, 256, nk * rbk, dtype=np.uint8)
        classifier.scatter(dev(resp), d_ik, nk, rbk, d_out_off, out)
        for j, f in enumerate(got):
            expect_out[exp_off[f]: exp_off[f] + rbk] = resp[j * rbk:(j + 1) * rbk]
    assert host(out, int(counts[K])).tobytes() == expect_out.tobytes()


def test_rejects_bad_arguments(classifier):
    L = srpc_amd._lib.lib()
    import ctypes as C
    out = C.c_uint64()
    assert L.srpc_frames_scratch_bytes(10, 0, C.byref(out)) == srpc_amd._lib.SRPC_E_INVALID
    assert L.srpc_frames_scratch_bytes(10, 17, C.byref(out)) == srpc_amd._lib.SRPC_E_INVALID
    # a string schema is not a fixed-size frame plan
    sp = GpuPacker(Schema("S", (("s", srpc_amd.STRING),)), b"\x00\x00\x00\x08xxxx")
    plans = (C.c_void_p * 1)(sp._h.value)
    rb = (C.c_uint32 * 1)(5)
    buf = empty(64)
    rc = L.srpc_frames_classify(plans, rb, 1, buf.data_ptr(), 8, buf.data_ptr(), 1, buf.data_ptr(), buf.data_ptr(),
                                buf.data_ptr(), buf.data_ptr(), buf.data_ptr(), 4096, None)
    assert rc == srpc_amd._lib.SRPC_E_INVALID


def test_offsets_past_the_buffer_are_unknown(classifier):
    """Offsets that run backwards or past buf_len (a caller bug, not a peer
    frame): those frames are UNKNOWN and no byte past the buffer is read --
    frame 1 is exactly one square request long but ends past buf_len."""
    pre = framed_request_prefix(METHODS[0][0], METHODS[0][1])
    one = pre + b"\x07\x00\x00\x00"
    buf = one * 4
    L = len(one)
    offs = np.array([0, L, 2 * L, L], np.uint32)
    n, K = 4, len(METHODS)
    d_buf = dev(np.frombuffer(buf, np.uint8))
    d_offs = dev(offs)
    d_cls, d_idx = empty(n + 16), empty(4 * K * n + 16)
    d_counts, d_out_off = empty(8 * (K + 2)), empty(8 * (n + 1))
    sb = classifier.scratch_bytes(n)
    scratch = torch.empty(sb, dtype=torch.uint8, device="cuda:0")
    # buf_len = 2L - 1 (the allocation holds four whole requests)
    classifier.classify(d_buf, 2 * L - 1, d_offs, n, d_cls, d_idx, d_counts, d_out_off, scratch, sb)
    # frame 0 [0, L): a square request; frame 1 [L, 2L): one request long but
    # ends past buf_len; frame 2 [2L, L): backwards; frame 3 [L, 2L - 1): short
    assert host(d_cls, n).tolist() == [0, UNKNOWN, UNKNOWN, UNKNOWN]
    counts = host(d_counts, 8 * (K + 2), np.uint64)
    assert int(counts[K + 1]) == 3 and int(counts[0]) == 1


def test_sixteen_methods_one_body():
    """SRPC_FRAMES_MAX_PLANS plans of the same body size (frames differ only in
    the method name): every bucket gets exactly its frames."""
    K = srpc_amd._lib.SRPC_FRAMES_MAX_PLANS
    methods = [(srpc_amd.NUMBER, f"Svc_servicer::m{k:02d}", 23) for k in range(K)]
    plans = [GpuPacker(s, framed_request_prefix(s, m)) for s, m, _ in methods]
    fc = FrameClassifier([(p, rb) for p, (_, _, rb) in zip(plans, methods)])
    n = 9001
    rng = np.random.default_rng(16)
    want = rng.integers(0, K + 1, n)  # K = a foreign method
    pres = [framed_request_prefix(s, m) for s, m, _ in methods]
    foreign = framed_request_prefix(srpc_amd.NUMBER, "Svc_servicer::zzz")
    assert all(len(q) == len(foreign) for q in pres)
    parts = [(pres[k] if k < K else foreign) + rng.bytes(4) for k in want]
    buf = b"".join(parts)
    offs = (np.arange(n, dtype=np.uint32) * len(parts[0])).astype(np.uint32)
    d_buf, d_offs = dev(np.frombuffer(buf, np.uint8)), dev(offs)
    d_cls, d_idx = empty(n + 16), empty(4 * K * n + 16)
    d_counts, d_out_off = empty(8 * (K + 2)), empty(8 * (n + 1))
    sb = fc.scratch_bytes(n)
    scratch = torch.empty(sb, dtype=torch.uint8, device="cuda:0")
    fc.classify(d_buf, len(buf), d_offs, n, d_cls, d_idx, d_counts, d_out_off, scratch, sb)
    counts = host(d_counts, 8 * (K + 2), np.uint64)
    cls = host(d_cls, n)
    exp_cls = np.where(want == K, UNKNOWN, want).astype(np.uint8)
    assert np.array_equal(cls, exp_cls)
    idx = host(d_idx, 4 * K * n, np.uint32).reshape(K, n)
    for k in range(K):
        nk = int(counts[k])
        assert nk == int((want == k).sum())
        assert np.array_equal(np.sort(idx[k, :nk]), np.flatnonzero(want == k).astype(np.uint32))
    assert int(counts[K + 1]) == int((want == K).sum()) and int(counts[K]) == 23 * int((want < K).sum())
