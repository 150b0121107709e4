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
  gathered records and the scattered responses byte for byte;
- methods with string fields (variable-length frames) among fixed ones:
  classified by prefix, BE32 and a walk of their fields, gathered with a
  record index, unpacked, answered, packed, framed and scattered into the
  reply stream the reference server writes (srpc_frames_gather_var /
  _scatter_var / _offsets)."""
import struct

import numpy as np
import pytest

import oracle
import srpc_amd
from srpc_amd import FrameClassifier, GpuPacker, Schema, framed_request_prefix, request_prefix

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

from tests.test_gpu_parity import dev, empty, host, read_status, status_buf  # noqa: E402

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
    # a plan without a prefix cannot be told apart from another method's frames
    # (string plans are accepted since ABI v4: register_var_method)
    sp = GpuPacker(Schema("S", (("s", srpc_amd.STRING),)))
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


# ---- methods with string fields (variable-length frames) -----------------------
MP = Schema("multiple_primitives", (("a1", srpc_amd.INT8), ("a2", srpc_amd.CHAR), ("a3", srpc_amd.INT64),
                                    ("s", srpc_amd.STRING)))
TS = Schema("TwoStr", (("x", srpc_amd.STRING), ("n", srpc_amd.INT32), ("y", srpc_amd.STRING)))
VAR_METHODS = [(MP, "Svc_servicer::echo"), (TS, "Svc_servicer::cat")]


def _var_frame(schema, method, vals):
    """BE32 | request record of one string-bodied request (vals: field values)."""
    body = request_prefix(method, schema.name)
    for (_, k), v in zip(schema.fields, vals):
        if k == srpc_amd.STRING:
            body += struct.pack("<Q", len(v)) + v
        else:
            body += np.array([v], oracle.KIND_DTYPE[k]).tobytes()
    return struct.pack(">I", len(body)) + body


def _rand_vals(schema, rng, maxlen):
    out = []
    for _, k in schema.fields:
        if k == srpc_amd.STRING:
            out.append(rng.bytes(int(rng.integers(0, maxlen + 1))))
        else:
            info = np.iinfo(oracle.KIND_DTYPE[k])
            out.append(int(rng.integers(info.min, info.max, endpoint=True)))
    return out


def _mixed_var_frames(n, rng, foreign_frac, maxlen=40):
    """Fixed methods (METHODS), string methods (VAR_METHODS) and foreign frames
    near the string ones: a string length past the frame, one trailing byte, a
    BE32 that disagrees with the frame, a payload shorter than the fixed part,
    a method name of the same length.  Returns (buf, offs, classes, values)."""
    pres = [framed_request_prefix(s, m) for s, m, _ in METHODS]
    K = len(METHODS)
    parts, cls, vals = [], [], []
    for i in range(n):
        u = rng.random()
        if u < foreign_frac:
            s, m = VAR_METHODS[int(rng.integers(0, 2))]
            kind = int(rng.integers(0, 5))
            v = _rand_vals(s, rng, maxlen)
            f = bytearray(_var_frame(s, m, v))
            if kind == 0:  # the first string's length runs past the frame
                at = 4 + len(request_prefix(m, s.name)) + (10 if s is MP else 0)
                f[at:at + 8] = struct.pack("<Q", len(f))
            elif kind == 1:  # a trailing byte (BE32 counts it)
                f += b"\x00"
                f[0:4] = struct.pack(">I", len(f) - 4)
            elif kind == 2:  # BE32 one short of the frame
                f[0:4] = struct.pack(">I", len(f) - 5)
            elif kind == 3:  # cut inside the fixed part
                f = f[:4 + len(request_prefix(m, s.name)) + 3]
                f[0:4] = struct.pack(">I", len(f) - 4)
            else:  # same-length method name, one byte changed
                f[4 + 8 + 3] ^= 0x20
            parts.append(bytes(f))
            cls.append(UNKNOWN)
            vals.append(None)
        elif u < foreign_frac + 0.5:
            j = int(rng.integers(0, 2))
            s, m = VAR_METHODS[j]
            v = _rand_vals(s, rng, maxlen)
            parts.append(_var_frame(s, m, v))
            cls.append(K + j)
            vals.append(v)
        else:
            k = int(rng.integers(0, K))
            parts.append(pres[k] + rng.bytes(METHODS[k][0].body_bytes))
            cls.append(k)
            vals.append(None)
    offs = np.zeros(n, np.uint32)
    if n:
        offs[1:] = np.cumsum([len(p) for p in parts[:-1]])
    return b"".join(parts), offs, np.array(cls, np.uint8), vals


@pytest.fixture(scope="module")
def mixed_classifier():
    fixed = [(GpuPacker(s, framed_request_prefix(s, m)), rb) for s, m, rb in METHODS]
    var = [(GpuPacker.for_request(s, m), 0) for s, m in VAR_METHODS]
    return FrameClassifier(fixed + var)


def _var_responses(schema, vals):
    """Host model of a string method's responses: ints + 1, every string with
    b"!" appended; returns (columns, str_offs) in record order."""
    cols, offs = [], []
    for f, (_, k) in enumerate(schema.fields):
        if k == srpc_amd.STRING:
            ss = [v[f] + b"!" for v in vals]
            o = np.zeros(len(ss) + 1, np.uint64)
            o[1:] = np.cumsum([len(x) for x in ss])
            cols.append(np.frombuffer(b"".join(ss) + b"\0", np.uint8))
            offs.append(o)
        else:
            dt = oracle.KIND_DTYPE[k]
            cols.append(np.array([v[f] for v in vals], np.int64).astype(dt) + dt(1))
            offs.append(None)
    return cols, offs


@pytest.mark.parametrize("n,foreign", [(1, 0.0), (5, 0.0), (777, 0.2), (50_001, 0.05), (20_000, 0.0)])
def test_string_methods_classify_gather_pack_scatter(mixed_classifier, n, foreign):
    """Fixed and string-bodied methods in one batch: classified on the device
    (string frames by prefix, BE32 and a walk of their fields), each string
    bucket gathered with its record index, unpacked, answered (host model of
    a handler), packed with srpc_gpu_pack_var, then the reply stream's offsets
    recomputed and every response scattered -- compared byte for byte with
    the reply stream the reference server would write."""
    rng = np.random.default_rng(n + 7)
    buf, offs, want, vals = _mixed_var_frames(n, rng, foreign)
    K, KV = len(METHODS), len(VAR_METHODS)
    KT = K + KV
    fc = mixed_classifier
    d_buf, d_offs = dev(np.frombuffer(buf, np.uint8)), dev(offs)
    d_cls, d_idx = empty(n + 16), empty(4 * KT * n + 16)
    d_counts, d_out_off = empty(8 * (KT + 2)), empty(8 * (n + 1))
    sb = fc.scratch_bytes(n)
    scratch = torch.empty(sb, dtype=torch.uint8, device="cuda:0")
    fc.classify(d_buf, len(buf), d_offs, n, d_cls, d_idx, d_counts, d_out_off, scratch, sb)
    assert np.array_equal(host(d_cls, n), want)
    counts = host(d_counts, 8 * (KT + 2), np.uint64)
    assert [int(c) for c in counts[:KT]] == [int((want == k).sum()) for k in range(KT)]
    idx = host(d_idx, 4 * KT * n, np.uint32).reshape(KT, n)
    # fixed methods: random response records, as test_classify_gather_scatter
    fixed_resp = {}
    for k in range(K):
        nk = int(counts[k])
        fixed_resp[k] = rng.integers(0, 256, nk * METHODS[k][2], dtype=np.uint8)
    # string methods: gather -> unpack_var -> host handler -> pack_var
    var_rec, var_wire, var_out = [None] * KT, {}, {}
    bnp = np.frombuffer(buf, np.uint8)
    for j, (schema, method) in enumerate(VAR_METHODS):
        k = K + j
        nk = int(counts[k])
        frames = idx[k, :nk]
        assert np.array_equal(np.sort(frames), np.flatnonzero(want == k).astype(np.uint32))
        if not nk:
            var_rec[k], var_wire[k], var_out[k] = empty(16), empty(16), []
            continue
        payloads = [bytes(bnp[offs[f] + 4: (offs[f + 1] if f + 1 < n else len(buf))]) for f in frames]
        total = sum(len(p) for p in payloads)
        g, rec = empty(total + 16), empty(8 * (nk + 1))
        gsb = fc.scratch_bytes(max(nk, 1))
        gs = torch.empty(gsb, dtype=torch.uint8, device="cuda:0")
        d_ik = d_idx[4 * k * n:]
        FrameClassifier.gather_var(d_buf, d_offs, d_ik, nk, g, rec, gs, gsb)
        exp_rec = np.zeros(nk + 1, np.uint64)
        exp_rec[1:] = np.cumsum([len(p) for p in payloads])
        assert np.array_equal(host(rec, 8 * (nk + 1), np.uint64), exp_rec), method
        assert host(g, total).tobytes() == b"".join(payloads), method
        req = GpuPacker.for_request(schema, method)
        kinds = schema.kinds
        cols = [empty(total + 16) if kk == srpc_amd.STRING else empty(nk * oracle.KIND_SIZE[kk] + 16) for kk in kinds]
        soffs = [empty(8 * (nk + 1)) if kk == srpc_amd.STRING else None for kk in kinds]
        usb = req.var_scratch_bytes(nk, total)
        us = torch.empty(max(usb, 8), dtype=torch.uint8, device="cuda:0")
        st = status_buf()
        req.unpack_var(g, total, nk, rec, cols, soffs, us, usb, st)
        assert read_status(st) == (0, 2**64 - 1)
        fv = [vals[f] for f in frames]
        for f, kk in enumerate(kinds):  # the unpacked request equals what the client sent
            if kk == srpc_amd.STRING:
                so = host(soffs[f], 8 * (nk + 1), np.uint64)
                assert host(cols[f], int(so[nk])).tobytes() == b"".join(v[f] for v in fv), (method, f)
            else:
                got = host(cols[f], nk * oracle.KIND_SIZE[kk], oracle.KIND_DTYPE[kk])
                assert got.tolist() == [v[f] for v in fv], (method, f)
        rcols, roffs = _var_responses(schema, fv)
        resp = GpuPacker.for_response(schema)
        exp = oracle.pack(kinds, rcols, nk, resp.prefix, roffs)
        cap = len(exp) + 16
        w, rrec = empty(cap), empty(8 * (nk + 1))
        psb = resp.var_scratch_bytes(nk, cap)
        ps = torch.empty(max(psb, 8), dtype=torch.uint8, device="cuda:0")
        resp.pack_var([dev(c) for c in rcols], [dev(o) if o is not None else None for o in roffs], nk, w, cap, rrec,
                      ps, psb)
        assert host(w, len(exp)).tobytes() == exp
        var_rec[k], var_wire[k] = rrec, w
        rr = host(rrec, 8 * (nk + 1), np.uint64)
        var_out[k] = [exp[int(rr[i]): int(rr[i + 1])] for i in range(nk)]
    total_d = empty(16)
    fc.offsets(d_cls, n, d_idx, d_counts, var_rec, d_out_off, total_d, scratch, sb)
    # the reference server's reply stream: one answer per classified frame, in order
    pos = {k: {int(f): i for i, f in enumerate(idx[k, :int(counts[k])])} for k in range(KT)}
    expect = []
    for i, c in enumerate(want):
        c = int(c)
        if c == UNKNOWN:
            continue
        if c < K:
            rb = METHODS[c][2]
            expect.append(fixed_resp[c][pos[c][i] * rb:(pos[c][i] + 1) * rb].tobytes())
        else:
            r = var_out[c][pos[c][i]]
            expect.append(struct.pack(">I", len(r)) + r)
    expect = b"".join(expect)
    assert int(host(total_d, 8, np.uint64)[0]) == len(expect)
    out_off = host(d_out_off, 8 * (n + 1), np.uint64)
    assert int(out_off[n]) == len(expect)
    out = empty(len(expect) + 16)
    for k in range(K):
        nk = int(counts[k])
        if nk:
            fc.scatter(dev(fixed_resp[k]), d_idx[4 * k * n:], nk, METHODS[k][2], d_out_off, out)
    for j in range(KV):
        k = K + j
        nk = int(counts[k])
        FrameClassifier.scatter_var(var_wire[k], var_rec[k], d_idx[4 * k * n:] if nk else empty(16), nk, d_out_off, out)
    assert host(out, len(expect)).tobytes() == expect
