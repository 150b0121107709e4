"""Fixed-size records packed from / unpacked into an array of structs on the
device (srpc_gpu_pack_aos / srpc_gpu_unpack_aos): the caller's own record
layout -- a C++ std::vector<T> copied as raw bytes, here a numpy structured
array with C alignment and padding -- instead of SoA columns.  The wire must
be byte-identical to the reference's `p << r` loop (oracle.pack, and the
reference-built all_kinds.bin fixture); unpack must write the leaf fields and
leave every other byte of the structs (padding, a vtable-pointer slot) as it
was."""
import os

import numpy as np
import pytest

import oracle
import srpc_amd
from srpc_amd import QUAD, SQUARE_METHOD, NUMBER, GpuPacker, Schema

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

from tests.test_gpu_parity import ALL_DT, ALL_KINDS, dev, empty, host, read_status, status_buf  # noqa: E402

NP_OF_KIND = {oracle.BOOL: np.uint8, oracle.INT8: np.int8, oracle.CHAR: np.int8, oracle.INT16: np.int16,
              oracle.INT32: np.int32, oracle.INT64: np.int64}


def struct_dtype(kinds, vptr=True):
    """A C++-like struct: an 8-byte vtable-pointer slot first (message_base is
    polymorphic), then the leaf fields with natural alignment and padding."""
    names, formats = (["_vptr"], [np.uint64]) if vptr else ([], [])
    for i, k in enumerate(kinds):
        names.append(f"f{i}")
        formats.append(NP_OF_KIND[k])
    return np.dtype({"names": names, "formats": formats}, align=True)


def random_records(kinds, n, rng, vptr=True):
    dt = struct_dtype(kinds, vptr)
    raw = rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8)  # garbage in padding and the vptr slot
    recs = raw.view(dt).copy()
    for i, k in enumerate(kinds):
        if k == oracle.BOOL:
            recs[f"f{i}"] &= 1
    return recs


def layout(recs, nfields):
    dt = recs.dtype
    return dt.itemsize, [dt.fields[f"f{i}"][1] for i in range(nfields)]


@pytest.mark.parametrize("n", [1, 15, 16, 17, 1000, 4099, 100_003])
@pytest.mark.parametrize("schema,envelope,vptr,shift", [
    ("quad", None, True, 0), ("all", None, True, 0), ("all", "request", True, 0), ("number", "response", True, 0),
    ("i64_i8", None, True, 0), ("wide", "request", True, 0),
    # no vtable slot: Quad's struct is its wire body (the tile-copy kernels);
    # Number's fields cover the struct (no read-back of the struct tile)
    ("quad", None, False, 0), ("number", "response", False, 0), ("all", "request", False, 0),
    # all six kinds, plain and behind a vtable slot, no envelope: the
    # compile-time layout kernels (aos.hip k_*_aos_lay; n = 1..100003 covers
    # the array's last, partial lane)
    ("all", None, False, 0),
    # runs of 8 / 24 / 32 bytes behind a vtable slot (structs of 16 / 32 /
    # 40 bytes): the run kernels, whole-line piece unpack
    ("pair", None, True, 0), ("i64x3", None, True, 0), ("i64x4", None, True, 0),
    # a struct array 8 bytes off 16-byte alignment: the per-field kernels
    ("quad", None, True, 8), ("all", "request", True, 8)])
def test_aos_pack_unpack_vs_oracle(n, schema, envelope, vptr, shift):
    kinds = {"quad": [oracle.INT32] * 4, "pair": [oracle.INT32] * 2, "i64x3": [oracle.INT64] * 3,
             "i64x4": [oracle.INT64] * 4,
             "all": [oracle.BOOL, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64],
             "number": [oracle.INT32], "i64_i8": [oracle.INT64, oracle.INT8],
             "wide": [oracle.INT8, oracle.INT64, oracle.INT16, oracle.INT8, oracle.INT32] * 3}[schema]
    sch = Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    p = (GpuPacker.for_request(sch, "Svc_servicer::m") if envelope == "request"
         else GpuPacker.for_response(sch, 0) if envelope == "response" else GpuPacker(sch))
    rng = np.random.default_rng(n + len(kinds))
    recs = random_records(kinds, n, rng, vptr)
    stride, offs = layout(recs, len(kinds))
    cols = [np.ascontiguousarray(recs[f"f{i}"]) for i in range(len(kinds))]
    want = bytes(oracle.pack(kinds, cols, n, p.prefix))

    def on_dev(a):  # the struct bytes at `shift` bytes into a 16-byte aligned allocation
        t = empty(a.nbytes + 32)
        t[shift:shift + a.nbytes].copy_(torch.from_numpy(a.view(np.uint8).reshape(-1).copy()))
        return t[shift:]

    d_recs = on_dev(recs)
    wire = empty(p.wire_bytes(n) + 16)
    p.pack_aos(d_recs, stride, offs, n, wire)
    assert host(wire, p.wire_bytes(n)).tobytes() == want
    # unpack into a device copy of different structs: only the leaf bytes change
    other = random_records(kinds, n, np.random.default_rng(7 + n), vptr)
    d_other = on_dev(other)
    st = status_buf()
    assert p.unpack_aos(dev(np.frombuffer(want, np.uint8)), len(want), n, d_other, stride, offs, st) == 0
    assert read_status(st) == (0, 2**64 - 1)
    back = host(d_other, n * stride).view(recs.dtype)
    for i in range(len(kinds)):
        assert back[f"f{i}"].tobytes() == recs[f"f{i}"].tobytes(), i
    if vptr:
        assert back["_vptr"].tobytes() == other["_vptr"].tobytes()
    # padding bytes are those of `other`
    mask = np.zeros(stride, bool)
    mask[0:8 if vptr else 0] = True
    for o, k in zip(offs, kinds):
        mask[o:o + oracle.KIND_SIZE[k]] = True
    pad = np.flatnonzero(~mask)
    if pad.size:
        b, o = back.view(np.uint8).reshape(n, stride), other.view(np.uint8).reshape(n, stride)
        assert np.array_equal(b[:, pad], o[:, pad])


@pytest.mark.parametrize("n", [1, 17, 4099, 100_003])
@pytest.mark.parametrize("schema,envelope,vptr,shift", [
    ("quad", None, True, 0),          # the run kernels (fields one run behind the vtable slot)
    ("pair", None, True, 0), ("i64x3", None, True, 0), ("i64x4", None, True, 0),
    ("all", None, True, 0), ("all", None, False, 0),  # layout kernels
    ("all", "request", True, 0), ("i64_i8", None, True, 0),  # staged kernels
    ("quad", None, False, 0),         # fields cover the struct: no fill needed
    ("quad", None, True, 8), ("all", "request", True, 8)])  # per-field kernels (+ a fill pass)
def test_aos_unpack_into_fresh_objects(n, schema, envelope, vptr, shift):
    """srpc_gpu_unpack_aos_fill: the leaf fields from the wire, every other
    struct byte from the fill record (a T{} image), whatever the array held."""
    kinds = {"quad": [oracle.INT32] * 4, "pair": [oracle.INT32] * 2, "i64x3": [oracle.INT64] * 3,
             "i64x4": [oracle.INT64] * 4,
             "all": [oracle.BOOL, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64],
             "i64_i8": [oracle.INT64, oracle.INT8]}[schema]
    sch = Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    p = GpuPacker.for_request(sch, "Svc_servicer::m") if envelope == "request" else GpuPacker(sch)
    rng = np.random.default_rng(31 * n + len(kinds))
    recs = random_records(kinds, n, rng, vptr)
    stride, offs = layout(recs, len(kinds))
    cols = [np.ascontiguousarray(recs[f"f{i}"]) for i in range(len(kinds))]
    want = bytes(oracle.pack(kinds, cols, n, p.prefix))
    fill = rng.integers(0, 256, stride, dtype=np.uint8).tobytes()
    t = empty(n * stride + 32)
    t[shift:shift + n * stride].copy_(torch.from_numpy(
        random_records(kinds, n, np.random.default_rng(5 + n), vptr).view(np.uint8).reshape(-1).copy()))
    d_other = t[shift:]
    st = status_buf()
    assert p.unpack_aos_fill(dev(np.frombuffer(want, np.uint8)), len(want), n, d_other, stride, offs, fill, st) == 0
    assert read_status(st) == (0, 2**64 - 1)
    back = host(d_other, n * stride).view(np.uint8).reshape(n, stride)
    expect = np.tile(np.frombuffer(fill, np.uint8), (n, 1))
    for o, k in zip(offs, kinds):
        expect[:, o:o + oracle.KIND_SIZE[k]] = recs.view(np.uint8).reshape(n, stride)[:, o:o + oracle.KIND_SIZE[k]]
    cover = sum(oracle.KIND_SIZE[k] for k in kinds) == stride
    if cover:  # nothing to fill: the fields are the struct
        expect = recs.view(np.uint8).reshape(n, stride)
    assert np.array_equal(back, expect)
    # the bytes after the array are untouched
    assert host(t, n * stride + 32)[shift + n * stride:].tobytes() == b"\xa5" * (32 - shift)


@pytest.mark.parametrize("schema", ["pair", "i64x3", "i64x4", "quad"])
def test_aos_run_unpack_refuses_wire_8_bytes_off_16(schema):
    """the run layouts' whole-line piece unpack loads the wire
    in 16-byte pieces.  A wire 8 bytes off 16-byte alignment never reaches it:
    both AoS unpack entry points refuse it (SRPC_E_ALIGN) before any launch,
    and the piece kernel's own dispatch requires a 16-byte aligned wire too;
    the aligned wire of the same batch decodes exactly."""
    kinds = {"quad": [oracle.INT32] * 4, "pair": [oracle.INT32] * 2, "i64x3": [oracle.INT64] * 3,
             "i64x4": [oracle.INT64] * 4}[schema]
    p = GpuPacker(Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
    n = 4099
    rng = np.random.default_rng(n + 77)
    recs = random_records(kinds, n, rng, True)
    stride, offs = layout(recs, len(kinds))
    cols = [np.ascontiguousarray(recs[f"f{i}"]) for i in range(len(kinds))]
    want = bytes(oracle.pack(kinds, cols, n))
    w = empty(len(want) + 32)
    w[8:8 + len(want)].copy_(torch.from_numpy(np.frombuffer(want, np.uint8).copy()))
    d_other = dev(random_records(kinds, n, np.random.default_rng(3 + n), True).view(np.uint8))
    fill = rng.integers(0, 256, stride, dtype=np.uint8).tobytes()
    with pytest.raises(srpc_amd.SrpcError, match="misaligned"):
        p.unpack_aos(w[8:], len(want), n, d_other, stride, offs)
    with pytest.raises(srpc_amd.SrpcError, match="misaligned"):
        p.unpack_aos_fill(w[8:], len(want), n, d_other, stride, offs, fill)
    st = status_buf()
    assert p.unpack_aos(dev(np.frombuffer(want, np.uint8)), len(want), n, d_other, stride, offs, st) == 0
    back = host(d_other, n * stride).view(recs.dtype)
    for i in range(len(kinds)):
        assert back[f"f{i}"].tobytes() == recs[f"f{i}"].tobytes(), i


def test_aos_all_kinds_reference_fixture(golden_dir):
    """The reference-built all_kinds.bin from structs instead of columns."""
    z = np.load(os.path.join(golden_dir, "all_kinds_in.npz"))
    cols = [z[k] for k in ("kb", "k8", "kc", "k16", "k32", "k64")]
    kinds = [oracle.BOOL, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64]
    recs = np.zeros(1000, struct_dtype(kinds))
    for i, c in enumerate(cols):
        recs[f"f{i}"] = c
    stride, offs = layout(recs, 6)
    p = GpuPacker(ALL_KINDS)
    wire = empty(17 * 1000 + 16)
    p.pack_aos(dev(recs.view(np.uint8)), stride, offs, 1000, wire)
    assert host(wire, 17 * 1000).tobytes() == open(os.path.join(golden_dir, "all_kinds.bin"), "rb").read()
    back = np.zeros(1000, recs.dtype)
    d_back = dev(back.view(np.uint8))
    p.unpack_aos(dev(np.frombuffer(open(os.path.join(golden_dir, "all_kinds.bin"), "rb").read(), np.uint8)), 17000,
                 1000, d_back, stride, offs)
    got = host(d_back, 1000 * stride).view(recs.dtype)
    for i, dt in enumerate(ALL_DT):
        assert got[f"f{i}"].astype(dt).tobytes() == cols[i].astype(dt).tobytes()


def test_aos_square_request_digest(manifest):
    """1M Calculator.square requests packed from Number structs hash to the
    reference digest."""
    import hashlib
    n = 1 << 20
    nums = np.zeros(n, struct_dtype([oracle.INT32]))
    nums["f0"] = oracle.square_inputs(n)
    ent = manifest["streams"]["square_requests_1M"]
    p = GpuPacker.for_request(NUMBER, SQUARE_METHOD)
    stride, offs = layout(nums, 1)
    wire = empty(p.wire_bytes(n) + 16)
    p.pack_aos(dev(nums.view(np.uint8)), stride, offs, n, wire)
    assert hashlib.sha256(host(wire, p.wire_bytes(n)).tobytes()).hexdigest() == ent["sha256"]


def test_aos_errors():
    kinds = [oracle.INT32] * 4
    p = GpuPacker(QUAD)
    recs = random_records(kinds, 100, np.random.default_rng(1))
    stride, offs = layout(recs, 4)
    d = dev(recs.view(np.uint8))
    wire = empty(16 * 100 + 16)
    with pytest.raises(srpc_amd.SrpcError):  # misaligned field offset
        p.pack_aos(d, stride, [offs[0] + 1] + offs[1:], 100, wire)
    with pytest.raises(srpc_amd.SrpcError):  # field past the struct
        p.pack_aos(d, 8, offs, 100, wire)
    with pytest.raises(srpc_amd.SrpcError):  # wire too small
        p.pack_aos(d, stride, offs, 100, wire, wire_cap=16 * 99)
    # truncated wire: records that fit are decoded, BOUNDS names the first missing one
    p.pack_aos(d, stride, offs, 100, wire)
    back = dev(np.zeros(100 * stride, np.uint8))
    st = status_buf()
    rc = p.unpack_aos(wire, 16 * 60 + 5, 100, back, stride, offs, st)
    assert rc == srpc_amd.SRPC_ERR_BOUNDS and read_status(st) == (srpc_amd.SRPC_STATUS_BOUNDS, 60)
    got = host(back, 100 * stride).view(recs.dtype)
    assert got["f2"][:60].tobytes() == recs["f2"][:60].tobytes() and not got["f2"][60:].any()
    # a foreign prefix byte is reported at its record
    pr = GpuPacker.for_request(QUAD, "Svc_servicer::m")
    w = empty(pr.wire_bytes(100) + 16)
    pr.pack_aos(d, stride, offs, 100, w)
    wb = bytearray(host(w, pr.wire_bytes(100)).tobytes())
    wb[pr.record_bytes * 42 + 9] ^= 0x20
    st = status_buf()
    pr.unpack_aos(dev(np.frombuffer(bytes(wb), np.uint8)), len(wb), 100, back, stride, offs, st)
    assert read_status(st) == (srpc_amd.SRPC_STATUS_PREFIX, 42)


LAY_UNPACK = {"staged_unpack": 0, "layout_unpack": 1, "piece_unpack": 2}


@pytest.fixture(params=list(LAY_UNPACK))
def lay_unpack(request):
    """srpc_debug_aos_lay_unpack: the all-kinds struct's unpack through the
    staged kernels, the compile-time layout kernel with a lane per four
    structs, or the layout kernel with a lane per 16-byte piece of the
    structs (whole-line stores, the default; the 24-byte struct falls back
    to the staged kernels), DESIGN.md §4.5."""
    import ctypes

    from srpc_amd import _lib
    hook = _lib.lib().srpc_debug_aos_lay_unpack
    hook.argtypes, hook.restype = [ctypes.c_int], ctypes.c_int
    prev = hook(LAY_UNPACK[request.param])
    yield request.param
    hook(prev)


@pytest.mark.parametrize("n", [1, 17, 255, 256, 257, 4099, 100_003])
@pytest.mark.parametrize("vptr", [True, False])
def test_aos_all_kinds_layout_kernels_both_unpacks(n, vptr, lay_unpack):
    """The all-kinds struct (with and without the vtable slot) in place and
    into fresh objects, by either unpack kernel family, against the oracle."""
    kinds = [oracle.BOOL, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64]
    sch = Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    p = GpuPacker(sch)
    rng = np.random.default_rng(17 * n + vptr)
    recs = random_records(kinds, n, rng, vptr)
    stride, offs = layout(recs, len(kinds))
    cols = [np.ascontiguousarray(recs[f"f{i}"]) for i in range(len(kinds))]
    want = bytes(oracle.pack(kinds, cols, n, p.prefix))
    other = random_records(kinds, n, np.random.default_rng(3 + n), vptr)
    d_other = dev(other.view(np.uint8).reshape(-1).copy())
    st = status_buf()
    assert p.unpack_aos(dev(np.frombuffer(want, np.uint8)), len(want), n, d_other, stride, offs, st) == 0
    assert read_status(st) == (0, 2**64 - 1)
    back = host(d_other, n * stride).view(recs.dtype)
    for i in range(len(kinds)):
        assert back[f"f{i}"].tobytes() == recs[f"f{i}"].tobytes(), i
    mask = np.zeros(stride, bool)
    mask[0:8 if vptr else 0] = True
    for o, k in zip(offs, kinds):
        mask[o:o + oracle.KIND_SIZE[k]] = True
    pad = np.flatnonzero(~mask)
    assert np.array_equal(back.view(np.uint8).reshape(n, stride)[:, pad],
                          other.view(np.uint8).reshape(n, stride)[:, pad])
    fill = rng.integers(0, 256, stride, dtype=np.uint8).tobytes()
    d_fresh = dev(other.view(np.uint8).reshape(-1).copy())
    assert p.unpack_aos_fill(dev(np.frombuffer(want, np.uint8)), len(want), n, d_fresh, stride, offs, fill, st) == 0
    assert read_status(st) == (0, 2**64 - 1)
    got = host(d_fresh, n * stride).view(np.uint8).reshape(n, stride)
    expect = np.tile(np.frombuffer(fill, np.uint8), (n, 1))
    for o, k in zip(offs, kinds):
        expect[:, o:o + oracle.KIND_SIZE[k]] = recs.view(np.uint8).reshape(n, stride)[:, o:o + oracle.KIND_SIZE[k]]
    assert np.array_equal(got, expect)
