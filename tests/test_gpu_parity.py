"""Parity of the HIP path (through the C ABI) with the CPU oracle and the
reference-produced fixtures.  Bit-exact: this is byte/integer work.

Small cases run against oracle/packer_oracle.c on the same seeded inputs;
full BASELINE.json sizes are checked against the reference's SHA-256 digests
(tests/golden/manifest.json) and by pack -> unpack round trips.
"""
import hashlib
import os

import numpy as np
import pytest

import oracle
import srpc_amd
from srpc_amd import (NUMBER, QUAD, SQUARE_METHOD, TWO_NUMBERS, GpuPacker, Schema,
                      SRPC_ERR_BOUNDS, SRPC_PATH_DWORD, SRPC_PATH_TILE, SRPC_STATUS_BOUNDS,
                      SRPC_STATUS_PREFIX)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")


def dev(a: np.ndarray) -> "torch.Tensor":
    """numpy -> device tensor with the same bytes (16-byte aligned allocation)."""
    b = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = torch.empty(max(b.size, 1), dtype=torch.uint8, device=DEV)
    if b.size:
        t[: b.size].copy_(torch.from_numpy(b.copy()))
    return t


def host(t, nbytes: int, dtype=np.uint8) -> np.ndarray:
    torch.cuda.synchronize()
    return t[:nbytes].cpu().numpy().view(dtype) if nbytes else np.zeros(0, dtype)


def empty(nbytes: int):
    return torch.full((max(nbytes, 1),), 0xA5, dtype=torch.uint8, device=DEV)


def status_buf():
    return torch.zeros(16, dtype=torch.uint8, device=DEV)


def read_status(t):
    b = host(t, 16)
    flags = int(b[:4].view(np.uint32)[0])
    first = int(b[8:16].view(np.uint64)[0])
    return flags, first


def gpu_pack(packer, cols, n):
    dcols = [dev(c) for c in cols]
    wire = empty(packer.wire_bytes(n))
    packer.pack(dcols, n, wire)
    return host(wire, packer.wire_bytes(n)).tobytes()


def gpu_unpack(packer, wire: bytes, n, dtypes, wire_len=None, status=None):
    w = dev(np.frombuffer(wire, np.uint8)) if len(wire) else empty(16)
    outs = [empty(n * np.dtype(dt).itemsize + 16) for dt in dtypes]
    rc = packer.unpack(w, len(wire) if wire_len is None else wire_len, n, outs, status)
    return rc, [host(o, n * np.dtype(dt).itemsize, dt) for o, dt in zip(outs, dtypes)]


def read(golden_dir, name):
    with open(os.path.join(golden_dir, name), "rb") as f:
        return f.read()


SIZES = [0, 1, 2, 15, 16, 17, 255, 256, 257, 1023, 1024, 1025, 4096 + 17, 100_003]


@pytest.mark.parametrize("path", [SRPC_PATH_DWORD, SRPC_PATH_TILE])
@pytest.mark.parametrize("n", SIZES)
def test_quad_pack_unpack_vs_oracle(n, path):
    p = GpuPacker(QUAD)
    assert p.path == SRPC_PATH_DWORD
    p.force_path(path)
    cols = oracle.splitmix_columns_i32(4, n)
    wire = gpu_pack(p, cols, n)
    assert wire == oracle.pack([oracle.INT32] * 4, cols, n)
    rc, back = gpu_unpack(p, wire, n, [np.int32] * 4)
    assert rc == 0
    for a, b in zip(cols, back):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("path", [SRPC_PATH_DWORD, SRPC_PATH_TILE])
def test_quad_golden_head_and_edges(golden_dir, path):
    p = GpuPacker(QUAD)
    p.force_path(path)
    cols = oracle.splitmix_columns_i32(4, 4096)
    assert gpu_pack(p, cols, 4096) == read(golden_dir, "quad_body_head4096.bin")
    z = np.load(os.path.join(golden_dir, "quad_edges_in.npz"))
    ecols = [z[k] for k in "abcd"]
    wire = read(golden_dir, "quad_edges.bin")
    assert gpu_pack(p, ecols, 256) == wire
    rc, back = gpu_unpack(p, wire, 256, [np.int32] * 4)
    assert rc == 0 and all(np.array_equal(a, b) for a, b in zip(ecols, back))


@pytest.mark.parametrize("path", [SRPC_PATH_DWORD, SRPC_PATH_TILE])
def test_number_and_two_numbers(golden_dir, manifest, path):
    p = GpuPacker(NUMBER)
    p.force_path(path)
    n = manifest["streams"]["number_body_1M"]["records"]
    num = oracle.splitmix_columns_i32(1, n)
    wire = gpu_pack(p, num, n)
    assert wire[: 4096 * 4] == read(golden_dir, "number_body_head4096.bin")
    assert hashlib.sha256(wire).hexdigest() == manifest["streams"]["number_body_1M"]["sha256"]
    rc, back = gpu_unpack(p, wire, n, [np.int32])
    assert rc == 0 and np.array_equal(back[0], num[0])
    p2 = GpuPacker(TWO_NUMBERS)
    p2.force_path(path)
    l, r = oracle.splitmix_columns_i32(2, 1000, seed=oracle.SEED + 1)
    assert gpu_pack(p2, [l, r], 1000) == read(golden_dir, "two_numbers.bin")


ALL_KINDS = Schema.of("all_kinds", ("k_bool", "bool"), ("k_i8", "int8"), ("k_char", "char"),
                      ("k_i16", "int16"), ("k_i32", "int32"), ("k_i64", "int64"))
ALL_DT = [np.uint8, np.int8, np.int8, np.int16, np.int32, np.int64]


def test_all_kinds_tile(golden_dir):
    p = GpuPacker(ALL_KINDS)
    assert p.path == SRPC_PATH_TILE and p.record_bytes == 17
    z = np.load(os.path.join(golden_dir, "all_kinds_in.npz"))
    cols = [z[k] for k in ("kb", "k8", "kc", "k16", "k32", "k64")]
    wire = read(golden_dir, "all_kinds.bin")
    assert gpu_pack(p, cols, 1000) == wire
    rc, back = gpu_unpack(p, wire, 1000, ALL_DT)
    assert rc == 0
    for a, b in zip(cols, back):
        assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("n", [1, 7, 16, 17, 333, 4099, 65537])
@pytest.mark.parametrize("schema", ["all", "i16x3", "i64x2", "i8", "mixed_dword"])
def test_random_schemas_vs_oracle(n, schema):
    kinds = {"all": [oracle.BOOL, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64],
             "i16x3": [oracle.INT16] * 3, "i64x2": [oracle.INT64] * 2, "i8": [oracle.INT8],
             "mixed_dword": [oracle.INT64, oracle.INT32, oracle.INT64]}[schema]
    rng = np.random.default_rng(n * 31 + len(kinds))
    cols = []
    for k in kinds:
        dt = np.dtype(oracle.KIND_DTYPE[k])
        c = rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt)
        if k == oracle.BOOL:
            c = (c & 1).astype(np.uint8)
        cols.append(c)
    p = GpuPacker(Schema("X", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
    paths = [p.path] + ([SRPC_PATH_TILE] if p.path == SRPC_PATH_DWORD else [])
    want = oracle.pack(kinds, cols, n)
    for path in paths:
        p.force_path(path)
        assert gpu_pack(p, cols, n) == want
        rc, back = gpu_unpack(p, want, n, [oracle.KIND_DTYPE[k] for k in kinds])
        assert rc == 0
        for a, b in zip(cols, back):
            assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("n", [1, 3, 5, 4097, 65539])
@pytest.mark.parametrize("kinds,prefix", [
    ([oracle.INT16, oracle.INT64], b"abc"),  # 13 B, prefix bytes between fields of odd offsets
    ([oracle.INT64, oracle.INT64, oracle.INT64, oracle.INT32, oracle.INT8], b""),  # 29 B
    ([oracle.INT8, oracle.INT16, oracle.INT8, oracle.INT32, oracle.INT8, oracle.INT64], b"\x01\x02"),  # 19 B
    ([oracle.INT16, oracle.INT32], b"q" * 24),  # 30 B, mostly prefix
])
def test_odd_stride_records_vs_oracle(n, kinds, prefix):
    """Small TILE records whose stride is not a multiple of 4 (2/4/8-byte
    values at odd image offsets): sizes that leave a partial last tile and a
    ragged wire tail, with and without an envelope."""
    rng = np.random.default_rng(n * 7 + len(kinds) + len(prefix))
    cols = [rng.integers(0, 256, n * oracle.KIND_SIZE[k], dtype=np.uint8).view(oracle.KIND_DTYPE[k])
            for k in kinds]
    p = GpuPacker(Schema("X", tuple((f"f{i}", k) for i, k in enumerate(kinds))), prefix)
    assert p.path == SRPC_PATH_TILE
    want = oracle.pack(kinds, cols, n, prefix)
    assert gpu_pack(p, cols, n) == want
    rc, back = gpu_unpack(p, want, n, [oracle.KIND_DTYPE[k] for k in kinds])
    assert rc == 0
    for a, b in zip(cols, back):
        assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("n", [1, 1000, 20_001])
@pytest.mark.parametrize("strings", [False, True])
def test_schema_at_the_limits_vs_oracle(n, strings):
    """SRPC_MAX_FIELDS leaf fields behind a SRPC_MAX_PREFIX-byte envelope (the
    widest schema this build accepts; one more field or prefix byte is refused,
    tests/test_abi.py): a 1280-byte fixed record on the TILE path, and the same
    with every fourth field a string on the VAR path."""
    kinds = [[oracle.INT64, oracle.INT8, oracle.INT32, oracle.INT16][i % 4] for i in range(srpc_amd._lib.SRPC_MAX_FIELDS)]
    if strings:
        kinds = [oracle.STRING if i % 4 == 1 else k for i, k in enumerate(kinds)]
    rng = np.random.default_rng(n)
    prefix = rng.integers(0, 256, srpc_amd._lib.SRPC_MAX_PREFIX, dtype=np.uint8).tobytes()
    p = GpuPacker(Schema("Wide", tuple((f"f{i}", k) for i, k in enumerate(kinds))), prefix)
    if not strings:
        assert p.path == SRPC_PATH_TILE and p.record_bytes == 1024 + 8 * 8 + 8 * 1 + 8 * 4 + 8 * 2
        cols = [rng.integers(0, 256, n * oracle.KIND_SIZE[k], dtype=np.uint8).view(oracle.KIND_DTYPE[k])
                for k in kinds]
        want = oracle.pack(kinds, cols, n, prefix)
        assert gpu_pack(p, cols, n) == want
        rc, back = gpu_unpack(p, want, n, [oracle.KIND_DTYPE[k] for k in kinds])
        assert rc == 0 and all(a.tobytes() == b.tobytes() for a, b in zip(cols, back))
        return
    cols, offs = _random_string_batch(kinds, n, rng, 24)
    want = oracle.pack(kinds, cols, n, prefix, list(offs))
    wire, rec, st = gpu_pack_var(p, kinds, cols, offs, n)
    assert st == (0, 2**64 - 1) and wire == bytes(want)
    back, boffs, st = gpu_unpack_var(p, kinds, wire, n, rec)
    assert st[0] == 0
    rc, ocols, ooffs, _, _ = oracle.unpack(kinds, want, n, prefix)
    assert rc == 0
    for f, k in enumerate(kinds):
        assert back[f].tobytes() == ocols[f].tobytes(), f
        if k == oracle.STRING:
            assert np.array_equal(boffs[f], ooffs[f]), f


@pytest.mark.parametrize("schema", ["quad", "number", "two", "i64x2"])
def test_dword_variants_identical(schema):
    sch = {"quad": QUAD, "number": NUMBER, "two": TWO_NUMBERS,
           "i64x2": Schema.of("L", ("x", "int64"), ("y", "int64"))}[schema]
    kinds = sch.kinds
    n = 3 * 4096 + 7  # exercises the x4 body and the 1-record tail
    rng = np.random.default_rng(11)
    cols = [rng.integers(0, 256, n * np.dtype(oracle.KIND_DTYPE[k]).itemsize, dtype=np.uint8)
            .view(oracle.KIND_DTYPE[k]) for k in kinds]
    want = oracle.pack(kinds, cols, n)
    p = GpuPacker(sch)
    variants = [(r, i, t, 0) for r in (1, 4) for i in (1, 2, 4, 8) for t in range(4)]
    variants += [(1, 1, 3, 7), (4, 2, 0, 3), (1, 4, 2, 1)]  # capped grids: grid-stride loops
    for rpl, it, nt, grid in variants:
        p.tune(rpl, it, nt, grid=grid)
        assert gpu_pack(p, cols, n) == want, (rpl, it, nt, grid)
        rc, back = gpu_unpack(p, want, n, [oracle.KIND_DTYPE[k] for k in kinds])
        assert rc == 0 and all(a.tobytes() == b.tobytes() for a, b in zip(cols, back)), (rpl, it, nt, grid)


# ---- envelopes (Calculator.square) ---------------------------------------------

def test_square_request_envelope(golden_dir, manifest):
    st = manifest["streams"]["square_requests_1M"]
    n = st["records"]
    p = GpuPacker.for_request(NUMBER, SQUARE_METHOD)
    assert p.record_bytes == 53 and p.path == SRPC_PATH_TILE
    nums = oracle.square_inputs(n)
    wire = gpu_pack(p, [nums], n)
    assert wire[: 1024 * 53] == read(golden_dir, "square_req_head1024.bin")
    assert hashlib.sha256(wire).hexdigest() == st["sha256"]
    s = status_buf()
    rc, back = gpu_unpack(p, wire, n, [np.int32], status=s)
    assert rc == 0 and np.array_equal(back[0], nums)
    assert read_status(s) == (0, 2**64 - 1)


def test_square_response_envelope(golden_dir, manifest):
    st = manifest["streams"]["square_responses_1M"]
    n = st["records"]
    p = GpuPacker.for_response(NUMBER, srpc_amd.RPC_SUCCESS)
    assert p.record_bytes == 19
    sq = (oracle.square_inputs(n).astype(np.int64) ** 2).astype(np.int32)
    wire = gpu_pack(p, [sq], n)
    assert wire[: 1024 * 19] == read(golden_dir, "square_resp_head1024.bin")
    assert hashlib.sha256(wire).hexdigest() == st["sha256"]


@pytest.mark.parametrize("bad", [0, 5, 143, 144, 145, 9999])
def test_request_prefix_mismatch_reported(bad):
    n = 10_000
    p = GpuPacker.for_request(NUMBER, SQUARE_METHOD)
    nums = np.arange(n, dtype=np.int32) - 5000
    pre = oracle.request_prefix(SQUARE_METHOD, "Number")
    wire = bytearray(oracle.pack([oracle.INT32], [nums], n, pre))
    wire[bad * 53 + 20] ^= 0x20          # corrupt the method name of record `bad`
    wire[min(n - 1, bad + 3) * 53 + 48] ^= 1   # and the message name of a later one
    s = status_buf()
    rc, back = gpu_unpack(p, bytes(wire), n, [np.int32], status=s)
    assert rc == 0
    flags, first = read_status(s)
    assert flags == SRPC_STATUS_PREFIX and first == bad
    # the oracle agrees on where decoding fails
    st, _, _, _, err = oracle.unpack([oracle.INT32], bytes(wire), n, pre)
    assert st == oracle.ORC_ERR_PREFIX and err == bad
    # fields are still decoded from their fixed positions
    assert np.array_equal(back[0], nums)


def test_truncated_wire_bounds():
    n = 1000
    p = GpuPacker.for_request(NUMBER, SQUARE_METHOD)
    nums = np.arange(n, dtype=np.int32)
    pre = oracle.request_prefix(SQUARE_METHOD, "Number")
    wire = oracle.pack([oracle.INT32], [nums], n, pre)
    s = status_buf()
    cut = len(wire) - 30
    rc, back = gpu_unpack(p, wire[:cut], n, [np.int32], status=s)
    assert rc == SRPC_ERR_BOUNDS
    flags, first = read_status(s)
    assert flags == SRPC_STATUS_BOUNDS and first == n - 1
    assert np.array_equal(back[0][: n - 1], nums[: n - 1])
    st, _, _, _, err = oracle.unpack([oracle.INT32], wire[:cut], n, pre)
    assert st == oracle.ORC_ERR_BOUNDS and err == n - 1


def test_alignment_and_capacity_errors():
    p = GpuPacker(QUAD)
    cols = [torch.zeros(64, dtype=torch.int32, device=DEV) for _ in range(4)]
    wire = torch.zeros(1024 + 16, dtype=torch.uint8, device=DEV)
    with pytest.raises(srpc_amd.SrpcError) as e:
        p.pack(cols, 64, wire[1:].data_ptr(), 1024)
    assert e.value.code == -2
    with pytest.raises(srpc_amd.SrpcError) as e:
        p.pack(cols, 64, wire, 1000)
    assert e.value.code == -5


def test_fill_splitmix_matches_numpy():
    n = 100_000
    cols = [torch.empty(n, dtype=torch.int32, device=DEV) for _ in range(4)]
    srpc_amd.fill_splitmix_i32(cols, n, oracle.SEED, first_record=12345)
    torch.cuda.synchronize()
    want = oracle.splitmix_columns_i32(4, n, first_record=12345)
    for c, w in zip(cols, want):
        assert np.array_equal(c.cpu().numpy(), w)


# ---- full BASELINE.json sizes ----------------------------------------------------

@pytest.mark.parametrize("path", [SRPC_PATH_DWORD, SRPC_PATH_TILE])
def test_kernel_timing_hook(path):
    """srpc_time_next_call: the armed call's kernels stamp begin/end into the
    events, the bytes are unchanged, and the hook is consumed by one call."""
    n = 1 << 20
    cols = oracle.splitmix_columns_i32(4, n, 0x5EED)
    p = GpuPacker(QUAD)
    p.force_path(path)
    dcols = [dev(c) for c in cols]
    wire = empty(n * 16)
    back = [empty(n * 4) for _ in range(4)]
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    for e in ev:
        e.record(s)
    torch.cuda.synchronize()
    srpc_amd.time_next_call(ev[0], ev[1])
    p.pack(dcols, n, wire, stream=s)
    srpc_amd.time_next_call(ev[2], ev[3])
    p.unpack(wire, n * 16, n, back, stream=s)
    ev[4].record(s)
    p.pack(dcols, n, wire, stream=s)  # not armed: must not restamp ev[3]
    torch.cuda.synchronize()
    t_pack, t_unpack = ev[0].elapsed_time(ev[1]), ev[2].elapsed_time(ev[3])
    assert 0 < t_pack < 100 and 0 < t_unpack < 100
    assert ev[3].elapsed_time(ev[4]) >= 0
    assert host(wire, n * 16).tobytes() == oracle.pack([oracle.INT32] * 4, cols, n)
    for c, b in zip(cols, back):
        np.testing.assert_array_equal(host(b, n * 4, np.int32), c)
    with pytest.raises(ValueError):
        srpc_amd.time_next_call(torch.cuda.Event(enable_timing=True), None)


@pytest.mark.slow
@pytest.mark.parametrize("label", ["quad_body_16M", "quad_body_64M"])
def test_quad_full_size_digest_and_roundtrip(manifest, label):
    st = manifest["streams"][label]
    n = st["records"]
    p = GpuPacker(QUAD)
    cols = [torch.empty(n, dtype=torch.int32, device=DEV) for _ in range(4)]
    srpc_amd.fill_splitmix_i32(cols, n, oracle.SEED)
    wire = torch.empty(n * 16, dtype=torch.uint8, device=DEV)
    p.pack(cols, n, wire)
    torch.cuda.synchronize()
    assert hashlib.sha256(wire.cpu().numpy().tobytes()).hexdigest() == st["sha256"]
    back = [torch.empty(n, dtype=torch.int32, device=DEV) for _ in range(4)]
    p.unpack(wire, n * 16, n, back)
    torch.cuda.synchronize()
    for a, b in zip(cols, back):
        assert torch.equal(a, b)
    # the TILE path produces the same bytes at full size
    p.force_path(SRPC_PATH_TILE)
    wire2 = torch.empty_like(wire)
    p.pack(cols, n, wire2)
    torch.cuda.synchronize()
    assert torch.equal(wire, wire2)


# ---- string fields (SRPC_PATH_VAR) -------------------------------------------------

MULTIPLE = Schema.of("multiple_primitives", ("arg1", "int8"), ("arg2", "char"), ("arg3", "int64"),
                     ("arg4", "string"))


def _dev_u64(a):
    return dev(np.ascontiguousarray(a, dtype=np.uint64))


def gpu_pack_var(p, kinds, cols, offs, n):
    """cols[f]: numpy column (fixed) or uint8 chars (string); offs[f]: n+1 offsets or None."""
    dcols = [dev(c) for c in cols]
    doffs = [_dev_u64(o) if o is not None else None for o in offs]
    total = int(sum(int(o[n] - o[0]) for o in offs if o is not None)) + n * (
        len(p.prefix) + sum(8 if k == oracle.STRING else oracle.KIND_SIZE[k] for k in kinds))
    wire = empty(total + 16)
    rec = empty(8 * (n + 1))
    sb = p.var_scratch_bytes(n, total)
    scratch = empty(sb + 16)
    st = status_buf()
    p.pack_var(dcols, doffs, n, wire, total, rec, scratch, sb, st)
    rec_h = host(rec, 8 * (n + 1), np.uint64)
    return host(wire, total).tobytes(), rec_h, read_status(st)


def gpu_unpack_var(p, kinds, wire: bytes, n, rec_offs, wire_len=None):
    w = dev(np.frombuffer(wire, np.uint8)) if len(wire) else empty(16)
    L = len(wire) if wire_len is None else wire_len
    outs, offs = [], []
    for k in kinds:
        if k == oracle.STRING:
            outs.append(empty(L + 16))
            offs.append(empty(8 * (n + 1)))
        else:
            outs.append(empty(n * oracle.KIND_SIZE[k] + 16))
            offs.append(None)
    sb = p.var_scratch_bytes(n, L)
    scratch = empty(sb + 16)
    st = status_buf()
    p.unpack_var(w, L, n, _dev_u64(rec_offs), outs, offs, scratch, sb, st)
    res = []
    res_offs = []
    for k, o, so in zip(kinds, outs, offs):
        if k == oracle.STRING:
            oh = host(so, 8 * (n + 1), np.uint64)
            res_offs.append(oh)
            res.append(host(o, int(oh[n])) if n else np.zeros(0, np.uint8))
        else:
            res_offs.append(None)
            res.append(host(o, n * oracle.KIND_SIZE[k], oracle.KIND_DTYPE[k]))
    return res, res_offs, read_status(st)


def _rec_offsets(kinds, offs, n, prefix_len=0):
    fixed = prefix_len + sum(8 if k == oracle.STRING else oracle.KIND_SIZE[k] for k in kinds)
    sizes = np.full(n, fixed, np.uint64)
    for k, o in zip(kinds, offs):
        if k == oracle.STRING:
            sizes += np.diff(o.astype(np.uint64))
    r = np.zeros(n + 1, np.uint64)
    r[1:] = np.cumsum(sizes)
    return r


def test_strings_reference_fixture(golden_dir):
    z = np.load(os.path.join(golden_dir, "multiple_strings_in.npz"))
    kinds = MULTIPLE.kinds
    cols = [z["a1"], z["a2"], z["a3"], z["chars"]]
    offs = [None, None, None, z["offs"]]
    n = len(z["a1"])
    p = GpuPacker(MULTIPLE)
    assert p.path == srpc_amd.SRPC_PATH_VAR and p.record_bytes == 0
    wire, rec, st = gpu_pack_var(p, kinds, cols, offs, n)
    assert st == (0, 2**64 - 1)
    assert wire == read(golden_dir, "multiple_strings.bin")
    assert np.array_equal(rec, _rec_offsets(kinds, offs, n))
    back, boffs, st = gpu_unpack_var(p, kinds, wire, n, rec)
    assert st == (0, 2**64 - 1)
    for a, b in zip(cols[:3], back[:3]):
        assert a.tobytes() == b.tobytes()
    assert np.array_equal(boffs[3], z["offs"]) and back[3].tobytes() == z["chars"].tobytes()


def _random_string_batch(kinds, n, rng, maxlen):
    cols, offs = [], []
    for k in kinds:
        if k == oracle.STRING:
            lens = rng.integers(0, maxlen + 1, n).astype(np.uint64)
            lens[rng.random(n) < 0.2] = 0  # plenty of empty strings
            o = np.zeros(n + 1, np.uint64)
            o[1:] = np.cumsum(lens)
            cols.append(rng.integers(0, 256, max(1, int(o[-1])), dtype=np.uint8))
            offs.append(o)
        else:
            dt = np.dtype(oracle.KIND_DTYPE[k])
            c = rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt)
            cols.append((c & 1).astype(np.uint8) if k == oracle.BOOL else c)
            offs.append(None)
    return cols, offs


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 2047, 2048, 2049, 30_001])
@pytest.mark.parametrize("schema,maxlen,envelope", [
    ("s", 40, None), ("s", 16, None), ("mixed", 300, None), ("two_str", 16, "request"), ("s", 5000, None),
    ("nested", 64, "response"), ("wide", 24, "request")])
@pytest.mark.parametrize("vk", [None, 0, 2], ids=["default", "walk", "tiles"])
def test_strings_random_vs_oracle(n, schema, maxlen, envelope, vk):
    kinds = {"s": [oracle.STRING],
             "mixed": [oracle.INT8, oracle.STRING, oracle.INT64, oracle.BOOL, oracle.STRING, oracle.INT16],
             "two_str": [oracle.STRING, oracle.INT32, oracle.STRING],
             "nested": [oracle.INT64, oracle.INT8, oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING],
             "wide": [oracle.STRING, oracle.INT8, oracle.INT16, oracle.STRING, oracle.INT32, oracle.INT64,
                      oracle.BOOL, oracle.STRING, oracle.CHAR, oracle.INT64, oracle.INT8]}[schema]
    if maxlen > 1000 and n > 3000:
        n = 3000
    rng = np.random.default_rng(n + maxlen)
    cols, offs = _random_string_batch(kinds, n, rng, maxlen)
    sch = Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    if envelope == "request":
        p = GpuPacker.for_request(sch, "Svc_servicer::m")
    elif envelope == "response":
        p = GpuPacker.for_response(sch, 2)
    else:
        p = GpuPacker(sch)
    if vk is not None:
        p.tune(var_kernel=vk)
    want = oracle.pack(kinds, cols, n, p.prefix, list(offs))
    wire, rec, st = gpu_pack_var(p, kinds, cols, offs, n)
    assert st[0] == 0
    assert wire == want
    assert np.array_equal(rec, _rec_offsets(kinds, offs, n, len(p.prefix)))
    back, boffs, st = gpu_unpack_var(p, kinds, want, n, rec)
    assert st[0] == 0
    rc, ocols, ooffs, _, _ = oracle.unpack(kinds, want, n, p.prefix)
    assert rc == 0
    for f, k in enumerate(kinds):
        assert back[f].tobytes() == ocols[f].tobytes(), f
        if k == oracle.STRING:
            assert np.array_equal(boffs[f], ooffs[f])


@pytest.mark.parametrize("schema,maxlen,envelope", [("mixed", 64, None), ("two_str", 32, "request")])
def test_strings_many_tiles_vs_oracle(schema, maxlen, envelope):
    """More 256-record tiles than the device holds workgroups (records of
    >= 40 bytes: the pack's resident grid loops over its tiles, each
    workgroup several times), byte for byte against the oracle; the stream
    decode of the same wire rebuilds the index."""
    kinds = {"mixed": [oracle.INT8, oracle.STRING, oracle.INT64, oracle.BOOL, oracle.STRING, oracle.INT16],
             "two_str": [oracle.STRING, oracle.INT32, oracle.STRING]}[schema]
    n = 700_001  # 2735 tiles
    rng = np.random.default_rng(7)
    cols, offs = _random_string_batch(kinds, n, rng, maxlen)
    sch = Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    p = GpuPacker.for_request(sch, "Svc_servicer::m") if envelope else GpuPacker(sch)
    want = oracle.pack(kinds, cols, n, p.prefix, list(offs))
    assert len(want) // n >= 40  # the looping pack
    wire, rec, st = gpu_pack_var(p, kinds, cols, offs, n)
    assert st[0] == 0 and wire == want
    assert np.array_equal(rec, _rec_offsets(kinds, offs, n, len(p.prefix)))
    back, boffs, st = gpu_unpack_var(p, kinds, want, n, rec)
    assert st[0] == 0
    for f, k in enumerate(kinds):
        if k == oracle.STRING:
            assert np.array_equal(boffs[f], offs[f] - offs[f][0])
            assert back[f].tobytes() == cols[f][:int(offs[f][n])].tobytes(), f
        else:
            assert back[f].tobytes() == cols[f].tobytes(), f
    from tests.test_gpu_stream import stream_unpack
    sback, sboffs, srec, sst = stream_unpack(p, kinds, want, n)
    assert sst == (0, 2**64 - 1) and np.array_equal(srec, rec)
    for f in range(len(kinds)):
        assert sback[f].tobytes() == back[f].tobytes(), f


@pytest.mark.parametrize("envelope", [None, "request"])
@pytest.mark.parametrize("n", [1, 7, 8, 9, 4099])
def test_long_records_pack_vs_oracle_and_capacity(n, envelope):
    """Records of 256 B or more on average (too long for the record tiles'
    LDS image: the output-chunk walk, k_pack_var) byte for byte against the
    oracle, and with a wire capacity short of the batch: exactly the bytes
    before the capacity are written, nothing past it, and BOUNDS is reported
    at the record that crosses it."""
    kinds = [oracle.INT16, oracle.STRING, oracle.INT8, oracle.STRING]
    rng = np.random.default_rng(n + 11)
    cols, offs = _random_string_batch(kinds, n, rng, 1400)
    sch = Schema("L", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    p = GpuPacker.for_request(sch, "Svc_servicer::m") if envelope else GpuPacker(sch)
    want = oracle.pack(kinds, cols, n, p.prefix, list(offs))
    if len(want) // n < 256:  # (a draw of short records: not this path)
        pytest.skip("average record under 256 B")
    wire, rec, st = gpu_pack_var(p, kinds, cols, offs, n)
    assert st == (0, 2**64 - 1) and wire == want
    # a capacity inside the batch
    cap = len(want) * 2 // 3 + 5
    dcols = [dev(c) for c in cols]
    doffs = [_dev_u64(o) if o is not None else None for o in offs]
    w = empty(len(want) + 64)
    recd = empty(8 * (n + 1))
    sb = p.var_scratch_bytes(n, cap)
    scratch = empty(sb + 16)
    stb = status_buf()
    p.pack_var(dcols, doffs, n, w, cap, recd, scratch, sb, stb)
    got = host(w, len(want) + 64).tobytes()
    assert got[:cap] == want[:cap]
    assert got[cap:] == bytes([0xA5]) * (len(want) + 64 - cap)
    flags, first = read_status(stb)
    starts = np.asarray(rec[:n], np.uint64)
    assert flags & srpc_amd.SRPC_STATUS_BOUNDS
    assert first == int(np.searchsorted(starts, cap, side="right")) - 1


@pytest.mark.parametrize("maxlens", [(0, 700), (3, 0, 900), (700, 2, 40), (0, 0)])
@pytest.mark.parametrize("n", [1, 257, 6000])
def test_strings_skewed_fields_vs_oracle(n, maxlens):
    """Multi-string unpack copies every field's chars in one launch, the
    fields' 4 KiB tiles interleaved: fields whose chars span very different
    tile counts (all empty, a few bytes, hundreds of bytes per record)."""
    kinds = []
    for i in range(len(maxlens)):
        kinds += [oracle.STRING, oracle.INT16 if i % 2 else oracle.INT64]
    rng = np.random.default_rng(n * 7 + len(maxlens))
    cols, offs = [], []
    for k in kinds:
        if k == oracle.STRING:
            m = maxlens[len([o for o in offs if o is not None])]
            lens = rng.integers(0, m + 1, n).astype(np.uint64)
            o = np.zeros(n + 1, np.uint64)
            o[1:] = np.cumsum(lens)
            cols.append(rng.integers(0, 256, max(1, int(o[-1])), dtype=np.uint8))
            offs.append(o)
        else:
            dt = np.dtype(oracle.KIND_DTYPE[k])
            cols.append(rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt))
            offs.append(None)
    sch = Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    p = GpuPacker.for_request(sch, "Svc_servicer::skew")
    want = oracle.pack(kinds, cols, n, p.prefix, list(offs))
    wire, rec, st = gpu_pack_var(p, kinds, cols, offs, n)
    assert st[0] == 0 and wire == want
    back, boffs, st = gpu_unpack_var(p, kinds, want, n, rec)
    assert st[0] == 0
    rc, ocols, ooffs, _, _ = oracle.unpack(kinds, want, n, p.prefix)
    assert rc == 0
    for f, k in enumerate(kinds):
        assert back[f].tobytes() == ocols[f].tobytes(), f
        if k == oracle.STRING:
            assert np.array_equal(boffs[f], ooffs[f])


@pytest.mark.parametrize("chars_shift,offs_shift", [(0, 0), (3, 8), (15, 8), (1, 0)])
def test_strings_unaligned_sources_and_long_strings(chars_shift, offs_shift):
    """Chars columns and offset arrays at any byte / 8-byte alignment, strings
    far longer than a 4 KiB tile, and a tiny-record run (many records per tile)."""
    kinds = [oracle.INT8, oracle.STRING, oracle.INT16]
    rng = np.random.default_rng(chars_shift * 31 + offs_shift)
    n = 3000
    lens = rng.integers(0, 24, n).astype(np.uint64)
    lens[100] = 70_000
    lens[101] = 9_000
    lens[2000:2600] = 0
    o = np.zeros(n + 1, np.uint64)
    o[1:] = np.cumsum(lens)
    chars = rng.integers(0, 256, int(o[-1]), dtype=np.uint8)
    c8 = rng.integers(-128, 128, n, dtype=np.int8)
    c16 = rng.integers(-2**15, 2**15, n, dtype=np.int16)
    p = GpuPacker(Schema("U", (("a", oracle.INT8), ("s", oracle.STRING), ("b", oracle.INT16))))
    want = oracle.pack(kinds, [c8, chars, c16], n, b"", [None, o, None])
    dchars = torch.zeros(len(chars) + 32, dtype=torch.uint8, device=DEV)
    dchars[chars_shift:chars_shift + len(chars)].copy_(torch.from_numpy(chars))
    doffs = torch.zeros(8 * (n + 1) + 16, dtype=torch.uint8, device=DEV)
    doffs[offs_shift:offs_shift + 8 * (n + 1)].copy_(torch.from_numpy(o.view(np.uint8)))
    wire = empty(len(want) + 16)
    rec = empty(8 * (n + 1))
    sb = p.var_scratch_bytes(n, len(want))
    scratch = empty(sb + 16)
    st = status_buf()
    p.pack_var([dev(c8), dchars[chars_shift:], dev(c16)], [None, doffs[offs_shift:], None], n, wire,
               len(want), rec, scratch, sb, st)
    assert read_status(st) == (0, 2**64 - 1)
    assert host(wire, len(want)).tobytes() == want


def _model_single_string(kinds, wire: bytes, n, rec, prefix: bytes):
    """The documented unpack_var semantics for a one-string schema on bad input
    (include/srpc_gpu.h): a BOUNDS record decodes its string as empty, a
    PREFIX-only record keeps its length.  Returns (str_offs, chars)."""
    fixed = len(prefix) + sum(8 if k == oracle.STRING else oracle.KIND_SIZE[k] for k in kinds)
    f = kinds.index(oracle.STRING)
    len_at = len(prefix) + sum(oracle.KIND_SIZE[k] for k in kinds[:f])
    offs, chars = [0], bytearray()
    for r in range(n):
        start, end = int(rec[r]), int(rec[r + 1])
        ln = 0
        if start <= end <= len(wire) and end - start >= fixed:
            ln = int.from_bytes(wire[start + len_at:start + len_at + 8], "little")
            if ln > end - (start + len_at + 8):
                ln = 0
            elif ln != end - start - fixed and wire[start:start + len(prefix)] == prefix:
                ln = 0  # size disagrees with the index: BOUNDS
            chars += wire[start + len_at + 8:start + len_at + 8 + ln]
        offs.append(offs[-1] + ln)
    return np.array(offs, np.uint64), bytes(chars)


def _check_single_string(kinds, back, boffs, wire, n, rec, prefix):
    mo, mc = _model_single_string(kinds, bytes(wire), n, rec, prefix)
    f = kinds.index(oracle.STRING)
    assert np.array_equal(boffs[f], mo)
    assert back[f].tobytes() == mc


@pytest.mark.parametrize("vk", [None, 0, 2], ids=["default", "walk", "tiles"])
def test_strings_errors(vk):
    kinds = [oracle.INT32, oracle.STRING]
    n = 1000
    rng = np.random.default_rng(5)
    cols, offs = _random_string_batch(kinds, n, rng, 30)
    p = GpuPacker.for_request(Schema("E", (("x", oracle.INT32), ("s", oracle.STRING))), "Svc::m")
    if vk is not None:
        p.tune(var_kernel=vk)
    wire = bytearray(oracle.pack(kinds, cols, n, p.prefix, list(offs)))
    rec = _rec_offsets(kinds, offs, n, len(p.prefix))
    # a length field pointing past its record
    bad = 417
    pos = int(rec[bad]) + len(p.prefix) + 4
    wire[pos:pos + 8] = (10**6).to_bytes(8, "little")
    back, boffs, st = gpu_unpack_var(p, kinds, bytes(wire), n, rec)
    assert st == (srpc_amd.SRPC_STATUS_BOUNDS, bad)
    _check_single_string(kinds, back, boffs, wire, n, rec, p.prefix)
    # prefix mismatch (method name) in a later record, length bug fixed
    wire[pos:pos + 8] = int(offs[1][bad + 1] - offs[1][bad]).to_bytes(8, "little")
    wire[int(rec[700]) + 9] ^= 0x40
    back, boffs, st = gpu_unpack_var(p, kinds, bytes(wire), n, rec)
    assert st == (SRPC_STATUS_PREFIX, 700)
    assert np.array_equal(back[0], cols[0])  # fields still decoded
    _check_single_string(kinds, back, boffs, wire, n, rec, p.prefix)
    # an index that disagrees with the record sizes
    rec2 = rec.copy()
    rec2[5] += 1
    back, boffs, st = gpu_unpack_var(p, kinds, bytes(wire), n, rec2)
    assert st[0] & srpc_amd.SRPC_STATUS_BOUNDS and st[1] == 4
    _check_single_string(kinds, back, boffs, wire, n, rec2, p.prefix)
    # a PREFIX record whose size also disagrees with the index keeps its length
    rec3 = rec.copy()
    rec3[701] += 2
    back, boffs, st = gpu_unpack_var(p, kinds, bytes(wire), n, rec3)
    assert st[0] & SRPC_STATUS_PREFIX and st[1] == 700
    _check_single_string(kinds, back, boffs, wire, n, rec3, p.prefix)
    # pack into too small a buffer: bounds flagged at the first record that does not fit
    dcols = [dev(c) for c in cols]
    doffs = [None, _dev_u64(offs[1])]
    recd = empty(8 * (n + 1))
    small = int(rec[600]) + 3
    sb = p.var_scratch_bytes(n, small)
    scratch = empty(sb + 16)
    s = status_buf()
    w = empty(int(rec[n]) + 16)
    p.pack_var(dcols, doffs, n, w, small, recd, scratch, sb, s)
    assert read_status(s) == (srpc_amd.SRPC_STATUS_BOUNDS, 600)
    got = host(w, int(rec[n])).tobytes()
    assert got[:small] == bytes(oracle.pack(kinds, cols, n, p.prefix, list(offs)))[:small]
    assert set(got[small:]) <= {0xA5}


@pytest.mark.parametrize("vk", [None, 2], ids=["default", "tiles"])
def test_strings_empty_frames_then_short_records(vk):
    """A block of zero-size records (empty frames: rec[i] == rec[i + 1]) in
    front of short valid records.  Every later record's fast-path output
    offset start - rec[0] - r * fixed_bytes would wrap below zero; the walk
    must treat those records as not exact (no copy of its own) and the
    general path must decode them as the model says."""
    kinds = [oracle.INT32, oracle.STRING]
    m, k = 2000, 700
    rng = np.random.default_rng(23)
    cols, offs = _random_string_batch(kinds, m, rng, 4)
    p = GpuPacker.for_request(Schema("E", (("x", oracle.INT32), ("s", oracle.STRING))), "Svc::m")
    if vk is not None:
        p.tune(var_kernel=vk)
    wire = bytes(oracle.pack(kinds, cols, m, p.prefix, list(offs)))
    rec = _rec_offsets(kinds, offs, m, len(p.prefix))
    for lead in (np.zeros(k, np.uint64), np.full(k, rec[m], np.uint64)):
        idx = np.concatenate([lead, rec]) if lead[0] == 0 else np.concatenate([rec, lead])
        n = m + k
        back, boffs, st = gpu_unpack_var(p, kinds, wire, n, idx)
        assert st[0] == srpc_amd.SRPC_STATUS_BOUNDS
        assert st[1] == (0 if lead[0] == 0 else m)
        _check_single_string(kinds, back, boffs, wire, n, idx, p.prefix)


def _model_multi_string(kinds, wire: bytes, n, rec, prefix: bytes):
    """The general (multi-string) unpack_var semantics on bad input, record
    by record as k_unpack_var_walk decodes it: BOUNDS (a record outside the
    wire or shorter than its fixed bytes, a length past the record end, a
    size that disagrees with the index) decodes every string of the record
    as empty; fixed fields read before the BOUNDS condition are written; a
    PREFIX-only record keeps everything.  Returns (status, fixed values
    {(f, r): bytes}, str_offs per string field, chars per string field)."""
    fixed = len(prefix) + sum(8 if k == oracle.STRING else oracle.KIND_SIZE[k] for k in kinds)
    W = len(wire)
    flags, first = 0, None
    vals = {}
    lens = {f: [] for f, k in enumerate(kinds) if k == oracle.STRING}
    chars = {f: bytearray() for f in lens}
    for r in range(n):
        start, end = int(rec[r]), int(rec[r + 1])
        flag = 0
        if start > end or end > W or end - start < fixed:
            flag = srpc_amd.SRPC_STATUS_BOUNDS
        if not flag and wire[start:start + len(prefix)] != prefix:
            flag = SRPC_STATUS_PREFIX
        pos = start + len(prefix)
        got = {}
        for f, k in enumerate(kinds):
            if k != oracle.STRING:
                sz = oracle.KIND_SIZE[k]
                # a field past the record end is not decoded (the size check flags the record)
                if flag != srpc_amd.SRPC_STATUS_BOUNDS and pos + sz <= end:
                    vals[(f, r)] = bytes(wire[pos:pos + sz])
                pos += sz
                continue
            ln = 0
            if flag != srpc_amd.SRPC_STATUS_BOUNDS and pos + 8 <= end:
                ln = int.from_bytes(wire[pos:pos + 8], "little")
                pos += 8
                if ln > end - pos:
                    flag, ln = srpc_amd.SRPC_STATUS_BOUNDS, 0
            else:
                flag = srpc_amd.SRPC_STATUS_BOUNDS
            got[f] = (pos, ln)
            pos += ln
        if not flag and pos != end:
            flag = srpc_amd.SRPC_STATUS_BOUNDS
        for f in lens:
            p0, ln = got[f]
            if flag == srpc_amd.SRPC_STATUS_BOUNDS:
                ln = 0
            lens[f].append(ln)
            chars[f] += wire[p0:p0 + ln]
        if flag:
            flags |= flag
            first = r if first is None else first
    offs = {f: np.concatenate([[0], np.cumsum(np.array(v, np.uint64))]).astype(np.uint64) for f, v in lens.items()}
    return (flags, first if first is not None else 2**64 - 1), vals, offs, {f: bytes(c) for f, c in chars.items()}


@pytest.mark.parametrize("vk", [None, 2], ids=["default", "tiles"])
@pytest.mark.parametrize("maxlen", [30, 200])
def test_multi_strings_errors(maxlen, vk):
    """Corrupt inputs through the multi-string unpack (the staged walk for
    short records, the global walk for long ones and for records outside a
    non-monotonic index) against the model of the general semantics."""
    kinds = [oracle.INT32, oracle.STRING, oracle.INT16, oracle.STRING, oracle.INT8]
    n = 3000
    rng = np.random.default_rng(17)
    cols, offs = _random_string_batch(kinds, n, rng, maxlen)
    sch = Schema("M", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    p = GpuPacker.for_request(sch, "Svc::multi")
    if vk is not None:
        p.tune(var_kernel=vk)
    clean = bytes(oracle.pack(kinds, cols, n, p.prefix, list(offs)))
    rec = _rec_offsets(kinds, offs, n, len(p.prefix))

    def check(wire, idx):
        back, boffs, st = gpu_unpack_var(p, kinds, bytes(wire), n, idx)
        want_st, vals, mo, mc = _model_multi_string(kinds, bytes(wire), n, idx, p.prefix)
        assert st == want_st
        for f, k in enumerate(kinds):
            if k == oracle.STRING:
                assert np.array_equal(boffs[f], mo[f]), f
                assert back[f].tobytes() == mc[f], f
            else:
                raw = back[f].tobytes()
                sz = oracle.KIND_SIZE[k]
                for (g, r), v in vals.items():
                    if g == f:
                        assert raw[r * sz:(r + 1) * sz] == v, (f, r)

    check(clean, rec)  # clean input: every record exact
    wire = bytearray(clean)
    # the second string's length pointing past its record
    bad = 1234
    pos = int(rec[bad]) + len(p.prefix) + 4 + 8 + int(offs[1][bad + 1] - offs[1][bad]) + 2
    wire[pos:pos + 8] = (10**6).to_bytes(8, "little")
    # the first string's length one byte short (record size then disagrees)
    pos2 = int(rec[2000]) + len(p.prefix) + 4
    ln = int(offs[1][2001] - offs[1][2000])
    if ln:
        wire[pos2:pos2 + 8] = (ln - 1).to_bytes(8, "little")
    # a prefix mismatch in an earlier record
    wire[int(rec[777]) + 5] ^= 0x01
    check(wire, rec)
    # an index that is not monotonic: records 299..300 point backwards
    rec4 = rec.copy()
    rec4[300] = rec[310]
    check(wire, rec4)
    # a truncated wire: the last records fall outside it
    check(bytes(wire[:int(rec[n - 5]) + 3]), rec)


WAVE_SCHEMAS = {
    "i8": ([oracle.INT8], b""),
    "i16_i8": ([oracle.INT16, oracle.INT8], b""),
    "bool_i32": ([oracle.BOOL, oracle.INT32], b""),
    "i64_i32_i16_i8": ([oracle.INT64, oracle.INT32, oracle.INT16, oracle.INT8], b""),
    "all_kinds": ([oracle.BOOL, oracle.INT8, oracle.CHAR, oracle.INT16, oracle.INT32, oracle.INT64], b""),
    "i16_i64_prefix": ([oracle.INT16, oracle.INT64], b"abc"),
    "quad": ([oracle.INT32] * 4, b""),
}


@pytest.mark.parametrize("wave", [0, 1024, 2048, 3072, 8192])
@pytest.mark.parametrize("n", [1, 15, 16, 17, 1023, 1025, 3001, 65_537])
@pytest.mark.parametrize("schema", sorted(WAVE_SCHEMAS))
def test_wave_tiles_vs_oracle(schema, n, wave):
    """TILE kernels with one wave per tile (SRPC_TUNE_WAVE_PACK_BYTES /
    WAVE_UNPACK_BYTES; 0 = workgroup tiles) at several tile sizes: partial
    last tiles, partial column chunks, enveloped records, against the oracle."""
    kinds, prefix = WAVE_SCHEMAS[schema]
    rng = np.random.default_rng(n * 13 + len(kinds) + wave)
    cols = []
    for k in kinds:
        c = rng.integers(0, 256, n * oracle.KIND_SIZE[k], dtype=np.uint8).view(oracle.KIND_DTYPE[k])
        cols.append((c & 1).astype(np.uint8) if k == oracle.BOOL else c)
    p = GpuPacker(Schema("X", tuple((f"f{i}", k) for i, k in enumerate(kinds))), prefix)
    p.force_path(SRPC_PATH_TILE)
    p.tune(wave_pack_bytes=wave, wave_unpack_bytes=wave)
    want = oracle.pack(kinds, cols, n, prefix)
    assert gpu_pack(p, cols, n) == want
    rc, back = gpu_unpack(p, want, n, [oracle.KIND_DTYPE[k] for k in kinds])
    assert rc == 0
    for a, b in zip(cols, back):
        assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("bad", [0, 63, 64, 1000])
def test_wave_tile_prefix_mismatch_reported(bad):
    """A corrupted envelope byte in a wave-tile unpack is reported at its
    record, as the oracle's cursor reports it."""
    kinds, prefix = WAVE_SCHEMAS["i16_i64_prefix"]
    n = 2000
    rng = np.random.default_rng(bad)
    cols = [rng.integers(0, 256, n * oracle.KIND_SIZE[k], dtype=np.uint8).view(oracle.KIND_DTYPE[k]) for k in kinds]
    p = GpuPacker(Schema("X", tuple((f"f{i}", k) for i, k in enumerate(kinds))), prefix)
    p.tune(wave_unpack_bytes=2048)
    wire = bytearray(oracle.pack(kinds, cols, n, prefix))
    wire[bad * p.record_bytes + 1] ^= 0x40
    st = status_buf()
    rc, _ = gpu_unpack(p, bytes(wire), n, [oracle.KIND_DTYPE[k] for k in kinds], status=st)
    flags, first = read_status(st)
    assert flags == SRPC_STATUS_PREFIX and first == bad
    st_o, _, _, _, err = oracle.unpack(kinds, bytes(wire), n, prefix)
    assert st_o == oracle.ORC_ERR_PREFIX and err == bad
