"""Index-free decode of a concatenated string-record stream on the GPU
(srpc_gpu_unpack_var_stream): the reference's own shared-cursor decode
(core.hpp:39, packer.hpp:210-222) of the bytes its packer appends, with no
record index.  Checked against the oracle's cursor (oracle/packer_oracle.c
orc_unpack) and the reference-produced fixtures:
- the reference's multiple_strings.bin (301 records, strings 0..300 bytes);
- the packer_test.cpp vectors repeated 100,003 times;
- random schemas, short and long strings (blocks inside one record pass
  their entry on), and zero-heavy data on which the speculative starts are
  often wrong (the chains are walked from every candidate of a block);
- adversarial streams at scale (1M-4M records: zero-heavy strings, records
  of zeros only, every phase of which parses), and long zero-filled strings
  whose ends no block can guess (the scan walks such a block from its entry);
- streams cut short, foreign prefixes, fewer records than asked for, and
  trailing bytes after the n-th record.
Tests taking the `path` fixture run once per table mode of the decoder
(sdx.hip; the srpc_debug_stream_tables test hook): "tables" as the library
runs it (every block's table holds the chains from every plausible position
of its first 64 bytes); "primary" tables holding only each block's first
speculated start and "walk" empty tables -- in both the first scan meets
positions no table holds, and the repair pass (round 6) gives every block
the exits of the block before as slots; "walk_norepair" empty tables and no
repair pass (every block the cursor enters is walked, the round-5 path, kept
as the fallback of a block whose exit slots overflow).  Every mode meets the
same cases.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import oracle
import srpc_amd
from srpc_amd import GpuPacker, Schema

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

from tests.streams import straddler_stream as _straddler_stream  # noqa: E402
from tests.test_gpu_parity import _random_string_batch, _rec_offsets, dev, empty, host, read_status, status_buf  # noqa: E402

RES_OFF, RES_MISS, RES_REPAIR, RES_OVER = 1, 2, 4, 8  # srpc_unpack_status.reserved bits (srpc_gpu.h)


MODES = {"tables": 0, "primary": 1, "walk": 2, "walk_norepair": 2 | 8}


@pytest.fixture(params=list(MODES))
def path(request):
    hook = srpc_amd._lib.lib().srpc_debug_stream_tables
    hook.argtypes, hook.restype = [ctypes.c_int], ctypes.c_int
    prev = hook(MODES[request.param])
    yield request.param
    hook(prev)


GPU_OF_ORC = {oracle.ORC_ERR_BOUNDS: srpc_amd.SRPC_STATUS_BOUNDS, oracle.ORC_ERR_PREFIX: srpc_amd.SRPC_STATUS_PREFIX}


def stream_unpack(p, kinds, wire: bytes, n):
    W = len(wire)
    w = dev(np.frombuffer(wire, np.uint8)) if W else empty(16)
    outs, offs = [], []
    for k in kinds:
        if k == oracle.STRING:
            outs.append(empty(W + 16))
            offs.append(empty(8 * (n + 1)))
        else:
            outs.append(empty(n * oracle.KIND_SIZE[k] + 16))
            offs.append(None)
    sb = p.var_stream_scratch_bytes(n, W)
    scratch = torch.empty(sb + 256, dtype=torch.uint8, device="cuda:0")
    base = (-scratch.data_ptr()) % 256
    rec = empty(8 * (n + 1))
    st = status_buf()
    p.unpack_var_stream(w, W, n, rec, outs, offs, scratch.data_ptr() + base, sb, st)
    rec_h = host(rec, 8 * (n + 1), np.uint64)
    stream_unpack.last_reserved = int(host(st, 8)[4:8].view(np.uint32)[0])
    res, res_offs = [], []
    for k, o, so in zip(kinds, outs, offs):
        if k == oracle.STRING:
            oh = host(so, 8 * (n + 1), np.uint64)
            res_offs.append(oh)
            res.append(host(o, int(oh[n])) if n else np.zeros(0, np.uint8))
        else:
            res_offs.append(None)
            res.append(host(o, n * oracle.KIND_SIZE[k], oracle.KIND_DTYPE[k]))
    return res, res_offs, rec_h, read_status(st)


def check_clean(p, kinds, wire, n):
    """A stream of exactly n well-formed records: everything equals the oracle."""
    back, boffs, rec, st = stream_unpack(p, kinds, wire, n)
    rc, ocols, ooffs, consumed, _ = oracle.unpack(kinds, wire, n, p.prefix)
    assert rc == oracle.ORC_OK
    assert st == (0, 2**64 - 1)
    for f, k in enumerate(kinds):
        assert back[f].tobytes() == ocols[f].tobytes(), f
        if k == oracle.STRING:
            assert np.array_equal(boffs[f], ooffs[f]), f
    return rec


def test_reference_fixture_without_index(golden_dir, path):
    z = np.load(os.path.join(golden_dir, "multiple_strings_in.npz"))
    kinds = [oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING]
    p = GpuPacker(Schema("multiple_primitives", tuple((f"a{i}", k) for i, k in enumerate(kinds))))
    wire = open(os.path.join(golden_dir, "multiple_strings.bin"), "rb").read()
    n = len(z["a1"])
    rec = check_clean(p, kinds, wire, n)
    assert np.array_equal(rec, _rec_offsets(kinds, [None, None, None, z["offs"]], n))


@pytest.mark.parametrize("reps", [1, 100_003])
@pytest.mark.parametrize("which", ["unpack request/multiple", "unpack response/nested"])
def test_packer_test_vectors_repeated(which, reps, path):
    with open(os.path.join(os.path.dirname(__file__), "golden", "packer_test_vectors.json")) as f:
        case = {c["section"]: c for c in json.load(f)}[which]
    one = bytes.fromhex(case["input"])
    if "multiple" in which:
        kinds = [oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING]
        p = GpuPacker.for_request(Schema("multiple_primitives", tuple((f"a{i}", k) for i, k in enumerate(kinds))),
                                  case["method"])
    else:
        kinds = [oracle.INT64, oracle.INT8, oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING]
        p = GpuPacker.for_response(Schema("nested_message", tuple((f"a{i}", k) for i, k in enumerate(kinds))),
                                   case["code"])
    rec = check_clean(p, kinds, one * reps, reps)
    assert np.array_equal(rec, np.arange(reps + 1, dtype=np.uint64) * np.uint64(len(one)))


KINDS = {"s": [oracle.STRING],
         "mixed": [oracle.INT8, oracle.STRING, oracle.INT64, oracle.BOOL, oracle.STRING, oracle.INT16],
         "two_str": [oracle.STRING, oracle.INT32, oracle.STRING],
         "nested": [oracle.INT64, oracle.INT8, oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING]}


@pytest.mark.parametrize("n", [0, 1, 2, 63, 1000, 30_001])
@pytest.mark.parametrize("schema,maxlen,envelope", [("s", 40, None), ("mixed", 300, None),
                                                    ("two_str", 16, "request"), ("s", 5000, None),
                                                    ("nested", 64, "response")])
def test_random_streams(n, schema, maxlen, envelope, path):
    kinds = KINDS[schema]
    if maxlen > 1000 and n > 3000:
        n = 3000
    rng = np.random.default_rng(n * 3 + maxlen)
    cols, offs = _random_string_batch(kinds, n, rng, maxlen)
    sch = Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    p = (GpuPacker.for_request(sch, "Svc_servicer::m") if envelope == "request"
         else GpuPacker.for_response(sch, 2) if envelope == "response" else GpuPacker(sch))
    wire = oracle.pack(kinds, cols, n, p.prefix, list(offs))
    rec = check_clean(p, kinds, wire, n)
    assert np.array_equal(rec, _rec_offsets(kinds, offs, n, len(p.prefix)))
    r = stream_unpack.last_reserved
    blocks = (len(wire) + 8191) // 8192
    if path == "tables":
        # a block's entry is almost always one of its table's slots (scan waves
        # that walked a block from global memory: bits 8-31)
        assert r >> 8 <= 1 + blocks // 20, (r >> 8, blocks)
    if path == "walk" and blocks > 64:
        assert r & RES_REPAIR, r
    if path == "walk_norepair" and blocks > 64:
        assert r & RES_MISS and r >> 8 >= 1, r


@pytest.mark.parametrize("n", [257, 20_000])
def test_zero_heavy_streams_misspeculate_and_fix(n, path):
    """Zero bytes everywhere: a string length read at a wrong offset is often
    0, so many chunks speculate a wrong start; the repair rounds walk them
    again, and what they leave wrong goes to the single pass.  The result
    must still be exact."""
    kinds = [oracle.INT8, oracle.STRING, oracle.INT16, oracle.STRING]
    rng = np.random.default_rng(n)
    cols, offs = [], []
    for k in kinds:
        if k == oracle.STRING:
            lens = rng.integers(0, 24, n).astype(np.uint64)
            lens[rng.random(n) < 0.5] = 0
            o = np.zeros(n + 1, np.uint64)
            o[1:] = np.cumsum(lens)
            c = np.zeros(max(1, int(o[-1])), np.uint8)
            c[rng.random(c.size) < 0.05] = 7
            cols.append(c)
            offs.append(o)
        else:
            dt = np.dtype(oracle.KIND_DTYPE[k])
            cols.append(np.zeros(n, dt))
            offs.append(None)
    p = GpuPacker(Schema("Z", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
    wire = oracle.pack(kinds, cols, n, b"", list(offs))
    rec = check_clean(p, kinds, wire, n)
    assert np.array_equal(rec, _rec_offsets(kinds, offs, n))
    r = stream_unpack.last_reserved
    if path == "tables" and n > 10_000:
        assert r & RES_OFF, "expected block entries off the speculation on zero-heavy data"


def _error_case(p, kinds, wire, n):
    """The first record the cursor cannot read is reported as the oracle meets
    it, and every record before it decodes exactly."""
    back, boffs, rec, st = stream_unpack(p, kinds, wire, n)
    rc, ocols, ooffs, consumed, err = oracle.unpack(kinds, wire, n, p.prefix)
    assert rc != oracle.ORC_OK
    assert st[1] == err and st[0] & GPU_OF_ORC[rc], (st, rc, err)
    assert int(rec[err]) == consumed or rc == oracle.ORC_ERR_BOUNDS
    for f, k in enumerate(kinds):
        if k == oracle.STRING:
            assert np.array_equal(boffs[f][:err + 1], ooffs[f][:err + 1]), f
            assert back[f].tobytes()[:int(ooffs[f][err])] == ocols[f].tobytes()[:int(ooffs[f][err])], f
        else:
            assert back[f][:err].tobytes() == ocols[f][:err].tobytes(), f


def test_stream_errors(path):
    kinds = KINDS["mixed"]
    n = 5000
    rng = np.random.default_rng(99)
    cols, offs = _random_string_batch(kinds, n, rng, 60)
    p = GpuPacker.for_request(Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds))), "Svc::stream")
    wire = bytes(oracle.pack(kinds, cols, n, p.prefix, list(offs)))
    rec = _rec_offsets(kinds, offs, n, len(p.prefix))
    # cut short at several places (inside a prefix, a length, chars, a fixed field)
    for cut in (int(rec[1234]) + 3, int(rec[2000]) + len(p.prefix) + 4, int(rec[4999]) + 40, int(rec[n]) - 1):
        _error_case(p, kinds, wire[:cut], n)
    # a foreign method name in record 3100
    bad = bytearray(wire)
    bad[int(rec[3100]) + 10] ^= 0x04
    _error_case(p, kinds, bytes(bad), n)
    # a string length past the end of the wire in record 17
    bad = bytearray(wire)
    at = int(rec[17]) + len(p.prefix) + 1
    bad[at:at + 8] = (2**40).to_bytes(8, "little")
    _error_case(p, kinds, bytes(bad), n)
    # more records asked for than the stream holds
    _error_case(p, kinds, wire, n + 7)


def test_trailing_bytes_after_n_records(path):
    kinds = KINDS["two_str"]
    n = 3000
    rng = np.random.default_rng(4)
    cols, offs = _random_string_batch(kinds, n, rng, 20)
    p = GpuPacker(Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
    wire = oracle.pack(kinds, cols, n, b"", list(offs))
    m = 2222
    back, boffs, rec, st = stream_unpack(p, kinds, wire, m)
    rc, ocols, ooffs, _, _ = oracle.unpack(kinds, wire, m, b"")
    assert rc == oracle.ORC_OK and st == (0, 2**64 - 1)
    assert np.array_equal(rec, _rec_offsets(kinds, offs, n)[:m + 1])
    for f, k in enumerate(kinds):
        assert back[f].tobytes() == ocols[f].tobytes(), f


@pytest.mark.parametrize("prefix", [b"\x07", b"abc", b"1234567", b"12345678"])
def test_short_custom_prefixes(prefix, path):
    """Prefixes shorter than the 8-byte filter word (and exactly 8): the scan's
    prefix filter masks the bytes it compares; plausibility then needs two
    records (a bare or short prefix) or one (8 bytes or more)."""
    kinds = KINDS["mixed"]
    n = 7001
    rng = np.random.default_rng(len(prefix))
    cols, offs = _random_string_batch(kinds, n, rng, 40)
    p = GpuPacker(Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds))), prefix)
    wire = oracle.pack(kinds, cols, n, p.prefix, list(offs))
    rec = check_clean(p, kinds, wire, n)
    assert np.array_equal(rec, _rec_offsets(kinds, offs, n, len(p.prefix)))


def _zero_heavy(kinds, n, rng, maxlen=24, p_empty=0.5, p_nonzero=0.05):
    cols, offs = [], []
    for k in kinds:
        if k == oracle.STRING:
            lens = rng.integers(0, maxlen, n).astype(np.uint64)
            lens[rng.random(n) < p_empty] = 0
            o = np.zeros(n + 1, np.uint64)
            o[1:] = np.cumsum(lens)
            c = np.zeros(max(1, int(o[-1])), np.uint8)
            c[rng.random(c.size) < p_nonzero] = 7
            cols.append(c)
            offs.append(o)
        else:
            cols.append(np.zeros(n, np.dtype(oracle.KIND_DTYPE[k])))
            offs.append(None)
    return cols, offs


@pytest.mark.parametrize("n,schema", [(1 << 20, "zh4"), (1 << 22, "zh4"), (1 << 20, "zeros"), (1 << 22, "zeros")])
def test_adversarial_streams_at_scale(n, schema, path):
    """Streams on which a speculated start is usually wrong, at 1M-4M records:
    zero-heavy strings (int8, string, int16, string), and records of zeros
    only (multiple_primitives with empty strings: every one of its 18 phases
    parses, to the end of the stream).  Checked against the oracle's cursor."""
    if path == "walk_norepair" and n >= 1 << 22:
        pytest.skip("no repair: every block walked from global memory: covered at 1M")
    rng = np.random.default_rng(n + len(schema))
    if schema == "zh4":
        kinds = [oracle.INT8, oracle.STRING, oracle.INT16, oracle.STRING]
        cols, offs = _zero_heavy(kinds, n, rng)
    else:
        kinds = [oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING]
        cols, offs = _zero_heavy(kinds, n, rng, maxlen=1, p_empty=1.0, p_nonzero=0.0)
    p = GpuPacker(Schema("Z", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
    wire = oracle.pack(kinds, cols, n, b"", list(offs))
    rec = check_clean(p, kinds, wire, n)
    assert np.array_equal(rec, _rec_offsets(kinds, offs, n))


@pytest.mark.parametrize("n", [300, 3000])
def test_long_zero_strings_entries_no_block_guesses(n, path):
    """Strings of 0-20000 zero bytes: inside one every position parses as an
    empty record, so a block's candidates are all wrong.  In the library's
    tables the record end that enters such a block is found by the zero-run
    rule (the window position congruent to it modulo the 8-byte empty record
    passes through it: no walk); with the test hook's tables it is walked
    from the block's entry, and each miss is counted.  Exact either way."""
    kinds = [oracle.STRING]
    rng = np.random.default_rng(n)
    lens = rng.integers(0, 20000, n).astype(np.uint64)
    o = np.zeros(n + 1, np.uint64)
    o[1:] = np.cumsum(lens)
    c = np.zeros(max(1, int(o[-1])), np.uint8)
    p = GpuPacker(Schema("L", (("s", oracle.STRING),)))
    wire = oracle.pack(kinds, [c], n, b"", [o])
    rec = check_clean(p, kinds, wire, n)
    assert np.array_equal(rec, _rec_offsets(kinds, [o], n))
    r = stream_unpack.last_reserved
    if path == "tables":
        assert r >> 8 == 0, r  # no block walked
    elif path == "walk_norepair" and n >= 3000:
        assert r & RES_MISS and r >> 8 > 0, r
    elif n >= 3000:
        # the repair ran; a block entered by a record that started two or more
        # blocks back (strings of up to 20000 B here) is not given that entry
        # as an exit slot and is walked
        assert r & RES_REPAIR, r


ZH4 = [oracle.INT8, oracle.STRING, oracle.INT16, oracle.STRING]



@pytest.mark.parametrize("n,lead,over,fill", [
    (1 << 22, (1, 960), (65, 1000), "zero"),    # the verdict's stream at 4M records
    (1 << 20, (1, 6000), (65, 6000), "zero"),   # straddlers of up to 12 KiB
    (1 << 16, (1, 960), (65, 1000), "zero"),
    (1 << 16, (1, 900), (65, 100), "heavy"),    # zero-heavy straddlers starting within 1 KiB: landing slots
    (1 << 18, (1, 6000), (65, 100), "heavy"),   # ... up to 6000 B before the edge: the repair pass (round 6)
    (1 << 20, (1, 6000), (65, 6000), "heavy")])
def test_straddling_records_at_every_block(n, lead, over, fill, path):
    """a record straddles EVERY 8 KiB boundary and
    ends past the block's window, where no speculated start is.  Records of
    zero bytes (the verdict's stream), whatever their length, are found by
    the zero-run rule -- nothing is walked in the library's tables mode
    (reserved >> 8 == 0).  Zero-heavy straddlers that start within 1 KiB of
    the edge end at landing slots; longer ones (57.9
    ms for 256K records, one block after another walked by one wave) send
    the call through the repair pass: every block's entry is then an exit
    slot, nothing is walked.  Exact in every mode."""
    if path == "walk_norepair" and n > 1 << 16:
        pytest.skip("no repair: every block walked, serially: covered at 64K records")
    rng = np.random.default_rng(n + lead[1] + over[1] + len(fill))
    cols, offs = _straddler_stream(n, rng, lead, over, fill)
    p = GpuPacker(Schema("Z", tuple((f"f{i}", k) for i, k in enumerate(ZH4))))
    wire = oracle.pack(ZH4, cols, n, b"", offs)
    rec = check_clean(p, ZH4, wire, n)
    assert np.array_equal(rec, _rec_offsets(ZH4, offs, n))
    r = stream_unpack.last_reserved
    if path == "tables" and (fill == "zero" or lead[1] < 1024):
        assert r >> 8 == 0 and not r & RES_REPAIR, (r >> 8, len(wire) // 8192)
    elif path == "walk_norepair" and len(wire) > 64 * 8192:
        assert r & RES_MISS, r
    elif path != "walk_norepair":
        # the repair pass ran where it had to, and nothing was walked unless a
        # block had more possible entries than its exit slots hold (reserved
        # bit 3: a few blocks of zero-filled straddlers in the test-hook modes,
        # where the zero-run rule is off)
        assert r >> 8 == 0 or r & RES_OVER, (r, len(wire) // 8192)
        assert r >> 8 <= len(wire) // 8192 // 1000 + 1, (r, len(wire) // 8192)


def test_records_across_block_edges_and_margin(path):
    """Record lengths around the block (8 KiB) and its staged margin (2 KiB):
    records that start in one block and end several blocks later, records
    that run past the staged bytes (their tails read from global memory), one
    record that covers a block exactly."""
    kinds = [oracle.INT32, oracle.STRING, oracle.INT8]
    lens = np.array([8192 - 21, 0, 2048, 2049, 2047, 8192, 8193, 16384 + 5, 3, 0, 7000, 9000, 1, 20000, 0, 5] * 7,
                    np.uint64)
    n = lens.size
    rng = np.random.default_rng(5)
    o = np.zeros(n + 1, np.uint64)
    o[1:] = np.cumsum(lens)
    chars = rng.integers(0, 256, int(o[-1]), dtype=np.uint8)
    cols = [rng.integers(-2**31, 2**31, n).astype(np.int32), chars, rng.integers(-128, 128, n).astype(np.int8)]
    p = GpuPacker(Schema("E", tuple((f"f{i}", k) for i, k in enumerate(kinds))))
    wire = oracle.pack(kinds, cols, n, b"", [None, o, None])
    rec = check_clean(p, kinds, wire, n)
    assert np.array_equal(rec, _rec_offsets(kinds, [None, o, None], n))


@pytest.mark.parametrize("nstr", [3, 4, 5])
def test_many_string_fields(nstr, path):
    """Three and four string fields (the decode carries chars of all but the
    last in its state), five (the record index, then the indexed decode)."""
    kinds = []
    for i in range(nstr):
        kinds += [oracle.STRING, [oracle.INT8, oracle.INT16, oracle.INT64][i % 3]]
    n = 20_011
    rng = np.random.default_rng(nstr)
    cols, offs = _random_string_batch(kinds, n, rng, 30)
    p = GpuPacker.for_request(Schema("M", tuple((f"f{i}", k) for i, k in enumerate(kinds))), "Svc_servicer::many")
    wire = oracle.pack(kinds, cols, n, p.prefix, list(offs))
    rec = check_clean(p, kinds, wire, n)
    assert np.array_equal(rec, _rec_offsets(kinds, offs, n, len(p.prefix)))
