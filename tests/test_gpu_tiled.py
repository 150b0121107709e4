"""The tile table (ABI 6: srpc_gpu_var_tile_table + srpc_gpu_unpack_var_tiled):
the multi-string unpack takes each 256-record tile's chars bases from a table
of the batch's chars prefixes instead of looking back at earlier tiles.  Checked
against the oracle's cursor (oracle/packer_oracle.c orc_unpack, restating
pipe_output<std::string>, packer.hpp:216-222), including tables that are
wrong (each tile checks its totals against the table: a wrong table is caught
and the batch decoded again with the look-back, bit-identically)."""
import numpy as np
import pytest

import oracle
from srpc_amd import GpuPacker, Schema

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

from tests.test_gpu_parity import (_dev_u64, _random_string_batch, _rec_offsets, dev, empty, host,  # noqa: E402
                                   read_status, status_buf)

SCHEMAS = {"two_str": [oracle.STRING, oracle.INT32, oracle.STRING],
           "mixed": [oracle.INT8, oracle.STRING, oracle.INT64, oracle.BOOL, oracle.STRING, oracle.INT16],
           "wide": [oracle.STRING, oracle.INT8, oracle.INT16, oracle.STRING, oracle.INT32, oracle.INT64,
                    oracle.BOOL, oracle.STRING, oracle.CHAR, oracle.INT64, oracle.INT8],
           "one": [oracle.INT8, oracle.CHAR, oracle.INT64, oracle.STRING]}


def _table_from(p, offs, n):
    words = p.var_tile_table_words(n)
    t = empty(8 * words + 16)
    p.var_tile_table([_dev_u64(o) if o is not None else None for o in offs], n, t)
    return t, words


def _unpack_tiled(p, kinds, wire: bytes, n, rec, table):
    w = dev(np.frombuffer(wire, np.uint8)) if len(wire) else empty(16)
    L = len(wire)
    outs, offs = [], []
    for k in kinds:
        outs.append(empty(L + 16) if k == oracle.STRING else empty(n * oracle.KIND_SIZE[k] + 16))
        offs.append(empty(8 * (n + 1)) if k == oracle.STRING else None)
    sb = p.var_scratch_bytes(n, L)
    scratch = empty(sb + 16)
    st = status_buf()
    p.unpack_var_tiled(w, L, n, _dev_u64(rec), table, outs, offs, scratch, sb, st)
    res, res_offs = [], []
    for k, o, so in zip(kinds, outs, offs):
        if k == oracle.STRING:
            oh = host(so, 8 * (n + 1), np.uint64)
            res_offs.append(oh)
            res.append(host(o, int(oh[n])) if n else np.zeros(0, np.uint8))
        else:
            res_offs.append(None)
            res.append(host(o, n * oracle.KIND_SIZE[k], oracle.KIND_DTYPE[k]))
    return res, res_offs, read_status(st)


def _case(schema, n, maxlen, envelope, seed):
    kinds = SCHEMAS[schema]
    rng = np.random.default_rng(seed)
    cols, offs = _random_string_batch(kinds, n, rng, maxlen)
    sch = Schema("S", tuple((f"f{i}", k) for i, k in enumerate(kinds)))
    p = GpuPacker.for_request(sch, "Svc_servicer::m") if envelope else GpuPacker(sch)
    wire = bytes(oracle.pack(kinds, cols, n, p.prefix, list(offs)))
    return kinds, cols, offs, p, wire


def _check(kinds, p, wire, n, back, boffs, st):
    assert st == (0, 2**64 - 1)
    rc, ocols, ooffs, _, _ = oracle.unpack(kinds, wire, n, p.prefix)
    assert rc == oracle.ORC_OK
    for f, k in enumerate(kinds):
        assert back[f].tobytes() == ocols[f].tobytes(), f
        if k == oracle.STRING:
            assert np.array_equal(boffs[f], ooffs[f]), f


@pytest.mark.parametrize("n", [0, 1, 255, 256, 257, 4097, 30_001])
@pytest.mark.parametrize("schema,maxlen,envelope", [("two_str", 32, True), ("mixed", 120, False),
                                                    ("wide", 24, True), ("one", 64, False)])
def test_tiled_unpack_vs_oracle(n, schema, maxlen, envelope):
    kinds, cols, offs, p, wire = _case(schema, n, maxlen, envelope, n * 7 + maxlen)
    table, words = _table_from(p, offs, n)
    t = host(table, 8 * words, np.uint64)
    # the table is the chars prefix of each string field at every 256th record
    ns = sum(k == oracle.STRING for k in kinds)
    so = [o for o in offs if o is not None]
    for tile in range(words // ns):
        for s in range(ns):
            assert t[tile * ns + s] == so[s][min(256 * tile, n)] - so[s][0]
    back, boffs, st = _unpack_tiled(p, kinds, wire, n, _rec_offsets(kinds, offs, n, len(p.prefix)), table)
    _check(kinds, p, wire, n, back, boffs, st)


@pytest.mark.parametrize("how", ["one_entry_off_by_one", "first_nonzero", "huge", "zeros", "swapped_fields"])
def test_wrong_table_is_caught(how):
    """Every kind of wrong table decodes exactly (the look-back pass reruns)."""
    kinds, cols, offs, p, wire = _case("two_str", 20_000, 40, True, 11)
    n = 20_000
    table, words = _table_from(p, offs, n)
    t = host(table, 8 * words, np.uint64).copy()
    if how == "one_entry_off_by_one":
        t[2 * 40 + 1] += 1
    elif how == "first_nonzero":
        t[:] += 3
    elif how == "huge":
        t[2 * 10] = 2**62
    elif how == "zeros":
        t[:] = 0
    else:
        t = t.reshape(-1, 2)[:, ::-1].reshape(-1).copy()
    back, boffs, st = _unpack_tiled(p, kinds, wire, n, _rec_offsets(kinds, offs, n, len(p.prefix)), _dev_u64(t))
    _check(kinds, p, wire, n, back, boffs, st)


def test_pack_then_tiled_unpack_round_trip():
    """The table from the pack call's own input offsets (srpc_gpu_pack_var ->
    srpc_gpu_var_tile_table -> srpc_gpu_unpack_var_tiled)."""
    from tests.test_gpu_parity import gpu_pack_var
    kinds, cols, offs, p, wire = _case("mixed", 50_000, 60, True, 5)
    n = 50_000
    got, rec, st = gpu_pack_var(p, kinds, cols, offs, n)
    assert got == wire and st[0] == 0
    table, _ = _table_from(p, offs, n)
    back, boffs, st = _unpack_tiled(p, kinds, got, n, rec, table)
    _check(kinds, p, wire, n, back, boffs, st)


def test_stalled_look_back_is_reported_and_a_retry_is_exact():
    """SRPC_STATUS_STALLED (srpc_gpu.h): a multi-string tile whose chars-offset
    look-back outwaits its budget gives up and says so -- the call returns, the
    status carries STALLED, and the caller's retry decodes exactly.  The test
    hook srpc_debug_var_spin_limit shrinks the budget to one poll so tiles give
    up whenever a predecessor has not published yet."""
    import ctypes

    from srpc_amd import _lib
    hook = _lib.lib().srpc_debug_var_spin_limit
    hook.argtypes, hook.restype = [ctypes.c_uint32], ctypes.c_int
    kinds, cols, offs, p, wire = _case("two_str", 200_000, 40, True, 3)
    n = 200_000
    rec = _rec_offsets(kinds, offs, n, len(p.prefix))
    assert hook(1) == 0
    try:
        back, boffs, st = _unpack_tiled(p, kinds, wire, n, rec, None)
    finally:
        assert hook(0) == 0
    stalled = 4  # SRPC_STATUS_STALLED (include/srpc_gpu.h)
    flags = st[0]
    assert flags & ~stalled == 0
    if not flags & stalled:  # no tile had to wait: the outputs are exact
        _check(kinds, p, wire, n, back, boffs, st)
    back, boffs, st = _unpack_tiled(p, kinds, wire, n, rec, None)  # the retry
    _check(kinds, p, wire, n, back, boffs, st)
