"""Schema-specialised TILE kernels (srpc_amd/csrc/rec.hip): the layouts that
have an instance -- all_kinds (17 B), Number behind the square request (53 B)
and response (19 B) envelopes, TwoNumbers behind request / response envelopes
-- packed and unpacked with the specialised kernels (whole tiles) plus the
generic ones (the tail), against the oracle and against the generic kernels
alone (SRPC_TUNE_REC_KERNEL 0), at sizes around the tile (1024 / 512 records)
and with prefix mismatches inside the specialised part and in the tail (the
first bad record's absolute index)."""
import numpy as np
import pytest

import oracle
import srpc_amd
from srpc_amd import GpuPacker, Schema

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

from tests.test_gpu_parity import gpu_pack, gpu_unpack, read_status, status_buf  # noqa: E402

I32 = srpc_amd.INT32
LAYOUTS = {
    "all_kinds": (Schema.of("all_kinds", ("a", "bool"), ("b", "int8"), ("c", "char"), ("d", "int16"), ("e", "int32"),
                            ("f", "int64")), None, 1024),
    "square_request": (srpc_amd.NUMBER, ("request", srpc_amd.SQUARE_METHOD), 512),
    "square_response": (srpc_amd.NUMBER, ("response", 0), 1024),
    "add_request": (srpc_amd.TWO_NUMBERS, ("request", "Calculator_servicer::add"), 512),
    "add_response": (srpc_amd.TWO_NUMBERS, ("response", 0), 1024),
}


def _packer(name):
    sch, env, _ = LAYOUTS[name]
    if env is None:
        return GpuPacker(sch)
    if env[0] == "request":
        return GpuPacker.for_request(sch, env[1])
    return GpuPacker.for_response(sch, env[1])


def _cols(sch, n, rng):
    out = []
    for k in sch.kinds:
        dt = np.dtype(oracle.KIND_DTYPE[k])
        c = rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt)
        if k == oracle.BOOL:
            c = c & 1
        out.append(c)
    return out


@pytest.mark.parametrize("name", list(LAYOUTS))
@pytest.mark.parametrize("tiles,extra", [(0, 1), (1, -1), (1, 0), (1, 1), (3, 17), (97, 5)])
def test_rec_kernels_vs_oracle(name, tiles, extra):
    sch, _, TR = LAYOUTS[name]
    n = tiles * TR + extra
    p = _packer(name)
    assert p.path == srpc_amd.SRPC_PATH_TILE
    rng = np.random.default_rng(n)
    cols = _cols(sch, n, rng)
    want = bytes(oracle.pack(sch.kinds, cols, n, p.prefix))
    assert gpu_pack(p, cols, n) == want
    st = status_buf()
    rc, back = gpu_unpack(p, want, n, [c.dtype for c in cols], status=st)
    assert rc == 0 and read_status(st) == (0, 2**64 - 1)
    for c, b in zip(cols, back):
        assert c.tobytes() == b.tobytes()
    # the generic kernels give the same bytes
    p.tune(rec_kernel=0)
    assert gpu_pack(p, cols, n) == want
    p.tune(rec_kernel=2)  # both directions, whichever the plan would choose


@pytest.mark.parametrize("name", ["square_request", "add_response"])
@pytest.mark.parametrize("where", ["first", "inside", "tail_only"])
def test_rec_prefix_mismatch_first_record(name, where):
    sch, _, TR = LAYOUTS[name]
    n = 5 * TR + 100
    p = _packer(name)
    rng = np.random.default_rng(11)
    cols = _cols(sch, n, rng)
    wire = bytearray(oracle.pack(sch.kinds, cols, n, p.prefix))
    stride = p.record_bytes
    bad = {"first": [0, 3 * TR + 7], "inside": [2 * TR + 5, 4 * TR + 1, 5 * TR + 50],
           "tail_only": [5 * TR + 3, 5 * TR + 99]}[where]
    for r in bad:
        wire[r * stride + 3] ^= 0x10  # a byte of the prefix
    st = status_buf()
    rc, back = gpu_unpack(p, bytes(wire), n, [c.dtype for c in cols], status=st)
    assert read_status(st) == (srpc_amd.SRPC_STATUS_PREFIX, min(bad))
    for c, b in zip(cols, back):  # fields still decoded from their places
        assert c.tobytes() == b.tobytes()
