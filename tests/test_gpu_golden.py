"""The reference's own 12 golden vectors through the HIP path.

tests/packer_test.cpp:91-436 (pack / unpack x request / response x
{single_primitive, multiple_primitives, nested_message}) is restated as data
in tests/golden/packer_test_vectors.json, produced by the reference build
(tests/golden/make_golden.py).  Each section runs through the C ABI:
single_primitive on the fixed-size path (srpc_gpu_pack / _unpack),
multiple_primitives and nested_message (flattened, as pack_struct inlines
nested members, packer.hpp:185-186) on the VAR path (srpc_gpu_pack_var /
_unpack_var).  Request prefixes use the method names of the test ("test",
and "test_method" for unpack request/multiple, packer_test.cpp:302-303),
responses the codes 0 / 2 / 1.  Each section is run as one record and as
100,003 copies of it: the wire must equal the vector (repeated) byte for
byte, and every decoded record, re-emitted as a bare body, must equal the
body the reference decoded from the same input.
"""
import json
import os

import numpy as np
import pytest

import oracle
from srpc_amd import GpuPacker, Schema, SRPC_PATH_VAR

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover - CPU container
    pytest.skip("no GPU", allow_module_level=True)

from tests.test_gpu_parity import gpu_pack, gpu_pack_var, gpu_unpack, gpu_unpack_var  # noqa: E402

I64MAX = 2**63 - 1
SINGLE = Schema.of("single_primitive", ("arg1", "int8"))
MULTIPLE = Schema.of("multiple_primitives", ("arg1", "int8"), ("arg2", "char"), ("arg3", "int64"),
                     ("arg4", "string"))
NESTED = Schema.of("nested_message", ("arg1", "int64"), ("arg2", SINGLE), ("arg3", MULTIPLE))
SCHEMA = {"single": SINGLE, "multiple": MULTIPLE, "nested": NESTED}
CODE = {"single": 0, "multiple": 2, "nested": 1}  # packer_test.cpp:191,214,249
REPS = [1, 100_003]


def _vectors():
    with open(os.path.join(os.path.dirname(__file__), "golden", "packer_test_vectors.json")) as f:
        return {c["section"]: c for c in json.load(f)}


def _values(which, reps):
    """The field values of the test's messages (packer_test.cpp make_* ), each
    column repeated `reps` times; strings as chars + n+1 offsets."""
    txt = np.frombuffer(b"testing_string", np.uint8)
    sp = [np.full(reps, 5, np.int8)]
    mp = [np.full(reps, 22, np.int8), np.full(reps, ord("z"), np.int8), np.full(reps, I64MAX, np.int64),
          np.tile(txt, reps)]
    offs = np.arange(reps + 1, dtype=np.uint64) * np.uint64(len(txt))
    if which == "single":
        return sp, [None]
    if which == "multiple":
        return mp, [None, None, None, offs]
    return [np.full(reps, I64MAX, np.int64)] + sp + mp, [None, None, None, None, None, offs]


def _packer(which, kind, method="test"):
    sch = SCHEMA[which]
    if kind == "request":
        return GpuPacker.for_request(sch, method)
    return GpuPacker.for_response(sch, CODE[which])


@pytest.mark.parametrize("reps", REPS)
@pytest.mark.parametrize("which", ["single", "multiple", "nested"])
@pytest.mark.parametrize("kind", ["request", "response"])
def test_pack_sections_on_gpu(kind, which, reps):
    want = bytes.fromhex(_vectors()[f"pack {kind}/{which}"]["bytes"])
    p = _packer(which, kind)
    cols, offs = _values(which, reps)
    if which == "single":
        assert p.record_bytes == len(want)
        got = gpu_pack(p, cols, reps)
    else:
        assert p.path == SRPC_PATH_VAR
        got, rec, st = gpu_pack_var(p, SCHEMA[which].kinds, cols, offs, reps)
        assert st == (0, 2**64 - 1)
        assert np.array_equal(rec, np.arange(reps + 1, dtype=np.uint64) * np.uint64(len(want)))
    assert got == want * reps


@pytest.mark.parametrize("reps", REPS)
@pytest.mark.parametrize("which", ["single", "multiple", "nested"])
@pytest.mark.parametrize("kind", ["request", "response"])
def test_unpack_sections_on_gpu(kind, which, reps):
    case = _vectors()[f"unpack {kind}/{which}"]
    one = bytes.fromhex(case["input"])
    body = bytes.fromhex(case["body"])  # what the reference decoded, re-emitted as a body
    if kind == "request":
        p = _packer(which, kind, case["method"])
    else:
        assert case["code"] == CODE[which]
        p = _packer(which, kind)
    kinds = SCHEMA[which].kinds
    wire = one * reps
    if which == "single":
        rc, back = gpu_unpack(p, wire, reps, [np.int8])
        assert rc == 0
        boffs = [None]
    else:
        rec = np.arange(reps + 1, dtype=np.uint64) * np.uint64(len(one))
        back, boffs, st = gpu_unpack_var(p, kinds, wire, reps, rec)
        assert st == (0, 2**64 - 1)
    # every decoded record re-emitted as a bare body (`p << value`) is the reference's body
    got = oracle.pack(kinds, back, reps, b"", list(boffs))
    assert got == body * reps
    cols, offs = _values(which, reps)
    for f, k in enumerate(kinds):
        assert back[f].tobytes() == cols[f].tobytes(), f
        if offs[f] is not None:
            assert np.array_equal(boffs[f], offs[f])


def test_unpack_request_multiple_other_method_is_prefix_error():
    """unpack request/multiple carries "test_method" (packer_test.cpp:302-303):
    a plan expecting "test" flags every record's envelope as foreign."""
    case = _vectors()["unpack request/multiple"]
    one = bytes.fromhex(case["input"])
    p = _packer("multiple", "request", "test")
    rec = np.arange(4, dtype=np.uint64) * np.uint64(len(one))
    _, _, st = gpu_unpack_var(p, MULTIPLE.kinds, one * 3, 3, rec)
    assert st[1] == 0 and st[0] != 0
