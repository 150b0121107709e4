"""The C-ABI library builds, loads and exports every symbol include/srpc_gpu.h
declares.  No compute calls (no GPU here)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from srpc_amd import _lib, build
from srpc_amd.packer import Schema, request_prefix, response_prefix
from srpc_amd.shard import shard_range, shard_ranges

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "srpc_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(srpc_\w+)\s*\(", src, re.M)))


def test_header_parses():
    fns = declared_functions()
    assert "srpc_gpu_pack" in fns and "srpc_gpu_unpack" in fns and "srpc_plan_create" in fns
    assert set(fns) == set(_lib.SIGNATURES), "ctypes table out of sync with the header"


def test_library_exports_every_symbol():
    so = build.build()
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True)
    exported = set(re.findall(r"\bT (srpc_\w+)", out.stdout))
    missing = set(declared_functions()) - exported
    assert not missing, f"not exported: {missing}"


def test_library_loads_and_answers_host_calls():
    L = _lib.lib()
    assert L.srpc_gpu_abi_version() == 8
    assert L.srpc_status_string(-2) == b"device pointer misaligned"
    assert L.srpc_status_string(2).startswith(b"wire shorter")
    # argument validation needs no device
    assert L.srpc_plan_create(None, 0, None) == _lib.SRPC_E_INVALID
    assert L.srpc_plan_destroy(None) == _lib.SRPC_E_INVALID
    assert L.srpc_gpu_pack(None, None, 0, None, 0, None) == _lib.SRPC_E_INVALID
    # ABI 7 host-terminated calls: a null plan is refused before any device work
    out = C.c_uint64()
    assert L.srpc_plan_host_scratch_bytes(None, 1024, 3, C.byref(out)) == _lib.SRPC_E_INVALID
    assert L.srpc_gpu_pack_host(None, None, 1, None, 0, 0, 1, None, 0, None) == _lib.SRPC_E_INVALID
    assert L.srpc_gpu_unpack_host(None, None, 0, 1, None, 0, 1, None, 0, None, None) == _lib.SRPC_E_INVALID
    # the timing hook only arms thread-local state; an invalid call consumes it
    assert L.srpc_time_next_call(None, None) == _lib.SRPC_OK
    assert L.srpc_time_next_call(C.c_void_p(1), None) == _lib.SRPC_OK
    assert L.srpc_gpu_pack(None, None, 0, None, 0, None) == _lib.SRPC_E_INVALID
    # schema limits (SRPC_MAX_FIELDS, SRPC_MAX_PREFIX) are refused before any device work
    kinds33 = (C.c_int32 * 33)(*([5] * 33))
    h = C.c_void_p()
    assert L.srpc_plan_create(C.byref(_lib.SchemaDesc(33, kinds33, None, 0)), 0, C.byref(h)) == _lib.SRPC_E_UNSUPPORTED
    pre = (C.c_uint8 * 1025)()
    assert L.srpc_plan_create(C.byref(_lib.SchemaDesc(1, kinds33, pre, 1025)), 0, C.byref(h)) == \
        _lib.SRPC_E_UNSUPPORTED
    assert L.srpc_plan_create(C.byref(_lib.SchemaDesc(0, kinds33, None, 0)), 0, C.byref(h)) == _lib.SRPC_E_INVALID
    # frame bucketing: scratch sizing is host arithmetic; bad plan counts are refused
    out = C.c_uint64()
    assert L.srpc_frames_scratch_bytes(1 << 20, 4, C.byref(out)) == _lib.SRPC_OK and out.value >= 4 << 20
    assert L.srpc_frames_scratch_bytes(10, 0, C.byref(out)) == _lib.SRPC_E_INVALID
    assert L.srpc_frames_scratch_bytes(10, 17, C.byref(out)) == _lib.SRPC_E_INVALID
    assert L.srpc_frames_classify(None, None, 1, None, 0, None, 0, None, None, None, None, None, 0,
                                  None) == _lib.SRPC_E_INVALID
    assert L.srpc_frames_gather(None, None, None, 0, 57, None, None) == _lib.SRPC_OK  # nothing to do
    assert L.srpc_frames_gather(None, None, None, 3, 57, None, None) == _lib.SRPC_E_INVALID


def test_library_is_gfx950_code_object():
    data = open(build.build(), "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data  # offload bundle entry id


def test_envelope_headers():
    assert request_prefix("Calculator_servicer::square", "Number") == (
        (27).to_bytes(8, "little") + b"Calculator_servicer::square" + (6).to_bytes(8, "little") + b"Number")
    assert response_prefix(0, "Number") == b"\x00" + (6).to_bytes(8, "little") + b"Number"


def test_schema_flattening_nested():
    sp = Schema.of("single_primitive", ("arg1", "int8"))
    mp = Schema.of("multiple_primitives", ("arg1", "int8"), ("arg2", "char"), ("arg3", "int64"),
                   ("arg4", "string"))
    nm = Schema.of("nested_message", ("arg1", "int64"), ("arg2", sp), ("arg3", mp))
    assert nm.kinds == [6, 2, 2, 3, 6, 7]
    assert nm.body_bytes == 0 and sp.body_bytes == 1
    assert Schema.of("Quad", *[(c, "int32") for c in "abcd"]).body_bytes == 16


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (17, 2), (1 << 24, 8), (1000, 3), (64, 8)])
def test_shard_ranges_cover(n, world):
    rs = shard_ranges(n, world)
    assert rs[0][0] == 0 and rs[-1][1] == n
    for (a, b), (c, d) in zip(rs, rs[1:]):
        assert b == c and a <= b
    for lo, _ in rs:
        assert lo % 16 == 0 or lo == n
    assert shard_range(n, 0, 1) == (0, n)


@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 1000, 4099, 1 << 24, (1 << 26) + 5, 2**63 + 11])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8])
def test_native_shard_range_matches_python_rule(n, world):
    """srpc_shard_range (C ABI, host arithmetic) == srpc_amd.shard.shard_range:
    contiguous, rank-ordered, every start a multiple of 16 records, so a
    shard's wire offset is lo * record_bytes and every shard is 16-byte aligned
    for 1-byte records (the alignment the TILE/DWORD kernels need)."""
    from srpc_amd.shard import native_shard_range
    got = [native_shard_range(n, r, world) for r in range(world)]
    assert got == shard_ranges(n, world)
    for lo, hi in got:
        assert lo % 16 == 0 or lo == n
    # byte offsets of a fixed record size reproduce the single-batch layout
    rb = 53
    offs = [lo * rb for lo, _ in got]
    assert offs[0] == 0 and all(o2 - o1 == (hi - lo) * rb for (lo, hi), o1, o2 in zip(got, offs, offs[1:] + [n * rb]))


def test_native_shard_range_rejects_bad_ranks():
    L = _lib.lib()
    lo, hi = C.c_uint64(), C.c_uint64()
    assert L.srpc_shard_range(10, 2, 2, C.byref(lo), C.byref(hi)) == _lib.SRPC_E_INVALID
    assert L.srpc_shard_range(10, -1, 2, C.byref(lo), C.byref(hi)) == _lib.SRPC_E_INVALID
    assert L.srpc_shard_range(10, 0, 0, C.byref(lo), C.byref(hi)) == _lib.SRPC_E_INVALID
    assert L.srpc_comm_destroy(None) == _lib.SRPC_E_INVALID
    assert L.srpc_gather_wire(None, None, 0, None, 0, None, 0, None) == _lib.SRPC_E_INVALID
