"""TEST INFRASTRUCTURE ONLY -- the checker, never the product.

Python bindings for
  * ``liboracle.so``        -- the plain-C restatement of the sRPC packer
                               (``oracle/packer_oracle.c``), and
  * ``_ref/libsrpc_ref.so`` -- the reference packer itself, compiled from the
                               unmodified headers under /root/reference by
                               ``oracle/Makefile`` (absent where it cannot be
                               built; it travels to the GPU box prebuilt).
plus the vectorised splitmix64 input definition of SURVEY.md §8c.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package.  ``srpc_amd`` never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libsrpc_ref.so")

# Field kinds (same numbering as include/srpc_gpu.h and packer_oracle.h).
BOOL, INT8, CHAR, INT16, INT32, INT64, STRING = 1, 2, 3, 4, 5, 6, 7
KIND_SIZE = {BOOL: 1, INT8: 1, CHAR: 1, INT16: 2, INT32: 4, INT64: 8, STRING: 0}
KIND_DTYPE = {BOOL: np.uint8, INT8: np.int8, CHAR: np.int8, INT16: np.int16,
              INT32: np.int32, INT64: np.int64}

ORC_OK, ORC_ERR_BOUNDS, ORC_ERR_PREFIX = 0, 1, 2

_u8p = C.POINTER(C.c_uint8)
_vp = C.c_void_p
_u64 = C.c_uint64


def build(quiet: bool = True) -> None:
    """Build liboracle.so (and _ref/ when /root/reference exists)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


_oracle = None
_ref = None


def oracle_lib() -> C.CDLL:
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            build()
        lib = C.CDLL(ORACLE_SO)
        lib.orc_pack.restype = _u64
        lib.orc_pack.argtypes = [_vp, C.c_int, _vp, _u64, _vp, _vp, _u64, _vp, _u64]
        lib.orc_unpack.restype = C.c_int
        lib.orc_unpack.argtypes = [_vp, C.c_int, _vp, _u64, _vp, _u64, _u64, _vp, _vp,
                                   C.POINTER(_u64), C.POINTER(_u64)]
        lib.orc_request_prefix.restype = _u64
        lib.orc_request_prefix.argtypes = [C.c_char_p, C.c_char_p, _vp]
        lib.orc_response_prefix.restype = _u64
        lib.orc_response_prefix.argtypes = [C.c_uint8, C.c_char_p, _vp]
        lib.orc_fixed_record_size.restype = _u64
        lib.orc_fixed_record_size.argtypes = [_vp, C.c_int, _u64]
        lib.orc_splitmix_i32.restype = None
        lib.orc_splitmix_i32.argtypes = [C.POINTER(_u64), _vp, _u64]
        _oracle = lib
    return _oracle


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref_lib() -> C.CDLL:
    """The reference packer (compiled from /root/reference).  Raises if absent."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_SO):
            raise FileNotFoundError(REF_SO + " not built (needs /root/reference)")
        lib = C.CDLL(REF_SO)
        D = C.POINTER(C.c_double)
        sig = {
            "ref_packer_test_vector": (_u64, [C.c_int, _vp, _u64]),
            "ref_packer_test_decode": (_u64, [C.c_int, C.c_int, _vp, _u64, _vp, _u64, C.c_char_p,
                                              C.POINTER(C.c_int)]),
            "ref_pack_number": (_u64, [_vp, _u64, _vp, _u64]),
            "ref_pack_two_numbers": (_u64, [_vp, _vp, _u64, _vp, _u64]),
            "ref_pack_all_kinds": (_u64, [_vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp, _u64]),
            "ref_pack_multiple": (_u64, [_vp, _vp, _vp, _vp, _vp, _u64, _vp, _u64]),
            "ref_unpack_multiple": (C.c_int, [_vp, _u64, _u64, _vp, _vp, _vp, _vp, _vp]),
            "ref_unpack_all_kinds": (C.c_int, [_vp, _u64, _u64, _vp, _vp, _vp, _vp, _vp, _vp]),
            "ref_pack_quad": (_u64, [_vp, _vp, _vp, _vp, _u64, _vp, _u64, D]),
            "ref_unpack_quad": (C.c_int, [_vp, _u64, _u64, _vp, _vp, _vp, _vp, D]),
            "ref_pack_quad_mt": (_u64, [_vp, _vp, _vp, _vp, _u64, _vp, C.c_int, D]),
            "ref_unpack_quad_mt": (C.c_int, [_vp, _u64, _vp, _vp, _vp, _vp, C.c_int, D]),
            "ref_pack_square_requests": (_u64, [_vp, _u64, _vp, _u64, D]),
            "ref_server_square": (_u64, [_vp, _u64, _u64, _vp, _u64, D]),
            "ref_unpack_square_responses": (C.c_int, [_vp, _u64, _u64, _vp, _vp]),
            "ref_geo_locate_responses": (_u64, [_u64, _u64, _vp, _u64]),
            "ref_geo_locate_requests": (_u64, [_u64, _u64, _vp, _u64]),
            "ref_server_echo": (_u64, [_u64, _vp, _u64, C.POINTER(_u64)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _ref = lib
    return _ref


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# --------------------------------------------------------------------------
# splitmix64 synthetic inputs, vectorised.
# --------------------------------------------------------------------------
SEED = 0x5EED
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def splitmix_u32(seed: int, start: int, count: int) -> np.ndarray:
    """Low 32 bits of splitmix64 draws number start..start+count-1."""
    out = np.empty(count, dtype=np.uint32)
    step = 1 << 24
    with np.errstate(over="ignore"):
        for lo in range(0, count, step):
            hi = min(count, lo + step)
            i = np.arange(start + lo + 1, start + hi + 1, dtype=np.uint64)
            z = np.uint64(seed) + i * _GOLD
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            out[lo:hi] = (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    return out


def splitmix_columns_i32(nfields: int, n: int, seed: int = SEED, first_record: int = 0):
    """F int32 columns; record i field f = draw i*F+f."""
    flat = splitmix_u32(seed, first_record * nfields, n * nfields).view(np.int32)
    m = flat.reshape(n, nfields)
    return [np.ascontiguousarray(m[:, f]) for f in range(nfields)]


def square_inputs(n: int, seed: int = SEED) -> np.ndarray:
    """num = next % 46341 with C++ truncating %, so |num| <= 46340."""
    v = splitmix_u32(seed, 0, n).view(np.int32).astype(np.int64)
    r = np.fmod(v, 46341)
    return r.astype(np.int32)


# --------------------------------------------------------------------------
# Oracle wrappers
# --------------------------------------------------------------------------

def request_prefix(method: str, name: str) -> bytes:
    buf = np.zeros(16 + len(method) + len(name), np.uint8)
    n = oracle_lib().orc_request_prefix(method.encode(), name.encode(), ptr(buf))
    return buf[:n].tobytes()


def response_prefix(code: int, name: str) -> bytes:
    buf = np.zeros(9 + len(name), np.uint8)
    n = oracle_lib().orc_response_prefix(code, name.encode(), ptr(buf))
    return buf[:n].tobytes()


def _kinds_arr(kinds):
    return np.asarray(kinds, dtype=np.int32)


def pack(kinds, cols, n: int, prefix: bytes = b"", str_offsets=None) -> bytes:
    """Oracle pack of n records.  cols[f]: numpy array (fixed) or uint8 chars (string)."""
    lib = oracle_lib()
    k = _kinds_arr(kinds)
    F = len(kinds)
    colp = (C.c_void_p * F)(*[ptr(c) for c in cols])
    offp = (C.c_void_p * F)()
    cap = len(prefix) * n
    for f, kind in enumerate(kinds):
        if kind == STRING:
            o = np.ascontiguousarray(str_offsets[f], dtype=np.uint64)
            str_offsets[f] = o
            offp[f] = ptr(o)
            cap += 8 * n + int(o[n] - o[0])
        else:
            cap += KIND_SIZE[kind] * n
    out = np.zeros(max(cap, 1), np.uint8)
    pre = np.frombuffer(prefix, np.uint8) if prefix else np.zeros(1, np.uint8)
    w = lib.orc_pack(ptr(k), F, ptr(pre), len(prefix), C.addressof(colp), C.addressof(offp),
                     n, ptr(out), cap)
    if w == 2**64 - 1:
        raise ValueError("oracle pack overflow")
    return out[:w].tobytes()


def unpack(kinds, wire: bytes, n: int, prefix: bytes = b""):
    """Oracle unpack.  Returns (status, cols, str_offsets, consumed, err_record)."""
    lib = oracle_lib()
    k = _kinds_arr(kinds)
    F = len(kinds)
    w = np.frombuffer(wire, np.uint8) if len(wire) else np.zeros(1, np.uint8)
    cols, offs = [], [None] * F
    colp = (C.c_void_p * F)()
    offp = (C.c_void_p * F)()
    for f, kind in enumerate(kinds):
        if kind == STRING:
            c = np.zeros(max(len(wire), 1), np.uint8)
            o = np.zeros(n + 1, np.uint64)
            offs[f] = o
            offp[f] = ptr(o)
        else:
            c = np.zeros(max(n, 1), KIND_DTYPE[kind])
        cols.append(c)
        colp[f] = ptr(c)
    pre = np.frombuffer(prefix, np.uint8) if prefix else np.zeros(1, np.uint8)
    consumed, err = _u64(0), _u64(0)
    st = lib.orc_unpack(ptr(k), F, ptr(pre), len(prefix), ptr(w), len(wire), n,
                        C.addressof(colp), C.addressof(offp), C.byref(consumed), C.byref(err))
    for f, kind in enumerate(kinds):
        if kind == STRING:
            cols[f] = cols[f][: int(offs[f][n])] if st == ORC_OK else cols[f]
        else:
            cols[f] = cols[f][:n]
    return st, cols, offs, consumed.value, err.value
