"""ctypes binding of the C ABI in include/srpc_gpu.h (libsrpc_gpu.so).

The HIP library is the only compute path: if it cannot be loaded, every call
raises.  There is no CPU fallback anywhere in ``srpc_amd``.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

from . import build as _build

_vp = C.c_void_p
_u64 = C.c_uint64
_i32 = C.c_int32

SRPC_OK = 0
SRPC_E_INVALID = -1
SRPC_E_ALIGN = -2
SRPC_E_HIP = -3
SRPC_E_UNSUPPORTED = -4
SRPC_E_CAPACITY = -5
SRPC_ERR_BOUNDS = 2

SRPC_STATUS_PREFIX = 1
SRPC_STATUS_BOUNDS = 2
SRPC_STATUS_STALLED = 4
SRPC_COMM_ID_BYTES = 128
SRPC_MAX_FIELDS = 32
SRPC_MAX_PREFIX = 1024
SRPC_FRAMES_MAX_PLANS = 16
SRPC_FRAME_UNKNOWN = 0xFF
SRPC_FRAMES_MAX_STRINGS = 16

SRPC_PATH_DWORD = 1
SRPC_PATH_TILE = 2
SRPC_PATH_VAR = 3

# Every symbol declared in include/srpc_gpu.h: (restype, argtypes)
SIGNATURES = {
    "srpc_plan_create": (C.c_int, [_vp, C.c_int, C.POINTER(_vp)]),
    "srpc_plan_destroy": (C.c_int, [_vp]),
    "srpc_plan_record_bytes": (C.c_int, [_vp, C.POINTER(_u64)]),
    "srpc_plan_path": (C.c_int, [_vp, C.POINTER(C.c_int)]),
    "srpc_plan_force_path": (C.c_int, [_vp, C.c_int]),
    "srpc_plan_tune": (C.c_int, [_vp, C.c_int, C.c_int]),
    "srpc_gpu_pack": (C.c_int, [_vp, _vp, _u64, _vp, _u64, _vp]),
    "srpc_gpu_unpack": (C.c_int, [_vp, _vp, _u64, _u64, _vp, _vp, _vp]),
    "srpc_plan_var_scratch_bytes": (C.c_int, [_vp, _u64, _u64, C.POINTER(_u64)]),
    "srpc_gpu_pack_var": (C.c_int, [_vp, _vp, _vp, _u64, _vp, _u64, _vp, _vp, _vp, _u64, _vp]),
    "srpc_gpu_unpack_var": (C.c_int, [_vp, _vp, _u64, _u64, _vp, _vp, _vp, _vp, _vp, _u64, _vp]),
    "srpc_gpu_fill_splitmix_i32": (C.c_int, [_vp, C.c_uint32, _u64, _u64, _u64, _vp]),
    "srpc_time_next_call": (C.c_int, [_vp, _vp]),
    "srpc_var_tile_table_words": (C.c_int, [_vp, _u64, C.POINTER(_u64)]),
    "srpc_gpu_var_tile_table": (C.c_int, [_vp, _vp, _u64, _vp, _vp]),
    "srpc_gpu_unpack_var_tiled": (C.c_int, [_vp, _vp, _u64, _u64, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp]),
    "srpc_plan_var_stream_scratch_bytes": (C.c_int, [_vp, _u64, _u64, C.POINTER(_u64)]),
    "srpc_gpu_unpack_var_stream": (C.c_int, [_vp, _vp, _u64, _u64, _vp, _vp, _vp, _vp, _vp, _u64, _vp]),
    "srpc_plan_host_scratch_bytes": (C.c_int, [_vp, _u64, C.c_uint32, C.POINTER(_u64)]),
    "srpc_gpu_pack_host": (C.c_int, [_vp, _vp, _u64, _vp, _u64, _u64, C.c_uint32, _vp, _u64, _vp]),
    "srpc_gpu_unpack_host": (C.c_int, [_vp, _vp, _u64, _u64, _vp, _u64, C.c_uint32, _vp, _u64, _vp, _vp]),
    "srpc_shard_range": (C.c_int, [_u64, C.c_int, C.c_int, C.POINTER(_u64), C.POINTER(_u64)]),
    "srpc_comm_unique_id": (C.c_int, [_vp]),
    "srpc_comm_init_rank": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.POINTER(_vp)]),
    "srpc_comm_init_all": (C.c_int, [_vp, C.c_int, _vp]),
    "srpc_comm_destroy": (C.c_int, [_vp]),
    "srpc_comm_rank": (C.c_int, [_vp, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "srpc_allgather_u64": (C.c_int, [_vp, _vp, _vp, _vp]),
    "srpc_gather_plan": (C.c_int, [C.c_int, C.c_int, C.c_int, _u64, _vp, _u64, _vp, C.c_int, C.POINTER(C.c_int)]),
    "srpc_gather_wire": (C.c_int, [_vp, _vp, _u64, _vp, _u64, _vp, C.c_int, _vp]),
    "srpc_group_gather_wire": (C.c_int, [_vp, C.c_int, _vp, _vp, _vp, _u64, C.c_int, _vp]),
    "srpc_group_pack_gather": (C.c_int, [_vp, _vp, C.c_int, _vp, _u64, _vp, _vp, _u64, C.c_int, _vp]),
    "srpc_gpu_pack_aos": (C.c_int, [_vp, _vp, _u64, _vp, _u64, _vp, _u64, _vp]),
    "srpc_gpu_unpack_aos": (C.c_int, [_vp, _vp, _u64, _u64, _vp, _u64, _vp, _vp, _vp]),
    "srpc_gpu_unpack_aos_fill": (C.c_int, [_vp, _vp, _u64, _u64, _vp, _u64, _vp, _vp, _vp, _vp]),
    "srpc_frames_scratch_bytes": (C.c_int, [_u64, C.c_int, C.POINTER(_u64)]),
    "srpc_frames_classify": (C.c_int, [_vp, _vp, C.c_int, _vp, _u64, _vp, _u64, _vp, _vp, _vp, _vp, _vp, _u64,
                                       _vp]),
    "srpc_frames_gather": (C.c_int, [_vp, _vp, _vp, _u64, C.c_uint32, _vp, _vp]),
    "srpc_frames_scatter": (C.c_int, [_vp, _vp, _u64, C.c_uint32, _vp, _vp, _vp]),
    "srpc_frames_gather_var": (C.c_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp, _u64, _vp]),
    "srpc_frames_scatter_var": (C.c_int, [_vp, _vp, _vp, _u64, _vp, _vp, _vp]),
    "srpc_frames_offsets": (C.c_int, [_vp, _vp, C.c_int, _vp, _u64, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp]),
    "srpc_status_string": (C.c_char_p, [C.c_int]),
    "srpc_gpu_abi_version": (C.c_int, []),
}


class SchemaDesc(C.Structure):
    _fields_ = [("nfields", C.c_uint32), ("kinds", C.POINTER(_i32)),
                ("prefix", C.POINTER(C.c_uint8)), ("prefix_len", C.c_uint32)]


class GatherOp(C.Structure):
    _fields_ = [("kind", _i32), ("peer", _i32), ("offset", _u64), ("bytes", _u64)]


SRPC_GATHER_SEND = 1
SRPC_GATHER_RECV = 2
SRPC_GATHER_COPY = 3


class UnpackStatus(C.Structure):
    _fields_ = [("flags", C.c_uint32), ("reserved", C.c_uint32),
                ("first_bad_record", C.c_uint64)]


class SrpcError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: srpc status {code} ({status_string(code)})")


_lock = threading.Lock()
_lib = None


def _preload_torch() -> None:
    # libsrpc_gpu.so binds the HIP runtime by soname (libamdhip64.so.7).  If
    # torch is used in this process its bundled runtime must be the one bound,
    # so import torch first when it is available.
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib() -> C.CDLL:
    global _lib
    with _lock:
        if _lib is None:
            path = os.environ.get("SRPC_GPU_LIB")  # A/B experiments: another build of the library
            if not path:
                if _build.needs_build():
                    _build.build()
                path = _build.SO
            _preload_torch()
            so = C.CDLL(path, mode=C.RTLD_GLOBAL)
            ab = bool(os.environ.get("SRPC_GPU_LIB"))
            for name, (res, args) in SIGNATURES.items():
                if ab and not hasattr(so, name):  # an A/B build older than this table: its symbols only
                    continue
                fn = getattr(so, name)
                fn.restype = res
                fn.argtypes = args
            _lib = so
    return _lib


def so_path() -> str:
    return os.path.abspath(os.environ.get("SRPC_GPU_LIB") or _build.SO)


def status_string(code: int) -> str:
    try:
        return lib().srpc_status_string(code).decode()
    except Exception:
        return "?"


def check(code: int, what: str) -> int:
    if code < 0:
        raise SrpcError(code, what)
    return code
