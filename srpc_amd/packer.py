"""Host-side batch packer over the HIP C ABI.

Mirrors the reference packer's vocabulary (include/srpc/packer.hpp):
``pack`` / ``unpack`` are the batched ``p << r`` / ``r.unpack(bp)`` loops,
``for_request`` / ``for_response`` build the constant envelope header that
``packer::pack_request`` (packer.hpp:77-82) and ``packer::pack_response``
(packer.hpp:86-91) emit in front of every body.

Device memory is passed as raw device pointers (ints) or as any object with a
``data_ptr()`` method (e.g. a torch tensor on the GPU); streams as a raw
``hipStream_t`` (int) or an object with ``cuda_stream``.
"""
from __future__ import annotations

import ctypes as C
import struct
from dataclasses import dataclass, field
from typing import Iterable, Sequence

from . import _lib
from ._lib import SrpcError, check

# IDL kinds (include/srpc_gpu.h, = the type table of parser.hpp:253-290)
BOOL, INT8, CHAR, INT16, INT32, INT64, STRING = 1, 2, 3, 4, 5, 6, 7
KIND_NAMES = {"bool": BOOL, "int8": INT8, "char": CHAR, "int16": INT16, "int32": INT32,
              "int64": INT64, "string": STRING}
KIND_SIZE = {BOOL: 1, INT8: 1, CHAR: 1, INT16: 2, INT32: 4, INT64: 8, STRING: 0}

# rpc_status_code (packer.hpp:16-20)
RPC_SUCCESS, RPC_ERR_FUNCTION_NOT_REGISTERED, RPC_ERR_RECV_TIMEOUT = 0, 1, 2


@dataclass(frozen=True)
class Schema:
    """A message type: its name (``T::name``) and its flattened fields in
    ``T::fields`` declaration order (nested messages inlined, as
    ``pack_arg`` does for message-typed members, packer.hpp:185-186)."""

    name: str
    fields: tuple = field(default_factory=tuple)  # ((field_name, kind), ...)

    @staticmethod
    def of(name: str, *fields) -> "Schema":
        out = []
        for fname, kind in fields:
            if isinstance(kind, Schema):  # nested message: inline its fields
                out.extend((f"{fname}.{n}", k) for n, k in kind.fields)
            else:
                out.append((fname, KIND_NAMES[kind] if isinstance(kind, str) else int(kind)))
        return Schema(name, tuple(out))

    @property
    def kinds(self) -> list[int]:
        return [k for _, k in self.fields]

    @property
    def body_bytes(self) -> int:
        """Fixed body size, 0 if the schema has a string field."""
        if any(k == STRING for k in self.kinds):
            return 0
        return sum(KIND_SIZE[k] for k in self.kinds)


def request_prefix(method: str, msg_name: str) -> bytes:
    """``u64 len(method) | method | u64 len(T::name) | T::name`` (packer.hpp:77-82,
    strings per pack_arg<std::string> 193-198 and pack_arg<const char*> 203-208)."""
    m, n = method.encode(), msg_name.encode()
    return struct.pack("<Q", len(m)) + m + struct.pack("<Q", len(n)) + n


def response_prefix(code: int, msg_name: str) -> bytes:
    """``u8 code | u64 len(T::name) | T::name`` (packer.hpp:86-91)."""
    n = msg_name.encode()
    return bytes([code & 0xFF]) + struct.pack("<Q", len(n)) + n


def _dptr(x) -> int:
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    raise TypeError(f"expected a device pointer or tensor, got {type(x)!r}")


def _stream(s) -> int:
    if s is None:
        return 0
    if isinstance(s, int):
        return s
    if hasattr(s, "cuda_stream"):
        return int(s.cuda_stream)
    raise TypeError(f"expected a hipStream_t handle or stream object, got {type(s)!r}")


class GpuPacker:
    """A plan for one record schema (+ optional envelope prefix) on one device."""

    def __init__(self, schema: Schema, prefix: bytes = b"", device: int = 0):
        self.schema = schema
        self.prefix = bytes(prefix)
        self.device = device
        L = _lib.lib()
        kinds = (C.c_int32 * len(schema.kinds))(*schema.kinds)
        pre = (C.c_uint8 * max(1, len(self.prefix))).from_buffer_copy(self.prefix or b"\0")
        desc = _lib.SchemaDesc(len(schema.kinds), kinds, pre, len(self.prefix))
        h = C.c_void_p()
        check(L.srpc_plan_create(C.byref(desc), device, C.byref(h)), "srpc_plan_create")
        self._h = h
        rb = C.c_uint64()
        check(L.srpc_plan_record_bytes(h, C.byref(rb)), "srpc_plan_record_bytes")
        self.record_bytes = rb.value

    @classmethod
    def for_request(cls, schema: Schema, method: str, device: int = 0) -> "GpuPacker":
        return cls(schema, request_prefix(method, schema.name), device)

    @classmethod
    def for_response(cls, schema: Schema, code: int = RPC_SUCCESS, device: int = 0) -> "GpuPacker":
        return cls(schema, response_prefix(code, schema.name), device)

    # -- plan info ---------------------------------------------------------
    @property
    def path(self) -> int:
        p = C.c_int()
        check(_lib.lib().srpc_plan_path(self._h, C.byref(p)), "srpc_plan_path")
        return p.value

    def force_path(self, path: int) -> None:
        check(_lib.lib().srpc_plan_force_path(self._h, path), "srpc_plan_force_path")

    def tune(self, records_per_lane: int | None = None, iters: int | None = None,
             nontemporal: int | None = None, tile_bytes: int | None = None,
             grid: int | None = None, pack_tile_bytes: int | None = None,
             var_kernel: int | None = None, var_image_bytes: int | None = None,
             var_chars_bytes: int | None = None, wave_pack_bytes: int | None = None,
             wave_unpack_bytes: int | None = None, rec_kernel: int | None = None) -> None:
        """Performance knobs (srpc_plan_tune); output bytes never change.
        var_kernel: VAR pack, 1 = record tiles (one pass), 0 = scan + chunk walk.
        rec_kernel: TILE schema-specialised kernels, 1 = where measured faster, 2 = both directions, 0 = off."""
        L = _lib.lib()
        for knob, val in ((1, records_per_lane), (2, iters), (3, nontemporal), (4, tile_bytes),
                          (5, grid), (9, pack_tile_bytes), (7, var_kernel), (8, var_image_bytes),
                          (10, var_chars_bytes), (11, wave_pack_bytes), (12, wave_unpack_bytes),
                          (13, rec_kernel)):
            if val is not None:
                check(L.srpc_plan_tune(self._h, knob, int(val)), "srpc_plan_tune")

    def wire_bytes(self, n: int) -> int:
        return n * self.record_bytes

    # -- hot path ----------------------------------------------------------
    def _cols(self, cols: Sequence) -> C.Array:
        if len(cols) != len(self.schema.kinds):
            raise ValueError(f"{self.schema.name}: expected {len(self.schema.kinds)} columns, "
                             f"got {len(cols)}")
        return (C.c_void_p * len(cols))(*[_dptr(c) for c in cols])

    def pack(self, cols: Sequence, n: int, wire, wire_cap: int | None = None, stream=None) -> int:
        """Pack n records from device columns into device wire bytes (async)."""
        arr = self._cols(cols)
        cap = self.wire_bytes(n) if wire_cap is None else wire_cap
        check(_lib.lib().srpc_gpu_pack(self._h, arr, n, _dptr(wire), cap, _stream(stream)),
              "srpc_gpu_pack")
        return self.wire_bytes(n)

    def unpack(self, wire, wire_len: int, n: int, cols: Sequence, status=None, stream=None) -> int:
        """Unpack n records from device wire bytes into device columns (async).
        ``status``: device pointer to a 16-byte srpc_unpack_status, or None.
        Returns SRPC_OK or SRPC_ERR_BOUNDS."""
        arr = self._cols(cols)
        return check(_lib.lib().srpc_gpu_unpack(self._h, _dptr(wire), wire_len, n, arr,
                                                _dptr(status), _stream(stream)),
                     "srpc_gpu_unpack")

    # -- host-terminated batches (ABI 7) ---------------------------------------
    def host_scratch_bytes(self, chunk_records: int, depth: int = 3) -> int:
        out = C.c_uint64()
        check(_lib.lib().srpc_plan_host_scratch_bytes(self._h, chunk_records, depth, C.byref(out)),
              "srpc_plan_host_scratch_bytes")
        return out.value

    def pack_host(self, h_cols: Sequence, n: int, h_wire, chunk_records: int, scratch, scratch_bytes: int,
                  depth: int = 3, wire_cap: int | None = None, stream=None) -> int:
        """Pack n records from HOST columns into HOST wire bytes, pipelined
        through `depth` device buffers of `chunk_records` (async on `stream`;
        host buffers: pinned tensors or addresses)."""
        arr = self._cols(h_cols)
        cap = self.wire_bytes(n) if wire_cap is None else wire_cap
        check(_lib.lib().srpc_gpu_pack_host(self._h, arr, n, _dptr(h_wire), cap, chunk_records, depth,
                                            _dptr(scratch), scratch_bytes, _stream(stream)), "srpc_gpu_pack_host")
        return self.wire_bytes(n)

    def unpack_host(self, h_wire, wire_len: int, n: int, h_cols: Sequence, chunk_records: int, scratch,
                    scratch_bytes: int, depth: int = 3, status=None, stream=None) -> int:
        """Unpack n records from HOST wire bytes into HOST columns (the mirror
        of pack_host).  Returns SRPC_OK or SRPC_ERR_BOUNDS."""
        arr = self._cols(h_cols)
        return check(_lib.lib().srpc_gpu_unpack_host(self._h, _dptr(h_wire), wire_len, n, arr, chunk_records, depth,
                                                     _dptr(scratch), scratch_bytes, _dptr(status), _stream(stream)),
                     "srpc_gpu_unpack_host")

    # -- records as structs (AoS) ---------------------------------------------
    def _offsets(self, field_offsets: Sequence[int]) -> C.Array:
        if len(field_offsets) != len(self.schema.kinds):
            raise ValueError(f"{self.schema.name}: expected {len(self.schema.kinds)} field offsets")
        return (C.c_uint32 * len(field_offsets))(*[int(o) for o in field_offsets])

    def pack_aos(self, records, record_stride: int, field_offsets: Sequence[int], n: int, wire,
                 wire_cap: int | None = None, stream=None) -> int:
        """Pack n records from a device array of structs (e.g. a numpy structured
        dtype's bytes): field f of record r at r * record_stride + field_offsets[f]."""
        cap = self.wire_bytes(n) if wire_cap is None else wire_cap
        check(_lib.lib().srpc_gpu_pack_aos(self._h, _dptr(records), record_stride, self._offsets(field_offsets), n,
                                           _dptr(wire), cap, _stream(stream)), "srpc_gpu_pack_aos")
        return self.wire_bytes(n)

    def unpack_aos(self, wire, wire_len: int, n: int, records, record_stride: int, field_offsets: Sequence[int],
                   status=None, stream=None) -> int:
        """Unpack n records into the leaf fields of a device array of structs
        (other bytes untouched).  Returns SRPC_OK or SRPC_ERR_BOUNDS."""
        return check(_lib.lib().srpc_gpu_unpack_aos(self._h, _dptr(wire), wire_len, n, _dptr(records), record_stride,
                                                    self._offsets(field_offsets), _dptr(status), _stream(stream)),
                     "srpc_gpu_unpack_aos")

    def unpack_aos_fill(self, wire, wire_len: int, n: int, records, record_stride: int,
                        field_offsets: Sequence[int], fill: bytes, status=None, stream=None) -> int:
        """As unpack_aos into fresh objects: every struct byte no leaf field
        covers is set from `fill` (record_stride bytes, e.g. a T{} image)."""
        if len(fill) != record_stride:
            raise ValueError("fill must be record_stride bytes")
        buf = C.create_string_buffer(bytes(fill), record_stride)
        return check(_lib.lib().srpc_gpu_unpack_aos_fill(self._h, _dptr(wire), wire_len, n, _dptr(records),
                                                         record_stride, self._offsets(field_offsets), buf,
                                                         _dptr(status), _stream(stream)),
                     "srpc_gpu_unpack_aos_fill")

    # -- string schemas (SRPC_PATH_VAR) -------------------------------------
    def var_scratch_bytes(self, n: int, wire_bytes: int) -> int:
        """Device scratch for pack_var (wire_bytes = wire_cap) / unpack_var (= wire_len)."""
        out = C.c_uint64()
        check(_lib.lib().srpc_plan_var_scratch_bytes(self._h, n, wire_bytes, C.byref(out)),
              "srpc_plan_var_scratch_bytes")
        return out.value

    def _str_offs(self, str_offs: Sequence) -> C.Array:
        ptrs = [_dptr(o) if (o is not None and k == STRING) else 0
                for o, k in zip(str_offs, self.schema.kinds)]
        return (C.c_void_p * len(ptrs))(*ptrs)

    def pack_var(self, cols: Sequence, str_offs: Sequence, n: int, wire, wire_cap: int, rec_offs,
                 scratch, scratch_bytes: int, status=None, stream=None) -> None:
        """Pack n records with string fields; writes rec_offs[0..n] (async).
        ``str_offs[f]``: n+1 u64 device offsets for string fields, None otherwise."""
        check(_lib.lib().srpc_gpu_pack_var(self._h, self._cols(cols), self._str_offs(str_offs), n,
                                           _dptr(wire), wire_cap, _dptr(rec_offs), _dptr(status),
                                           _dptr(scratch), scratch_bytes, _stream(stream)),
              "srpc_gpu_pack_var")

    def unpack_var(self, wire, wire_len: int, n: int, rec_offs, cols: Sequence, str_offs: Sequence,
                   scratch, scratch_bytes: int, status=None, stream=None) -> None:
        """Unpack n records whose starts are rec_offs[0..n] (async).  String
        field f's chars go to cols[f] (room for wire_len bytes), its n+1
        offsets to str_offs[f]."""
        check(_lib.lib().srpc_gpu_unpack_var(self._h, _dptr(wire), wire_len, n, _dptr(rec_offs),
                                             self._cols(cols), self._str_offs(str_offs),
                                             _dptr(status), _dptr(scratch), scratch_bytes,
                                             _stream(stream)),
              "srpc_gpu_unpack_var")

    def var_tile_table_words(self, n: int) -> int:
        """u64 words of a batch's tile table (srpc_gpu_var_tile_table)."""
        out = C.c_uint64()
        check(_lib.lib().srpc_var_tile_table_words(self._h, n, C.byref(out)), "srpc_var_tile_table_words")
        return out.value

    def var_tile_table(self, str_offs: Sequence, n: int, table, stream=None) -> None:
        """The tile table of n records from their string offsets (async)."""
        check(_lib.lib().srpc_gpu_var_tile_table(self._h, self._str_offs(str_offs), n, _dptr(table), _stream(stream)),
              "srpc_gpu_var_tile_table")

    def unpack_var_tiled(self, wire, wire_len: int, n: int, rec_offs, table, cols: Sequence, str_offs: Sequence,
                         scratch, scratch_bytes: int, status=None, stream=None) -> None:
        """unpack_var with the batch's tile table (output bases without the look-back)."""
        check(_lib.lib().srpc_gpu_unpack_var_tiled(self._h, _dptr(wire), wire_len, n, _dptr(rec_offs), _dptr(table),
                                                   self._cols(cols), self._str_offs(str_offs), _dptr(status),
                                                   _dptr(scratch), scratch_bytes, _stream(stream)),
              "srpc_gpu_unpack_var_tiled")

    def var_stream_scratch_bytes(self, n: int, wire_len: int) -> int:
        """Device scratch for unpack_var_stream (256-byte aligned)."""
        out = C.c_uint64()
        check(_lib.lib().srpc_plan_var_stream_scratch_bytes(self._h, n, wire_len, C.byref(out)),
              "srpc_plan_var_stream_scratch_bytes")
        return out.value

    def unpack_var_stream(self, wire, wire_len: int, n: int, rec_offs, cols: Sequence, str_offs: Sequence,
                          scratch, scratch_bytes: int, status=None, stream=None) -> None:
        """Unpack n records from a concatenated stream with no index (the
        reference's shared-cursor decode); writes rec_offs[0..n] (async)."""
        check(_lib.lib().srpc_gpu_unpack_var_stream(self._h, _dptr(wire), wire_len, n, _dptr(rec_offs),
                                                    self._cols(cols), self._str_offs(str_offs),
                                                    _dptr(status), _dptr(scratch), scratch_bytes,
                                                    _stream(stream)),
              "srpc_gpu_unpack_var_stream")

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().srpc_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fill_splitmix_i32(cols: Iterable, n: int, seed: int, first_record: int = 0, stream=None) -> None:
    """Synthetic int32 columns on the device (SURVEY.md §8c splitmix64 stream)."""
    ptrs = [_dptr(c) for c in cols]
    arr = (C.c_void_p * len(ptrs))(*ptrs)
    check(_lib.lib().srpc_gpu_fill_splitmix_i32(arr, len(ptrs), n, seed, first_record,
                                                _stream(stream)), "srpc_gpu_fill_splitmix_i32")


def time_next_call(start=None, stop=None) -> None:
    """Arm srpc_time_next_call: the kernels of the next pack/unpack call made
    on this thread stamp their dispatch begin (first kernel) and end (last
    kernel) into ``start`` / ``stop``.  Each is a torch.cuda.Event created
    with enable_timing=True and recorded at least once (torch creates the HIP
    event lazily, on first record), or a raw hipEvent_t handle."""
    def handle(e):
        if e is None:
            return None
        if hasattr(e, "cuda_event"):
            if not e.cuda_event:
                raise ValueError("time_next_call: record the event once first (torch creates it lazily)")
            return e.cuda_event
        return int(e)

    check(_lib.lib().srpc_time_next_call(handle(start), handle(stop)), "srpc_time_next_call")


def framed_request_prefix(schema: Schema, method: str) -> bytes:
    """``BE32 payload | str(method) | str(T::name)``: the constant head of every
    frame Calculator_stub-style clients send for a fixed-size request
    (transport.hpp send_data + packer.hpp:77-82)."""
    pre = request_prefix(method, schema.name)
    return struct.pack(">I", len(pre) + schema.body_bytes) + pre


def framed_response_prefix(schema: Schema, code: int = RPC_SUCCESS) -> bytes:
    pre = response_prefix(code, schema.name)
    return struct.pack(">I", len(pre) + schema.body_bytes) + pre


class FrameClassifier:
    """Buckets a batch of socket frames by method on the device
    (srpc_frames_classify / _gather / _scatter): ``methods`` is a list of
    (request GpuPacker with a framed prefix, response record bytes)."""

    def __init__(self, methods: Sequence[tuple["GpuPacker", int]]):
        self.methods = list(methods)
        k = len(self.methods)
        self._plans = (C.c_void_p * k)(*[m[0]._h.value for m in self.methods])
        self._rb = (C.c_uint32 * k)(*[int(m[1]) for m in self.methods])

    def scratch_bytes(self, nframes: int) -> int:
        out = C.c_uint64()
        check(_lib.lib().srpc_frames_scratch_bytes(nframes, len(self.methods), C.byref(out)),
              "srpc_frames_scratch_bytes")
        return out.value

    def classify(self, buf, buf_len: int, offs, nframes: int, cls, index, counts, out_off, scratch,
                 scratch_bytes: int, stream=None) -> None:
        check(_lib.lib().srpc_frames_classify(self._plans, self._rb, len(self.methods), _dptr(buf), buf_len,
                                              _dptr(offs), nframes, _dptr(cls), _dptr(index), _dptr(counts),
                                              _dptr(out_off), _dptr(scratch), scratch_bytes, _stream(stream)),
              "srpc_frames_classify")

    @staticmethod
    def gather(buf, offs, index, n: int, record_bytes: int, out, stream=None) -> None:
        check(_lib.lib().srpc_frames_gather(_dptr(buf), _dptr(offs), _dptr(index), n, record_bytes, _dptr(out),
                                            _stream(stream)), "srpc_frames_gather")

    @staticmethod
    def scatter(resp, index, n: int, record_bytes: int, out_off, out, stream=None) -> None:
        check(_lib.lib().srpc_frames_scatter(_dptr(resp), _dptr(index), n, record_bytes, _dptr(out_off),
                                             _dptr(out), _stream(stream)), "srpc_frames_scatter")

    # string plans (request GpuPackers built with request_prefix, no BE32):
    @staticmethod
    def gather_var(buf, offs, index, n: int, out, rec_offs, scratch, scratch_bytes: int, stream=None) -> None:
        check(_lib.lib().srpc_frames_gather_var(_dptr(buf), _dptr(offs), _dptr(index), n, _dptr(out), _dptr(rec_offs),
                                                _dptr(scratch), scratch_bytes, _stream(stream)),
              "srpc_frames_gather_var")

    @staticmethod
    def scatter_var(resp, rec_offs, index, n: int, out_off, out, stream=None) -> None:
        check(_lib.lib().srpc_frames_scatter_var(_dptr(resp), _dptr(rec_offs), _dptr(index), n, _dptr(out_off),
                                                 _dptr(out), _stream(stream)), "srpc_frames_scatter_var")

    def offsets(self, cls, nframes: int, index, counts, var_rec_offs, out_off, total, scratch, scratch_bytes: int,
                stream=None) -> None:
        """var_rec_offs: per method, the response index of a string method's
        bucket (device buffer) or None for a fixed one."""
        k = len(self.methods)
        vr = (C.c_void_p * k)(*[_dptr(v) if v is not None else None for v in var_rec_offs])
        check(_lib.lib().srpc_frames_offsets(self._plans, self._rb, k, _dptr(cls), nframes, _dptr(index), _dptr(counts),
                                             vr, _dptr(out_off), _dptr(total), _dptr(scratch), scratch_bytes,
                                             _stream(stream)), "srpc_frames_offsets")


__all__ = ["Schema", "GpuPacker", "SrpcError", "request_prefix", "response_prefix",
           "fill_splitmix_i32", "time_next_call", "framed_request_prefix", "framed_response_prefix",
           "FrameClassifier", "BOOL", "INT8", "CHAR", "INT16", "INT32", "INT64", "STRING",
           "RPC_SUCCESS", "RPC_ERR_FUNCTION_NOT_REGISTERED", "RPC_ERR_RECV_TIMEOUT"]
