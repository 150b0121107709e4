"""srpc_amd -- MI355X-native batched packer for the sRPC wire format.

The compute path is the HIP library ``srpc_amd/libsrpc_gpu.so`` (C ABI in
``include/srpc_gpu.h``); this package is the thin host-side binding used by the
tests and ``bench.py``.  C++ callers use ``include/srpc/gpu.hpp`` instead.
"""
from .packer import (BOOL, CHAR, INT8, INT16, INT32, INT64, RPC_ERR_FUNCTION_NOT_REGISTERED,
                     RPC_ERR_RECV_TIMEOUT, RPC_SUCCESS, STRING, GpuPacker, Schema, SrpcError,
                     fill_splitmix_i32, request_prefix, response_prefix, time_next_call,
                     FrameClassifier, framed_request_prefix, framed_response_prefix)
from ._lib import (SRPC_ERR_BOUNDS, SRPC_PATH_DWORD, SRPC_PATH_TILE, SRPC_PATH_VAR, SRPC_STATUS_BOUNDS,
                   SRPC_STATUS_PREFIX, UnpackStatus)

# Schemas used by the reference's example and by the benchmark.
NUMBER = Schema.of("Number", ("num", "int32"))                       # examples/calculator.contract:1-3
TWO_NUMBERS = Schema.of("TwoNumbers", ("left", "int32"), ("right", "int32"))  # :5-8
QUAD = Schema.of("Quad", ("a", "int32"), ("b", "int32"), ("c", "int32"), ("d", "int32"))
SQUARE_METHOD = "Calculator_servicer::square"  # generator.hpp:84 naming, calculator_srpc.cpp:123

__all__ = ["GpuPacker", "Schema", "SrpcError", "fill_splitmix_i32", "time_next_call", "request_prefix",
           "response_prefix", "NUMBER", "TWO_NUMBERS", "QUAD", "SQUARE_METHOD", "BOOL", "INT8",
           "CHAR", "INT16", "INT32", "INT64", "STRING", "RPC_SUCCESS",
           "RPC_ERR_FUNCTION_NOT_REGISTERED", "RPC_ERR_RECV_TIMEOUT", "SRPC_ERR_BOUNDS",
           "SRPC_PATH_DWORD", "SRPC_PATH_TILE", "SRPC_PATH_VAR", "SRPC_STATUS_BOUNDS", "SRPC_STATUS_PREFIX",
           "UnpackStatus", "FrameClassifier", "framed_request_prefix", "framed_response_prefix"]
