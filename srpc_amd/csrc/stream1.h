// stream1.h -- internal: the single-pass decode of a concatenated record
// stream (stream1.hip), the bounded path of srpc_gpu_unpack_var_stream
// (stream.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "plan.h"

namespace srpc_impl {

// Schemas whose chars the single pass carries itself (at most 4 string
// fields); others get the record index only (rec_offs) and an indexed decode.
bool stream1_decodes(const srpc_plan* p);
// Device scratch of one call (256-byte aligned).
uint64_t stream1_scratch_bytes(const srpc_plan* p, uint64_t wire_len);
// Stream-ordered launches; every kernel returns at once while `gate` (device
// word, may be NULL = always) is 0.  Writes rec_offs, and for schemas it
// decodes the columns, str_offs and *st; SRPC_E_UNSUPPORTED for wires of 1 TiB
// or more.
int stream1_launch(const srpc_plan* p, const uint8_t* wire, uint64_t wire_len, uint64_t n, uint64_t* rec_offs,
                   void* const* cols, uint64_t* const* str_offs, srpc_unpack_status* st, void* scratch,
                   const uint32_t* gate, hipStream_t s);
// ORs the single pass's diagnostics into st->reserved (gated likewise).
int stream1_note(const srpc_plan* p, uint64_t wire_len, void* scratch, srpc_unpack_status* st, const uint32_t* gate,
                 hipStream_t s);

}  // namespace srpc_impl
