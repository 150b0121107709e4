// sdec.h -- internal: the speculative single-pass decode of a concatenated
// record stream (sdec.hip), the first path of srpc_gpu_unpack_var_stream
// (stream.hip).  Not part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "plan.h"

namespace srpc_impl {

// Schemas it decodes (1..4 string fields, records of >= 8 bytes).
bool sdec_supports(const srpc_plan* p);
// Device scratch of one call (256-byte aligned).
uint64_t sdec_scratch_bytes(const srpc_plan* p, uint64_t wire_len);
// Stream-ordered launches: decodes the whole stream (rec_offs, columns,
// str_offs, *st) in one pass over the wire, or nothing while the device word
// *gate is 0 (gate NULL: always).  *abort_out is set to the address of a
// device word that is nonzero when the decode gave up (the stream needs the
// bounded decode of stream1.hip, which the caller gates on it; 0 when the
// gate kept this decode from running).  miss_limit: blocks entered where no
// chain of theirs starts before it gives up (0: the default share of the
// blocks, ~0u: never).
int sdec_launch(const srpc_plan* p, const uint8_t* wire, uint64_t wire_len, uint64_t n, uint64_t* rec_offs,
                void* const* cols, uint64_t* const* str_offs, srpc_unpack_status* st, void* scratch,
                uint32_t miss_limit, const uint32_t* gate, const uint32_t** abort_out, hipStream_t s);

}  // namespace srpc_impl
