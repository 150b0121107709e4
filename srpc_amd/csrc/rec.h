// rec.h -- schema-specialised TILE kernels (rec.hip), internal API.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "srpc_gpu.h"

struct srpc_plan;

namespace srpc_impl {

// The instance for the plan's layout (prefix length and field sizes), or -1.
int rec_kernel_for(const srpc_plan* p);
// Whether instance `id`'s pack / unpack kernel beat the generic TILE kernels
// (tools/bench_paths.py --rec-ab, profiles/r03_paths_rec_ab.log).
bool rec_default(int id, bool pack);
// Records per tile of instance `id`'s pack / unpack kernel (they cover whole
// tiles only).
uint64_t rec_tile_records(int id, bool pack);
// The first tiles * rec_tile_records(id) records; columns 16-byte aligned.
int rec_pack(int id, const srpc_plan* p, const void* const* cols, uint64_t tiles, uint8_t* wire, hipStream_t s);
int rec_unpack(int id, const srpc_plan* p, const uint8_t* wire, uint64_t tiles, void* const* cols,
               srpc_unpack_status* st, hipStream_t s);

}  // namespace srpc_impl
