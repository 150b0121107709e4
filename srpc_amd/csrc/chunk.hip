// chunk.hip -- fixed-size schemas of any stride: register-assembled wire chunks
// (the TILE path's CHUNK kernel, SRPC_TUNE_TILE_KERNEL = 1).
//
// Wire bytes of a fixed schema are periodic: with stride S, the 16-byte
// chunks of one period of L = lcm(S, 16) bytes (P = L/16 chunks, rpp = L/S
// records) repeat with the records' values substituted.  The plan holds, per
// phase ph of the period, the chunk's constant bytes (prefix template, zeros
// elsewhere), the prefix byte mask, and the list of field occurrences
// (record q of the period, field f, byte position pos of the field's first
// byte relative to the chunk, in [-7, 15]).  A workgroup takes a tile of R
// records (R a multiple of 16, so the tile's wire span and every column
// slice are 16-byte aligned):
//
// PACK   1. each field's column slice -> an LDS slab, aligned 16-byte loads
//           and stores (8 loads in flight per lane);
//        2. lane per wire chunk: template | each occurrence's value (aligned
//           LDS read) shifted into place; one aligned 16-byte store.
// UNPACK 1. lane per wire chunk: one aligned 16-byte load, prefix bytes
//           compared under the mask, each occurrence's bytes shifted out into
//           its slab element (an aligned LDS store; the bytes of an element
//           that straddles two chunks are written by both lanes, byte-wise);
//        2. slabs -> columns, aligned 16-byte stores.
// So every global access is an aligned, coalesced 16-byte access and every
// LDS access is naturally aligned -- the TILE image kernels' stride-S
// scatter/gather in LDS is unaligned (a replayed access per element,
// cdna_hip_programming.md Guideline 17).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "plan.h"
#include "srpc_gpu.h"

namespace srpc_impl {

namespace {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
constexpr int kChunkLoadBatch = 8;    // pack: column slice loads in flight per lane
constexpr int kUnpackLoadBatch = 4;  // unpack: wire chunks in flight per lane (register budget)
#ifndef SRPC_PACK_CHUNKS
#define SRPC_PACK_CHUNKS 4
#endif
constexpr int kPackChunks = SRPC_PACK_CHUNKS;  // pack: chunks assembled per lane at a time

// Occurrence entry (plan.h, chunk_entry): q | lg << 8 | (pos + 8) << 10 | slab offset << 15;
// 0 = padding (every phase has exactly a.emax entries).
__device__ __forceinline__ uint32_t e_q(uint32_t e) { return e & 0xff; }
__device__ __forceinline__ uint32_t e_lg(uint32_t e) { return (e >> 8) & 3; }
__device__ __forceinline__ int e_pos(uint32_t e) { return static_cast<int>((e >> 10) & 31) - 8; }
__device__ __forceinline__ uint32_t e_slab(uint32_t e) { return e >> 15; }

__device__ __forceinline__ uint64_t size_mask(uint32_t lg) {
    return lg == 3 ? ~0ull : (1ull << (8u << lg)) - 1;
}

// The element at LDS byte address p (naturally aligned, 1 << lg bytes): one
// aligned 8-byte read, shifted and masked (no branch on the size).
__device__ __forceinline__ uint64_t lds_element(const uint8_t* base, uint32_t off, uint32_t lg) {
    const uint64_t w = *reinterpret_cast<const uint64_t*>(base + (off & ~7u));
    return (w >> (8 * (off & 7))) & size_mask(lg);
}

// v placed at byte pos (-7..15) of a 16-byte chunk (lo, hi), with selects.
__device__ __forceinline__ void place(uint64_t v, int pos, uint64_t& lo, uint64_t& hi) {
    const int s = 8 * pos;  // -56 .. 120
    const uint64_t l = s < 0 ? v >> ((-s) & 63) : (s < 64 ? v << (s & 63) : 0);
    const uint64_t h = s >= 64 ? v << ((s - 64) & 63) : (s > 0 ? v >> ((64 - s) & 63) : 0);
    lo |= l;
    hi |= h;
}

// 8 bytes from byte pos (0..15) of the 24 bytes (lo, hi, nx).
__device__ __forceinline__ uint64_t extract(uint64_t lo, uint64_t hi, uint64_t nx, int pos) {
    const int s = 8 * pos;  // 0 .. 120
    const uint64_t a = s < 64 ? lo : hi, b = s < 64 ? hi : nx;
    const int t = s & 63;
    return t ? (a >> t) | (b << (64 - t)) : a;
}

// LDS: slabs [R * field_bytes] | tmpl [P][16] | pmask [P][16] | ent [P][emax] u32
struct ChunkLds {
    uint8_t* slab;
    const uint8_t* tmpl;
    const uint8_t* pmask;
    const uint32_t* ent;
};

// (Fields are passed by value: taking the address of the by-value kernel
// argument block would copy it to scratch.)
__device__ __forceinline__ ChunkLds chunk_lds(const uint8_t* table, uint32_t table_bytes, uint32_t slab_bytes,
                                              uint32_t P, uint8_t* lds) {
    ChunkLds L;
    L.slab = lds;
    uint8_t* t = lds + slab_bytes;  // slab_bytes is a multiple of 16
    const uint32_t nq = table_bytes / 16;
    for (uint32_t i = threadIdx.x; i < nq; i += kBlock)
        reinterpret_cast<u64x2*>(t)[i] = reinterpret_cast<const u64x2*>(table)[i];
    L.tmpl = t;
    L.pmask = t + 16 * P;
    L.ent = reinterpret_cast<const uint32_t*>(t + 32 * P);
    return L;
}

}  // namespace

__global__ __launch_bounds__(kBlock) void k_pack_chunk(ChunkArgs a, uint8_t* __restrict__ wire, uint64_t n,
                                                       uint64_t ntiles) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const ChunkLds L = chunk_lds(a.table, a.table_bytes, a.slab_bytes, a.P, lds);
    const uint32_t cstep_ph = kBlock % a.P, cstep_per = kBlock / a.P;
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t rbase = tile * a.R;
        const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
        __syncthreads();  // the table is in LDS; the previous tile's slabs are consumed
        // 1. column slices -> slabs (aligned 16-byte blocks; a block holding one
        //    valid byte of a column never crosses a page)
        for (uint32_t f = 0; f < a.nfields; ++f) {
            const uint32_t sz = 1u << a.lg[f];
            const u64x2* src = reinterpret_cast<const u64x2*>(a.col[f] + rbase * sz);
            u64x2* dst = reinterpret_cast<u64x2*>(L.slab + a.slab_off[f]);
            const uint32_t nb = (nr * sz + 15) / 16;
            for (uint32_t c0 = threadIdx.x; c0 < nb; c0 += kBlock * kChunkLoadBatch) {
                u64x2 v[kChunkLoadBatch];
#pragma unroll
                for (int u = 0; u < kChunkLoadBatch; ++u) {
                    const uint32_t c = c0 + u * kBlock;
                    if (c < nb) v[u] = __builtin_nontemporal_load(src + c);
                }
#pragma unroll
                for (int u = 0; u < kChunkLoadBatch; ++u) {
                    const uint32_t c = c0 + u * kBlock;
                    if (c < nb) dst[c] = v[u];
                }
            }
        }
        __syncthreads();
        // 2. lane per wire chunk
        const uint32_t tbytes = nr * a.stride;
        const uint32_t nch = (tbytes + 15) / 16;
        uint8_t* out = wire + rbase * a.stride;  // 16-byte aligned: R * stride is
        uint32_t ph = threadIdx.x % a.P, per = threadIdx.x / a.P;
        // kPackChunks chunks per lane at a time: their LDS chains (template,
        // entry, element) are independent and overlap
        for (uint32_t c0 = threadIdx.x; c0 < nch; c0 += kBlock * kPackChunks) {
            uint64_t lo[kPackChunks], hi[kPackChunks];
#pragma unroll
            for (int u = 0; u < kPackChunks; ++u) {
                const u64x2 t = *reinterpret_cast<const u64x2*>(L.tmpl + 16 * ph);
                lo[u] = t.x;
                hi[u] = t.y;
                const uint32_t q0 = per * a.rpp;
                for (uint32_t j = 0; j < a.emax; ++j) {  // uniform trip count
                    const uint32_t en = L.ent[ph * a.emax + j];
                    const uint32_t k = q0 + e_q(en), lg = e_lg(en);
                    uint64_t v = lds_element(L.slab, e_slab(en) + (k << lg), lg);
                    v = (en && k < nr) ? v : 0;
                    place(v, e_pos(en), lo[u], hi[u]);
                }
                ph += cstep_ph;
                per += cstep_per;
                if (ph >= a.P) {
                    ph -= a.P;
                    ++per;
                }
            }
#pragma unroll
            for (int u = 0; u < kPackChunks; ++u) {
                const uint32_t c = c0 + u * kBlock;
                if (16 * c + 16 <= tbytes) {
                    __builtin_nontemporal_store(u64x2{lo[u], hi[u]}, reinterpret_cast<u64x2*>(out + 16 * c));
                } else if (16 * c < tbytes) {
                    for (uint32_t i = 0; 16 * c + i < tbytes; ++i)
                        out[16 * c + i] = static_cast<uint8_t>(i < 8 ? lo[u] >> (8 * i) : hi[u] >> (8 * (i - 8)));
                }
            }
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_unpack_chunk(ChunkArgs a, const uint8_t* __restrict__ wire, uint64_t n,
                                                         uint64_t ntiles, srpc_unpack_status* st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const ChunkLds L = chunk_lds(a.table, a.table_bytes, a.slab_bytes, a.P, lds);
    const uint32_t cstep_ph = kBlock % a.P, cstep_per = kBlock / a.P;
    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t rbase = tile * a.R;
        const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
        __syncthreads();  // the table is in LDS; the previous tile's slabs are stored
        // 1. lane per wire chunk: prefix check, fields into the slabs
        const uint32_t tbytes = nr * a.stride;
        const uint32_t nch = (tbytes + 15) / 16;
        const u64x2* src = reinterpret_cast<const u64x2*>(wire + rbase * a.stride);
        uint32_t ph = threadIdx.x % a.P, per = threadIdx.x / a.P;
        for (uint32_t c0 = threadIdx.x; c0 < nch; c0 += kBlock * kUnpackLoadBatch) {
            u64x2 v[kUnpackLoadBatch];
#pragma unroll
            for (int u = 0; u < kUnpackLoadBatch; ++u) {
                const uint32_t c = c0 + u * kBlock;
                if (c < nch) v[u] = __builtin_nontemporal_load(src + c);  // aligned: never crosses a page
            }
#pragma unroll
            for (int u = 0; u < kUnpackLoadBatch; ++u) {
                const uint32_t c = c0 + u * kBlock;
                if (c < nch) {
                    const uint64_t lo = v[u].x, hi = v[u].y;
                    if (a.prefix_len && st) {
                        const u64x2 t = *reinterpret_cast<const u64x2*>(L.tmpl + 16 * ph);
                        const u64x2 m = *reinterpret_cast<const u64x2*>(L.pmask + 16 * ph);
                        uint64_t dlo = (lo ^ t.x) & m.x, dhi = (hi ^ t.y) & m.y;
                        const uint32_t valid = tbytes - 16 * c;  // bytes of this chunk inside the tile
                        if (valid < 16) {
                            if (valid <= 8) {
                                dlo &= valid == 8 ? ~0ull : (1ull << (8 * valid)) - 1;
                                dhi = 0;
                            } else {
                                dhi &= (1ull << (8 * (valid - 8))) - 1;
                            }
                        }
                        if (dlo | dhi) {
                            const uint32_t b = dlo ? __builtin_ctzll(dlo) >> 3 : 8 + (__builtin_ctzll(dhi) >> 3);
                            report_bad(st, SRPC_STATUS_PREFIX, rbase + (16 * c + b) / a.stride);
                        }
                    }
                    // the next chunk's first 8 bytes: from the next lane, or (lane 63) a load
                    uint64_t nx = __shfl_down(lo, 1, 64);
                    if ((threadIdx.x & 63) == 63 && c + 1 < nch) nx = reinterpret_cast<const uint64_t*>(src + c + 1)[0];
                    const uint32_t q0 = per * a.rpp;
                    for (uint32_t j = 0; j < a.emax; ++j) {  // uniform trip count
                        const uint32_t en = L.ent[ph * a.emax + j];
                        const uint32_t k = q0 + e_q(en), lg = e_lg(en);
                        const int pos = e_pos(en);
                        // the element whose first byte is in this chunk is written whole by this lane
                        if (!en || k >= nr || pos < 0) continue;
                        const uint64_t x = extract(lo, hi, nx, pos);
                        uint8_t* dst = L.slab + e_slab(en) + (k << lg);
                        switch (lg) {
                        case 0: *dst = static_cast<uint8_t>(x); break;
                        case 1: *reinterpret_cast<uint16_t*>(dst) = static_cast<uint16_t>(x); break;
                        case 2: *reinterpret_cast<uint32_t*>(dst) = static_cast<uint32_t>(x); break;
                        default: *reinterpret_cast<uint64_t*>(dst) = x; break;
                        }
                    }
                }
                ph += cstep_ph;
                per += cstep_per;
                if (ph >= a.P) {
                    ph -= a.P;
                    ++per;
                }
            }
        }
        __syncthreads();
        // 2. slabs -> columns
        for (uint32_t f = 0; f < a.nfields; ++f) {
            const uint32_t sz = 1u << a.lg[f];
            const uint32_t nbytes = nr * sz;
            uint8_t* dstc = const_cast<uint8_t*>(a.col[f]) + rbase * sz;
            const uint8_t* slab = L.slab + a.slab_off[f];
            for (uint32_t c = threadIdx.x; 16 * c < nbytes; c += kBlock) {
                if (16 * c + 16 <= nbytes) {
                    __builtin_nontemporal_store(*reinterpret_cast<const u64x2*>(slab + 16 * c),
                                                reinterpret_cast<u64x2*>(dstc + 16 * c));
                } else {  // the column's last, partial block
                    for (uint32_t i = 16 * c; i < nbytes; ++i) dstc[i] = slab[i];
                }
            }
        }
    }
}

}  // namespace srpc_impl
