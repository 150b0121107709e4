// srpc_gpu.hip -- MI355X (gfx950) batched record packer for sRPC wire format.
//
// Implements include/srpc_gpu.h.  Two kernel families for fixed-size schemas:
//
//  DWORD path  (every field 4 or 8 bytes, no envelope prefix, record <= 32 B)
//      One record per lane.  Each record dword is read straight from its field
//      column (lanes of a wave read consecutive elements: 256 B coalesced per
//      wave instruction), assembled in VGPRs and stored as the widest aligned
//      vector (dwordx4 for 16-byte records: a wave writes 1 KiB contiguous).
//      Unpack is the transpose back.  Pure HBM streaming; no LDS, no MFMA.
//
//  TILE path   (any fixed-size schema: 1/2/8-byte fields, odd record strides
//               such as the 53-byte Calculator.square request)
//      A workgroup owns a tile of R records (R*stride bytes, a multiple of 16).
//      Pack: 16-byte column loads -> scatter of each element into an LDS image
//      of the tile's wire bytes -> 16-byte aligned stores of the image, with
//      the constant envelope prefix merged from a periodic template.  Unpack:
//      16-byte wire loads (prefix checked against the template/mask) -> LDS
//      image -> gather of each column's elements -> 16-byte column stores.
//
// Wire format (reference include/srpc/packer.hpp): fields are raw LE bytes in
// declaration order with no padding (pack_arg 183-191, pack_struct 172-178);
// request/response envelopes are a constant header for a batch of one message
// type and one method (pack_request 77-82, pack_response 86-91).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "plan.h"
#include "rec.h"
#include "srpc_gpu.h"

namespace {
using namespace srpc_impl;


// ---------------------------------------------------------------------------
// Kernel argument blocks (all wave-uniform: they live in SGPRs / kernarg).
// ---------------------------------------------------------------------------
struct DwordMap {
    // Record dword k = dword (r << lg[k]) of src[k]: src[k] already points at
    // the right half of an 8-byte field, lg[k] is 0 for 4-byte fields and 1
    // for 8-byte ones.
    const uint32_t* src[kMaxDwords];
    uint32_t lg[kMaxDwords];
};



struct TileArgs {
    const uint8_t* col[kMaxFields];  // field column base (pack: src, unpack: dst)
    uint32_t size[kMaxFields];       // field bytes: 1, 2, 4 or 8
    uint32_t lgsize[kMaxFields];     // log2(size)
    uint32_t off[kMaxFields];        // field byte offset inside the record (prefix included)
    const uint8_t* period;           // device template | mask of one period (2L bytes; prefix_len > 0)
    uint32_t nfields;
    uint32_t stride;                 // record bytes
    uint32_t prefix_len;
    uint32_t R;                      // records per tile (multiple of 16)
    uint32_t L;                      // template period lcm(stride, 16), divides R*stride
    uint64_t base;                   // unpack: index of the wire's first record (status reports)
};


// ---------------------------------------------------------------------------
// DWORD path
// ---------------------------------------------------------------------------
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));


template <int NT, typename T>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (NT & kNtLoad) return __builtin_nontemporal_load(p);
    else return *p;
}

template <int NT, typename T>
__device__ __forceinline__ void st(T* p, T v) {
    if constexpr (NT & kNtStore) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// W dwords of one record to/from its (4W-byte aligned) wire slot, using the
// widest vector the record alignment allows.
template <int W, int NT>
__device__ __forceinline__ void store_record(uint8_t* p, const uint32_t (&v)[W]) {
    if constexpr (W % 4 == 0) {
#pragma unroll
        for (int k = 0; k < W; k += 4)
            st<NT>(reinterpret_cast<u32x4*>(p + 4 * k), u32x4{v[k], v[k + 1], v[k + 2], v[k + 3]});
    } else if constexpr (W % 2 == 0) {
#pragma unroll
        for (int k = 0; k < W; k += 2) st<NT>(reinterpret_cast<u32x2*>(p + 4 * k), u32x2{v[k], v[k + 1]});
    } else {
#pragma unroll
        for (int k = 0; k < W; ++k) st<NT>(reinterpret_cast<uint32_t*>(p) + k, v[k]);
    }
}

template <int W, int NT>
__device__ __forceinline__ void load_record(const uint8_t* p, uint32_t (&v)[W]) {
    if constexpr (W % 4 == 0) {
#pragma unroll
        for (int k = 0; k < W; k += 4) {
            const u32x4 q = ld<NT>(reinterpret_cast<const u32x4*>(p + 4 * k));
            v[k] = q.x; v[k + 1] = q.y; v[k + 2] = q.z; v[k + 3] = q.w;
        }
    } else if constexpr (W % 2 == 0) {
#pragma unroll
        for (int k = 0; k < W; k += 2) {
            const u32x2 q = ld<NT>(reinterpret_cast<const u32x2*>(p + 4 * k));
            v[k] = q.x; v[k + 1] = q.y;
        }
    } else {
#pragma unroll
        for (int k = 0; k < W; ++k) v[k] = ld<NT>(reinterpret_cast<const uint32_t*>(p) + k);
    }
}

// One record per lane.  ITER records per lane, spaced one workgroup-width
// apart, so every wave instruction touches consecutive elements (256 B per
// column load, 64*4W B per record store) while each lane keeps ITER*W
// independent loads in flight.
template <int W, int ITER, int NT>
__global__ __launch_bounds__(kBlock) void k_pack_dword(DwordMap m, uint8_t* __restrict__ wire,
                                                       uint64_t n) {
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * (kBlock * ITER);
    for (uint64_t r0 = static_cast<uint64_t>(blockIdx.x) * (kBlock * ITER) + threadIdx.x; r0 < n; r0 += step) {
        uint32_t v[ITER][W];
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const uint64_t r = r0 + static_cast<uint64_t>(it) * kBlock;
            if (r < n) {
#pragma unroll
                for (int k = 0; k < W; ++k) v[it][k] = ld<NT>(m.src[k] + (r << m.lg[k]));
            }
        }
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const uint64_t r = r0 + static_cast<uint64_t>(it) * kBlock;
            if (r < n) store_record<W, NT>(wire + r * (4 * W), v[it]);
        }
    }
}

template <int W, int ITER, int NT>
__global__ __launch_bounds__(kBlock) void k_unpack_dword(DwordMap m, const uint8_t* __restrict__ wire,
                                                         uint64_t n) {
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * (kBlock * ITER);
    for (uint64_t r0 = static_cast<uint64_t>(blockIdx.x) * (kBlock * ITER) + threadIdx.x; r0 < n; r0 += step) {
        uint32_t v[ITER][W];
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const uint64_t r = r0 + static_cast<uint64_t>(it) * kBlock;
            if (r < n) load_record<W, NT>(wire + r * (4 * W), v[it]);
        }
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const uint64_t r = r0 + static_cast<uint64_t>(it) * kBlock;
            if (r < n) {
#pragma unroll
                for (int k = 0; k < W; ++k) st<NT>(const_cast<uint32_t*>(m.src[k]) + (r << m.lg[k]), v[it][k]);
            }
        }
    }
}

// Four consecutive records per lane (all fields 4 bytes, 16-byte aligned
// columns): one 16-byte load per column, a register transpose, and W 16-byte
// stores of the lane's 4 contiguous records.  Records past n are handled by
// the one-record-per-lane kernel of the same variant (the host splits n).
template <int W, int ITER, int NT>
__global__ __launch_bounds__(kBlock) void k_pack_dword_x4(DwordMap m, uint8_t* __restrict__ wire,
                                                          uint64_t nq) {
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * (kBlock * ITER);
    for (uint64_t q0 = static_cast<uint64_t>(blockIdx.x) * (kBlock * ITER) + threadIdx.x; q0 < nq; q0 += step) {
        u32x4 c[ITER][W];
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const uint64_t q = q0 + static_cast<uint64_t>(it) * kBlock;
            if (q < nq) {
#pragma unroll
                for (int k = 0; k < W; ++k) c[it][k] = ld<NT>(reinterpret_cast<const u32x4*>(m.src[k]) + q);
            }
        }
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const uint64_t q = q0 + static_cast<uint64_t>(it) * kBlock;
            if (q < nq) {
                uint32_t o[4 * W];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int k = 0; k < W; ++k) o[i * W + k] = c[it][k][i];
                u32x4* dst = reinterpret_cast<u32x4*>(wire + q * (16 * W));
#pragma unroll
                for (int j = 0; j < W; ++j)
                    st<NT>(dst + j, u32x4{o[4 * j], o[4 * j + 1], o[4 * j + 2], o[4 * j + 3]});
            }
        }
    }
}

template <int W, int ITER, int NT>
__global__ __launch_bounds__(kBlock) void k_unpack_dword_x4(DwordMap m, const uint8_t* __restrict__ wire,
                                                            uint64_t nq) {
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * (kBlock * ITER);
    for (uint64_t q0 = static_cast<uint64_t>(blockIdx.x) * (kBlock * ITER) + threadIdx.x; q0 < nq; q0 += step) {
        u32x4 c[ITER][W];
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const uint64_t q = q0 + static_cast<uint64_t>(it) * kBlock;
            if (q < nq) {
                const u32x4* src = reinterpret_cast<const u32x4*>(wire + q * (16 * W));
#pragma unroll
                for (int j = 0; j < W; ++j) c[it][j] = ld<NT>(src + j);
            }
        }
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const uint64_t q = q0 + static_cast<uint64_t>(it) * kBlock;
            if (q < nq) {
                uint32_t o[4 * W];
#pragma unroll
                for (int j = 0; j < W; ++j)
#pragma unroll
                    for (int e = 0; e < 4; ++e) o[4 * j + e] = c[it][j][e];
#pragma unroll
                for (int k = 0; k < W; ++k)
                    st<NT>(reinterpret_cast<u32x4*>(const_cast<uint32_t*>(m.src[k])) + q,
                           u32x4{o[k], o[W + k], o[2 * W + k], o[3 * W + k]});
            }
        }
    }
}

// ---------------------------------------------------------------------------
// TILE path
// ---------------------------------------------------------------------------
// Independent 16-byte global loads each lane issues before using any of them.
constexpr int kLoadBatch = 8;

// LDS layout (dynamic, 16-byte aligned base): image[R*stride] | tmpl[L] | mask[L]
// The template and mask of one period are built once per plan in device
// memory (plan.d_period); each workgroup copies them with 16-byte loads.
__device__ __forceinline__ void build_template(const TileArgs& a, uint8_t* tmpl, uint8_t*) {
    const uint32_t nch = (2 * a.L) >> 4;
    for (uint32_t i = threadIdx.x; i < nch; i += kBlock)
        reinterpret_cast<uint4*>(tmpl)[i] = reinterpret_cast<const uint4*>(a.period)[i];
}

__device__ __forceinline__ uint4 and_not_or(uint4 v, uint4 m, uint4 t) {
    return make_uint4((v.x & ~m.x) | t.x, (v.y & ~m.y) | t.y, (v.z & ~m.z) | t.z, (v.w & ~m.w) | t.w);
}

// Scatter the elements of one 16-byte column chunk into the tile image.
template <int S>
__device__ __forceinline__ void scatter_chunk(uint8_t* img, const uint4& q, uint32_t e0, uint32_t ne,
                                              uint32_t stride, uint32_t off) {
    const uint8_t* b = reinterpret_cast<const uint8_t*>(&q);
#pragma unroll
    for (int j = 0; j < 16 / S; ++j)
        if (static_cast<uint32_t>(j) < ne) __builtin_memcpy(img + (e0 + j) * stride + off, b + j * S, S);
}

template <int S>
__device__ __forceinline__ uint4 gather_chunk(const uint8_t* img, uint32_t e0, uint32_t ne,
                                              uint32_t stride, uint32_t off) {
    uint4 q = make_uint4(0, 0, 0, 0);
    uint8_t* b = reinterpret_cast<uint8_t*>(&q);
#pragma unroll
    for (int j = 0; j < 16 / S; ++j)
        if (static_cast<uint32_t>(j) < ne) __builtin_memcpy(b + j * S, img + (e0 + j) * stride + off, S);
    return q;
}

// LB: 16-byte column loads in flight per lane (the host sizes it to the
// tile: fewer slots, fewer VGPRs, more resident workgroups).
template <int LB>
__global__ __launch_bounds__(kBlock) void k_pack_tile(TileArgs a, uint8_t* __restrict__ wire, uint64_t n,
                                                      uint64_t ntiles) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t T = a.R * a.stride;
    uint8_t* img = lds;
    uint8_t* tmpl = lds + T;
    uint8_t* mask = tmpl + a.L;
    if (a.prefix_len) build_template(a, tmpl, mask);

    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t rbase = tile * a.R;
        const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
        // 1. columns -> image
        for (uint32_t f = 0; f < a.nfields; ++f) {
            const uint32_t s = a.size[f], lg = a.lgsize[f];
            const uint8_t* src = a.col[f] + rbase * s;
            const uint32_t nbytes = nr * s;
            const uint32_t nchunks = (nbytes + 15) >> 4;
            for (uint32_t c0 = threadIdx.x; c0 < nchunks; c0 += kBlock * LB) {
                uint4 qq[LB];
#pragma unroll
                for (int u = 0; u < LB; ++u) {
                    const uint32_t c = c0 + u * kBlock;
                    if ((c + 1) * 16 <= nbytes) qq[u] = *reinterpret_cast<const uint4*>(src + 16 * c);
                }
#pragma unroll
                for (int u = 0; u < LB; ++u) {
                    const uint32_t c = c0 + u * kBlock;
                    if (c >= nchunks) break;
                    const uint32_t e0 = (16 * c) >> lg;
                    const uint32_t ne = min<uint32_t>(16u >> lg, nr - e0);
                    if ((c + 1) * 16 > nbytes) {  // the column's last, partial chunk: whole elements, bytewise
                        for (uint32_t e = e0; e < nr; ++e)
                            for (uint32_t i = 0; i < s; ++i) img[e * a.stride + a.off[f] + i] = src[e * s + i];
                        continue;
                    }
                    switch (s) {
                    case 1: scatter_chunk<1>(img, qq[u], e0, ne, a.stride, a.off[f]); break;
                    case 2: scatter_chunk<2>(img, qq[u], e0, ne, a.stride, a.off[f]); break;
                    case 4: scatter_chunk<4>(img, qq[u], e0, ne, a.stride, a.off[f]); break;
                    default: scatter_chunk<8>(img, qq[u], e0, ne, a.stride, a.off[f]); break;
                    }
                }
            }
        }
        __syncthreads();
        // 2. image (+ prefix template) -> wire, 16-byte aligned stores
        uint8_t* dst = wire + rbase * a.stride;
        const uint32_t tbytes = nr * a.stride;
        const uint32_t full = tbytes >> 4;
        for (uint32_t c = threadIdx.x; c < full; c += kBlock) {
            uint4 v = *reinterpret_cast<const uint4*>(img + 16 * c);
            if (a.prefix_len) {
                const uint32_t ph = (16 * c) % a.L;
                v = and_not_or(v, *reinterpret_cast<const uint4*>(mask + ph),
                               *reinterpret_cast<const uint4*>(tmpl + ph));
            }
            // non-temporal: the wire is written once (Quad on TILE 112 -> 93 us
            // with the full grid, r01_tile_grid_nt_ab.log)
            __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(dst + 16 * c));
        }
        if (threadIdx.x == 0) {
            for (uint32_t i = full * 16; i < tbytes; ++i) {
                const uint32_t ph = i % a.L;
                dst[i] = a.prefix_len && mask[ph] ? tmpl[ph] : img[i];
            }
        }
        __syncthreads();
    }
}

// Multi-field pack with every field's column slice loaded in ONE batch.
// k_pack_tile walks the fields one after another, so a tile pays one memory
// round trip per field (6 for the 17-byte all-kinds record: 87 % of its wave
// cycles stalled, profiles/r02_pmc_before_all_kinds.txt).  Here the tile's
// 16-byte column chunks of all fields are numbered as one list (field f owns
// chunks [cs[f], cs[f+1])) and lane t takes chunks t, t + 256, ..., t + 256(K-1):
// all K loads are in flight before the first scatter, and consecutive lanes
// still read consecutive chunks of one column (coalesced).  K is sized by the
// host to the tile's chunk count (<= 256 K).
struct FieldLds {
    const uint8_t* col;
    uint32_t size, lg, off, pad;
};

#ifndef SRPC_FLAT_WAVES
#define SRPC_FLAT_WAVES 0  // A/B: amdgpu_waves_per_eu floor for the flat pack (0 = compiler's choice)
#endif
#if SRPC_FLAT_WAVES
#define SRPC_FLAT_ATTR __attribute__((amdgpu_waves_per_eu(SRPC_FLAT_WAVES)))
#else
#define SRPC_FLAT_ATTR
#endif
template <int K>
__global__ __launch_bounds__(kBlock) SRPC_FLAT_ATTR void k_pack_tile_flat(TileArgs a, uint8_t* __restrict__ wire, uint64_t n,
                                                           uint64_t ntiles) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t T = a.R * a.stride;
    uint8_t* img = lds;
    uint8_t* tmpl = lds + T;
    uint8_t* mask = tmpl + a.L;
    __shared__ FieldLds fl[kMaxFields];
    if (a.prefix_len) build_template(a, tmpl, mask);
    if (threadIdx.x < a.nfields)
        fl[threadIdx.x] = {a.col[threadIdx.x], a.size[threadIdx.x], a.lgsize[threadIdx.x], a.off[threadIdx.x], 0};
    __syncthreads();

    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t rbase = tile * a.R;
        const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
        // item g -> (field, chunk of its column slice): fields' chunk counts
        // summed uniformly (the last tile is short), no indexed arrays
        uint32_t fk[K], ck[K];
        uint32_t total = 0;
#pragma unroll
        for (int u = 0; u < K; ++u) fk[u] = ck[u] = 0;
        for (uint32_t f = 0; f < a.nfields; ++f) {
#pragma unroll
            for (int u = 0; u < K; ++u) {
                const uint32_t g = threadIdx.x + u * kBlock;
                if (g >= total) {
                    fk[u] = f;
                    ck[u] = g - total;
                }
            }
            total += (nr * a.size[f] + 15) >> 4;
        }
        uint4 qq[K];
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const uint32_t g = threadIdx.x + u * kBlock;
            if (g < total) {
                const uint32_t f = fk[u], c = ck[u];
                const uint32_t s = fl[f].size;
                const uint8_t* src = fl[f].col + rbase * s;
                if ((c + 1) * 16 <= nr * s) qq[u] = *reinterpret_cast<const uint4*>(src + 16 * c);
            }
        }
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const uint32_t g = threadIdx.x + u * kBlock;
            if (g >= total) break;
            const uint32_t f = fk[u], c = ck[u];
            const uint32_t s = fl[f].size, lg = fl[f].lg, off = fl[f].off;
            const uint32_t e0 = (16 * c) >> lg;
            const uint32_t ne = min<uint32_t>(16u >> lg, nr - e0);
            if ((c + 1) * 16 > nr * s) {  // the column's last, partial chunk: whole elements, bytewise
                const uint8_t* src = fl[f].col + rbase * s;
                for (uint32_t e = e0; e < nr; ++e)
                    for (uint32_t i = 0; i < s; ++i) img[e * a.stride + off + i] = src[e * s + i];
                continue;
            }
            switch (s) {
            case 1: scatter_chunk<1>(img, qq[u], e0, ne, a.stride, off); break;
            case 2: scatter_chunk<2>(img, qq[u], e0, ne, a.stride, off); break;
            case 4: scatter_chunk<4>(img, qq[u], e0, ne, a.stride, off); break;
            default: scatter_chunk<8>(img, qq[u], e0, ne, a.stride, off); break;
            }
        }
        __syncthreads();
        uint8_t* dst = wire + rbase * a.stride;
        const uint32_t tbytes = nr * a.stride;
        const uint32_t full = tbytes >> 4;
        for (uint32_t c = threadIdx.x; c < full; c += kBlock) {
            uint4 v = *reinterpret_cast<const uint4*>(img + 16 * c);
            if (a.prefix_len) {
                const uint32_t ph = (16 * c) % a.L;
                v = and_not_or(v, *reinterpret_cast<const uint4*>(mask + ph),
                               *reinterpret_cast<const uint4*>(tmpl + ph));
            }
            __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(dst + 16 * c));
        }
        if (threadIdx.x == 0) {
            for (uint32_t i = full * 16; i < tbytes; ++i) {
                const uint32_t ph = i % a.L;
                dst[i] = a.prefix_len && mask[ph] ? tmpl[ph] : img[i];
            }
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Wave tiles: one wave owns a tile of R records (a workgroup of one wave), so
// no phase waits on other waves -- the image needs only the wave's own LDS
// ordering (s_waitcnt lgkmcnt(0)), never an s_barrier.  A workgroup tile's
// stores cannot start until its slowest wave's loads are back; here every
// wave streams load -> scatter -> store on its own, and the small image
// (~4 KiB) lets 8 waves per SIMD stay resident.
// ---------------------------------------------------------------------------
constexpr int kWave = 64;

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void wave_template(const TileArgs& a, uint8_t* tmpl) {
    const uint32_t nch = (2 * a.L) >> 4;
    for (uint32_t i = threadIdx.x; i < nch; i += kWave)
        reinterpret_cast<uint4*>(tmpl)[i] = reinterpret_cast<const uint4*>(a.period)[i];
}

// Item g of a tile -> (column pointer, element bytes, record offset, chunk):
// every field's 16-byte column chunks numbered as one list, K items per lane
// (g = lane + 64u).  Field values come from uniform (scalar) reads of the
// kernarg arrays inside the uniform field loop.
template <int K>
struct WaveItems {
    const uint8_t* col[K];
    uint32_t sz[K], off[K], c[K];
    uint32_t total;
};

template <int K>
__device__ __forceinline__ void wave_items(const TileArgs& a, uint64_t rbase, uint32_t nr, WaveItems<K>& w) {
    const uint32_t lane = threadIdx.x;
    uint32_t total = 0;
#pragma unroll
    for (int u = 0; u < K; ++u) {
        w.col[u] = nullptr;
        w.sz[u] = w.off[u] = w.c[u] = 0;
    }
    for (uint32_t f = 0; f < a.nfields; ++f) {
        const uint32_t s = a.size[f];
        const uint8_t* base = a.col[f] + rbase * s;
        const uint32_t off = a.off[f];
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const uint32_t g = lane + u * kWave;
            if (g >= total) {
                w.col[u] = base;
                w.sz[u] = s;
                w.off[u] = off;
                w.c[u] = g - total;
            }
        }
        total += (nr * s + 15) >> 4;
    }
    w.total = total;
}

template <int K>
__global__ __launch_bounds__(kWave) void k_pack_tile_wave(TileArgs a, uint8_t* __restrict__ wire, uint64_t n) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x;
    const uint32_t T = a.R * a.stride;
    uint8_t* img = lds;
    uint8_t* tmpl = lds + T;
    uint8_t* mask = tmpl + a.L;
    const uint64_t rbase = static_cast<uint64_t>(blockIdx.x) * a.R;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
    WaveItems<K> w;
    wave_items<K>(a, rbase, nr, w);
    uint4 qq[K];
#pragma unroll
    for (int u = 0; u < K; ++u) {
        const uint32_t g = lane + u * kWave;
        if (g < w.total && (w.c[u] + 1) * 16 <= nr * w.sz[u])
            qq[u] = reinterpret_cast<const uint4*>(w.col[u])[w.c[u]];
    }
    if (a.prefix_len) wave_template(a, tmpl);
#pragma unroll
    for (int u = 0; u < K; ++u) {
        const uint32_t g = lane + u * kWave;
        if (g >= w.total) break;
        const uint32_t s = w.sz[u], off = w.off[u], c = w.c[u];
        const uint32_t lg = s == 1 ? 0 : s == 2 ? 1 : s == 4 ? 2 : 3;
        const uint32_t e0 = (16 * c) >> lg;
        const uint32_t ne = min<uint32_t>(16u >> lg, nr - e0);
        if ((c + 1) * 16 > nr * s) {  // the column's last, partial chunk: whole elements, bytewise
            for (uint32_t e = e0; e < nr; ++e)
                for (uint32_t i = 0; i < s; ++i) img[e * a.stride + off + i] = w.col[u][e * s + i];
            continue;
        }
        switch (s) {
        case 1: scatter_chunk<1>(img, qq[u], e0, ne, a.stride, off); break;
        case 2: scatter_chunk<2>(img, qq[u], e0, ne, a.stride, off); break;
        case 4: scatter_chunk<4>(img, qq[u], e0, ne, a.stride, off); break;
        default: scatter_chunk<8>(img, qq[u], e0, ne, a.stride, off); break;
        }
    }
    wave_lds_sync();
    uint8_t* dst = wire + rbase * a.stride;
    const uint32_t tbytes = nr * a.stride;
    const uint32_t full = tbytes >> 4;
    for (uint32_t c = lane; c < full; c += kWave) {
        uint4 v = *reinterpret_cast<const uint4*>(img + 16 * c);
        if (a.prefix_len) {
            const uint32_t ph = (16 * c) % a.L;
            v = and_not_or(v, *reinterpret_cast<const uint4*>(mask + ph), *reinterpret_cast<const uint4*>(tmpl + ph));
        }
        __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(dst + 16 * c));
    }
    if (lane == 0) {
        for (uint32_t i = full * 16; i < tbytes; ++i) {
            const uint32_t ph = i % a.L;
            dst[i] = a.prefix_len && mask[ph] ? tmpl[ph] : img[i];
        }
    }
}

// Unpack of a wave tile: wire chunks (KW per lane, every prefix byte checked)
// -> LDS image -> every field's column chunks as one list (K per lane).
template <int K, int KW>
__global__ __launch_bounds__(kWave) void k_unpack_tile_wave(TileArgs a, const uint8_t* __restrict__ wire, uint64_t n,
                                                            srpc_unpack_status* st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t lane = threadIdx.x;
    const uint32_t T = a.R * a.stride;
    uint8_t* img = lds;
    uint8_t* tmpl = lds + T;
    uint8_t* mask = tmpl + a.L;
    const uint64_t rbase = static_cast<uint64_t>(blockIdx.x) * a.R;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
    const uint8_t* src = wire + rbase * a.stride;
    const uint32_t tbytes = nr * a.stride;
    const uint32_t full = tbytes >> 4;
    uint4 vv[KW];
#pragma unroll
    for (int u = 0; u < KW; ++u) {
        const uint32_t c = lane + u * kWave;
        if (c < full) vv[u] = reinterpret_cast<const uint4*>(src)[c];
    }
    if (a.prefix_len) wave_template(a, tmpl);
    wave_lds_sync();
#pragma unroll
    for (int u = 0; u < KW; ++u) {
        const uint32_t c = lane + u * kWave;
        if (c >= full) break;
        const uint4 v = vv[u];
        if (a.prefix_len && st) {
            const uint32_t ph = (16 * c) % a.L;
            const uint4 m = *reinterpret_cast<const uint4*>(mask + ph);
            const uint4 t = *reinterpret_cast<const uint4*>(tmpl + ph);
            const uint32_t d0 = (v.x & m.x) ^ t.x, d1 = (v.y & m.y) ^ t.y;
            const uint32_t d2 = (v.z & m.z) ^ t.z, d3 = (v.w & m.w) ^ t.w;
            if (d0 | d1 | d2 | d3) {
                const uint32_t wd = d0 ? 0 : d1 ? 1 : d2 ? 2 : 3;
                const uint32_t dw = d0 ? d0 : d1 ? d1 : d2 ? d2 : d3;
                const uint32_t i = 16 * c + 4 * wd + (__builtin_ctz(dw) >> 3);
                report_bad(st, SRPC_STATUS_PREFIX, a.base + rbase + i / a.stride);
            }
        }
        *reinterpret_cast<uint4*>(img + 16 * c) = v;
    }
    if (lane == 0) {
        for (uint32_t i = full * 16; i < tbytes; ++i) {
            const uint8_t b = src[i];
            const uint32_t ph = i % a.L;
            if (a.prefix_len && st && (b & mask[ph]) != tmpl[ph]) report_bad(st, SRPC_STATUS_PREFIX, a.base + rbase + i / a.stride);
            img[i] = b;
        }
    }
    wave_lds_sync();
    WaveItems<K> w;
    wave_items<K>(a, rbase, nr, w);
#pragma unroll
    for (int u = 0; u < K; ++u) {
        const uint32_t g = lane + u * kWave;
        if (g >= w.total) break;
        const uint32_t s = w.sz[u], off = w.off[u], c = w.c[u];
        const uint32_t lg = s == 1 ? 0 : s == 2 ? 1 : s == 4 ? 2 : 3;
        const uint32_t e0 = (16 * c) >> lg;
        const uint32_t ne = min<uint32_t>(16u >> lg, nr - e0);
        uint8_t* dstc = const_cast<uint8_t*>(w.col[u]);
        if ((c + 1) * 16 > nr * s) {  // the column's last, partial chunk: whole elements, bytewise
            for (uint32_t e = e0; e < nr; ++e)
                for (uint32_t i = 0; i < s; ++i) dstc[e * s + i] = img[e * a.stride + off + i];
            continue;
        }
        uint4 q;
        switch (s) {
        case 1: q = gather_chunk<1>(img, e0, ne, a.stride, off); break;
        case 2: q = gather_chunk<2>(img, e0, ne, a.stride, off); break;
        case 4: q = gather_chunk<4>(img, e0, ne, a.stride, off); break;
        default: q = gather_chunk<8>(img, e0, ne, a.stride, off); break;
        }
        __builtin_nontemporal_store(u32x4{q.x, q.y, q.z, q.w}, reinterpret_cast<u32x4*>(dstc) + c);
    }
}

__global__ __launch_bounds__(kBlock) void k_unpack_tile(TileArgs a, const uint8_t* __restrict__ wire,
                                                        uint64_t n, uint64_t ntiles,
                                                        srpc_unpack_status* st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const uint32_t T = a.R * a.stride;
    uint8_t* img = lds;
    uint8_t* tmpl = lds + T;
    uint8_t* mask = tmpl + a.L;
    if (a.prefix_len) build_template(a, tmpl, mask);
    __syncthreads();

    for (uint64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const uint64_t rbase = tile * a.R;
        const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
        // 1. wire -> image, checking every prefix byte against the template
        const uint8_t* src = wire + rbase * a.stride;
        const uint32_t tbytes = nr * a.stride;
        const uint32_t full = tbytes >> 4;
        // kLoadBatch independent 16-byte loads in flight per lane before any is used
        for (uint32_t c0 = threadIdx.x; c0 < full; c0 += kBlock * kLoadBatch) {
            uint4 vv[kLoadBatch];
#pragma unroll
            for (int u = 0; u < kLoadBatch; ++u) {
                const uint32_t c = c0 + u * kBlock;
                if (c < full) vv[u] = *reinterpret_cast<const uint4*>(src + 16 * c);
            }
#pragma unroll
            for (int u = 0; u < kLoadBatch; ++u) {
                const uint32_t c = c0 + u * kBlock;
                if (c >= full) break;
                const uint4 v = vv[u];
                if (a.prefix_len && st) {
                    const uint32_t ph = (16 * c) % a.L;
                    const uint4 m = *reinterpret_cast<const uint4*>(mask + ph);
                    const uint4 t = *reinterpret_cast<const uint4*>(tmpl + ph);
                    const uint32_t d0 = (v.x & m.x) ^ t.x, d1 = (v.y & m.y) ^ t.y;
                    const uint32_t d2 = (v.z & m.z) ^ t.z, d3 = (v.w & m.w) ^ t.w;
                    if (d0 | d1 | d2 | d3) {
                        // first record touched by a differing byte of this chunk
                        const uint32_t w = d0 ? 0 : d1 ? 1 : d2 ? 2 : 3;
                        const uint32_t dw = d0 ? d0 : d1 ? d1 : d2 ? d2 : d3;
                        const uint32_t i = 16 * c + 4 * w + (__builtin_ctz(dw) >> 3);
                        report_bad(st, SRPC_STATUS_PREFIX, a.base + rbase + i / a.stride);
                    }
                }
                *reinterpret_cast<uint4*>(img + 16 * c) = v;
            }
        }
        if (threadIdx.x == 0) {
            for (uint32_t i = full * 16; i < tbytes; ++i) {
                const uint8_t b = src[i];
                const uint32_t ph = i % a.L;
                if (a.prefix_len && st && (b & mask[ph]) != tmpl[ph])
                    report_bad(st, SRPC_STATUS_PREFIX, a.base + rbase + i / a.stride);
                img[i] = b;
            }
        }
        __syncthreads();
        // 2. image -> columns
        for (uint32_t f = 0; f < a.nfields; ++f) {
            const uint32_t s = a.size[f], lg = a.lgsize[f];
            uint8_t* dstc = const_cast<uint8_t*>(a.col[f]) + rbase * s;
            const uint32_t nbytes = nr * s;
            const uint32_t nchunks = (nbytes + 15) >> 4;
            for (uint32_t c = threadIdx.x; c < nchunks; c += kBlock) {
                const uint32_t e0 = (16 * c) >> lg;
                const uint32_t ne = min<uint32_t>(16u >> lg, nr - e0);
                uint4 q;
                switch (s) {
                case 1: q = gather_chunk<1>(img, e0, ne, a.stride, a.off[f]); break;
                case 2: q = gather_chunk<2>(img, e0, ne, a.stride, a.off[f]); break;
                case 4: q = gather_chunk<4>(img, e0, ne, a.stride, a.off[f]); break;
                default: q = gather_chunk<8>(img, e0, ne, a.stride, a.off[f]); break;
                }
                if ((c + 1) * 16 <= nbytes) {
                    // non-temporal: Quad on TILE 99 -> 79 us (r01_tile_unpack_nt_ab.log)
                    __builtin_nontemporal_store(u32x4{q.x, q.y, q.z, q.w}, reinterpret_cast<u32x4*>(dstc + 16 * c));
                } else {  // the column's last, partial chunk: whole elements, bytewise from the image
                    for (uint32_t e = e0; e < nr; ++e)
                        for (uint32_t i = 0; i < s; ++i) dstc[e * s + i] = img[e * a.stride + a.off[f] + i];
                }
            }
        }
        __syncthreads();
    }
}

__global__ void k_set_status(srpc_unpack_status* st, uint32_t flags, uint64_t first_bad) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        if (flags) {
            atomicOr(&st->flags, flags);
            atomicMin(reinterpret_cast<unsigned long long*>(&st->first_bad_record),
                      static_cast<unsigned long long>(first_bad));
        } else {
            st->flags = 0;
            st->reserved = 0;
            st->first_bad_record = ~0ull;
        }
    }
}

// ---------------------------------------------------------------------------
// Synthetic input generator (SURVEY.md §8c splitmix64)
// ---------------------------------------------------------------------------
struct FillArgs {
    uint32_t* col[kMaxFields];
};

__global__ __launch_bounds__(kBlock) void k_fill_splitmix(FillArgs a, uint32_t nfields, uint64_t n,
                                                          uint64_t seed, uint64_t first) {
    const uint64_t gsz = static_cast<uint64_t>(gridDim.x) * kBlock;
    for (uint64_t r = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; r < n; r += gsz) {
        for (uint32_t f = 0; f < nfields; ++f) {
            uint64_t z = seed + ((first + r) * nfields + f + 1) * 0x9E3779B97F4A7C15ull;
            z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
            z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
            z ^= z >> 31;
            a.col[f][r] = static_cast<uint32_t>(z);
        }
    }
}

}  // namespace

// ===========================================================================
// Host side: plans and the C ABI
// ===========================================================================

namespace {
using namespace srpc_impl;

// TILE pack of multi-field records: the flat kernel (all fields' column
// loads in one batch) unless built with -DSRPC_TILE_PACK_FLAT=0 (A/B).
#ifndef SRPC_TILE_PACK_FLAT
#define SRPC_TILE_PACK_FLAT 1
#endif
constexpr bool kTilePackFlat = SRPC_TILE_PACK_FLAT != 0;

template <int W, int ITER, int NT>
int launch_dword_v(bool pack, const DwordMap& m, uint8_t* wire, uint64_t n, int rpl, int max_grid, hipStream_t s) {
    const uint64_t per = static_cast<uint64_t>(kBlock) * ITER;
    // kernels are grid-stride: max_grid > 0 caps the workgroup count
    auto cap = [max_grid](uint64_t g) { return max_grid > 0 ? std::min<uint64_t>(g, max_grid) : g; };
    uint64_t done = 0;
    if (rpl == 4) {
        const uint64_t nq = n / 4;
        if (nq) {
            const uint64_t grid = cap((nq + per - 1) / per);
            if (grid > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
            if (pack)
                launch(k_pack_dword_x4<W, ITER, NT>, dim3(static_cast<uint32_t>(grid)),
                                   dim3(kBlock), 0, s, m, wire, nq);
            else
                launch(k_unpack_dword_x4<W, ITER, NT>, dim3(static_cast<uint32_t>(grid)),
                                   dim3(kBlock), 0, s, m, wire, nq);
            done = nq * 4;
        }
    }
    if (done < n) {
        // remaining records (all of them for rpl == 1): shift the map to `done`
        DwordMap t = m;
        for (int k = 0; k < W; ++k) t.src[k] += done << t.lg[k];
        const uint64_t rest = n - done;
        const uint64_t grid = cap((rest + per - 1) / per);
        if (grid > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
        if (pack)
            launch(k_pack_dword<W, ITER, NT>, dim3(static_cast<uint32_t>(grid)), dim3(kBlock),
                               0, s, t, wire + done * 4 * W, rest);
        else
            launch(k_unpack_dword<W, ITER, NT>, dim3(static_cast<uint32_t>(grid)), dim3(kBlock),
                               0, s, t, wire + done * 4 * W, rest);
    }
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

// Tuning matrix (ITER x NT) is instantiated only for the record widths that
// matter for throughput (Number, TwoNumbers, Quad); other widths run the
// default variant.
template <int W>
int launch_dword(bool pack, const DwordMap& m, uint8_t* wire, uint64_t n, const DwordVariant& v,
                 hipStream_t s) {
    if constexpr (W == 1 || W == 2 || W == 4) {
#define SRPC_NT_CASES(IT)                                                        \
    switch (v.nt) {                                                              \
    case 0: return launch_dword_v<W, IT, 0>(pack, m, wire, n, v.rpl, v.grid, s);         \
    case 1: return launch_dword_v<W, IT, 1>(pack, m, wire, n, v.rpl, v.grid, s);         \
    case 2: return launch_dword_v<W, IT, 2>(pack, m, wire, n, v.rpl, v.grid, s);         \
    default: return launch_dword_v<W, IT, 3>(pack, m, wire, n, v.rpl, v.grid, s);        \
    }
        switch (v.iter) {
        case 1: SRPC_NT_CASES(1)
        case 2: SRPC_NT_CASES(2)
        case 8: SRPC_NT_CASES(8)
        default: SRPC_NT_CASES(4)
        }
#undef SRPC_NT_CASES
    } else {
        return launch_dword_v<W, 4, 0>(pack, m, wire, n, 1, v.grid, s);
    }
}

int launch_dword_any(bool pack, const DwordMap& m, uint8_t* wire, uint64_t n, uint32_t W,
                     const DwordVariant& v, hipStream_t s) {
    switch (W) {
    case 1: return launch_dword<1>(pack, m, wire, n, v, s);
    case 2: return launch_dword<2>(pack, m, wire, n, v, s);
    case 3: return launch_dword<3>(pack, m, wire, n, v, s);
    case 4: return launch_dword<4>(pack, m, wire, n, v, s);
    case 5: return launch_dword<5>(pack, m, wire, n, v, s);
    case 6: return launch_dword<6>(pack, m, wire, n, v, s);
    case 7: return launch_dword<7>(pack, m, wire, n, v, s);
    case 8: return launch_dword<8>(pack, m, wire, n, v, s);
    default: return SRPC_E_UNSUPPORTED;
    }
}

DwordMap make_dword_map(const srpc_plan* p, const void* const* cols) {
    DwordMap m{};
    uint32_t k = 0;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        const uint32_t dw = p->size[f] / 4;
        for (uint32_t j = 0; j < dw; ++j, ++k) {
            m.src[k] = static_cast<const uint32_t*>(cols[f]) + j;
            m.lg[k] = dw == 2 ? 1 : 0;
        }
    }
    return m;
}

TileArgs make_tile_args(const srpc_plan* p, const void* const* cols, bool pack) {
    TileArgs a{};
    for (uint32_t f = 0; f < p->nfields; ++f) {
        a.col[f] = static_cast<const uint8_t*>(cols[f]);
        a.size[f] = p->size[f];
        a.lgsize[f] = ilog2(p->size[f]);
        a.off[f] = p->off[f];
    }
    a.period = p->d_period;
    a.nfields = p->nfields;
    a.stride = static_cast<uint32_t>(p->stride);
    a.prefix_len = p->prefix_len;
    a.R = pack ? p->ptile_R : p->tile_R;
    a.L = p->tile_L;
    return a;
}

bool check_cols_aligned(const void* const* cols, uint32_t nf, uintptr_t a) {
    for (uint32_t f = 0; f < nf; ++f)
        if (!aligned(cols[f], a)) return false;
    return true;
}

int check_cols(const srpc_plan* p, const void* const* cols, uint64_t n) {
    if (n == 0) return SRPC_OK;
    if (!cols) return SRPC_E_INVALID;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        if (!cols[f]) return SRPC_E_INVALID;
        const uintptr_t need = p->path == SRPC_PATH_TILE ? 16 : 4;
        if (!aligned(cols[f], need)) return SRPC_E_ALIGN;
    }
    return SRPC_OK;
}

// DWORD variant per record width, from the interleaved A/B sweeps of
// profiles/r01_sweep_{quad,number,two}.log and the bench loop (r01_tune.log):
// 1-dword records want 16-byte column loads (4 records per lane); 2-dword
// records two records per lane-iteration with non-temporal loads; 4-dword
// records one per lane with non-temporal loads and stores.
DwordVariant default_dword_variant(uint32_t W) {
    DwordVariant v;
    if (W == 1) {
        v.rpl = 4;
        v.iter = 1;
        v.nt = kNtLoad;
    } else if (W == 4) {
        v.rpl = 1;
        v.iter = 1;
        v.nt = kNtLoad | kNtStore;
    } else {
        v.rpl = 1;
        v.iter = 2;
        v.nt = kNtLoad;
    }
    return v;
}

// TILE geometry: R records per tile (a multiple of 16, so every tile's wire
// span is 16-byte aligned) with an image of about `target` bytes, the
// template period L = lcm(stride, 16), and a grid-stride grid of as many
// workgroups as can be resident.
int upload_period(srpc_plan* p) {
    if (!p->prefix_len || p->d_period) return SRPC_OK;
    const uint32_t L = p->tile_L, S = static_cast<uint32_t>(p->stride);
    std::vector<uint8_t> h(2 * static_cast<size_t>(L), 0);
    for (uint32_t i = 0; i < L; ++i) {
        const uint32_t pos = i % S;
        if (pos < p->prefix_len) {
            h[i] = p->h_prefix[pos];
            h[L + i] = 0xFF;
        }
    }
    DeviceGuard g(p->device);
    if (hipMalloc(&p->d_period, h.size()) != hipSuccess) {
        p->d_period = nullptr;
        return SRPC_E_HIP;
    }
    if (hipMemcpy(p->d_period, h.data(), h.size(), hipMemcpyHostToDevice) != hipSuccess) return SRPC_E_HIP;
    return SRPC_OK;
}

// The pack image kernel's own tile (its best size differs from unpack's:
// profiles/r01_sweep_tile.log) and its column load slots per lane, sized to
// the widest field's slice of a tile (fewer slots, fewer VGPRs, more
// resident workgroups).
void configure_pack_tile(srpc_plan* p, uint32_t target) {
    const uint32_t S = static_cast<uint32_t>(p->stride);
    const uint32_t R = 16 * std::max<uint32_t>(1, target / (16 * S));
    p->ptile_R = R;
    p->ptile_lds = static_cast<size_t>(R) * S + (p->prefix_len ? 2 * p->tile_L : 0);
    uint32_t maxc = 1, allc = 0;
    bool mixed = false;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        maxc = std::max(maxc, (R * p->size[f] + 15) / 16);
        allc += (R * p->size[f] + 15) / 16;
        mixed |= p->size[f] != p->size[0];
    }
    p->tile_lb = maxc <= kBlock ? 1 : maxc <= 2 * kBlock ? 2 : maxc <= 4 * kBlock ? 4 : 8;
    // flat kernel: all fields' chunks in one batch of K loads per lane, for
    // records of mixed field widths (17-byte all-kinds pack 125 -> 111 us;
    // equal widths keep the per-field kernel: Quad on TILE 80 -> 84 us with
    // the flat one, profiles/r02_tile_flat_ab.log)
    const uint32_t k = (allc + kBlock - 1) / kBlock;
    p->tile_flat_k = mixed && kTilePackFlat ? (k <= 1 ? 1 : k <= 2 ? 2 : k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : 0) : 0;
}

inline int pow2_slots(uint32_t k) { return k <= 1 ? 1 : k <= 2 ? 2 : k <= 4 ? 4 : k <= 8 ? 8 : k <= 16 ? 16 : 0; }

// Wave tiles of about `target` image bytes (0: workgroup tiles): R records, a
// multiple of 16 (R*stride is then a multiple of 16), and the column and wire
// chunk slots per lane.
int configure_wave_tile(srpc_plan* p, srpc_plan::WaveTile& w, uint32_t target) {
    w = srpc_plan::WaveTile{};
    if (!target) return SRPC_OK;
    const uint32_t S = static_cast<uint32_t>(p->stride);
    const uint32_t R = 16 * std::max<uint32_t>(1, target / (16 * S));
    uint32_t allc = 0;
    for (uint32_t f = 0; f < p->nfields; ++f) allc += (R * p->size[f] + 15) / 16;
    const int k = pow2_slots((allc + kWave - 1) / kWave);
    const int kw = pow2_slots((R * S / 16 + kWave - 1) / kWave);
    const size_t lds = static_cast<size_t>(R) * S + (p->prefix_len ? 2 * p->tile_L : 0);
    if (!k || !kw || lds > 65536) return SRPC_E_INVALID;
    w.R = R;
    w.lds = lds;
    w.k = k;
    w.kw = kw;
    return SRPC_OK;
}

void configure_tile(srpc_plan* p, uint32_t target) {
    const uint32_t S = static_cast<uint32_t>(p->stride);
    const uint32_t R = 16 * std::max<uint32_t>(1, target / (16 * S));
    p->tile_R = R;
    p->tile_L = S / gcd_u32(S, 16) * 16;
    p->tile_lds = static_cast<size_t>(R) * S + (p->prefix_len ? 2 * p->tile_L : 0);
    configure_pack_tile(p, target);
    int per_cu = 0, cus = 0;
    DeviceGuard g(p->device);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_pack_tile<8>, kBlock, p->tile_lds) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, p->device) != hipSuccess) {
        per_cu = 4;
        cus = 256;
    }
    p->tile_grid = std::max(1, std::min(per_cu, 8)) * std::max(cus, 1);
    // Image kernels: one workgroup per tile beat a resident grid-stride grid
    // on every TILE schema (square request unpack 193 -> 167 us, response
    // 78 -> 70 us; profiles/r01_tile_grid_nt_ab.log).  A grid-stride variant
    // that issued the next tile's loads before draining the current image
    // (kept in flight across the tile loop) lost to both (r01_tile_pipe_ab.log).
    p->tile_full_grid = true;
}

// Device copy of the constant prefix with 16 zero bytes on both sides, so a
// 16-byte load at any offset in [-15, prefix_len) stays inside the buffer.
int upload_prefix(srpc_plan* p) {
    if (!p->prefix_len) return SRPC_OK;
    const size_t bytes = p->prefix_len + 32;
    if (hipMalloc(&p->d_prefix_alloc, bytes) != hipSuccess) {
        p->d_prefix_alloc = nullptr;
        return SRPC_E_HIP;
    }
    if (hipMemset(p->d_prefix_alloc, 0, bytes) != hipSuccess ||
        hipMemcpy(p->d_prefix_alloc + 16, p->h_prefix, p->prefix_len, hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(p->d_prefix_alloc);
        p->d_prefix_alloc = nullptr;
        return SRPC_E_HIP;
    }
    p->d_prefix = p->d_prefix_alloc + 16;
    return SRPC_OK;
}

// Schema-specialised kernels (rec.hip): mode 1 = in the directions where the
// instance measured faster, 2 = both, 0 = none.
void set_rec(srpc_plan* p, int mode) {
    p->rec_id = mode ? rec_kernel_for(p) : -1;
    p->rec_pack = p->rec_id >= 0 && (mode == 2 || rec_default(p->rec_id, true));
    p->rec_unpack = p->rec_id >= 0 && (mode == 2 || rec_default(p->rec_id, false));
}

}  // namespace

extern "C" {

int srpc_gpu_abi_version(void) { return SRPC_GPU_ABI_VERSION; }

int srpc_time_next_call(void* start_event, void* stop_event) {
    LaunchTimer& t = launch_timer();
    t = LaunchTimer{};
    t.start = static_cast<hipEvent_t>(start_event);
    t.stop = static_cast<hipEvent_t>(stop_event);
    t.armed = start_event || stop_event;
    return SRPC_OK;
}

const char* srpc_status_string(int code) {
    switch (code) {
    case SRPC_OK: return "ok";
    case SRPC_E_INVALID: return "invalid argument or schema";
    case SRPC_E_ALIGN: return "device pointer misaligned";
    case SRPC_E_HIP: return "HIP runtime error";
    case SRPC_E_UNSUPPORTED: return "not supported (a schema or layout this build has no kernel for, or a chunked host call in a stream capture)";
    case SRPC_E_CAPACITY: return "output buffer too small";
    case SRPC_ERR_BOUNDS: return "wire shorter than the requested records";
    default: return "unknown status";
    }
}

int srpc_plan_create(const srpc_schema_desc* d, int device, srpc_plan** out) {
    if (!d || !out) return SRPC_E_INVALID;
    *out = nullptr;
    if (d->nfields == 0 || !d->kinds || (d->prefix_len && !d->prefix)) return SRPC_E_INVALID;
    if (d->nfields > static_cast<uint32_t>(kMaxFields) || d->prefix_len > kMaxPrefix) return SRPC_E_UNSUPPORTED;
    auto* p = new (std::nothrow) srpc_plan();
    if (!p) return SRPC_E_INVALID;
    p->device = device;
    p->nfields = d->nfields;
    p->prefix_len = d->prefix_len;
    if (d->prefix_len) std::memcpy(p->h_prefix, d->prefix, d->prefix_len);
    uint64_t o = d->prefix_len;
    // The DWORD path has no envelope support: prefixed schemas use TILE.
    bool dword_ok = d->prefix_len == 0;
    bool all4_fields = true;
    for (uint32_t f = 0; f < d->nfields; ++f) {
        const int s = kind_size(d->kinds[f]);
        if (s < 0) {
            delete p;
            return SRPC_E_INVALID;
        }
        p->kinds[f] = d->kinds[f];
        p->size[f] = static_cast<uint32_t>(s);
        p->off[f] = static_cast<uint32_t>(o);
        if (s == 0) p->has_string = true;
        if (s != 4 && s != 8) dword_ok = false;
        if (s != 4) all4_fields = false;
        o += static_cast<uint64_t>(s);
    }
    if (p->has_string) {
        p->path = SRPC_PATH_VAR;
        for (uint32_t f = 0; f < d->nfields; ++f) p->nstrings += p->size[f] == 0;
        p->fixed_bytes = static_cast<uint32_t>(o + 8ull * p->nstrings);
        p->stride = 0;
        DeviceGuard g(device);
        if (upload_prefix(p) != SRPC_OK) {
            delete p;
            return SRPC_E_HIP;
        }
        *out = p;
        return SRPC_OK;
    }
    p->stride = o;
    p->all4 = all4_fields;
    p->dword_ok = dword_ok && (o / 4) <= static_cast<uint64_t>(kMaxDwords);
    p->path = p->dword_ok ? SRPC_PATH_DWORD : (o <= kMaxTileStride ? SRPC_PATH_TILE : 0);
    if (!p->path) {
        delete p;
        return SRPC_E_UNSUPPORTED;
    }
    DeviceGuard g(device);
    if (upload_prefix(p) != SRPC_OK) {
        delete p;
        return SRPC_E_HIP;
    }
    if (p->dword_ok) p->dv = default_dword_variant(static_cast<uint32_t>(o / 4));
    // TILE unpack image: 32 KiB, within 3 % of the best of 4-32 KiB for every
    // record width swept on MI355X (profiles/r01_sweep_tile.log).
    if (o <= kMaxTileStride) {
        configure_tile(p, 32768);
        // pack image: 24 KiB tiles for enveloped records, 16 KiB otherwise --
        // the best or within 2 % of it with the columns cache-resident (pack
        // after pack) and cold (pack after an unpack that streamed the wire
        // through the caches) for the square request/response and Quad
        // (profiles/r01_ab_pack_tile.log, r01_sweep_tile.log)
        configure_pack_tile(p, p->prefix_len ? 24576 : 16384);
        // records under 16 bytes without an envelope: wave tiles (pack 2 KiB,
        // unpack 3 KiB images) -- 3-15-byte schemas 5-32 % faster both ways,
        // 16-53-byte and enveloped ones as fast or slower, a lone int16 column
        // unpacks faster with workgroup tiles (profiles/r02_wave_tile_sweep.log)
        if (!p->prefix_len && o < 16) {
            (void)configure_wave_tile(p, p->wtp, 2048);
            if (o != 2) (void)configure_wave_tile(p, p->wtu, 3072);
        }
        if (upload_period(p) != SRPC_OK) {
            (void)srpc_plan_destroy(p);
            return SRPC_E_HIP;
        }
        if (p->path == SRPC_PATH_TILE) set_rec(p, 1);
    }
    *out = p;
    return SRPC_OK;
}

int srpc_plan_destroy(srpc_plan* p) {
    if (!p) return SRPC_E_INVALID;
    if (p->d_prefix_alloc) {
        DeviceGuard g(p->device);
        (void)hipFree(p->d_prefix_alloc);
    }
    if (p->d_period) {
        DeviceGuard g(p->device);
        (void)hipFree(p->d_period);
    }
    delete p;
    return SRPC_OK;
}

int srpc_plan_record_bytes(const srpc_plan* p, uint64_t* out) {
    if (!p || !out) return SRPC_E_INVALID;
    *out = p->has_string ? 0 : p->stride;
    return SRPC_OK;
}

int srpc_plan_path(const srpc_plan* p, int* out) {
    if (!p || !out) return SRPC_E_INVALID;
    *out = p->path;
    return SRPC_OK;
}

int srpc_plan_force_path(srpc_plan* p, int path) {
    if (!p) return SRPC_E_INVALID;
    if (path == SRPC_PATH_DWORD && p->dword_ok) {
        p->path = path;
        return SRPC_OK;
    }
    if (path == SRPC_PATH_TILE && p->tile_R) {
        p->path = path;
        set_rec(p, 1);
        return SRPC_OK;
    }
    return SRPC_E_UNSUPPORTED;
}

int srpc_plan_tune(srpc_plan* p, int knob, int value) {
    if (!p) return SRPC_E_INVALID;
    switch (knob) {
    case SRPC_TUNE_RECORDS_PER_LANE:
        if (value != 1 && value != 4) return SRPC_E_INVALID;
        p->dv.rpl = value;
        return SRPC_OK;
    case SRPC_TUNE_ITER:
        if (value != 1 && value != 2 && value != 4 && value != 8) return SRPC_E_INVALID;
        p->dv.iter = value;
        return SRPC_OK;
    case SRPC_TUNE_NONTEMPORAL:
        if (value < 0 || value > 3) return SRPC_E_INVALID;
        p->dv.nt = value;
        return SRPC_OK;
    case SRPC_TUNE_GRID:
        if (value < 0) return SRPC_E_INVALID;
        p->dv.grid = value;
        return SRPC_OK;
    case SRPC_TUNE_TILE_BYTES:
        if (value < 1024 || value > 49152 || p->has_string || p->stride > kMaxTileStride) return SRPC_E_INVALID;
        configure_tile(p, static_cast<uint32_t>(value));
        return SRPC_OK;
    case SRPC_TUNE_VAR_KERNEL:
        if (value < 0 || value > 2 || !p->has_string) return SRPC_E_INVALID;
        p->var_kernel = value ? 1 : 0;
        p->var_rt_general = value == 2;
        return SRPC_OK;
    case SRPC_TUNE_VAR_IMAGE_BYTES:
        if (value < 8192 || value > 65536 || value % 16 || !p->has_string) return SRPC_E_INVALID;
        p->rt_img_cap = static_cast<uint32_t>(value);
        return SRPC_OK;
    case SRPC_TUNE_VAR_CHARS_BYTES:
        if (value < 0 || value > 65536 || value % 16 || !p->has_string) return SRPC_E_INVALID;
        p->rt_ch_cap = static_cast<uint32_t>(value);
        p->rt_ch_cap_auto = false;
        return SRPC_OK;
    case SRPC_TUNE_WAVE_PACK_BYTES:
        if (value < 0 || value > 65536 || p->has_string || p->stride > kMaxTileStride) return SRPC_E_INVALID;
        return configure_wave_tile(p, p->wtp, static_cast<uint32_t>(value));
    case SRPC_TUNE_WAVE_UNPACK_BYTES:
        if (value < 0 || value > 65536 || p->has_string || p->stride > kMaxTileStride) return SRPC_E_INVALID;
        return configure_wave_tile(p, p->wtu, static_cast<uint32_t>(value));
    case SRPC_TUNE_REC_KERNEL:
        if (value < 0 || value > 2 || p->has_string) return SRPC_E_INVALID;
        set_rec(p, p->path == SRPC_PATH_TILE ? value : 0);
        return SRPC_OK;
    case SRPC_TUNE_PACK_TILE_BYTES:
        if (value < 1024 || value > 49152 || p->has_string || p->stride > kMaxTileStride) return SRPC_E_INVALID;
        configure_pack_tile(p, static_cast<uint32_t>(value));
        return SRPC_OK;
    default: return SRPC_E_INVALID;
    }
}

int srpc_gpu_pack(const srpc_plan* p, const void* const* cols, uint64_t n, uint8_t* wire,
                  uint64_t wire_cap, void* stream) {
    const TimedCall timed;
    if (!p || p->has_string) return SRPC_E_INVALID;  // string schemas: srpc_gpu_pack_var
    if (n == 0) return SRPC_OK;
    if (!wire) return SRPC_E_INVALID;
    if (n > UINT64_MAX / p->stride || n * p->stride > wire_cap) return SRPC_E_CAPACITY;
    if (!aligned(wire, 16)) return SRPC_E_ALIGN;
    int rc = check_cols(p, cols, n);
    if (rc) return rc;
    auto s = static_cast<hipStream_t>(stream);
    if (p->path == SRPC_PATH_DWORD) {
        const DwordMap m = make_dword_map(p, cols);
        const bool x4 = p->dv.rpl == 4 && p->all4 && check_cols_aligned(cols, p->nfields, 16);
        DwordVariant v = p->dv;
        v.rpl = x4 ? 4 : 1;
        return launch_dword_any(true, m, wire, n, static_cast<uint32_t>(p->stride / 4), v, s);
    }
    // schema-specialised kernels (rec.hip) for the whole tiles, the generic
    // ones for the rest
    const void* rest[kMaxFields];
    if (p->rec_pack && check_cols_aligned(cols, p->nfields, 16)) {
        const uint64_t TR = rec_tile_records(p->rec_id, true), tiles = n / TR;
        if (tiles) {
            if (int rc2 = rec_pack(p->rec_id, p, cols, tiles, wire, s)) return rc2;
            const uint64_t done = tiles * TR;
            if (done == n) return SRPC_OK;
            for (uint32_t f = 0; f < p->nfields; ++f) rest[f] = static_cast<const uint8_t*>(cols[f]) + done * p->size[f];
            cols = rest;
            n -= done;
            wire += done * p->stride;
        }
    }
    if (p->wtp.R && n / p->wtp.R < (1ull << 26)) {
        TileArgs a = make_tile_args(p, cols, true);
        a.R = p->wtp.R;
        const uint32_t grid = static_cast<uint32_t>((n + a.R - 1) / a.R);
        const size_t lds = p->wtp.lds;
        switch (p->wtp.k) {
        case 1: launch(k_pack_tile_wave<1>, dim3(grid), dim3(kWave), lds, s, a, wire, n); break;
        case 2: launch(k_pack_tile_wave<2>, dim3(grid), dim3(kWave), lds, s, a, wire, n); break;
        case 4: launch(k_pack_tile_wave<4>, dim3(grid), dim3(kWave), lds, s, a, wire, n); break;
        case 8: launch(k_pack_tile_wave<8>, dim3(grid), dim3(kWave), lds, s, a, wire, n); break;
        default: launch(k_pack_tile_wave<16>, dim3(grid), dim3(kWave), lds, s, a, wire, n); break;
        }
        return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    }
    const TileArgs a = make_tile_args(p, cols, true);
    const uint64_t ptiles = (n + p->ptile_R - 1) / p->ptile_R;
    const uint32_t pgrid = static_cast<uint32_t>(std::min<uint64_t>(ptiles, p->tile_full_grid ? (1u << 30) : p->tile_grid));
    const size_t lds = p->ptile_lds;
    switch (p->tile_flat_k) {
    case 1: launch(k_pack_tile_flat<1>, dim3(pgrid), dim3(kBlock), lds, s, a, wire, n, ptiles); break;
    case 2: launch(k_pack_tile_flat<2>, dim3(pgrid), dim3(kBlock), lds, s, a, wire, n, ptiles); break;
    case 4: launch(k_pack_tile_flat<4>, dim3(pgrid), dim3(kBlock), lds, s, a, wire, n, ptiles); break;
    case 8: launch(k_pack_tile_flat<8>, dim3(pgrid), dim3(kBlock), lds, s, a, wire, n, ptiles); break;
    case 16: launch(k_pack_tile_flat<16>, dim3(pgrid), dim3(kBlock), lds, s, a, wire, n, ptiles); break;
    default: break;
    }
    if (p->tile_flat_k) return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    switch (p->tile_lb) {
    case 1: launch(k_pack_tile<1>, dim3(pgrid), dim3(kBlock), lds, s, a, wire, n, ptiles); break;
    case 2: launch(k_pack_tile<2>, dim3(pgrid), dim3(kBlock), lds, s, a, wire, n, ptiles); break;
    case 4: launch(k_pack_tile<4>, dim3(pgrid), dim3(kBlock), lds, s, a, wire, n, ptiles); break;
    default: launch(k_pack_tile<8>, dim3(pgrid), dim3(kBlock), lds, s, a, wire, n, ptiles); break;
    }
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int srpc_gpu_unpack(const srpc_plan* p, const uint8_t* wire, uint64_t wire_len, uint64_t n,
                    void* const* cols, srpc_unpack_status* st, void* stream) {
    const TimedCall timed;
    if (!p || p->has_string) return SRPC_E_INVALID;  // string schemas: srpc_gpu_unpack_var
    auto s = static_cast<hipStream_t>(stream);
    if (st) {
        hipLaunchKernelGGL(k_set_status, dim3(1), dim3(64), 0, s, st, 0u, 0ull);
        if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
    }
    if (n == 0) return SRPC_OK;
    if (!wire) return SRPC_E_INVALID;
    if (!aligned(wire, 16)) return SRPC_E_ALIGN;
    int rc = check_cols(p, reinterpret_cast<const void* const*>(cols), n);
    if (rc) return rc;
    uint64_t n_fit = wire_len / p->stride;
    int ret = SRPC_OK;
    if (n_fit < n) {
        if (st) {
            hipLaunchKernelGGL(k_set_status, dim3(1), dim3(64), 0, s, st, SRPC_STATUS_BOUNDS, n_fit);
            if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
        }
        ret = SRPC_ERR_BOUNDS;
    } else {
        n_fit = n;
    }
    if (n_fit == 0) return ret;
    void* rest[kMaxFields];
    uint64_t base = 0;  // records before `wire` (status reports of the generic kernels)
    if (p->path == SRPC_PATH_TILE && p->rec_unpack &&
        check_cols_aligned(reinterpret_cast<const void* const*>(cols), p->nfields, 16)) {
        const uint64_t TR = rec_tile_records(p->rec_id, false), tiles = n_fit / TR;
        if (tiles) {
            if (int rc2 = rec_unpack(p->rec_id, p, wire, tiles, cols, st, s)) return rc2;
            base = tiles * TR;
            if (base == n_fit) return ret;
            for (uint32_t f = 0; f < p->nfields; ++f) rest[f] = static_cast<uint8_t*>(cols[f]) + base * p->size[f];
            cols = rest;
            n_fit -= base;
            wire += base * p->stride;
        }
    }
    if (p->path == SRPC_PATH_DWORD) {
        const DwordMap m = make_dword_map(p, reinterpret_cast<const void* const*>(cols));
        const bool x4 = p->dv.rpl == 4 && p->all4 &&
                        check_cols_aligned(reinterpret_cast<const void* const*>(cols), p->nfields, 16);
        DwordVariant v = p->dv;
        v.rpl = x4 ? 4 : 1;
        rc = launch_dword_any(false, m, const_cast<uint8_t*>(wire), n_fit,
                              static_cast<uint32_t>(p->stride / 4), v, s);
        return rc ? rc : ret;
    }
    if (p->wtu.R && n_fit / p->wtu.R < (1ull << 26)) {
        TileArgs a = make_tile_args(p, reinterpret_cast<const void* const*>(cols), false);
        a.R = p->wtu.R;
        a.base = base;
        const uint32_t grid = static_cast<uint32_t>((n_fit + a.R - 1) / a.R);
        const size_t lds = p->wtu.lds;
#define SRPC_UW(K, KW) launch(k_unpack_tile_wave<K, KW>, dim3(grid), dim3(kWave), lds, s, a, wire, n_fit, st)
#define SRPC_UWK(K)                          \
    switch (p->wtu.kw) {                   \
    case 1: SRPC_UW(K, 1); break;            \
    case 2: SRPC_UW(K, 2); break;            \
    case 4: SRPC_UW(K, 4); break;            \
    case 8: SRPC_UW(K, 8); break;            \
    default: SRPC_UW(K, 16); break;          \
    }
        switch (p->wtu.k) {
        case 1: SRPC_UWK(1); break;
        case 2: SRPC_UWK(2); break;
        case 4: SRPC_UWK(4); break;
        case 8: SRPC_UWK(8); break;
        default: SRPC_UWK(16); break;
        }
#undef SRPC_UWK
#undef SRPC_UW
        if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
        return ret;
    }
    const uint64_t ntiles = (n_fit + p->tile_R - 1) / p->tile_R;
    TileArgs a = make_tile_args(p, reinterpret_cast<const void* const*>(cols), false);
    a.base = base;
    const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(ntiles, p->tile_full_grid ? (1u << 30) : p->tile_grid));
    launch(k_unpack_tile, dim3(grid), dim3(kBlock), p->tile_lds, s, a, wire, n_fit, ntiles, st);
    if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
    return ret;
}

int srpc_gpu_fill_splitmix_i32(int32_t* const* cols, uint32_t nfields, uint64_t n, uint64_t seed,
                               uint64_t first_record, void* stream) {
    if (nfields == 0 || nfields > static_cast<uint32_t>(kMaxFields) || !cols) return SRPC_E_INVALID;
    if (n == 0) return SRPC_OK;
    FillArgs a{};
    for (uint32_t f = 0; f < nfields; ++f) {
        if (!cols[f]) return SRPC_E_INVALID;
        a.col[f] = reinterpret_cast<uint32_t*>(cols[f]);
    }
    const uint64_t blocks = std::min<uint64_t>((n + kBlock - 1) / kBlock, 8192);
    hipLaunchKernelGGL(k_fill_splitmix, dim3(static_cast<uint32_t>(blocks)), dim3(kBlock), 0,
                       static_cast<hipStream_t>(stream), a, nfields, n, seed, first_record);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

}  // extern "C"
