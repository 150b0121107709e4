// scan.h -- device-wide exclusive scan of n counts (u32 or u64) into u64
// offsets out[0..n], out[n] = the total: per 2048 values a block total
// (xscan_reduce), one workgroup scanning the block totals in place
// (xscan_partials), then the apply pass (xscan_apply).  Used for the
// response offsets of a frame batch (frames.hip).  Scratch: xscan_parts(n)
// u64 words.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "plan.h"

namespace srpc_impl {
namespace {

constexpr uint32_t kXScanPer = kBlock * 8;  // values per block

inline uint64_t xscan_parts(uint64_t n) { return (n + kXScanPer - 1) / kXScanPer + 1; }

template <typename T>
__global__ __launch_bounds__(kBlock) void k_xscan_reduce(const T* __restrict__ v, uint64_t n,
                                                         uint64_t* __restrict__ part) {
    __shared__ uint64_t ws[kBlock / 64];
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kXScanPer;
    uint64_t s = 0;
    for (uint32_t j = threadIdx.x; j < kXScanPer; j += kBlock)
        if (base + j < n) s += v[base + j];
    for (int d = 32; d > 0; d >>= 1) s += __shfl_down(s, d, 64);
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// One workgroup of B threads: exclusive scan of the nb block totals in place,
// thread t owning a contiguous run of them; *total = their sum.  Each run is
// read and written 8 words per batch (independent loads in flight: a run of
// 32 read word by word, one round trip each, took 17 us).
template <int B>
__global__ __launch_bounds__(B) void k_xscan_partials(uint64_t* __restrict__ part, uint64_t nb,
                                                      uint64_t* __restrict__ total) {
    __shared__ uint64_t ws[B / 64];
    const uint64_t per = (nb + B - 1) / B;
    const uint64_t lo = min<uint64_t>(threadIdx.x * per, nb), hi = min<uint64_t>(lo + per, nb);
    uint64_t s = 0;
    uint64_t b = lo;
    for (; b + 8 <= hi; b += 8) {
        uint64_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = part[b + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j];
    }
    for (; b < hi; ++b) s += part[b];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint64_t run = inc - s;
    for (int w = 0; w < wave; ++w) run += ws[w];
    b = lo;
    for (; b + 8 <= hi; b += 8) {
        uint64_t v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = part[b + j];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            part[b + j] = run;
            run += v[j];
        }
    }
    for (; b < hi; ++b) {
        const uint64_t x = part[b];
        part[b] = run;
        run += x;
    }
    if (threadIdx.x == B - 1) {
        uint64_t t = 0;
        for (int w = 0; w < B / 64; ++w) t += ws[w];
        *total = t;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_xscan_apply(const T* __restrict__ v, uint64_t n,
                                                        const uint64_t* __restrict__ part, const uint64_t* total,
                                                        uint64_t* __restrict__ out) {
    __shared__ uint64_t vals[kXScanPer];
    __shared__ uint64_t ws[kBlock / 64];
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kXScanPer;
    for (uint32_t j = threadIdx.x; j < kXScanPer; j += kBlock) vals[j] = base + j < n ? v[base + j] : 0;
    __syncthreads();
    uint64_t loc[8];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        loc[j] = s;
        s += vals[threadIdx.x * 8 + j];
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = s;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint64_t before = n ? part[blockIdx.x] : 0;
    for (int w = 0; w < wave; ++w) before += ws[w];
    before += inc - s;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint64_t f = base + threadIdx.x * 8 + j;
        if (f < n) out[f] = before + loc[j];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = *total;
}

// Launches the three passes on stream s: out[0..n] from v[0..n); part has
// xscan_parts(n) words, *total one more word.
template <typename T>
inline void xscan(const T* v, uint64_t n, uint64_t* part, uint64_t* total, uint64_t* out, hipStream_t s) {
    const uint64_t nb = (n + kXScanPer - 1) / kXScanPer;
    if (nb) launch(k_xscan_reduce<T>, dim3(static_cast<uint32_t>(nb)), dim3(kBlock), 0, s, v, n, part);
    launch(k_xscan_partials<kBlock>, dim3(1), dim3(kBlock), 0, s, part, nb, total);
    launch(k_xscan_apply<T>, dim3(static_cast<uint32_t>(nb ? nb : 1)), dim3(kBlock), 0, s, v, n,
           static_cast<const uint64_t*>(part), static_cast<const uint64_t*>(total), out);
}

}  // namespace
}  // namespace srpc_impl
