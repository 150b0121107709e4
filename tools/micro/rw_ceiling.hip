// Microbenchmark: the HBM ceilings of the TILE path's traffic shapes on gfx950.
// The Calculator.square request pack reads 4 B and writes 53 B per record (and
// unpack the reverse), so its bound is closer to a pure write (read) stream
// than to a copy.  Every kernel moves 16-byte aligned chunks, one per lane,
// grid of one chunk per lane (the TILE kernels' access shape):
//   W   write-only 16-B stores           (plain / non-temporal)
//   R   read-only 16-B loads, xor-reduced (plain / non-temporal)
//   C   1:1 copy                          (plain / non-temporal)
//   P   read 1 B : write 13.25 B (4 B column element per 53 B wire)
//   U   read 13.25 B : write 1 B
// and variants of P that locate its cost: K chunks per lane, pipelined
// grid-stride, no load, wave-coalesced load + shuffle, a load independent of
// the store, cache-resident loads, plain (cacheable) vs non-temporal loads.
// (A variant that phased reads and writes with a grid barrier was dropped:
// a spin on a counter in coarse-grained memory does not see other XCDs'
// increments, so the bounded spins time out.)
// Bytes: 16M records' worth (request wire = 889,192,448 B).  Prints GB/s of
// bytes moved (read + written), median of 10 after 3 warm-ups.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_write(u32x4* dst, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) st<NT>(dst + i, u32x4{uint32_t(i), 1u, 2u, 3u});
}

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const u32x4* src, uint64_t n, uint32_t* sink) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) {
        const u32x4 v = ld<NT>(src + i);
        const uint32_t x = v.x ^ v.y ^ v.z ^ v.w;
        if (x == 0x9E3779B9u) sink[0] = x;  // never true for the fill below: keeps the load
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const u32x4* src, u32x4* dst, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) st<NT>(dst + i, ld<NT>(src + i));
}

// wire chunk i takes the 4-byte element of its record (16 i / 53): the pack shape
__global__ __launch_bounds__(256) void k_expand(const uint32_t* col, u32x4* wire, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) {
        const uint32_t v = __builtin_nontemporal_load(col + (16 * i) / 53);
        __builtin_nontemporal_store(u32x4{v, 0x11u, 0x22u, 0x33u}, wire + i);
    }
}

// pack shape, K chunks per lane (K*256 consecutive chunks per workgroup):
// all K column loads issued before the first store
template <int K>
__global__ __launch_bounds__(256) void k_expand_k(const uint32_t* col, u32x4* wire, uint64_t n) {
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * 256 * K + threadIdx.x;
    uint32_t v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t i = base + 256 * k;
        v[k] = i < n ? __builtin_nontemporal_load(col + (16 * i) / 53) : 0;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t i = base + 256 * k;
        if (i < n) __builtin_nontemporal_store(u32x4{v[k], 0x11u, 0x22u, 0x33u}, wire + i);
    }
}

// pack shape, grid-stride with the next iteration's column element loaded
// before the current chunk is stored
__global__ __launch_bounds__(256) void k_expand_pipe(const uint32_t* col, u32x4* wire, uint64_t n) {
    const uint64_t step = static_cast<uint64_t>(gridDim.x) * 256;
    uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    uint32_t v = i < n ? __builtin_nontemporal_load(col + (16 * i) / 53) : 0;
    for (; i < n; i += step) {
        const uint64_t j = i + step;
        const uint32_t nv = j < n ? __builtin_nontemporal_load(col + (16 * j) / 53) : 0;
        __builtin_nontemporal_store(u32x4{v, 0x11u, 0x22u, 0x33u}, wire + i);
        v = nv;
    }
}

// pack shape without the load: the element is computed (a store-only kernel
// with the same index arithmetic)
__global__ __launch_bounds__(256) void k_expand_noload(u32x4* wire, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(u32x4{static_cast<uint32_t>((16 * i) / 53), 0x11u, 0x22u, 0x33u}, wire + i);
}

// pack shape, wave-coalesced: a wave loads 64 consecutive column elements (one
// 256-byte load) and writes the 212 wire chunks of those 64 records (53*64/16),
// each lane taking its chunk's element from the owning lane by a shuffle
__global__ __launch_bounds__(256) void k_expand_wave(const uint32_t* col, u32x4* wire, uint64_t nrec) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x) >> 6;
    const uint64_t r0 = wave * 64;
    if (r0 >= nrec) return;
    const uint32_t v = __builtin_nontemporal_load(col + r0 + lane);
    u32x4* dst = wire + r0 * 53 / 16;  // 64 records = 3392 bytes = 212 chunks, 16-byte aligned
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t c = lane + 64 * k;
        const uint32_t src = min(c * 16 / 53, 63u);
        const uint32_t x = __shfl(v, static_cast<int>(src));
        if (c < 212) __builtin_nontemporal_store(u32x4{x, 0x11u, 0x22u, 0x33u}, dst + c);
    }
}

// pack shape, the load not feeding the store (used only by a never-taken branch)
__global__ __launch_bounds__(256) void k_expand_indep(const uint32_t* col, u32x4* wire, uint64_t n, uint32_t* sink) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) {
        const uint32_t v = __builtin_nontemporal_load(col + (16 * i) / 53);
        __builtin_nontemporal_store(u32x4{static_cast<uint32_t>(i), 0x11u, 0x22u, 0x33u}, wire + i);
        if (v == 0x9E3779B9u) sink[0] = v;
    }
}

// pack shape reading a 1 MiB column window (cache-resident: no HBM reads)
__global__ __launch_bounds__(256) void k_expand_cached(const uint32_t* col, u32x4* wire, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) {
        const uint32_t v = col[((16 * i) / 53) & ((1u << 18) - 1)];
        __builtin_nontemporal_store(u32x4{v, 0x11u, 0x22u, 0x33u}, wire + i);
    }
}

// pack shape with plain (cacheable) column loads
__global__ __launch_bounds__(256) void k_expand_plain(const uint32_t* col, u32x4* wire, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(u32x4{col[(16 * i) / 53], 0x11u, 0x22u, 0x33u}, wire + i);
}

// the unpack shape: every wire chunk is read, the chunks holding a record's
// body write its element
__global__ __launch_bounds__(256) void k_contract(const u32x4* wire, uint32_t* col, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n) {
        const u32x4 v = __builtin_nontemporal_load(wire + i);
        const uint64_t r = (16 * i) / 53;
        if ((16 * (i + 1)) / 53 != r || i == 0) __builtin_nontemporal_store(v.x ^ v.w, col + (16 * (i + 1)) / 53);
    }
}

int main() {
    const uint64_t nrec = 1ull << 24;
    const uint64_t wbytes = nrec * 53;
    const uint64_t nch = wbytes / 16;
    u32x4 *a, *b;
    uint32_t *col, *sink;
    hipMalloc(&a, wbytes + 4096);
    hipMalloc(&b, wbytes + 4096);
    hipMalloc(&col, nrec * 4 + 4096);
    hipMalloc(&sink, 64);
    hipMemset(a, 1, wbytes + 4096);
    hipMemset(b, 0, wbytes + 4096);
    hipMemset(col, 2, nrec * 4 + 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, double moved, auto&& launch) {
        std::vector<float> ms;
        for (int r = 0; r < 13; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float t;
            hipEventElapsedTime(&t, e0, e1);
            if (r >= 3) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double t = ms[ms.size() / 2] * 1e-3;
        printf("%-44s %8.1f us  %7.1f GB/s  (%.3f of 8 TB/s)\n", name, t * 1e6, moved / t / 1e9,
               moved / t / 8e12);
    };
    const dim3 grid(static_cast<uint32_t>((nch + 255) / 256)), blk(256);
    const double wb = 16.0 * nch;
    run("W write 16B plain", wb, [&] { k_write<false><<<grid, blk>>>(b, nch); });
    run("W write 16B nt", wb, [&] { k_write<true><<<grid, blk>>>(b, nch); });
    run("R read 16B plain", wb, [&] { k_read<false><<<grid, blk>>>(a, nch, sink); });
    run("R read 16B nt", wb, [&] { k_read<true><<<grid, blk>>>(a, nch, sink); });
    run("C copy 16B plain", 2 * wb, [&] { k_copy<false><<<grid, blk>>>(a, b, nch); });
    run("C copy 16B nt", 2 * wb, [&] { k_copy<true><<<grid, blk>>>(a, b, nch); });
    run("P 4B col -> 53B wire (pack shape)", wb + 4.0 * nrec, [&] { k_expand<<<grid, blk>>>(col, b, nch); });
    run("P K=4", wb + 4.0 * nrec, [&] { k_expand_k<4><<<dim3((nch + 1023) / 1024), blk>>>(col, b, nch); });
    run("P K=8", wb + 4.0 * nrec, [&] { k_expand_k<8><<<dim3((nch + 2047) / 2048), blk>>>(col, b, nch); });
    run("P K=16", wb + 4.0 * nrec, [&] { k_expand_k<16><<<dim3((nch + 4095) / 4096), blk>>>(col, b, nch); });
    for (uint32_t g : {1024u, 2048u, 4096u, 8192u})
        run(g == 1024 ? "P pipe grid 1024" : g == 2048 ? "P pipe grid 2048" : g == 4096 ? "P pipe grid 4096" : "P pipe grid 8192",
            wb + 4.0 * nrec, [&] { k_expand_pipe<<<dim3(g), blk>>>(col, b, nch); });
    run("P no load (computed element)", wb + 4.0 * nrec, [&] { k_expand_noload<<<grid, blk>>>(b, nch); });
    run("P wave-coalesced + shuffle", wb + 4.0 * nrec, [&] { k_expand_wave<<<dim3((nrec / 64 + 3) / 4), blk>>>(col, b, nrec); });
    run("P load independent of the store", wb + 4.0 * nrec, [&] { k_expand_indep<<<grid, blk>>>(col, b, nch, sink); });
    run("P load from a cached 1 MiB window", wb + 4.0 * nrec, [&] { k_expand_cached<<<grid, blk>>>(col, b, nch); });
    // MALL prefetch: the column read in a pass of its own (pure reads), then the
    // pack shape with plain loads -- does HBM then see only the writes?
    {
        const uint64_t cch = nrec * 4 / 16;
        const dim3 cg(static_cast<uint32_t>((cch + 255) / 256));
        run("col read pass alone (64 MiB)", 4.0 * nrec, [&] { k_read<false><<<cg, blk>>>(reinterpret_cast<const u32x4*>(col), cch, sink); });
        run("P plain loads alone", wb + 4.0 * nrec, [&] { k_expand_plain<<<grid, blk>>>(col, b, nch); });
        run("col read pass + P (two kernels)", wb + 4.0 * nrec, [&] {
            k_read<false><<<cg, blk>>>(reinterpret_cast<const u32x4*>(col), cch, sink);
            k_expand_plain<<<grid, blk>>>(col, b, nch);
        });
        run("col read pass + P nt-store", wb + 4.0 * nrec, [&] {
            k_read<false><<<cg, blk>>>(reinterpret_cast<const u32x4*>(col), cch, sink);
            k_expand_plain<<<grid, blk>>>(col, b, nch);
        });
    }
    run("U 53B wire -> 4B col (unpack shape)", wb + 4.0 * nrec, [&] { k_contract<<<grid, blk>>>(a, col, nch); });
    run("hipMemsetD32 of the wire", wb, [&] { hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(b), 7, nch * 4); });
    hipDeviceSynchronize();
    return 0;
}
