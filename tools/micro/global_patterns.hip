// Microbenchmark: HBM copy rate of the access patterns a string packer can
// use on gfx950 (256 MiB moved per kernel, out of place, median of 10):
//   A  coalesced 16-B loads and stores, both 16-byte aligned (memcpy shape)
//   B  coalesced 16-B loads at +3 bytes (unaligned), aligned stores
//   C  aligned loads, coalesced 16-B stores at +3 bytes
//   D  one 48-byte record per lane at a stride of S bytes (S = 50: records
//      back to back): 3 x 16-B unaligned loads and stores per lane
//   E  one S-byte string per lane (S = 512), 16-B steps, unaligned
//   F  D's records copied by groups of 4 lanes (lane j of a group moves
//      bytes [16j, 16j+16) of the group's record; 16 records per wave)
//   G  8-byte loads/stores at a stride of 50 bytes per lane (field-sized)
//   H  1-byte loads/stores at a stride of 50 bytes per lane
// Prints GB/s of bytes moved (read + written).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

template <typename T>
__device__ __forceinline__ T ldu(const uint8_t* p) {
    typedef T Tu __attribute__((aligned(1)));
    return *reinterpret_cast<__attribute__((address_space(1))) const Tu*>(reinterpret_cast<uintptr_t>(p));
}

template <typename T>
__device__ __forceinline__ void stu(uint8_t* p, T v) {
    typedef T Tu __attribute__((aligned(1)));
    *reinterpret_cast<__attribute__((address_space(1))) Tu*>(reinterpret_cast<uintptr_t>(p)) = v;
}

__global__ void k_coalesced(const uint8_t* src, uint8_t* dst, uint64_t nchunks, int soff, int doff) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < nchunks) stu<u64x2>(dst + 16 * i + doff, ldu<u64x2>(src + 16 * i + soff));
}

// one record of `len` bytes per lane, records `stride` apart, 16-byte steps
__global__ void k_per_lane(const uint8_t* src, uint8_t* dst, uint64_t nrec, uint32_t stride, uint32_t len) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= nrec) return;
    const uint8_t* s = src + i * stride + 1;
    uint8_t* d = dst + i * stride + 3;
    for (uint32_t j = 0; j + 16 <= len; j += 16) stu<u64x2>(d + j, ldu<u64x2>(s + j));
}

// groups of G lanes per record
template <int G>
__global__ void k_grouped(const uint8_t* src, uint8_t* dst, uint64_t nrec, uint32_t stride, uint32_t len) {
    const uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t i = t / G;
    const uint32_t j = 16 * (t % G);
    if (i >= nrec) return;
    const uint8_t* s = src + i * stride + 1;
    uint8_t* d = dst + i * stride + 3;
    for (uint32_t q = j; q + 16 <= len; q += 16 * G) stu<u64x2>(d + q, ldu<u64x2>(s + q));
}

template <typename T>
__global__ void k_field(const uint8_t* src, uint8_t* dst, uint64_t nrec, uint32_t stride) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < nrec) stu<T>(dst + i * stride + 3, ldu<T>(src + i * stride + 1));
}

int main() {
    const uint64_t bytes = 256ull << 20;
    uint8_t *src, *dst;
    hipMalloc(&src, bytes + 4096);
    hipMalloc(&dst, bytes + 4096);
    hipMemset(src, 1, bytes + 4096);
    hipMemset(dst, 0, bytes + 4096);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    auto run = [&](const char* name, double moved, auto&& launch) {
        std::vector<float> ms;
        for (int r = 0; r < 13; ++r) {
            hipEventRecord(a);
            launch();
            hipEventRecord(b);
            hipEventSynchronize(b);
            float t;
            hipEventElapsedTime(&t, a, b);
            if (r >= 3) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double t = ms[ms.size() / 2] * 1e-3;
        printf("%-58s %8.1f us  %7.1f GB/s\n", name, t * 1e6, moved / t / 1e9);
    };
    const uint64_t nch = bytes / 16;
    const dim3 blk(256);
    auto grid = [&](uint64_t threads) { return dim3(static_cast<uint32_t>((threads + 255) / 256)); };
    run("A coalesced 16B, aligned", 2.0 * bytes, [&] { k_coalesced<<<grid(nch), blk>>>(src, dst, nch, 0, 0); });
    run("B coalesced 16B, loads +3", 2.0 * bytes, [&] { k_coalesced<<<grid(nch), blk>>>(src, dst, nch, 3, 0); });
    run("C coalesced 16B, stores +3", 2.0 * bytes, [&] { k_coalesced<<<grid(nch), blk>>>(src, dst, nch, 0, 3); });
    run("B+C coalesced 16B, both unaligned", 2.0 * bytes, [&] { k_coalesced<<<grid(nch), blk>>>(src, dst, nch, 1, 3); });
    for (uint32_t stride : {50u, 64u}) {
        const uint64_t nrec = bytes / stride;
        char nm[96];
        snprintf(nm, sizeof nm, "D 48B record per lane, stride %u", stride);
        run(nm, 2.0 * 48 * nrec, [&] { k_per_lane<<<grid(nrec), blk>>>(src, dst, nrec, stride, 48); });
        snprintf(nm, sizeof nm, "F 48B record per 4-lane group, stride %u", stride);
        run(nm, 2.0 * 48 * nrec, [&] { k_grouped<4><<<grid(nrec * 4), blk>>>(src, dst, nrec, stride, 48); });
        snprintf(nm, sizeof nm, "G 8B field per lane, stride %u", stride);
        run(nm, 2.0 * 8 * nrec, [&] { k_field<uint64_t><<<grid(nrec), blk>>>(src, dst, nrec, stride); });
        snprintf(nm, sizeof nm, "H 1B field per lane, stride %u", stride);
        run(nm, 2.0 * 1 * nrec, [&] { k_field<uint8_t><<<grid(nrec), blk>>>(src, dst, nrec, stride); });
    }
    {
        const uint32_t stride = 528, len = 512;
        const uint64_t nrec = bytes / stride;
        run("E 512B string per lane, stride 528", 2.0 * len * nrec,
            [&] { k_per_lane<<<grid(nrec), blk>>>(src, dst, nrec, stride, len); });
        run("E' 512B string per 32-lane group, stride 528", 2.0 * len * nrec,
            [&] { k_grouped<32><<<grid(nrec * 32), blk>>>(src, dst, nrec, stride, len); });
        run("E'' 512B string per 8-lane group, stride 528", 2.0 * len * nrec,
            [&] { k_grouped<8><<<grid(nrec * 8), blk>>>(src, dst, nrec, stride, len); });
    }
    hipDeviceSynchronize();
    return 0;
}
