// Microbenchmark: cost of LDS accesses at unaligned addresses on gfx950.
// One workgroup per CU, 256 threads; each lane copies 16 (or 8) bytes
// LDS->LDS per iteration at byte offset `mis` from 16-byte alignment, with a
// per-lane stride of `stride` bytes.  Prints cycles per wave-iteration.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int W>
__global__ __launch_bounds__(256) void k(uint32_t mis, uint32_t stride, uint32_t iters, uint64_t* out) {
    __shared__ __attribute__((aligned(16))) uint8_t buf[65536];
    for (uint32_t i = threadIdx.x; i < 65536; i += 256) buf[i] = static_cast<uint8_t>(i);
    __syncthreads();
    const uint32_t lane = threadIdx.x;
    uint32_t src = (lane * stride) % 28672 + mis, dst = 32768 + (lane * stride) % 28672 + mis;
    const uint64_t t0 = clock64();
    for (uint32_t it = 0; it < iters; ++it) {
        if constexpr (W == 16) {
            uint4 v;
            __builtin_memcpy(&v, buf + src, 16);
            v.x += it;
            __builtin_memcpy(buf + dst, &v, 16);
        } else if constexpr (W == 8) {
            uint2 v;
            __builtin_memcpy(&v, buf + src, 8);
            v.x += it;
            __builtin_memcpy(buf + dst, &v, 8);
        } else {
            uint32_t v;
            __builtin_memcpy(&v, buf + src, 4);
            v += it;
            __builtin_memcpy(buf + dst, &v, 4);
        }
        src = (src + 64) & 32767;
        dst = 32768 + ((dst + 64) & 32767);
    }
    __syncthreads();
    const uint64_t t1 = clock64();
    if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0 + buf[lane];
}

int main() {
    uint64_t* d;
    hipMalloc(&d, 256 * 8);
    uint64_t h[256];
    const uint32_t iters = 4096;
    for (int w : {4, 8, 16}) {
        for (uint32_t stride : {16u, 48u, 50u}) {
            for (uint32_t mis : {0u, 1u, 4u, 8u}) {
                if (w == 4) hipLaunchKernelGGL(k<4>, dim3(256), dim3(256), 0, 0, mis, stride, iters, d);
                if (w == 8) hipLaunchKernelGGL(k<8>, dim3(256), dim3(256), 0, 0, mis, stride, iters, d);
                if (w == 16) hipLaunchKernelGGL(k<16>, dim3(256), dim3(256), 0, 0, mis, stride, iters, d);
                hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
                uint64_t s = 0;
                for (int i = 0; i < 256; ++i) s += h[i];
                printf("width %2d stride %2u misalign %u: %.1f cycles per iteration (4 waves)\n", w, stride, mis,
                       double(s) / 256 / iters);
            }
        }
    }
    return 0;
}
