// frames.hip -- server-side batches of framed requests of several methods
// (SURVEY §8 f1).  The reference server dispatches every request by its
// method name (server.hpp:58-69: recv_data -> `>> funcname` -> call); a batch
// read from a socket holds frames of any registered method, in any order.
// srpc_frames_classify buckets such a batch on the GPU: frame i belongs to
// request plan k when it is exactly one record of that plan (its length is
// the plan's record bytes and it starts with the plan's constant prefix --
// BE32 length | str(method) | str(Req::name) for a framed request plan), the
// first matching plan winning.  Each bucket is then gathered into a
// contiguous batch for the plan's ordinary unpack, and the packed responses
// are scattered back into request order (srpc_frames_gather / _scatter).
// Frames no plan matches are left to the caller (the CPU server).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "plan.h"
#include "scan.h"
#include "srpc_gpu.h"

namespace srpc_impl {
namespace {

constexpr uint32_t kNoClass = SRPC_FRAME_UNKNOWN;
constexpr int kMaxPlans = SRPC_FRAMES_MAX_PLANS;

struct ClassArgs {
    const uint8_t* prefix[kMaxPlans];  // device prefix of plan k
    uint32_t prefix_len[kMaxPlans];
    uint32_t frame_bytes[kMaxPlans];   // the plan's record bytes (the whole frame)
    uint32_t resp_bytes[kMaxPlans];    // bytes of one response of plan k
    uint32_t nplans;
};

template <typename T>
__device__ __forceinline__ T ldu(const uint8_t* p) {
    T v;
    __builtin_memcpy(&v, p, sizeof(T));
    return v;
}

// One lane per frame: class, bucket slot (wave-aggregated atomics: one add per
// wave and plan), response bytes; block sums of the response bytes.
__global__ __launch_bounds__(kBlock) void k_classify(ClassArgs a, const uint8_t* __restrict__ buf, uint64_t buf_len,
                                                     const uint32_t* __restrict__ offs, uint64_t nf,
                                                     uint8_t* __restrict__ cls, uint32_t* __restrict__ index,
                                                     uint64_t* __restrict__ counts, uint32_t* __restrict__ rb) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    uint32_t k = kNoClass;
    if (i < nf) {
        const uint64_t o = offs[i];
        const uint64_t end = i + 1 < nf ? offs[i + 1] : buf_len;
        // offsets out of order or past the buffer: the frame is no plan's (the
        // caller answers it), and no byte outside [0, buf_len) is read
        const bool inside = o <= end && end <= buf_len;
        for (uint32_t p = 0; inside && p < a.nplans && k == kNoClass; ++p) {
            if (end - o != a.frame_bytes[p] || a.prefix_len[p] > end - o) continue;
            const uint8_t* f = buf + o;
            const uint8_t* q = a.prefix[p];
            bool eq = true;
            uint32_t b = 0;
            for (; b + 8 <= a.prefix_len[p] && eq; b += 8) eq = ldu<uint64_t>(f + b) == ldu<uint64_t>(q + b);
            for (; b < a.prefix_len[p] && eq; ++b) eq = f[b] == q[b];
            if (eq) k = p;
        }
        cls[i] = static_cast<uint8_t>(k);
        rb[i] = k == kNoClass ? 0 : a.resp_bytes[k];
    }
    // bucket slots: per plan, the wave's matching lanes take consecutive slots
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t p = 0; p < a.nplans; ++p) {
        const uint64_t m = __ballot(k == p);
        if (!m) continue;
        const uint32_t leader = __builtin_ctzll(m);
        uint64_t base = 0;
        if (lane == leader) base = atomicAdd(reinterpret_cast<unsigned long long*>(&counts[p]),
                                             static_cast<unsigned long long>(__popcll(m)));
        base = __shfl(base, leader, 64);
        if (k == p) index[p * nf + base + __popcll(m & ((1ull << lane) - 1))] = static_cast<uint32_t>(i);
    }
    const uint64_t mu = __ballot(i < nf && k == kNoClass);
    if (mu && lane == __builtin_ctzll(mu))
        atomicAdd(reinterpret_cast<unsigned long long*>(&counts[a.nplans + 1]), static_cast<unsigned long long>(__popcll(mu)));
}

// Bucket -> contiguous batch: 4 bytes per lane of the output (n records of
// rec bytes); record j is frame index[j].
__global__ __launch_bounds__(kBlock) void k_gather(const uint8_t* __restrict__ buf, const uint32_t* __restrict__ offs,
                                                   const uint32_t* __restrict__ index, uint64_t n, uint32_t rec,
                                                   uint8_t* __restrict__ out) {
    const uint64_t total = n * rec;
    const uint64_t gs = static_cast<uint64_t>(gridDim.x) * kBlock * 4;
    for (uint64_t x = (static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x) * 4; x < total; x += gs) {
        uint32_t w = 0;
        for (uint32_t b = 0; b < 4 && x + b < total; ++b) {
            const uint64_t j = (x + b) / rec, k = (x + b) - j * rec;
            w |= static_cast<uint32_t>(buf[offs[index[j]] + k]) << (8 * b);
        }
        if (x + 4 <= total) *reinterpret_cast<uint32_t*>(out + x) = w;
        else
            for (uint32_t b = 0; x + b < total; ++b) out[x + b] = static_cast<uint8_t>(w >> (8 * b));
    }
}

// Packed responses (n records of rec bytes) -> their frames' places.
__global__ __launch_bounds__(kBlock) void k_scatter(const uint8_t* __restrict__ resp, const uint32_t* __restrict__ index,
                                                    uint64_t n, uint32_t rec, const uint64_t* __restrict__ out_off,
                                                    uint8_t* __restrict__ out) {
    const uint64_t total = n * rec;
    const uint64_t gs = static_cast<uint64_t>(gridDim.x) * kBlock;
    for (uint64_t x = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; x < total; x += gs) {
        const uint64_t j = x / rec, k = x - j * rec;
        out[out_off[index[j]] + k] = resp[x];
    }
}

__global__ void k_zero_counts(uint64_t* c, uint32_t n) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) c[i] = 0;
}

uint32_t grid_for(uint64_t work, uint64_t per) {
    return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>((work + per - 1) / per, 1u << 20)));
}

}  // namespace
}  // namespace srpc_impl

using namespace srpc_impl;

extern "C" {

int srpc_frames_scratch_bytes(uint64_t nframes, int nplans, uint64_t* out) {
    if (!out || nplans <= 0 || nplans > kMaxPlans) return SRPC_E_INVALID;
    *out = 4 * nframes + 8 * xscan_parts(nframes) + 256;
    return SRPC_OK;
}

int srpc_frames_classify(const srpc_plan* const* req_plans, const uint32_t* resp_bytes, int nplans,
                         const uint8_t* d_buf, uint64_t buf_len, const uint32_t* d_offs, uint64_t nframes,
                         uint8_t* d_class, uint32_t* d_index, uint64_t* d_counts, uint64_t* d_out_off,
                         void* d_scratch, uint64_t scratch_bytes, void* stream) {
    if (!req_plans || !resp_bytes || nplans <= 0 || nplans > kMaxPlans || !d_counts || !d_out_off) return SRPC_E_INVALID;
    uint64_t need = 0;
    srpc_frames_scratch_bytes(nframes, nplans, &need);
    if (!d_scratch || scratch_bytes < need || !aligned(d_scratch, 8)) return SRPC_E_CAPACITY;
    if (nframes && (!d_buf || !d_offs || !d_class || !d_index)) return SRPC_E_INVALID;
    if (nframes > 0xffffffffull) return SRPC_E_UNSUPPORTED;
    ClassArgs a{};
    for (int k = 0; k < nplans; ++k) {
        const srpc_plan* p = req_plans[k];
        if (!p || p->has_string || p->prefix_len == 0) return SRPC_E_INVALID;  // fixed-size framed plans
        a.prefix[k] = p->d_prefix;
        a.prefix_len[k] = p->prefix_len;
        a.frame_bytes[k] = static_cast<uint32_t>(p->stride);
        a.resp_bytes[k] = resp_bytes[k];
    }
    a.nplans = static_cast<uint32_t>(nplans);
    auto s = static_cast<hipStream_t>(stream);
    auto* rb = static_cast<uint32_t*>(d_scratch);
    auto* part = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(d_scratch) + ((4 * nframes + 7) & ~7ull));
    hipLaunchKernelGGL(k_zero_counts, dim3(1), dim3(64), 0, s, d_counts, static_cast<uint32_t>(nplans + 2));
    if (nframes) {
        hipLaunchKernelGGL(k_classify, dim3(grid_for(nframes, kBlock)), dim3(kBlock), 0, s, a, d_buf, buf_len, d_offs,
                           nframes, d_class, d_index, d_counts, rb);
    }
    xscan(static_cast<const uint32_t*>(rb), nframes, part, d_counts + nplans, d_out_off, s);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int srpc_frames_gather(const uint8_t* d_buf, const uint32_t* d_offs, const uint32_t* d_index, uint64_t n,
                       uint32_t record_bytes, uint8_t* d_out, void* stream) {
    if (!n) return SRPC_OK;
    if (!d_buf || !d_offs || !d_index || !d_out || !record_bytes) return SRPC_E_INVALID;
    hipLaunchKernelGGL(k_gather, dim3(grid_for(n * record_bytes, kBlock * 4)), dim3(kBlock), 0,
                       static_cast<hipStream_t>(stream), d_buf, d_offs, d_index, n, record_bytes, d_out);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int srpc_frames_scatter(const uint8_t* d_resp, const uint32_t* d_index, uint64_t n, uint32_t record_bytes,
                        const uint64_t* d_out_off, uint8_t* d_out, void* stream) {
    if (!n) return SRPC_OK;
    if (!d_resp || !d_index || !d_out_off || !d_out || !record_bytes) return SRPC_E_INVALID;
    hipLaunchKernelGGL(k_scatter, dim3(grid_for(n * record_bytes, kBlock)), dim3(kBlock), 0,
                       static_cast<hipStream_t>(stream), d_resp, d_index, n, record_bytes, d_out_off, d_out);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

}  // extern "C"
