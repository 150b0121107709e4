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
//
// Methods with string fields (variable-length frames) take var plans whose
// prefix is `str(method) | str(Req::name)` after the frame's BE32 length: a
// frame is such a plan's when its BE32 is its payload length, the payload
// starts with the prefix, and its fields walk to exactly the frame's end
// (every string length inside the frame) -- the one record of that plan the
// reference server would unpack from it (server.hpp:58-69, packer.hpp:216-222).
// Their payloads are gathered with a record index (srpc_frames_gather_var)
// for srpc_gpu_unpack_var, the packed responses are framed and scattered by
// the response index srpc_gpu_pack_var writes (srpc_frames_scatter_var), and
// the reply stream's offsets are recomputed once those sizes are known
// (srpc_frames_offsets).
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
constexpr int kMaxStr = SRPC_FRAMES_MAX_STRINGS;

struct ClassArgs {
    const uint8_t* prefix[kMaxPlans];  // device prefix of plan k
    uint32_t prefix_len[kMaxPlans];
    uint32_t frame_bytes[kMaxPlans];   // fixed plans: the record bytes (the whole frame); var: the least payload
    uint32_t resp_bytes[kMaxPlans];    // bytes of one response of plan k (0 for var plans)
    // var plans: fixed bytes before string s's length word (after the prefix or
    // the previous string's chars), gap[k][nstr[k]] = fixed bytes after the last
    uint16_t gap[kMaxPlans][kMaxStr + 1];
    uint8_t nstr[kMaxPlans];           // 0: a fixed plan
    uint32_t nplans;
};

__device__ __forceinline__ uint32_t be32_at(const uint8_t* b) {
    return (static_cast<uint32_t>(b[0]) << 24) | (static_cast<uint32_t>(b[1]) << 16) |
           (static_cast<uint32_t>(b[2]) << 8) | static_cast<uint32_t>(b[3]);
}

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
            const uint32_t ns = a.nstr[p];
            const uint64_t len = end - o;
            if (ns == 0 ? len != a.frame_bytes[p] : (len < 4 + uint64_t{a.frame_bytes[p]} || be32_at(buf + o) != len - 4))
                continue;
            const uint64_t at = ns ? o + 4 : o;  // var plans: the prefix follows the BE32 length
            if (a.prefix_len[p] > end - at) continue;
            const uint8_t* f = buf + at;
            const uint8_t* q = a.prefix[p];
            bool eq = true;
            uint32_t b = 0;
            for (; b + 8 <= a.prefix_len[p] && eq; b += 8) eq = ldu<uint64_t>(f + b) == ldu<uint64_t>(q + b);
            for (; b < a.prefix_len[p] && eq; ++b) eq = f[b] == q[b];
            if (eq && ns) {  // the record's walk ends exactly at the frame's end
                uint64_t c = at + a.prefix_len[p];
                for (uint32_t t = 0; t < ns && eq; ++t) {
                    c += a.gap[p][t];
                    if (c + 8 > end) {
                        eq = false;
                        break;
                    }
                    const uint64_t sl = ldu<uint64_t>(buf + c);
                    c += 8;
                    if (sl > end - c) eq = false;
                    else c += sl;
                }
                eq = eq && c + a.gap[p][ns] == end;
            }
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

// Payload bytes (the frame after its BE32) of bucket record j.
__global__ __launch_bounds__(kBlock) void k_payload_lens(const uint8_t* __restrict__ buf, const uint32_t* __restrict__ offs,
                                                         const uint32_t* __restrict__ index, uint64_t n,
                                                         uint32_t* __restrict__ lens) {
    const uint64_t j = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (j < n) lens[j] = be32_at(buf + offs[index[j]]);
}

// A wave per record (grid-stride): payload j -> out + rec_offs[j].
__global__ __launch_bounds__(kBlock) void k_gather_var(const uint8_t* __restrict__ buf, const uint32_t* __restrict__ offs,
                                                       const uint32_t* __restrict__ index, uint64_t n,
                                                       const uint64_t* __restrict__ rec_offs, uint8_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
    for (uint64_t j = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + threadIdx.x / 64; j < n; j += waves) {
        const uint8_t* src = buf + offs[index[j]] + 4;
        const uint64_t o = rec_offs[j], len = rec_offs[j + 1] - o;
        for (uint64_t b = lane; b < len; b += 64) out[o + b] = src[b];
    }
}

// A wave per response (grid-stride): BE32(len) | response j at out + out_off[index[j]].
__global__ __launch_bounds__(kBlock) void k_scatter_var(const uint8_t* __restrict__ resp,
                                                        const uint64_t* __restrict__ rec_offs,
                                                        const uint32_t* __restrict__ index, uint64_t n,
                                                        const uint64_t* __restrict__ out_off, uint8_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t waves = static_cast<uint64_t>(gridDim.x) * (kBlock / 64);
    for (uint64_t j = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + threadIdx.x / 64; j < n; j += waves) {
        const uint64_t r = rec_offs[j], len = rec_offs[j + 1] - r;
        uint8_t* dst = out + out_off[index[j]];
        if (lane < 4) dst[lane] = static_cast<uint8_t>(len >> (8 * (3 - lane)));
        for (uint64_t b = lane; b < len; b += 64) dst[4 + b] = resp[r + b];
    }
}

struct VarOffs {
    const uint64_t* rec[kMaxPlans];  // response index of var plan k (NULL: a fixed plan)
};

// Response bytes of every frame: resp_bytes[k] for a fixed plan's frame, 0 for
// an unknown one (var plans' frames: k_var_sizes).
__global__ __launch_bounds__(kBlock) void k_fixed_sizes(const uint8_t* __restrict__ cls, uint64_t nf, ClassArgs a,
                                                        uint32_t* __restrict__ sizes) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= nf) return;
    const uint32_t c = cls[i];
    sizes[i] = c < a.nplans && a.nstr[c] == 0 ? a.resp_bytes[c] : 0;
}

// blockIdx.y = plan: BE32 + response bytes of each frame of a var plan's bucket.
__global__ __launch_bounds__(kBlock) void k_var_sizes(const uint32_t* __restrict__ index, uint64_t nf,
                                                      const uint64_t* __restrict__ counts, VarOffs v,
                                                      uint32_t* __restrict__ sizes) {
    const uint32_t k = blockIdx.y;
    const uint64_t* rec = v.rec[k];
    if (!rec) return;
    const uint64_t nk = counts[k];
    for (uint64_t j = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; j < nk;
         j += static_cast<uint64_t>(gridDim.x) * kBlock)
        sizes[index[k * nf + j]] = static_cast<uint32_t>(4 + rec[j + 1] - rec[j]);
}

__global__ void k_zero_counts(uint64_t* c, uint32_t n) {
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) c[i] = 0;
}

// The plans' match rules (see the file comment); SRPC_E_INVALID for a plan
// without a prefix, SRPC_E_UNSUPPORTED past SRPC_FRAMES_MAX_STRINGS strings.
int class_args(const srpc_plan* const* plans, const uint32_t* resp_bytes, int nplans, ClassArgs* a) {
    for (int k = 0; k < nplans; ++k) {
        const srpc_plan* p = plans[k];
        if (!p || p->prefix_len == 0) return SRPC_E_INVALID;
        a->prefix[k] = p->d_prefix;
        a->prefix_len[k] = p->prefix_len;
        if (!p->has_string) {
            a->frame_bytes[k] = static_cast<uint32_t>(p->stride);
            a->resp_bytes[k] = resp_bytes ? resp_bytes[k] : 0;
            continue;
        }
        if (p->nstrings > static_cast<uint32_t>(kMaxStr)) return SRPC_E_UNSUPPORTED;
        a->frame_bytes[k] = p->fixed_bytes;
        a->nstr[k] = static_cast<uint8_t>(p->nstrings);
        uint32_t t = 0, run = 0;
        for (uint32_t f = 0; f < p->nfields; ++f) {
            if (p->kinds[f] == SRPC_KIND_STRING) {
                a->gap[k][t++] = static_cast<uint16_t>(run);
                run = 0;
            } else {
                run += p->size[f];
            }
        }
        a->gap[k][t] = static_cast<uint16_t>(run);
    }
    a->nplans = static_cast<uint32_t>(nplans);
    return SRPC_OK;
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
    if (int rc = class_args(req_plans, resp_bytes, nplans, &a)) return rc;
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

int srpc_frames_gather_var(const uint8_t* d_buf, const uint32_t* d_offs, const uint32_t* d_index, uint64_t n,
                           uint8_t* d_out, uint64_t* d_rec_offs, void* d_scratch, uint64_t scratch_bytes,
                           void* stream) {
    if (!d_rec_offs || (n && (!d_buf || !d_offs || !d_index || !d_out))) return SRPC_E_INVALID;
    uint64_t need = 0;
    srpc_frames_scratch_bytes(n, 1, &need);
    if (!d_scratch || scratch_bytes < need || !aligned(d_scratch, 8)) return SRPC_E_CAPACITY;
    if (!aligned(d_rec_offs, 8)) return SRPC_E_ALIGN;
    auto s = static_cast<hipStream_t>(stream);
    auto* lens = static_cast<uint32_t*>(d_scratch);
    auto* part = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(d_scratch) + ((4 * n + 7) & ~7ull));
    if (n) hipLaunchKernelGGL(k_payload_lens, dim3(grid_for(n, kBlock)), dim3(kBlock), 0, s, d_buf, d_offs, d_index, n, lens);
    xscan(static_cast<const uint32_t*>(lens), n, part, part + xscan_parts(n), d_rec_offs, s);
    if (n)
        hipLaunchKernelGGL(k_gather_var, dim3(grid_for(n, kBlock / 64)), dim3(kBlock), 0, s, d_buf, d_offs, d_index, n,
                           static_cast<const uint64_t*>(d_rec_offs), d_out);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int srpc_frames_scatter_var(const uint8_t* d_resp, const uint64_t* d_rec_offs, const uint32_t* d_index, uint64_t n,
                            const uint64_t* d_out_off, uint8_t* d_out, void* stream) {
    if (!n) return SRPC_OK;
    if (!d_resp || !d_rec_offs || !d_index || !d_out_off || !d_out) return SRPC_E_INVALID;
    hipLaunchKernelGGL(k_scatter_var, dim3(grid_for(n, kBlock / 64)), dim3(kBlock), 0, static_cast<hipStream_t>(stream),
                       d_resp, d_rec_offs, d_index, n, d_out_off, d_out);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int srpc_frames_offsets(const srpc_plan* const* req_plans, const uint32_t* resp_bytes, int nplans,
                        const uint8_t* d_class, uint64_t nframes, const uint32_t* d_index, const uint64_t* d_counts,
                        const uint64_t* const* d_var_rec_offs, uint64_t* d_out_off, uint64_t* d_total,
                        void* d_scratch, uint64_t scratch_bytes, void* stream) {
    if (!req_plans || !resp_bytes || nplans <= 0 || nplans > kMaxPlans || !d_counts || !d_out_off || !d_total ||
        !d_var_rec_offs)
        return SRPC_E_INVALID;
    uint64_t need = 0;
    srpc_frames_scratch_bytes(nframes, nplans, &need);
    if (!d_scratch || scratch_bytes < need || !aligned(d_scratch, 8)) return SRPC_E_CAPACITY;
    if (nframes && (!d_class || !d_index)) return SRPC_E_INVALID;
    if (nframes > 0xffffffffull) return SRPC_E_UNSUPPORTED;
    ClassArgs a{};
    if (int rc = class_args(req_plans, resp_bytes, nplans, &a)) return rc;
    VarOffs v{};
    for (int k = 0; k < nplans; ++k) {
        if (a.nstr[k] && !d_var_rec_offs[k]) return SRPC_E_INVALID;
        v.rec[k] = a.nstr[k] ? d_var_rec_offs[k] : nullptr;
    }
    auto s = static_cast<hipStream_t>(stream);
    auto* sizes = static_cast<uint32_t*>(d_scratch);
    auto* part = reinterpret_cast<uint64_t*>(static_cast<uint8_t*>(d_scratch) + ((4 * nframes + 7) & ~7ull));
    if (nframes) {
        hipLaunchKernelGGL(k_fixed_sizes, dim3(grid_for(nframes, kBlock)), dim3(kBlock), 0, s, d_class, nframes, a, sizes);
        hipLaunchKernelGGL(k_var_sizes, dim3(std::min<uint32_t>(grid_for(nframes, kBlock), 1024), nplans), dim3(kBlock), 0,
                           s, d_index, nframes, d_counts, v, sizes);
    }
    xscan(static_cast<const uint32_t*>(sizes), nframes, part, d_total, d_out_off, s);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

}  // extern "C"
