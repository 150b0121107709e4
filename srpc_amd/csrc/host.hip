// host.hip -- the host-terminated path (ABI 7): columns and wire bytes in
// HOST memory, the way the reference's batches start and end (packer.hpp's
// byte vector handed to transport.hpp:94-123's socket writes, and the
// received bytes the generated unpack reads).  One call moves a fixed-width
// batch host -> HBM -> kernel -> HBM -> host as a pipeline of chunks over
// three HIP streams (H2D copies / kernels / D2H copies) and a ring of `depth`
// device buffers carved from the caller's scratch, so the H2D of chunk k+1,
// the kernel of chunk k and the D2H of chunk k-1 overlap (PCIe is full
// duplex).  Enqueued natively: a chunk costs a few HIP calls, not a Python
// round of torch copies and events, so chunks can be small enough that the
// pipeline's fill and drain are a small part of the call.
//
// Stream semantics: the call is ordered after the work already on `stream`
// and everything it does is ordered before the work enqueued on `stream`
// after it (the internal streams wait on an event of `stream` first; `stream`
// waits on the last D2H).  The internal streams and events are per host
// thread and device, created once.  Host buffers should be pinned (pageable
// ones work, without overlap).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <map>
#include <vector>

#include "plan.h"
#include "srpc_gpu.h"

namespace srpc_impl {
namespace {

constexpr uint64_t kAlignScratch = 256;

uint64_t r256(uint64_t x) { return (x + kAlignScratch - 1) & ~(kAlignScratch - 1); }

struct Pipe {
    hipStream_t in = nullptr, k = nullptr, out = nullptr;
    hipEvent_t start = nullptr;
    std::vector<hipEvent_t> ev;  // 3 per ring slot: input copied, kernel done, output copied
    bool ok = false;
};

// The calling thread's streams and events on `device` (ring of `depth`).
Pipe* pipe_for(int device, uint32_t depth) {
    thread_local std::map<int, Pipe> pipes;
    Pipe& p = pipes[device];
    if (!p.ok) {
        const unsigned fl = hipStreamNonBlocking;
        if (hipStreamCreateWithFlags(&p.in, fl) != hipSuccess || hipStreamCreateWithFlags(&p.k, fl) != hipSuccess ||
            hipStreamCreateWithFlags(&p.out, fl) != hipSuccess ||
            hipEventCreateWithFlags(&p.start, hipEventDisableTiming) != hipSuccess)
            return nullptr;
        p.ok = true;
    }
    while (p.ev.size() < 3ull * depth) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
        p.ev.push_back(e);
    }
    return &p;
}

// A chunk's status folded into the call's: flags OR'ed, its first failing
// record (chunk-relative) offset by the chunk's first record.
__global__ void k_merge_status(srpc_unpack_status* dst, const srpc_unpack_status* src, uint64_t first) {
    if (threadIdx.x) return;
    const uint32_t f = src->flags;
    if (!f) return;
    atomicOr(&dst->flags, f);
    const uint64_t b = src->first_bad_record;
    if (b != UINT64_MAX) atomicMin(reinterpret_cast<unsigned long long*>(&dst->first_bad_record),
                                   static_cast<unsigned long long>(first + b));
}

__global__ void k_host_status(srpc_unpack_status* st, uint32_t flags, uint64_t first_bad) {
    if (threadIdx.x) return;
    st->flags = flags;
    st->reserved = 0;
    st->first_bad_record = first_bad;
}

// Scratch layout of one ring slot: each column's chunk, the chunk's wire
// bytes, the chunk's status (unpack), every piece 256-byte aligned.
struct SlotLayout {
    uint64_t col[kMaxFields];
    uint64_t wire, status, bytes;
};

SlotLayout slot_layout(const srpc_plan* p, uint64_t chunk) {
    SlotLayout L{};
    uint64_t at = 0;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        L.col[f] = at;
        at += r256(chunk * p->size[f]);
    }
    L.wire = at;
    at += r256(chunk * p->stride);
    L.status = at;
    at += r256(sizeof(srpc_unpack_status));
    L.bytes = at;
    return L;
}

// A/B (SRPC_HOST_STREAMS=2, read per call): the kernels on the H2D stream --
// one cross-stream wait per chunk less (the H2D of the next chunk queues
// behind a kernel of a few microseconds).
bool two_streams() {
    const char* e = std::getenv("SRPC_HOST_STREAMS");
    return e && e[0] == '2';
}

int check_pipe_args(const srpc_plan* p, uint64_t chunk, uint32_t depth) {
    if (!p) return SRPC_E_INVALID;
    if (p->has_string) return SRPC_E_UNSUPPORTED;  // string batches have no fixed chunk size
    if (depth == 0 || depth > 16) return SRPC_E_INVALID;
    if (chunk > (1ull << 40) / p->stride) return SRPC_E_CAPACITY;
    return SRPC_OK;
}

// Direct mode (chunk_records == 0): the device addresses of page-locked,
// device-mapped host buffers (hipHostMalloc / hipHostRegister -- what
// torch's pin_memory allocates), or false when any buffer is not one: the
// kernels then read and write the host memory in place over PCIe, both
// directions at once, with no copies and no chunks.
bool mapped(const void* h, void** d) {
    if (!h) return false;
    hipPointerAttribute_t at{};
    if (hipPointerGetAttributes(&at, h) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    if (at.type != hipMemoryTypeHost) return false;
    if (hipHostGetDevicePointer(d, const_cast<void*>(h), 0) != hipSuccess || !*d) {
        (void)hipGetLastError();
        return false;
    }
    return true;
}

}  // namespace
}  // namespace srpc_impl

using namespace srpc_impl;

extern "C" {

int srpc_plan_host_scratch_bytes(const srpc_plan* p, uint64_t chunk_records, uint32_t depth, uint64_t* out) {
    if (!out) return SRPC_E_INVALID;
    if (int rc = check_pipe_args(p, chunk_records, depth)) return rc;
    *out = chunk_records ? depth * slot_layout(p, chunk_records).bytes : 0;
    return SRPC_OK;
}

int srpc_gpu_pack_host(const srpc_plan* p, const void* const* h_cols, uint64_t n, uint8_t* h_wire,
                       uint64_t wire_cap, uint64_t chunk_records, uint32_t depth, void* d_scratch,
                       uint64_t scratch_bytes, void* stream) {
    if (int rc = check_pipe_args(p, chunk_records, depth)) return rc;
    if (n == 0) return SRPC_OK;
    if (!h_cols || !h_wire) return SRPC_E_INVALID;
    for (uint32_t f = 0; f < p->nfields; ++f)
        if (!h_cols[f]) return SRPC_E_INVALID;
    if (n > UINT64_MAX / p->stride || n * p->stride > wire_cap) return SRPC_E_CAPACITY;
    if (chunk_records == 0) {
        DeviceGuard g(p->device);
        const void* dc[kMaxFields];
        void* dw = nullptr;
        for (uint32_t f = 0; f < p->nfields; ++f) {
            void* d = nullptr;
            if (!mapped(h_cols[f], &d)) return SRPC_E_INVALID;
            dc[f] = d;
        }
        if (!mapped(h_wire, &dw)) return SRPC_E_INVALID;
        return srpc_gpu_pack(p, dc, n, static_cast<uint8_t*>(dw), wire_cap, stream);
    }
    if (!d_scratch) return SRPC_E_INVALID;
    const SlotLayout L = slot_layout(p, chunk_records);
    if (scratch_bytes < depth * L.bytes) return SRPC_E_CAPACITY;
    if (reinterpret_cast<uintptr_t>(d_scratch) % kAlignScratch) return SRPC_E_ALIGN;
    DeviceGuard g(p->device);
    Pipe* P = pipe_for(p->device, depth);
    if (!P) return SRPC_E_HIP;
    const bool two = two_streams();
    hipStream_t ks = two ? P->in : P->k;
    auto s = static_cast<hipStream_t>(stream);
    auto* base = static_cast<uint8_t*>(d_scratch);
    if (hipEventRecord(P->start, s) != hipSuccess) return SRPC_E_HIP;
    for (hipStream_t q : {P->in, P->k, P->out}) (void)hipStreamWaitEvent(q, P->start, 0);
    const uint64_t nch = (n + chunk_records - 1) / chunk_records;
    for (uint64_t i = 0; i < nch; ++i) {
        const uint32_t sl = static_cast<uint32_t>(i % depth);
        hipEvent_t ev_in = P->ev[3 * sl], ev_k = P->ev[3 * sl + 1], ev_out = P->ev[3 * sl + 2];
        uint8_t* slot = base + sl * L.bytes;
        const uint64_t lo = i * chunk_records, cnt = std::min<uint64_t>(chunk_records, n - lo);
        if (i >= depth) {  // the slot's previous chunk: its kernel read the columns, its D2H drained the wire
            if (two) {
                (void)hipStreamWaitEvent(P->in, ev_out, 0);
            } else {
                (void)hipStreamWaitEvent(P->in, ev_k, 0);
                (void)hipStreamWaitEvent(P->k, ev_out, 0);
            }
        }
        const void* dcols[kMaxFields];
        for (uint32_t f = 0; f < p->nfields; ++f) {
            dcols[f] = slot + L.col[f];
            if (hipMemcpyAsync(slot + L.col[f], static_cast<const uint8_t*>(h_cols[f]) + lo * p->size[f],
                               cnt * p->size[f], hipMemcpyHostToDevice, P->in) != hipSuccess)
                return SRPC_E_HIP;
        }
        if (!two) {
            (void)hipEventRecord(ev_in, P->in);
            (void)hipStreamWaitEvent(P->k, ev_in, 0);
        }
        if (int rc = srpc_gpu_pack(p, dcols, cnt, slot + L.wire, cnt * p->stride, ks)) return rc;
        (void)hipEventRecord(ev_k, ks);
        (void)hipStreamWaitEvent(P->out, ev_k, 0);
        if (hipMemcpyAsync(h_wire + lo * p->stride, slot + L.wire, cnt * p->stride, hipMemcpyDeviceToHost, P->out) !=
            hipSuccess)
            return SRPC_E_HIP;
        (void)hipEventRecord(ev_out, P->out);
    }
    // the caller's stream after the last D2H (the copy stream runs them in order)
    (void)hipStreamWaitEvent(s, P->ev[3 * ((nch - 1) % depth) + 2], 0);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int srpc_gpu_unpack_host(const srpc_plan* p, const uint8_t* h_wire, uint64_t wire_len, uint64_t n,
                         void* const* h_cols, uint64_t chunk_records, uint32_t depth, void* d_scratch,
                         uint64_t scratch_bytes, srpc_unpack_status* d_status, void* stream) {
    if (int rc = check_pipe_args(p, chunk_records, depth)) return rc;
    DeviceGuard g(p->device);
    auto s = static_cast<hipStream_t>(stream);
    uint64_t n_fit = wire_len / p->stride;
    int ret = SRPC_OK;
    if (n_fit < n) {
        ret = SRPC_ERR_BOUNDS;
    } else {
        n_fit = n;
    }
    if (d_status) {
        hipLaunchKernelGGL(k_host_status, dim3(1), dim3(64), 0, s, d_status, ret ? SRPC_STATUS_BOUNDS : 0u,
                           ret ? n_fit : UINT64_MAX);
        if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
    }
    if (n_fit == 0) return ret;
    if (!h_cols || !h_wire) return SRPC_E_INVALID;
    for (uint32_t f = 0; f < p->nfields; ++f)
        if (!h_cols[f]) return SRPC_E_INVALID;
    if (chunk_records == 0) {
        void* dc[kMaxFields];
        void* dw = nullptr;
        for (uint32_t f = 0; f < p->nfields; ++f)
            if (!mapped(h_cols[f], &dc[f])) return SRPC_E_INVALID;
        if (!mapped(h_wire, &dw)) return SRPC_E_INVALID;
        const int rc = srpc_gpu_unpack(p, static_cast<const uint8_t*>(dw), wire_len, n, dc, d_status, stream);
        return rc;
    }
    if (!d_scratch) return SRPC_E_INVALID;
    const SlotLayout L = slot_layout(p, chunk_records);
    if (scratch_bytes < depth * L.bytes) return SRPC_E_CAPACITY;
    if (reinterpret_cast<uintptr_t>(d_scratch) % kAlignScratch) return SRPC_E_ALIGN;
    Pipe* P = pipe_for(p->device, depth);
    if (!P) return SRPC_E_HIP;
    const bool two = two_streams();
    hipStream_t ks = two ? P->in : P->k;
    auto* base = static_cast<uint8_t*>(d_scratch);
    if (hipEventRecord(P->start, s) != hipSuccess) return SRPC_E_HIP;
    for (hipStream_t q : {P->in, P->k, P->out}) (void)hipStreamWaitEvent(q, P->start, 0);
    const uint64_t nch = (n_fit + chunk_records - 1) / chunk_records;
    for (uint64_t i = 0; i < nch; ++i) {
        const uint32_t sl = static_cast<uint32_t>(i % depth);
        hipEvent_t ev_in = P->ev[3 * sl], ev_k = P->ev[3 * sl + 1], ev_out = P->ev[3 * sl + 2];
        uint8_t* slot = base + sl * L.bytes;
        const uint64_t lo = i * chunk_records, cnt = std::min<uint64_t>(chunk_records, n_fit - lo);
        if (i >= depth) {  // the slot's previous chunk: its kernel read the wire, its D2H drained the columns
            if (two) {
                (void)hipStreamWaitEvent(P->in, ev_out, 0);
            } else {
                (void)hipStreamWaitEvent(P->in, ev_k, 0);
                (void)hipStreamWaitEvent(P->k, ev_out, 0);
            }
        }
        if (hipMemcpyAsync(slot + L.wire, h_wire + lo * p->stride, cnt * p->stride, hipMemcpyHostToDevice, P->in) !=
            hipSuccess)
            return SRPC_E_HIP;
        if (!two) {
            (void)hipEventRecord(ev_in, P->in);
            (void)hipStreamWaitEvent(P->k, ev_in, 0);
        }
        void* dcols[kMaxFields];
        for (uint32_t f = 0; f < p->nfields; ++f) dcols[f] = slot + L.col[f];
        auto* cst = d_status ? reinterpret_cast<srpc_unpack_status*>(slot + L.status) : nullptr;
        const int rc = srpc_gpu_unpack(p, slot + L.wire, cnt * p->stride, cnt, dcols, cst, ks);
        if (rc != SRPC_OK) return rc;
        if (cst) {
            hipLaunchKernelGGL(k_merge_status, dim3(1), dim3(64), 0, ks, d_status, cst, lo);
            if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
        }
        (void)hipEventRecord(ev_k, ks);
        (void)hipStreamWaitEvent(P->out, ev_k, 0);
        for (uint32_t f = 0; f < p->nfields; ++f)
            if (hipMemcpyAsync(static_cast<uint8_t*>(h_cols[f]) + lo * p->size[f], slot + L.col[f], cnt * p->size[f],
                               hipMemcpyDeviceToHost, P->out) != hipSuccess)
                return SRPC_E_HIP;
        (void)hipEventRecord(ev_out, P->out);
    }
    (void)hipStreamWaitEvent(s, P->ev[3 * ((nch - 1) % depth) + 2], 0);
    return hipGetLastError() == hipSuccess ? ret : SRPC_E_HIP;
}

}  // extern "C"
