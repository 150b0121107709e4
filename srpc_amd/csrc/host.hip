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
// waits on the last D2H; after an error part way through, on everything the
// call enqueued).  The internal streams and events come from a per-device pool
// (a call borrows a pipe and returns it), created on first use.  Host buffers
// should be pinned (pageable ones work, without overlap).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdint>
#include <map>
#include <mutex>
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
    hipEvent_t fence[3] = {};    // an error's drain: the last work of each internal stream
    hipStream_t caller = nullptr;  // the caller stream of the call that last used it
    std::vector<hipEvent_t> ev;  // 3 per ring slot: input copied, kernel done, output copied
};

// Pipes are pooled per device: a call borrows one and returns
// it once its work is ENQUEUED, but a returned pipe may still be moving that
// call's bytes for milliseconds.  So a call takes, in order:
// a free pipe last used with its own caller stream (its work is ordered
// behind that stream's earlier calls anyway: nothing is serialised that was
// not already), else a free pipe whose streams are idle (hipStreamQuery of
// each), else a new pipe.  Calls on different caller streams therefore
// never queue their copies behind each other on shared internal streams while
// the other's are in flight; the pool grows to the number of calls in flight
// at once, not with the threads that made them, and a thread that exits
// leaks nothing.  Pipes live for the process (destroying streams while HIP
// tears down at exit is not safe).
struct PipePool {
    std::mutex mu;
    std::map<int, std::vector<Pipe*>> free;
    std::map<int, uint64_t> made;
};
PipePool& pool() {
    static PipePool* P = new PipePool;  // never destroyed (see above)
    return *P;
}

Pipe* make_pipe() {
    auto* p = new Pipe;
    const unsigned fl = hipStreamNonBlocking;
    bool ok = hipStreamCreateWithFlags(&p->in, fl) == hipSuccess && hipStreamCreateWithFlags(&p->k, fl) == hipSuccess &&
              hipStreamCreateWithFlags(&p->out, fl) == hipSuccess &&
              hipEventCreateWithFlags(&p->start, hipEventDisableTiming) == hipSuccess;
    for (auto& e : p->fence) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    if (ok) return p;
    for (hipStream_t q : {p->in, p->k, p->out})
        if (q) (void)hipStreamDestroy(q);
    for (hipEvent_t e : {p->start, p->fence[0], p->fence[1], p->fence[2]})
        if (e) (void)hipEventDestroy(e);
    delete p;
    (void)hipGetLastError();
    return nullptr;
}

// True when every piece of work enqueued on the pipe's streams has run.  (Not
// by events recorded at the pipe's return: with those, the reuse test saw a
// new pipe made after a device synchronize, i.e. no idle pipe found.)  A
// not-ready query leaves no error behind for the call's final hipGetLastError.
bool pipe_idle(Pipe* p) {
    for (hipStream_t q : {p->in, p->k, p->out}) {
        if (hipStreamQuery(q) == hipSuccess) continue;
        (void)hipGetLastError();
        return false;
    }
    return true;
}

thread_local const Pipe* t_last_pipe = nullptr;  // test hook: the pipe this thread's last call used

// A pipe of `device` (the current device) with a ring of `depth` for a call
// on `caller`, returned by ~Lease (see the pool's comment for the choice).
struct Lease {
    int device;
    hipStream_t caller;
    Pipe* p = nullptr;
    Lease(int dev, uint32_t depth, hipStream_t s) : device(dev), caller(s) {
        {
            std::lock_guard<std::mutex> lk(pool().mu);
            auto& v = pool().free[dev];
            size_t pick = v.size();
            for (size_t i = 0; i < v.size() && pick == v.size(); ++i)
                if (v[i]->caller == s) pick = i;
            for (size_t i = 0; i < v.size() && pick == v.size(); ++i)
                if (pipe_idle(v[i])) pick = i;
            if (pick < v.size()) {
                p = v[pick];
                v.erase(v.begin() + static_cast<std::ptrdiff_t>(pick));
            }
        }
        if (!p) {
            p = make_pipe();
            if (!p) return;
            std::lock_guard<std::mutex> lk(pool().mu);
            ++pool().made[dev];
        }
        t_last_pipe = p;
        while (p->ev.size() < 3ull * depth) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
                release();
                return;
            }
            p->ev.push_back(e);
        }
    }
    void release() {
        if (!p) return;
        p->caller = caller;
        std::lock_guard<std::mutex> lk(pool().mu);
        pool().free[device].push_back(p);
        p = nullptr;
    }
    ~Lease() { release(); }
};

// The chunked ring records events on `stream` and makes the pool's streams
// wait on them: inside a stream capture that would pull the pool's streams
// into the caller's graph (and a later call's copies with them), so the
// chunked mode refuses a capturing stream instead (SRPC_E_UNSUPPORTED).
bool capturing(hipStream_t s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return cs != hipStreamCaptureStatusNone;
}

// After an error part way through a ring: `stream` waits on everything already
// enqueued on the internal streams, so a caller that sees the error and then
// reuses its host buffers or scratch (in stream order) cannot race copies that
// are still in flight into them.  Returns rc.
int drain(Pipe* P, hipStream_t s, int rc) {
    hipStream_t q[3] = {P->in, P->k, P->out};
    for (int i = 0; i < 3; ++i)
        if (hipEventRecord(P->fence[i], q[i]) == hipSuccess) (void)hipStreamWaitEvent(s, P->fence[i], 0);
    return rc;
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

// Test hook (srpc_debug_host_fail_at(k), not in include/; off unless a test
// arms it): the chunked ring fails at chunk k as a HIP error would, after
// chunks 0..k-1 are enqueued -- the error path's drain is tested with copies
// really in flight.  Nothing in the environment can make a real call fail.
std::atomic<uint64_t> g_fail_at{UINT64_MAX};
uint64_t fail_at() { return g_fail_at.load(std::memory_order_relaxed); }

int check_pipe_args(const srpc_plan* p, uint64_t chunk, uint32_t depth) {
    if (!p) return SRPC_E_INVALID;
    if (p->has_string) return SRPC_E_UNSUPPORTED;  // string batches have no fixed chunk size
    if (depth == 0 || depth > 16) return SRPC_E_INVALID;
    if (chunk > (1ull << 40) / p->stride) return SRPC_E_CAPACITY;
    return SRPC_OK;
}

// Direct mode (chunk_records == 0): the device address of a page-locked,
// device-mapped host buffer (hipHostMalloc / hipHostRegister -- what torch's
// pin_memory allocates) whose allocation covers [h, h + bytes), or false: the
// kernels then read and write the host memory in place over PCIe, both
// directions at once, with no copies and no chunks.  The allocation's range
// is the runtime's own record of the pinned block (hipMemGetAddressRange), so
// a buffer shorter than the batch is refused instead of being read or written
// past its end.
bool mapped(const void* h, uint64_t bytes, void** d) {
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
    // the allocation's range, asked of the runtime four ways (hipHostMalloc
    // blocks answer the first; hipHostRegister'ed ranges may answer only the
    // pointer attributes), each in the address space it was asked in
    const void* at_ptr[2] = {*d, h};
    for (int i = 0; i < 4; ++i) {
        const void* q = at_ptr[i & 1];
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        bool ok;
        if (i < 2) {
            ok = hipMemGetAddressRange(&base, &size, const_cast<void*>(q)) == hipSuccess;
        } else {
            ok = hipPointerGetAttribute(&base, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                                        reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(q))) == hipSuccess &&
                 hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                                        reinterpret_cast<hipDeviceptr_t>(const_cast<void*>(q))) == hipSuccess;
        }
        if (!ok) (void)hipGetLastError();
        if (!ok || !base || !size) continue;
        const uintptr_t b = reinterpret_cast<uintptr_t>(base), lo = reinterpret_cast<uintptr_t>(q);
        if (lo < b || lo - b > size) continue;  // an answer about another range
        return bytes <= size - (lo - b);
    }
    return false;
}

__global__ void k_or_bounds(srpc_unpack_status* st, uint64_t at) {
    if (threadIdx.x) return;
    atomicOr(&st->flags, SRPC_STATUS_BOUNDS);
    atomicMin(reinterpret_cast<unsigned long long*>(&st->first_bad_record), static_cast<unsigned long long>(at));
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

// Every argument is checked before anything is enqueued; an error part way
// through the ring drains what was enqueued into `stream` (drain()).
int srpc_gpu_pack_host(const srpc_plan* p, const void* const* h_cols, uint64_t n, uint8_t* h_wire,
                       uint64_t wire_cap, uint64_t chunk_records, uint32_t depth, void* d_scratch,
                       uint64_t scratch_bytes, void* stream) {
    if (int rc = check_pipe_args(p, chunk_records, depth)) return rc;
    if (n == 0) return SRPC_OK;
    if (!h_cols || !h_wire) return SRPC_E_INVALID;
    for (uint32_t f = 0; f < p->nfields; ++f)
        if (!h_cols[f]) return SRPC_E_INVALID;
    if (n > UINT64_MAX / p->stride || n * p->stride > wire_cap) return SRPC_E_CAPACITY;
    DeviceGuard g(p->device);
    if (chunk_records == 0) {
        const void* dc[kMaxFields];
        void* dw = nullptr;
        for (uint32_t f = 0; f < p->nfields; ++f) {
            void* d = nullptr;
            if (!mapped(h_cols[f], n * p->size[f], &d)) return SRPC_E_INVALID;
            dc[f] = d;
        }
        if (!mapped(h_wire, n * p->stride, &dw)) return SRPC_E_INVALID;
        return srpc_gpu_pack(p, dc, n, static_cast<uint8_t*>(dw), n * p->stride, stream);
    }
    if (!d_scratch) return SRPC_E_INVALID;
    const SlotLayout L = slot_layout(p, chunk_records);
    if (scratch_bytes < depth * L.bytes) return SRPC_E_CAPACITY;
    if (reinterpret_cast<uintptr_t>(d_scratch) % kAlignScratch) return SRPC_E_ALIGN;
    auto s = static_cast<hipStream_t>(stream);
    if (capturing(s)) return SRPC_E_UNSUPPORTED;
    Lease lease(p->device, depth, s);
    Pipe* P = lease.p;
    if (!P) return SRPC_E_HIP;
    const bool two = two_streams();
    hipStream_t ks = two ? P->in : P->k;
    auto* base = static_cast<uint8_t*>(d_scratch);
    if (hipEventRecord(P->start, s) != hipSuccess) return SRPC_E_HIP;
    for (hipStream_t q : {P->in, P->k, P->out}) (void)hipStreamWaitEvent(q, P->start, 0);
    const uint64_t nch = (n + chunk_records - 1) / chunk_records, fail = fail_at();
    for (uint64_t i = 0; i < nch; ++i) {
        if (i == fail) return drain(P, s, SRPC_E_HIP);
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
                return drain(P, s, SRPC_E_HIP);
        }
        if (!two) {
            (void)hipEventRecord(ev_in, P->in);
            (void)hipStreamWaitEvent(P->k, ev_in, 0);
        }
        if (int rc = srpc_gpu_pack(p, dcols, cnt, slot + L.wire, cnt * p->stride, ks)) return drain(P, s, rc);
        (void)hipEventRecord(ev_k, ks);
        (void)hipStreamWaitEvent(P->out, ev_k, 0);
        if (hipMemcpyAsync(h_wire + lo * p->stride, slot + L.wire, cnt * p->stride, hipMemcpyDeviceToHost, P->out) !=
            hipSuccess)
            return drain(P, s, SRPC_E_HIP);
        (void)hipEventRecord(ev_out, P->out);
    }
    // the caller's stream after the last D2H (the copy stream runs them in order)
    (void)hipStreamWaitEvent(s, P->ev[3 * ((nch - 1) % depth) + 2], 0);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

// A wire shorter than n records: the records that fit are decoded, SRPC_ERR_
// BOUNDS is returned and the status says BOUNDS at record n_fit (srpc_gpu_
// unpack's own semantics, in either mode).
int srpc_gpu_unpack_host(const srpc_plan* p, const uint8_t* h_wire, uint64_t wire_len, uint64_t n,
                         void* const* h_cols, uint64_t chunk_records, uint32_t depth, void* d_scratch,
                         uint64_t scratch_bytes, srpc_unpack_status* d_status, void* stream) {
    if (int rc = check_pipe_args(p, chunk_records, depth)) return rc;
    uint64_t n_fit = wire_len / p->stride;
    const int ret = n_fit < n ? SRPC_ERR_BOUNDS : SRPC_OK;
    n_fit = std::min(n_fit, n);
    // arguments first: nothing is launched for a call that returns SRPC_E_*
    if (n_fit && (!h_cols || !h_wire)) return SRPC_E_INVALID;
    for (uint32_t f = 0; n_fit && f < p->nfields; ++f)
        if (!h_cols[f]) return SRPC_E_INVALID;
    DeviceGuard g(p->device);
    auto s = static_cast<hipStream_t>(stream);
    void* dc[kMaxFields];
    void* dw = nullptr;
    if (n_fit && chunk_records == 0) {
        for (uint32_t f = 0; f < p->nfields; ++f)
            if (!mapped(h_cols[f], n_fit * p->size[f], &dc[f])) return SRPC_E_INVALID;
        if (!mapped(h_wire, n_fit * p->stride, &dw)) return SRPC_E_INVALID;
    }
    const SlotLayout L = slot_layout(p, chunk_records ? chunk_records : 1);
    if (n_fit && chunk_records) {
        if (!d_scratch) return SRPC_E_INVALID;
        if (scratch_bytes < depth * L.bytes) return SRPC_E_CAPACITY;
        if (reinterpret_cast<uintptr_t>(d_scratch) % kAlignScratch) return SRPC_E_ALIGN;
        if (capturing(s)) return SRPC_E_UNSUPPORTED;
    }
    if (n_fit == 0) {
        if (d_status) {
            hipLaunchKernelGGL(k_host_status, dim3(1), dim3(64), 0, s, d_status, ret ? SRPC_STATUS_BOUNDS : 0u,
                               ret ? 0ull : UINT64_MAX);
            if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
        }
        return ret;
    }
    if (chunk_records == 0) {
        // the n_fit records that fit, then the short wire's BOUNDS on top
        const int rc = srpc_gpu_unpack(p, static_cast<const uint8_t*>(dw), n_fit * p->stride, n_fit, dc, d_status,
                                       stream);
        if (rc != SRPC_OK) return rc;
        if (ret && d_status) {
            hipLaunchKernelGGL(k_or_bounds, dim3(1), dim3(64), 0, s, d_status, n_fit);
            if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
        }
        return ret;
    }
    Lease lease(p->device, depth, s);
    Pipe* P = lease.p;
    if (!P) return SRPC_E_HIP;
    const bool two = two_streams();
    hipStream_t ks = two ? P->in : P->k;
    auto* base = static_cast<uint8_t*>(d_scratch);
    if (d_status) {
        hipLaunchKernelGGL(k_host_status, dim3(1), dim3(64), 0, s, d_status, ret ? SRPC_STATUS_BOUNDS : 0u,
                           ret ? n_fit : UINT64_MAX);
        if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
    }
    if (hipEventRecord(P->start, s) != hipSuccess) return SRPC_E_HIP;
    for (hipStream_t q : {P->in, P->k, P->out}) (void)hipStreamWaitEvent(q, P->start, 0);
    const uint64_t nch = (n_fit + chunk_records - 1) / chunk_records, fail = fail_at();
    for (uint64_t i = 0; i < nch; ++i) {
        if (i == fail) return drain(P, s, SRPC_E_HIP);
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
            return drain(P, s, SRPC_E_HIP);
        if (!two) {
            (void)hipEventRecord(ev_in, P->in);
            (void)hipStreamWaitEvent(P->k, ev_in, 0);
        }
        void* dcols[kMaxFields];
        for (uint32_t f = 0; f < p->nfields; ++f) dcols[f] = slot + L.col[f];
        auto* cst = d_status ? reinterpret_cast<srpc_unpack_status*>(slot + L.status) : nullptr;
        const int rc = srpc_gpu_unpack(p, slot + L.wire, cnt * p->stride, cnt, dcols, cst, ks);
        if (rc != SRPC_OK) return drain(P, s, rc);
        if (cst) {
            hipLaunchKernelGGL(k_merge_status, dim3(1), dim3(64), 0, ks, d_status, cst, lo);
            if (hipGetLastError() != hipSuccess) return drain(P, s, SRPC_E_HIP);
        }
        (void)hipEventRecord(ev_k, ks);
        (void)hipStreamWaitEvent(P->out, ev_k, 0);
        for (uint32_t f = 0; f < p->nfields; ++f)
            if (hipMemcpyAsync(static_cast<uint8_t*>(h_cols[f]) + lo * p->size[f], slot + L.col[f], cnt * p->size[f],
                               hipMemcpyDeviceToHost, P->out) != hipSuccess)
                return drain(P, s, SRPC_E_HIP);
        (void)hipEventRecord(ev_out, P->out);
    }
    (void)hipStreamWaitEvent(s, P->ev[3 * ((nch - 1) % depth) + 2], 0);
    return hipGetLastError() == hipSuccess ? ret : SRPC_E_HIP;
}

}  // extern "C"

// Test hook (not in include/): pipes the host-terminated calls have created on
// `device` (the pool's size), to check that it grows with concurrency, not with
// the number of threads that made calls.
extern "C" __attribute__((visibility("default"))) uint64_t srpc_debug_host_pipes(int device) {
    std::lock_guard<std::mutex> lk(pool().mu);
    auto it = pool().made.find(device);
    return it == pool().made.end() ? 0 : it->second;
}

// Test hooks (not in include/): arm the chunked ring's injected failure at
// chunk k (UINT64_MAX disarms), and the pipe this thread's last chunked call
// borrowed (an opaque id: which calls shared a pipe).
extern "C" __attribute__((visibility("default"))) void srpc_debug_host_fail_at(uint64_t k) {
    g_fail_at.store(k, std::memory_order_relaxed);
}
extern "C" __attribute__((visibility("default"))) uint64_t srpc_debug_host_last_pipe(void) {
    return reinterpret_cast<uintptr_t>(t_last_pipe);
}

// Test hook: how many pipes this process has made (every device).
extern "C" __attribute__((visibility("default"))) uint64_t srpc_debug_host_pipes_made(void) {
    std::lock_guard<std::mutex> lk(pool().mu);
    uint64_t n = 0;
    for (const auto& kv : pool().made) n += kv.second;
    return n;
}
