// srpc/gpu_server.hpp -- GPU-batched request serving.
//
// The reference server (include/srpc/server.hpp:45-74) handles one request at
// a time: recv_data -> `>> funcname` -> call -> getv<I> -> method ->
// pack_response -> send_data.  For streams of requests of methods with
// fixed-size bodies (Calculator.square: 57-byte frames = u32 BE 53 | 53-byte
// request), batch_server serves whole batches on the GPU with the same frames
// on the wire:
//
//   socket -> pinned host buffer (the CPU only walks the BE32 frame lengths)
//   -> H2D -> srpc_frames_classify (each frame against every registered
//   method's constant `BE32 len | str(method) | str(Req::name)` prefix and
//   length; per-method buckets; each response's offset in the reply stream)
//   -> per method: srpc_frames_gather -> srpc_gpu_unpack -> user device
//   handler -> srpc_gpu_pack (`BE32 len | code | str(Resp::name) | body`
//   frames) -> srpc_frames_scatter into request order -> D2H -> socket.
//
// A batch of one method skips the gather and scatter (its frames are already
// the plan's contiguous records).  A frame no registered method matches
// (another method, a string body, a corrupt header) is answered on the CPU
// by an ordinary srpc::server, in its place in the reply order; only those
// frames leave the GPU path.  A frame longer than the batch buffer is read on
// its own and answered the same way.
#pragma once

#include <hip/hip_runtime_api.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <sys/uio.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "gpu.hpp"
#include "server.hpp"
#include "transport.hpp"

namespace srpc::gpu {

inline std::vector<uint8_t> be32(uint32_t v) {
    return {static_cast<uint8_t>(v >> 24), static_cast<uint8_t>(v >> 16), static_cast<uint8_t>(v >> 8),
            static_cast<uint8_t>(v)};
}

/// A plan over an explicit prefix (used for framed envelopes).
class raw_plan {
public:
    raw_plan(std::vector<int32_t> const& kinds, std::vector<uint8_t> const& prefix, int device) {
        srpc_schema_desc d{static_cast<uint32_t>(kinds.size()), kinds.data(), prefix.empty() ? nullptr : prefix.data(),
                           static_cast<uint32_t>(prefix.size())};
        if (int rc = srpc_plan_create(&d, device, &_p); rc != SRPC_OK) throw plan_error("srpc_plan_create", rc);
        srpc_plan_record_bytes(_p, &_rb);
    }
    raw_plan(raw_plan const&) = delete;
    raw_plan& operator=(raw_plan const&) = delete;
    ~raw_plan() {
        if (_p) srpc_plan_destroy(_p);
    }
    srpc_plan* get() const { return _p; }
    uint64_t record_bytes() const { return _rb; }

private:
    srpc_plan* _p = nullptr;
    uint64_t _rb = 0;
};

template <SrpcMessage T>
uint64_t body_bytes() {
    uint64_t s = 0;
    T probe{};
    for_each_leaf<T>(probe, [&](const auto& v) { s += sizeof(v); });
    return s;
}

/// Constant prefix of a framed request: BE32(payload) | str(method) | str(T::name).
template <SrpcMessage T>
std::vector<uint8_t> framed_request_prefix(std::string const& method) {
    std::vector<uint8_t> hdr = request_prefix<T>(method);
    std::vector<uint8_t> out = be32(static_cast<uint32_t>(hdr.size() + body_bytes<T>()));
    out.insert(out.end(), hdr.begin(), hdr.end());
    return out;
}

/// Constant prefix of a framed response: BE32(payload) | code | str(T::name).
template <SrpcMessage T>
std::vector<uint8_t> framed_response_prefix(rpc_status_code code) {
    std::vector<uint8_t> hdr = response_prefix<T>(code);
    std::vector<uint8_t> out = be32(static_cast<uint32_t>(hdr.size() + body_bytes<T>()));
    out.insert(out.end(), hdr.begin(), hdr.end());
    return out;
}

struct batch_stats {
    uint64_t requests = 0;           // frames answered
    uint64_t gpu_batches = 0;        // batches that went through the GPU path
    uint64_t gpu_requests = 0;       // frames answered from the GPU
    uint64_t fallback_requests = 0;  // frames answered on the CPU (unknown method / shape)
    uint64_t oversize_requests = 0;  // of those, frames longer than the batch buffer
    uint64_t mixed_batches = 0;      // GPU batches that needed the gather / scatter
    uint64_t h2d_bytes = 0;
    uint64_t d2h_bytes = 0;
    double gpu_seconds = 0;  // H2D + classify + unpack + handler + pack + D2H, host-timed per batch
    double classify_seconds = 0;     // of which: H2D + classify + the counts' D2H (first sync)
    double first_batch_seconds = 0;  // gpu_seconds of the connection's first batch
    double recv_seconds = 0;
    double send_seconds = 0;
    double fallback_seconds = 0;
};

class batch_server {
public:
    /// handler(d_req_cols, d_resp_cols, n, stream): a method over a batch on
    /// the device (one column per flattened field of Req / Resp).
    using handler_t = std::function<int(void* const*, void* const*, uint64_t, hipStream_t)>;

    /// max_batch: frames per GPU batch; fallback: the CPU server for frames
    /// no registered method matches (nullptr: answered with
    /// RPC_ERR_FUNCTION_NOT_REGISTERED, as the reference does for an unknown name).
    explicit batch_server(uint64_t max_batch = 1u << 20, int device = 0, server* fallback = nullptr)
        : _fallback(fallback), _max(std::max<uint64_t>(max_batch, 1)), _dev(device) {
        check(hipSetDevice(device));
        check(hipStreamCreateWithFlags(&_s, hipStreamNonBlocking));
    }
    /// One method (the round-1 form).
    template <SrpcMessage Req, SrpcMessage Resp>
    static std::unique_ptr<batch_server> single(std::string method, handler_t handler, uint64_t max_batch = 1u << 20,
                                                int device = 0, server* fallback = nullptr) {
        auto s = std::make_unique<batch_server>(max_batch, device, fallback);
        s->register_method<Req, Resp>(std::move(method), std::move(handler));
        return s;
    }
    batch_server(batch_server const&) = delete;
    batch_server& operator=(batch_server const&) = delete;
    ~batch_server() {
        release();
        for (auto& m : _m) {
            for (void* p : m->req_cols) (void)hipFree(p);
            for (void* p : m->resp_cols) (void)hipFree(p);
        }
        (void)hipStreamDestroy(_s);
    }

    /// Serve `method` (frames `BE32 | str(method) | str(Req::name) | Req body`)
    /// with `handler` on the device; answers are `BE32 | RPC_SUCCESS |
    /// str(Resp::name) | Resp body` frames.  Up to SRPC_FRAMES_MAX_PLANS methods.
    template <SrpcMessage Req, SrpcMessage Resp>
    void register_method(std::string method, handler_t handler) {
        if (_m.size() >= SRPC_FRAMES_MAX_PLANS) throw plan_error("batch_server::register_method", SRPC_E_UNSUPPORTED);
        check(hipSetDevice(_dev));
        auto m = std::make_unique<method_entry>();
        m->name = std::move(method);
        m->handler = std::move(handler);
        m->in = std::make_unique<raw_plan>(flat_kinds<Req>(), framed_request_prefix<Req>(m->name), _dev);
        m->out = std::make_unique<raw_plan>(flat_kinds<Resp>(), framed_response_prefix<Resp>(RPC_SUCCESS), _dev);
        m->fin = m->in->record_bytes();
        m->fout = m->out->record_bytes();
        Req rq{};
        for_each_leaf<Req>(rq, [&](const auto& v) {
            m->req_bytes.push_back(_max * sizeof(v) + 16);
            m->req_cols.push_back(alloc(m->req_bytes.back()));
        });
        Resp rs{};
        for_each_leaf<Resp>(rs, [&](const auto& v) {
            m->resp_bytes.push_back(_max * sizeof(v) + 16);
            m->resp_cols.push_back(alloc(m->resp_bytes.back()));
        });
        _m.push_back(std::move(m));
        release();  // buffers are sized for the largest frames on the next serve
    }

    uint64_t request_frame_bytes(size_t k = 0) const { return _m.at(k)->fin; }
    uint64_t response_frame_bytes(size_t k = 0) const { return _m.at(k)->fout; }
    /// Bytes of the receive buffer: max_batch frames of the longest method.
    uint64_t buffer_bytes() const { return _max * max_fin(); }

    /// Serve one connected socket until the peer closes it.
    batch_stats serve_connection(int fd) {
        if (_m.empty()) throw plan_error("batch_server::serve_connection (no methods)", SRPC_E_INVALID);
        check(hipSetDevice(_dev));
        ensure();
        batch_stats st;
        const uint64_t cap = _cap;
        uint64_t have = 0;     // bytes in _h_in
        uint64_t walked = 0;   // bytes of whole frames found so far (frames _h_offs[0..nf))
        uint64_t nf = 0;
        bool eof = false;
        while (true) {
            if (!eof) {
                // cap - have > 0 here: a full buffer is always consumed below,
                // so recv returning 0 is the peer's orderly shutdown
                auto t0 = clock::now();
                ssize_t k = recv(fd, _h_in + have, cap - have, 0);
                if (k < 0 && errno == EINTR) continue;
                st.recv_seconds += secs(t0);
                if (k <= 0) eof = true;
                else have += static_cast<uint64_t>(k);
            }
            // frame boundaries (the only per-frame CPU work on the fast path)
            uint64_t next_len = 0;
            bool next_hdr = false;
            while (nf < _max && have - walked >= 4) {
                next_len = 4 + static_cast<uint64_t>(be32_at(_h_in + walked));
                next_hdr = true;
                if (have - walked < next_len) break;
                _h_offs[nf++] = static_cast<uint32_t>(walked);
                walked += next_len;
                next_hdr = false;
            }
            const bool oversize = next_hdr && next_len > cap;
            const bool full = nf == _max || have == cap || oversize;
            if (_trace)
                std::fprintf(stderr, "recv: have %llu walked %llu nf %llu next %llu%s%s\n", (unsigned long long)have,
                             (unsigned long long)walked, (unsigned long long)nf, (unsigned long long)next_len,
                             eof ? " eof" : "", full ? " full" : "");
            if (nf == 0 && !oversize) {
                if (eof) break;
                continue;
            }
            if (!full && !eof && more_pending(fd)) continue;  // fill the batch while data streams in
            if (nf) process(fd, nf, walked, st);
            std::memmove(_h_in, _h_in + walked, have - walked);
            have -= walked;
            walked = 0;
            nf = 0;
            if (oversize) {
                if (!serve_oversize(fd, have, st)) return st;
                have = 0;
            }
        }
        return st;  // bytes of a cut final frame are dropped, as the reference's recv_data does
    }

private:
    using clock = std::chrono::steady_clock;
    struct method_entry {
        std::string name;
        handler_t handler;
        std::unique_ptr<raw_plan> in, out;
        uint64_t fin = 0, fout = 0;
        std::vector<void*> req_cols, resp_cols;
        std::vector<uint64_t> req_bytes, resp_bytes;
    };
    void memset_cols(std::vector<void*> const& cols, std::vector<uint64_t> const& bytes) {
        for (size_t f = 0; f < cols.size(); ++f) check(hipMemsetAsync(cols[f], 0, bytes[f], _s));
    }

    static double secs(clock::time_point t0) { return std::chrono::duration<double>(clock::now() - t0).count(); }
    static void check(hipError_t e) {
        if (e != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e));
    }
    static void check_srpc(int rc, const char* what) {
        if (rc < 0) throw plan_error(what, rc);
    }
    static uint32_t be32_at(const uint8_t* b) {
        return (uint32_t(b[0]) << 24) | (uint32_t(b[1]) << 16) | (uint32_t(b[2]) << 8) | uint32_t(b[3]);
    }
    void* alloc(size_t b) {
        void* p = nullptr;
        check(hipMalloc(&p, b));
        return p;
    }
    static bool more_pending(int fd) {
        int avail = 0;
        return ::ioctl(fd, FIONREAD, &avail) == 0 && avail > 0;
    }
    uint64_t max_fin() const {
        uint64_t f = 0;
        for (auto const& m : _m) f = std::max(f, m->fin);
        return f;
    }
    uint64_t max_fout() const {
        uint64_t f = 0;
        for (auto const& m : _m) f = std::max(f, m->fout);
        return f;
    }

    void ensure() {
        if (_h_in) return;
        const uint64_t K = _m.size();
        _cap = _max * max_fin();
        if (_cap > 0xffffffffull) throw plan_error("batch_server: batch buffer over 4 GiB", SRPC_E_UNSUPPORTED);
        const uint64_t out_cap = _max * max_fout();
        check(hipHostMalloc(reinterpret_cast<void**>(&_h_in), _cap + 16, hipHostMallocDefault));
        check(hipHostMalloc(reinterpret_cast<void**>(&_h_offs), 4 * _max + 16, hipHostMallocDefault));
        check(hipHostMalloc(reinterpret_cast<void**>(&_h_out), out_cap + 16, hipHostMallocDefault));
        check(hipHostMalloc(reinterpret_cast<void**>(&_h_cls), _max + 16, hipHostMallocDefault));
        check(hipHostMalloc(reinterpret_cast<void**>(&_h_counts), 8 * (K + 2) + 16, hipHostMallocDefault));
        check(hipHostMalloc(reinterpret_cast<void**>(&_h_status), sizeof(srpc_unpack_status), hipHostMallocDefault));
        check(hipMalloc(&_d_in, _cap + 16));
        check(hipMalloc(&_d_offs, 4 * _max + 16));
        check(hipMalloc(&_d_cls, _max + 16));
        check(hipMalloc(&_d_index, 4 * K * _max + 16));
        check(hipMalloc(&_d_counts, 8 * (K + 2) + 16));
        check(hipMalloc(&_d_out_off, 8 * (_max + 1) + 16));
        check(hipMalloc(&_d_gather, _cap + 16));
        check(hipMalloc(&_d_resp, out_cap + 16));
        check(hipMalloc(&_d_out, out_cap + 16));
        check(hipMalloc(&_d_status, sizeof(srpc_unpack_status)));
        check_srpc(srpc_frames_scratch_bytes(_max, static_cast<int>(K), &_scratch_bytes), "srpc_frames_scratch_bytes");
        check(hipMalloc(&_d_scratch, _scratch_bytes));
        _in_plans.clear();
        _resp_bytes.clear();
        for (auto const& m : _m) {
            _in_plans.push_back(m->in->get());
            _resp_bytes.push_back(static_cast<uint32_t>(m->fout));
        }
        warm_up();
    }

    /// One-frame run of every kernel the batches use (the library's and each
    /// handler, on one all-zero record) and one copy through every staging
    /// buffer, at serve start: first uses cost milliseconds that otherwise land
    /// on the connection's first batch (profiles/r02_e2e_warmup.log).
    void warm_up() {
        const int K = static_cast<int>(_m.size());
        const uint64_t out_cap = _max * max_fout();
        check(hipMemsetAsync(_d_out, 0, out_cap + 16, _s));
        check(hipMemsetAsync(_d_resp, 0, out_cap + 16, _s));
        check(hipMemsetAsync(_d_gather, 0, _cap + 16, _s));
        check(hipMemsetAsync(_d_index, 0, 4 * _m.size() * _max + 16, _s));
        check(hipMemsetAsync(_d_out_off, 0, 8 * (_max + 1) + 16, _s));
        check(hipMemsetAsync(_d_cls, 0, _max + 16, _s));
        check(hipMemsetAsync(_d_scratch, 0, _scratch_bytes, _s));
        for (auto const& m : _m) {
            memset_cols(m->req_cols, m->req_bytes);
            memset_cols(m->resp_cols, m->resp_bytes);
        }
        std::memset(_h_in, 0, _cap);
        std::memset(_h_offs, 0, 4 * _max);
        // a batch's exact sequence of copies and launches on one all-zero frame,
        // twice (the first pass pays the first uses; whole buffers move)
        for (int pass = 0; pass < 2; ++pass) {
            check(hipMemcpyAsync(_d_in, _h_in, _cap, hipMemcpyHostToDevice, _s));
            check(hipMemcpyAsync(_d_offs, _h_offs, 4 * _max, hipMemcpyHostToDevice, _s));
            check_srpc(srpc_frames_classify(_in_plans.data(), _resp_bytes.data(), K, static_cast<const uint8_t*>(_d_in),
                                            8, static_cast<const uint32_t*>(_d_offs), 1, static_cast<uint8_t*>(_d_cls),
                                            static_cast<uint32_t*>(_d_index), static_cast<uint64_t*>(_d_counts),
                                            static_cast<uint64_t*>(_d_out_off), _d_scratch, _scratch_bytes, _s),
                       "srpc_frames_classify");
            check(hipMemcpyAsync(_h_counts, _d_counts, 8 * (K + 2), hipMemcpyDeviceToHost, _s));
            check(hipStreamSynchronize(_s));
            check(hipMemsetAsync(_d_status, 0, sizeof(srpc_unpack_status), _s));
            for (auto const& m : _m) {
                check_srpc(srpc_frames_gather(static_cast<const uint8_t*>(_d_in), static_cast<const uint32_t*>(_d_offs),
                                              static_cast<const uint32_t*>(_d_index), 1, static_cast<uint32_t>(m->fin),
                                              static_cast<uint8_t*>(_d_gather), _s),
                           "srpc_frames_gather");
                (void)srpc_gpu_unpack(m->in->get(), static_cast<const uint8_t*>(_d_gather), m->fin, 1,
                                      m->req_cols.data(), _d_status, _s);  // a prefix error on the zero frame: expected
                // the handler's own kernels load their code object on first use
                // too: it runs on the one zero record (its output is never sent)
                check_srpc(m->handler(m->req_cols.data(), m->resp_cols.data(), 1, _s), "batch handler (warm-up)");
                check_srpc(srpc_gpu_pack(m->out->get(), m->resp_cols.data(), 1, static_cast<uint8_t*>(_d_out), m->fout,
                                         _s),
                           "srpc_gpu_pack");
                check_srpc(srpc_gpu_pack(m->out->get(), m->resp_cols.data(), 1, static_cast<uint8_t*>(_d_resp), m->fout,
                                         _s),
                           "srpc_gpu_pack");
                check_srpc(srpc_frames_scatter(static_cast<const uint8_t*>(_d_resp),
                                               static_cast<const uint32_t*>(_d_index), 1, static_cast<uint32_t>(m->fout),
                                               static_cast<const uint64_t*>(_d_out_off), static_cast<uint8_t*>(_d_out),
                                               _s),
                           "srpc_frames_scatter");
            }
            check(hipMemcpyAsync(_h_out, _d_out, out_cap, hipMemcpyDeviceToHost, _s));
            check(hipMemcpyAsync(_h_cls, _d_cls, _max, hipMemcpyDeviceToHost, _s));
            check(hipMemcpyAsync(_h_status, _d_status, sizeof(srpc_unpack_status), hipMemcpyDeviceToHost, _s));
            check(hipStreamSynchronize(_s));
        }
    }
    void release() {
        for (void* p : {_d_in, _d_offs, _d_cls, _d_index, _d_counts, _d_out_off, _d_gather, _d_resp, _d_out,
                        static_cast<void*>(_d_status), _d_scratch})
            if (p) (void)hipFree(p);
        for (void* p : {static_cast<void*>(_h_in), static_cast<void*>(_h_offs), static_cast<void*>(_h_out),
                        static_cast<void*>(_h_cls), static_cast<void*>(_h_counts), static_cast<void*>(_h_status)})
            if (p) (void)hipHostFree(p);
        _d_in = _d_offs = _d_cls = _d_index = _d_counts = _d_out_off = _d_gather = _d_resp = _d_out = _d_scratch =
            nullptr;
        _d_status = nullptr;
        _h_in = _h_out = _h_cls = nullptr;
        _h_offs = nullptr;
        _h_counts = nullptr;
        _h_status = nullptr;
    }

    /// The GPU path for the nf whole frames in _h_in[0, used).
    void process(int fd, uint64_t nf, uint64_t used, batch_stats& st) {
        auto t0 = clock::now();
        auto mark = [&](const char* what) {
            if (_trace) std::fprintf(stderr, "batch %llu nf %llu %-10s %.3f ms\n", (unsigned long long)st.gpu_batches,
                                    (unsigned long long)nf, what, 1e3 * secs(t0));
        };
        const int K = static_cast<int>(_m.size());
        auto* d_in = static_cast<uint8_t*>(_d_in);
        auto* d_offs = static_cast<uint32_t*>(_d_offs);
        auto* d_idx = static_cast<uint32_t*>(_d_index);
        auto* d_counts = static_cast<uint64_t*>(_d_counts);
        auto* d_out_off = static_cast<uint64_t*>(_d_out_off);
        check(hipMemcpyAsync(d_in, _h_in, used, hipMemcpyHostToDevice, _s));
        check(hipMemcpyAsync(d_offs, _h_offs, 4 * nf, hipMemcpyHostToDevice, _s));
        mark("h2d");
        check_srpc(srpc_frames_classify(_in_plans.data(), _resp_bytes.data(), K, d_in, used, d_offs, nf,
                                        static_cast<uint8_t*>(_d_cls), d_idx, d_counts, d_out_off, _d_scratch,
                                        _scratch_bytes, _s),
                   "srpc_frames_classify");
        check(hipMemcpyAsync(_h_counts, d_counts, 8 * (K + 2), hipMemcpyDeviceToHost, _s));
        mark("classify");
        check(hipStreamSynchronize(_s));
        mark("sync1");
        st.classify_seconds += secs(t0);
        const uint64_t total = _h_counts[K], unknown = _h_counts[K + 1];
        bool mixed = false;
        check(hipMemsetAsync(_d_status, 0, sizeof(srpc_unpack_status), _s));
        for (int k = 0; k < K; ++k) {
            const uint64_t n = _h_counts[k];
            if (!n) continue;
            method_entry& m = *_m[static_cast<size_t>(k)];
            const bool whole = n == nf;  // every frame is method k: they already are its contiguous records
            mixed |= !whole;
            const uint8_t* src = d_in;
            if (!whole) {
                check_srpc(srpc_frames_gather(d_in, d_offs, d_idx + static_cast<uint64_t>(k) * nf, n,
                                              static_cast<uint32_t>(m.fin), static_cast<uint8_t*>(_d_gather), _s),
                           "srpc_frames_gather");
                src = static_cast<const uint8_t*>(_d_gather);
            }
            check_srpc(srpc_gpu_unpack(m.in->get(), src, n * m.fin, n, m.req_cols.data(), _d_status, _s),
                       "srpc_gpu_unpack");
            mark("unpack");
            check_srpc(m.handler(m.req_cols.data(), m.resp_cols.data(), n, _s), "batch handler");
            mark("handler");
            auto* dst = static_cast<uint8_t*>(whole ? _d_out : _d_resp);
            check_srpc(srpc_gpu_pack(m.out->get(), m.resp_cols.data(), n, dst, n * m.fout, _s), "srpc_gpu_pack");
            mark("pack");
            if (!whole)
                check_srpc(srpc_frames_scatter(dst, d_idx + static_cast<uint64_t>(k) * nf, n,
                                               static_cast<uint32_t>(m.fout), d_out_off, static_cast<uint8_t*>(_d_out),
                                               _s),
                           "srpc_frames_scatter");
        }
        if (total) check(hipMemcpyAsync(_h_out, _d_out, total, hipMemcpyDeviceToHost, _s));
        mark("d2h_out");
        if (unknown) check(hipMemcpyAsync(_h_cls, _d_cls, nf, hipMemcpyDeviceToHost, _s));
        check(hipMemcpyAsync(_h_status, _d_status, sizeof(srpc_unpack_status), hipMemcpyDeviceToHost, _s));
        mark("d2h");
        check(hipStreamSynchronize(_s));
        mark("sync2");
        // classification already matched every prefix and length: an unpack
        // status here means the buckets and the plans disagree
        if (_h_status->flags) throw plan_error("batch_server: classified frame failed to unpack", SRPC_E_INVALID);
        const double dt = secs(t0);
        if (st.gpu_batches == 0 && st.fallback_requests == 0) st.first_batch_seconds = dt;
        st.gpu_seconds += dt;
        st.h2d_bytes += used + 4 * nf;
        st.d2h_bytes += total + (unknown ? nf : 0);
        if (total) {
            st.gpu_batches += 1;
            st.mixed_batches += mixed ? 1 : 0;
        }
        st.gpu_requests += nf - unknown;
        st.requests += nf - unknown;
        auto t1 = clock::now();
        if (!unknown) {
            transport::send_all(fd, _h_out, total);
            st.send_seconds += secs(t1);
            return;
        }
        // GPU answers in runs, the CPU's in their places, one gathered send
        // (separate small sends would meet Nagle + delayed ACK on the socket)
        _arena.clear();
        _pieces.clear();
        uint64_t run = 0, pos = 0;
        for (uint64_t i = 0; i < nf; ++i) {
            const uint8_t c = _h_cls[i];
            if (c != SRPC_FRAME_UNKNOWN) {
                run += _m[c]->fout;
                continue;
            }
            if (run > pos) _pieces.push_back({true, pos, run - pos});
            pos = run;
            const uint64_t o = _h_offs[i];
            const uint64_t a0 = _arena.size();
            answer_cpu(_h_in + o + 4, be32_at(_h_in + o), st);
            _pieces.push_back({false, a0, _arena.size() - a0});
        }
        if (run > pos) _pieces.push_back({true, pos, run - pos});
        send_pieces(fd);
        st.send_seconds += secs(t1);
    }

    struct piece {
        bool gpu;  // _h_out or _arena
        uint64_t off, len;
    };

    /// sendmsg over the pieces, IOV_MAX at a time, resuming partial sends.
    void send_pieces(int fd) {
        if (_pieces.size() > 4096) {  // many short runs: one copy beats ~170 ns per iovec in the kernel
            _flat.resize(0);
            for (piece const& p : _pieces) {
                const uint8_t* b = (p.gpu ? _h_out : _arena.data()) + p.off;
                _flat.insert(_flat.end(), b, b + p.len);
            }
            transport::send_all(fd, _flat.data(), _flat.size());
            return;
        }
        std::vector<iovec> iov;
        iov.reserve(_pieces.size());
        for (piece const& p : _pieces)
            iov.push_back({(p.gpu ? _h_out : _arena.data()) + p.off, static_cast<size_t>(p.len)});
        size_t at = 0;
        while (at < iov.size()) {
            msghdr mh{};
            mh.msg_iov = iov.data() + at;
            mh.msg_iovlen = std::min<size_t>(iov.size() - at, 1024);
            ssize_t k = sendmsg(fd, &mh, MSG_NOSIGNAL);
            if (k < 0 && errno == EINTR) continue;
            if (k <= 0) return;  // the peer is gone; the recv side ends the connection
            auto left = static_cast<size_t>(k);
            while (at < iov.size() && left >= iov[at].iov_len) left -= iov[at++].iov_len;
            if (left) {
                iov[at].iov_base = static_cast<uint8_t*>(iov[at].iov_base) + left;
                iov[at].iov_len -= left;
            }
        }
    }

    /// A frame longer than the batch buffer: `have` bytes of it are at the
    /// start of _h_in; read the rest and answer it on the CPU.  False at EOF.
    bool serve_oversize(int fd, uint64_t have, batch_stats& st) {
        const uint64_t len = be32_at(_h_in);
        std::vector<uint8_t> payload(len);
        std::memcpy(payload.data(), _h_in + 4, have - 4);
        auto t0 = clock::now();
        const bool ok = transport::recv_all(fd, payload.data() + (have - 4), len - (have - 4));
        st.recv_seconds += secs(t0);
        if (!ok) return false;
        st.oversize_requests += 1;
        _arena.clear();
        answer_cpu(payload.data(), len, st);
        transport::send_all(fd, _arena.data(), _arena.size());
        return true;
    }

    /// One frame's payload through the scalar server (reference server.hpp:58-69);
    /// the framed answer (BE32 | response, as transport::send_data) goes to _arena.
    void answer_cpu(const uint8_t* payload, uint64_t len, batch_stats& st) {
        auto t0 = clock::now();
        packer::ptr r;
        if (_fallback) {
            packer::ptr p = std::make_shared<packer>(payload, len);
            std::string fn;
            (*p) >> fn;
            r = _fallback->call(fn, p);
        } else {
            r = std::make_shared<packer>();
            (*r) << static_cast<uint8_t>(RPC_ERR_FUNCTION_NOT_REGISTERED);
        }
        const std::vector<uint8_t> hdr = be32(static_cast<uint32_t>(r->size()));
        _arena.insert(_arena.end(), hdr.begin(), hdr.end());
        _arena.insert(_arena.end(), r->data(), r->data() + r->size());
        st.fallback_requests += 1;
        st.requests += 1;
        st.fallback_seconds += secs(t0);
    }

    server* _fallback;
    uint64_t _max;
    int _dev;
    hipStream_t _s = nullptr;
    std::vector<std::unique_ptr<method_entry>> _m;
    std::vector<const srpc_plan*> _in_plans;
    std::vector<uint32_t> _resp_bytes;
    std::vector<uint8_t> _arena;  // CPU answers of the batch being sent
    std::vector<piece> _pieces;
    std::vector<uint8_t> _flat;
    uint64_t _cap = 0, _scratch_bytes = 0;
    bool _trace = std::getenv("SRPC_SERVER_TRACE") != nullptr;  // per-recv / per-batch timeline on stderr
    uint8_t* _h_in = nullptr;
    uint32_t* _h_offs = nullptr;
    uint8_t* _h_out = nullptr;
    uint8_t* _h_cls = nullptr;
    uint64_t* _h_counts = nullptr;
    srpc_unpack_status* _h_status = nullptr;
    void *_d_in = nullptr, *_d_offs = nullptr, *_d_cls = nullptr, *_d_index = nullptr, *_d_counts = nullptr,
         *_d_out_off = nullptr, *_d_gather = nullptr, *_d_resp = nullptr, *_d_out = nullptr, *_d_scratch = nullptr;
    srpc_unpack_status* _d_status = nullptr;
};

}  // namespace srpc::gpu
