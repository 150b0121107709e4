// srpc/gpu_server.hpp -- GPU-batched request serving for one method.
//
// The reference server (include/srpc/server.hpp:45-74) handles one request at
// a time: recv_data -> `>> funcname` -> call -> getv<I> -> method ->
// pack_response -> send_data.  For a stream of requests of ONE method with a
// fixed-size body (Calculator.square: 57-byte frames = u32 BE 53 | 53-byte
// request), batch_server<Req, Resp> serves them in batches on the GPU with
// the same frames on the wire:
//
//   socket -> pinned host buffer -> H2D -> srpc_gpu_unpack (checks, for every
//   frame, the constant `BE32 len | str(method) | str(Req::name)` prefix and
//   extracts the body into SoA columns) -> user device handler (e.g. a square
//   kernel) -> srpc_gpu_pack (writes `BE32 len | code | str(Resp::name) | body`
//   frames) -> D2H -> socket.
//
// The frame header is simply part of the plan's constant prefix, so no CPU
// parsing happens on the fast path.  A batch in which any frame differs from
// the expected prefix (another method, another length) is replayed frame by
// frame through an ordinary srpc::server on the CPU, so mixed traffic is
// still answered correctly and in order.
#pragma once

#include <hip/hip_runtime_api.h>
#include <sys/ioctl.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <functional>
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
    uint64_t requests = 0;
    uint64_t gpu_batches = 0;
    uint64_t fallback_requests = 0;
    uint64_t h2d_bytes = 0;
    uint64_t d2h_bytes = 0;
    double gpu_seconds = 0;  // H2D + unpack + handler + pack + D2H, host-timed per batch
    double recv_seconds = 0;
    double send_seconds = 0;
};

template <SrpcMessage Req, SrpcMessage Resp>
class batch_server {
public:
    /// handler(d_req_cols, d_resp_cols, n, stream): the method over a batch on
    /// the device (one column per flattened field of Req / Resp).
    using handler_t = std::function<int(void* const*, void* const*, uint64_t, hipStream_t)>;

    batch_server(std::string method, handler_t handler, uint64_t max_batch = 1u << 20, int device = 0,
                 server* fallback = nullptr)
        : _method(std::move(method)),
          _handler(std::move(handler)),
          _fallback(fallback),
          _max(max_batch),
          _in(flat_kinds<Req>(), framed_request_prefix<Req>(_method), device),
          _out(flat_kinds<Resp>(), framed_response_prefix<Resp>(RPC_SUCCESS), device) {
        _fin = _in.record_bytes();
        _fout = _out.record_bytes();
        check(hipSetDevice(device));
        check(hipStreamCreateWithFlags(&_s, hipStreamNonBlocking));
        check(hipHostMalloc(reinterpret_cast<void**>(&_h_in), _max * _fin + _fin, hipHostMallocDefault));
        check(hipHostMalloc(reinterpret_cast<void**>(&_h_out), _max * _fout + 16, hipHostMallocDefault));
        check(hipMalloc(&_d_in, _max * _fin + 16));
        check(hipMalloc(&_d_out, _max * _fout + 16));
        check(hipMalloc(reinterpret_cast<void**>(&_d_status), sizeof(srpc_unpack_status)));
        Req rq{};
        for_each_leaf<Req>(rq, [&](const auto& v) { _req_cols.push_back(alloc(_max * sizeof(v) + 16)); });
        Resp rs{};
        for_each_leaf<Resp>(rs, [&](const auto& v) { _resp_cols.push_back(alloc(_max * sizeof(v) + 16)); });
    }
    batch_server(batch_server const&) = delete;
    batch_server& operator=(batch_server const&) = delete;
    ~batch_server() {
        for (void* p : _req_cols) (void)hipFree(p);
        for (void* p : _resp_cols) (void)hipFree(p);
        (void)hipFree(_d_in);
        (void)hipFree(_d_out);
        (void)hipFree(_d_status);
        (void)hipHostFree(_h_in);
        (void)hipHostFree(_h_out);
        (void)hipStreamDestroy(_s);
    }

    uint64_t request_frame_bytes() const { return _fin; }
    uint64_t response_frame_bytes() const { return _fout; }

    /// Serve one connected socket until the peer closes it.
    batch_stats serve_connection(int fd) {
        batch_stats st;
        uint64_t have = 0;
        const uint64_t cap = _max * _fin;
        while (true) {
            auto t0 = clock::now();
            ssize_t k = recv(fd, _h_in + have, cap - have, 0);
            if (k < 0 && errno == EINTR) continue;
            st.recv_seconds += secs(t0);
            if (k <= 0) break;
            have += static_cast<uint64_t>(k);
            const uint64_t nf = have / _fin;
            if (nf == 0) continue;
            if (have < cap && nf < _max && more_pending(fd)) continue;  // fill the batch while data streams in
            uint64_t used = process(fd, nf, have, st);
            std::memmove(_h_in, _h_in + used, have - used);
            have -= used;
        }
        if (have && _fallback) fallback_frames(fd, have, st);
        return st;
    }

private:
    using clock = std::chrono::steady_clock;
    static double secs(clock::time_point t0) { return std::chrono::duration<double>(clock::now() - t0).count(); }
    static void check(hipError_t e) {
        if (e != hipSuccess) throw std::runtime_error(std::string("HIP: ") + hipGetErrorString(e));
    }
    static void check_srpc(int rc, const char* what) {
        if (rc < 0) throw plan_error(what, rc);
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

    /// GPU path for nf frames at the start of _h_in; returns bytes consumed.
    uint64_t process(int fd, uint64_t nf, uint64_t have, batch_stats& st) {
        auto t0 = clock::now();
        const uint64_t in_b = nf * _fin, out_b = nf * _fout;
        check(hipMemcpyAsync(_d_in, _h_in, in_b, hipMemcpyHostToDevice, _s));
        check_srpc(srpc_gpu_unpack(_in.get(), static_cast<const uint8_t*>(_d_in), in_b, nf, _req_cols.data(),
                                   _d_status, _s),
                   "srpc_gpu_unpack");
        check_srpc(_handler(_req_cols.data(), _resp_cols.data(), nf, _s), "batch handler");
        check_srpc(srpc_gpu_pack(_out.get(), _resp_cols.data(), nf, static_cast<uint8_t*>(_d_out), out_b, _s),
                   "srpc_gpu_pack");
        check(hipMemcpyAsync(_h_out, _d_out, out_b, hipMemcpyDeviceToHost, _s));
        srpc_unpack_status hs{};
        check(hipMemcpyAsync(&hs, _d_status, sizeof(hs), hipMemcpyDeviceToHost, _s));
        check(hipStreamSynchronize(_s));
        st.gpu_seconds += secs(t0);
        st.h2d_bytes += in_b;
        st.d2h_bytes += out_b;
        if (hs.flags == 0) {
            auto t1 = clock::now();
            transport::send_all(fd, _h_out, out_b);
            st.send_seconds += secs(t1);
            st.requests += nf;
            st.gpu_batches += 1;
            return in_b;
        }
        // Some frame is not `method` with a fixed-size body: answer the frames
        // before the first bad one from the GPU result, the rest on the CPU.
        const uint64_t good = hs.first_bad_record < nf ? hs.first_bad_record : nf;
        transport::send_all(fd, _h_out, good * _fout);
        st.requests += good;
        return good * _fin + fallback_frames(fd, have - good * _fin, st, good * _fin);
    }

    /// Scalar path over whole frames in _h_in[off, off+len); returns bytes consumed.
    uint64_t fallback_frames(int fd, uint64_t len, batch_stats& st, uint64_t off = 0) {
        uint64_t pos = 0;
        const uint8_t* b = _h_in + off;
        while (len - pos >= 4) {
            const uint32_t flen = (uint32_t(b[pos]) << 24) | (uint32_t(b[pos + 1]) << 16) |
                                  (uint32_t(b[pos + 2]) << 8) | uint32_t(b[pos + 3]);
            if (len - pos - 4 < flen) break;
            packer::ptr p = std::make_shared<packer>(b + pos + 4, flen);
            packer::ptr r;
            if (_fallback) {
                std::string fn;
                (*p) >> fn;
                r = _fallback->call(fn, p);
            } else {
                r = std::make_shared<packer>();
                (*r) << static_cast<uint8_t>(RPC_ERR_FUNCTION_NOT_REGISTERED);
            }
            transport::send_data(fd, r->data(), r->size());
            pos += 4 + flen;
            st.fallback_requests += 1;
            st.requests += 1;
        }
        return pos;
    }

    std::string _method;
    handler_t _handler;
    server* _fallback;
    uint64_t _max;
    raw_plan _in, _out;
    uint64_t _fin = 0, _fout = 0;
    hipStream_t _s = nullptr;
    uint8_t* _h_in = nullptr;
    uint8_t* _h_out = nullptr;
    void* _d_in = nullptr;
    void* _d_out = nullptr;
    srpc_unpack_status* _d_status = nullptr;
    std::vector<void*> _req_cols, _resp_cols;
};

}  // namespace srpc::gpu
