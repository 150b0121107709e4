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
// the plan's contiguous records).  Methods with string fields
// (register_var_method) take the variable-length form of each step:
// srpc_frames_classify matches their frames by `str(method) | str(Req::name)`
// after the BE32 and walks their fields to the frame's end;
// srpc_frames_gather_var strips the BE32s and builds the record index ->
// srpc_gpu_unpack_var -> the user's var handler (chars + offsets per string
// field) -> srpc_gpu_pack_var -> srpc_frames_offsets (the reply stream's
// offsets, now that the responses' sizes are known) ->
// srpc_frames_scatter_var (`BE32 len | response` into request order).
// A frame no registered method matches (another method, a corrupt header or
// string length, trailing bytes) is answered on the CPU by an ordinary
// srpc::server, in its place in the reply order; only those frames leave the
// GPU path.  A frame longer than the batch buffer is read on its own and
// answered the same way.
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

/// Bytes of a record of T with every string empty (prefix excluded): the
/// fixed leaves plus 8 (the length) per string.
template <SrpcMessage T>
uint64_t min_body_bytes() {
    uint64_t s = 0;
    T probe{};
    for_each_leaf<T>(probe, [&](const auto& v) {
        using F = std::remove_cvref_t<decltype(v)>;
        s += std::is_same_v<F, std::string> ? 8 : sizeof(F);
    });
    return s;
}

/// A batch of a string-bodied method on the device, one entry per flattened
/// field of Req / Resp: a fixed field is n values; a string field is its
/// chars back to back (`*_cols[f]`) plus n+1 u64 offsets (`*_str_offs[f]`,
/// nullptr for fixed fields) -- the layout of srpc_gpu_unpack_var /
/// srpc_gpu_pack_var.  The handler writes every response column and the n+1
/// offsets of every response string field (offs[0] need not be 0; at most
/// resp_cap[f] chars).
struct var_batch {
    uint64_t n = 0;
    void* const* req_cols = nullptr;
    const uint64_t* const* req_str_offs = nullptr;
    void* const* resp_cols = nullptr;
    uint64_t* const* resp_str_offs = nullptr;
    const uint64_t* resp_cap = nullptr;  // bytes of each response column
};

/// Sizing of a string-bodied method's buffers (per request of a batch).
struct var_limits {
    uint64_t max_request_bytes = 512;  // frame bytes the receive buffer is sized for
    uint64_t max_response_chars = 256; // chars of one response's string field (batch average)
};

struct batch_stats {
    uint64_t requests = 0;           // frames answered
    uint64_t gpu_batches = 0;        // batches that went through the GPU path
    uint64_t gpu_requests = 0;       // frames answered from the GPU
    uint64_t fallback_requests = 0;  // frames answered on the CPU (unknown method / shape)
    uint64_t oversize_requests = 0;  // of those, frames longer than the batch buffer
    uint64_t overflow_batches = 0;   // string-method buckets answered on the CPU: responses past max_response_chars
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
    /// handler(batch, stream) for a method with string fields (var_batch).
    using var_handler_t = std::function<int(var_batch const&, hipStream_t)>;

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
            if (m->var) continue;  // released with the batch buffers
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

    /// Serve `method` whose request and/or response has string fields: frames
    /// `BE32 | str(method) | str(Req::name) | Req record`, answered with
    /// `BE32 | RPC_SUCCESS | str(Resp::name) | Resp record` frames; `handler`
    /// runs on whole batches of them (var_batch).  The receive buffer holds
    /// max_batch frames of lim.max_request_bytes; longer frames still batch
    /// while they fit, and one longer than the whole buffer is answered on
    /// the CPU.  Up to SRPC_FRAMES_MAX_STRINGS string fields in Req.
    template <SrpcMessage Req, SrpcMessage Resp>
    void register_var_method(std::string method, var_handler_t handler, var_limits lim = {}) {
        if (_m.size() >= SRPC_FRAMES_MAX_PLANS) throw plan_error("batch_server::register_var_method", SRPC_E_UNSUPPORTED);
        check(hipSetDevice(_dev));
        auto m = std::make_unique<method_entry>();
        m->var = true;
        m->name = std::move(method);
        m->vhandler = std::move(handler);
        const std::vector<uint8_t> rq = request_prefix<Req>(m->name), rs = response_prefix<Resp>(RPC_SUCCESS);
        m->in = std::make_unique<raw_plan>(flat_kinds<Req>(), rq, _dev);
        m->out = std::make_unique<raw_plan>(flat_kinds<Resp>(), rs, _dev);
        m->req_prefix = rq;
        m->min_in = rq.size() + min_body_bytes<Req>();
        m->min_out = rs.size() + min_body_bytes<Resp>();
        m->fin = std::max<uint64_t>(lim.max_request_bytes, 4 + m->min_in);
        m->fout = 0;  // response frames vary
        m->lim = lim;
        Req rq0{};
        for_each_leaf<Req>(rq0, [&](const auto& v) {
            using F = std::remove_cvref_t<decltype(v)>;
            m->req_string.push_back(std::is_same_v<F, std::string>);
            m->req_size.push_back(std::is_same_v<F, std::string> ? 0 : sizeof(F));
        });
        Resp rs0{};
        for_each_leaf<Resp>(rs0, [&](const auto& v) {
            using F = std::remove_cvref_t<decltype(v)>;
            m->resp_string.push_back(std::is_same_v<F, std::string>);
            m->resp_size.push_back(std::is_same_v<F, std::string> ? 0 : sizeof(F));
        });
        _m.push_back(std::move(m));
        release();
    }

    uint64_t request_frame_bytes(size_t k = 0) const { return _m.at(k)->fin; }
    uint64_t response_frame_bytes(size_t k = 0) const { return _m.at(k)->fout; }
    /// Bytes of the receive buffer: max_batch frames of the longest method.
    uint64_t buffer_bytes() const { return _max * max_fin(); }

    /// Serve one connected socket until the peer closes it.
    ///
    /// Servers whose methods are all fixed-size run two batches in flight:
    /// batch k's copies and kernels are enqueued (process_begin) and the next
    /// batch is received into the other half of the double-buffered pinned
    /// staging while they run; batch k's answers are sent (process_end) once
    /// batch k + 1 is enqueued -- or before any recv that would block, so a
    /// peer that waits for every answer before it closes is never kept
    /// waiting.  Answers leave in request order.
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
        bool buffered = false;  // whole frames already wait in _h_in: walk them before blocking in recv
        int cur = 0;            // the staging slot frames are received into
        use_slot(cur);
        pending pend;
        auto finish = [&] {
            if (!pend.valid) return;
            use_slot(pend.slot);
            process_end(fd, pend, st);
            pend.valid = false;
            use_slot(cur);
        };
        while (true) {
            if (!eof && !buffered) {
                // answer a batch in flight before a recv that would block
                if (pend.valid && !more_pending(fd)) finish();
                // cap - have > 0 here: a full buffer is always consumed below,
                // so recv returning 0 is the peer's orderly shutdown
                auto t0 = clock::now();
                ssize_t k = recv(fd, _h_in + have, cap - have, 0);
                if (k < 0 && errno == EINTR) continue;
                st.recv_seconds += secs(t0);
                if (k <= 0) eof = true;
                else have += static_cast<uint64_t>(k);
            }
            buffered = false;
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
            if (nf) {
                if (_nslots == 2) {
                    pending p = process_begin(nf, walked, st);
                    p.slot = cur;
                    finish();  // the previous batch's answers: its work ran while this one arrived
                    pend = p;
                    // the rest of the buffer (a cut frame) continues in the other slot
                    const int nxt = cur ^ 1;
                    std::memcpy(_slots[nxt].h_in, _h_in + walked, have - walked);
                    cur = nxt;
                    use_slot(cur);
                } else {
                    pending p = process_begin(nf, walked, st);
                    p.slot = cur;
                    process_end(fd, p, st);
                    std::memmove(_h_in, _h_in + walked, have - walked);
                }
            } else {
                std::memmove(_h_in, _h_in + walked, have - walked);
            }
            have -= walked;
            walked = 0;
            nf = 0;
            if (oversize) {
                finish();
                if (!serve_oversize(fd, have, st)) return st;
                have = 0;
            }
            // A batch ends at max_batch frames, so the buffer can still hold
            // whole frames (frames shorter than the method's fin) while the
            // peer, having sent everything, waits for their answers: serve
            // them before the next recv, which would block.
            buffered = have >= 4 && have - 4 >= be32_at(_h_in);
        }
        finish();
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
        // string-bodied methods (register_var_method); their device buffers are
        // sized with the batch buffer (ensure / release)
        bool var = false;
        var_handler_t vhandler;
        var_limits lim;
        std::vector<uint8_t> req_prefix;           // str(method) | str(Req::name)
        uint64_t min_in = 0, min_out = 0;          // records with empty strings
        std::vector<bool> req_string, resp_string;
        std::vector<uint64_t> req_size, resp_size;  // fixed leaves' bytes
        std::vector<uint64_t*> req_offs, resp_offs; // string leaves' n+1 offsets (nullptr: fixed)
        uint8_t* resp_wire = nullptr;               // packed responses and their index
        uint64_t resp_wire_cap = 0;
        uint64_t* resp_rec = nullptr;
        uint64_t* h_ends = nullptr;                 // pinned: per response field, offs[0] and offs[n]
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
    /// Bytes of a batch's reply stream: every frame of the widest fixed
    /// response, plus every string method's framed responses.
    uint64_t out_cap() const {
        uint64_t c = _max * max_fout();
        for (auto const& m : _m)
            if (m->var) c += m->resp_wire_cap + 4 * _max;
        return c;
    }
    bool any_var_method() const {
        for (auto const& m : _m)
            if (m->var) return true;
        return false;
    }

    /// A string method's device buffers for batches of _max frames in _cap bytes.
    void alloc_var(method_entry& m) {
        m.req_cols.clear();
        m.req_bytes.clear();
        m.req_offs.clear();
        for (size_t f = 0; f < m.req_string.size(); ++f) {
            m.req_bytes.push_back(m.req_string[f] ? _cap + 16 : _max * m.req_size[f] + 16);
            m.req_cols.push_back(alloc(m.req_bytes.back()));
            m.req_offs.push_back(m.req_string[f] ? static_cast<uint64_t*>(alloc(8 * (_max + 1) + 16)) : nullptr);
        }
        m.resp_cols.clear();
        m.resp_bytes.clear();
        m.resp_offs.clear();
        m.resp_wire_cap = _max * m.min_out + 16;
        for (size_t f = 0; f < m.resp_string.size(); ++f) {
            const uint64_t b = m.resp_string[f] ? _max * m.lim.max_response_chars + 16 : _max * m.resp_size[f] + 16;
            if (m.resp_string[f]) m.resp_wire_cap += b;
            m.resp_bytes.push_back(b);
            m.resp_cols.push_back(alloc(b));
            m.resp_offs.push_back(m.resp_string[f] ? static_cast<uint64_t*>(alloc(8 * (_max + 1) + 16)) : nullptr);
        }
        m.resp_wire = static_cast<uint8_t*>(alloc(m.resp_wire_cap));
        m.resp_rec = static_cast<uint64_t*>(alloc(8 * (_max + 1) + 16));
        check(hipHostMalloc(reinterpret_cast<void**>(&m.h_ends), 16 * m.resp_string.size() + 16, hipHostMallocDefault));
        uint64_t a = 0, b = 0;
        check_srpc(srpc_plan_var_scratch_bytes(m.in->get(), _max, _cap, &a), "srpc_plan_var_scratch_bytes");
        check_srpc(srpc_plan_var_scratch_bytes(m.out->get(), _max, m.resp_wire_cap, &b), "srpc_plan_var_scratch_bytes");
        _var_scratch_bytes = std::max({_var_scratch_bytes, a, b});
    }
    void free_var(method_entry& m) {
        for (void* p : m.req_cols) (void)hipFree(p);
        for (void* p : m.resp_cols) (void)hipFree(p);
        for (uint64_t* p : m.req_offs)
            if (p) (void)hipFree(p);
        for (uint64_t* p : m.resp_offs)
            if (p) (void)hipFree(p);
        if (m.resp_wire) (void)hipFree(m.resp_wire);
        if (m.resp_rec) (void)hipFree(m.resp_rec);
        if (m.h_ends) (void)hipHostFree(m.h_ends);
        m.h_ends = nullptr;
        m.req_cols.clear();
        m.resp_cols.clear();
        m.req_offs.clear();
        m.resp_offs.clear();
        m.resp_wire = nullptr;
        m.resp_rec = nullptr;
    }

    void ensure() {
        if (_h_in) return;
        const uint64_t K = _m.size();
        _cap = _max * max_fin();
        if (_cap > 0xffffffffull) throw plan_error("batch_server: batch buffer over 4 GiB", SRPC_E_UNSUPPORTED);
        _var_scratch_bytes = 0;
        for (auto& m : _m)
            if (m->var) alloc_var(*m);
        if (_var_scratch_bytes) _d_var_scratch = alloc(_var_scratch_bytes);
        if (any_var_method()) {
            _d_var_rec = alloc(8 * (_max + 1) + 16);
            check(hipHostMalloc(reinterpret_cast<void**>(&_h_out_off), 8 * (_max + 1) + 16, hipHostMallocDefault));
        }
        const uint64_t out_cap = this->out_cap();
        // two staging slots (two batches in flight) unless a string method's
        // batches need the host between their kernels (SRPC_SERVER_SLOTS=1:
        // one batch at a time, the A/B baseline)
        const char* slots_env = std::getenv("SRPC_SERVER_SLOTS");
        _nslots = any_var_method() || (slots_env && slots_env[0] == '1') ? 1 : 2;
        for (int i = 0; i < _nslots; ++i) {
            slot& z = _slots[i];
            check(hipHostMalloc(reinterpret_cast<void**>(&z.h_in), _cap + 16, hipHostMallocDefault));
            check(hipHostMalloc(reinterpret_cast<void**>(&z.h_offs), 4 * _max + 16, hipHostMallocDefault));
            check(hipHostMalloc(reinterpret_cast<void**>(&z.h_out), out_cap + 16, hipHostMallocDefault));
            check(hipHostMalloc(reinterpret_cast<void**>(&z.h_cls), _max + 16, hipHostMallocDefault));
            // per method: its unpack status [k], its pack status [K + k] (each
            // call resets its own, so methods never clear each other's)
            check(hipHostMalloc(reinterpret_cast<void**>(&z.h_status), 2 * K * sizeof(srpc_unpack_status),
                                hipHostMallocDefault));
            check(hipEventCreateWithFlags(&z.done, hipEventDisableTiming));
        }
        use_slot(0);
        check(hipHostMalloc(reinterpret_cast<void**>(&_h_counts), 8 * (K + 2) + 16, hipHostMallocDefault));
        check(hipMalloc(&_d_in, _cap + 16));
        check(hipMalloc(&_d_offs, 4 * _max + 16));
        check(hipMalloc(&_d_cls, _max + 16));
        check(hipMalloc(&_d_index, 4 * K * _max + 16));
        check(hipMalloc(&_d_counts, 8 * (K + 2) + 16));
        check(hipMalloc(&_d_out_off, 8 * (_max + 1) + 16));
        check(hipMalloc(&_d_gather, _cap + 16));
        check(hipMalloc(&_d_resp, out_cap + 16));
        check(hipMalloc(&_d_out, out_cap + 16));
        check(hipMalloc(&_d_status, 2 * K * sizeof(srpc_unpack_status)));
        check_srpc(srpc_frames_scratch_bytes(_max, static_cast<int>(K), &_scratch_bytes), "srpc_frames_scratch_bytes");
        check(hipMalloc(&_d_scratch, _scratch_bytes));
        _in_plans.clear();
        _resp_bytes.clear();
        _var_rec.clear();
        _var_idx.clear();
        for (auto const& m : _m) {
            if (m->var) _var_idx.push_back(_in_plans.size());
            _in_plans.push_back(m->in->get());
            _resp_bytes.push_back(static_cast<uint32_t>(m->fout));
            _var_rec.push_back(m->var ? m->resp_rec : nullptr);
        }
        warm_up();
    }

    /// One-frame run of every kernel the batches use (the library's and each
    /// handler, on one all-zero record) and one copy through every staging
    /// buffer, at serve start: first uses cost milliseconds that otherwise land
    /// on the connection's first batch (profiles/r02_e2e_warmup.log).
    void warm_up() {
        const int K = static_cast<int>(_m.size());
        const uint64_t out_cap = this->out_cap();
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
            for (uint64_t* p : m->req_offs)
                if (p) check(hipMemsetAsync(p, 0, 8 * (_max + 1), _s));
            for (uint64_t* p : m->resp_offs)
                if (p) check(hipMemsetAsync(p, 0, 8 * (_max + 1), _s));
        }
        if (_d_var_scratch) check(hipMemsetAsync(_d_var_scratch, 0, _var_scratch_bytes, _s));
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
            check(hipMemsetAsync(_d_status, 0, 2 * _m.size() * sizeof(srpc_unpack_status), _s));
            for (size_t k = 0; k < _m.size(); ++k) {
                auto const& m = _m[k];
                if (m->var) {
                    warm_up_var(*m, k);
                    continue;
                }
                check_srpc(srpc_frames_gather(static_cast<const uint8_t*>(_d_in), static_cast<const uint32_t*>(_d_offs),
                                              static_cast<const uint32_t*>(_d_index), 1, static_cast<uint32_t>(m->fin),
                                              static_cast<uint8_t*>(_d_gather), _s),
                           "srpc_frames_gather");
                (void)srpc_gpu_unpack(m->in->get(), static_cast<const uint8_t*>(_d_gather), m->fin, 1,
                                      m->req_cols.data(), _d_status + k, _s);  // a prefix error on the zero frame: expected
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
            check(hipMemcpyAsync(_h_status, _d_status, 2 * _m.size() * sizeof(srpc_unpack_status), hipMemcpyDeviceToHost,
                                 _s));
            check(hipStreamSynchronize(_s));
        }
    }
    /// One string-method batch on one well-formed request with empty strings
    /// (its prefix, zeros): every kernel of the var path and the handler load
    /// their code objects here, not on the first batch.
    void warm_up_var(method_entry& m, size_t k) {
        std::vector<uint8_t> f = be32(static_cast<uint32_t>(m.min_in));
        f.insert(f.end(), m.req_prefix.begin(), m.req_prefix.end());
        f.resize(4 + m.min_in, 0);
        check(hipMemcpyAsync(_d_in, f.data(), f.size(), hipMemcpyHostToDevice, _s));
        check(hipMemsetAsync(_d_index, 0, 4, _s));
        check(hipMemsetAsync(_d_offs, 0, 4, _s));
        check_srpc(srpc_frames_gather_var(static_cast<const uint8_t*>(_d_in), static_cast<const uint32_t*>(_d_offs),
                                          static_cast<const uint32_t*>(_d_index), 1, static_cast<uint8_t*>(_d_gather),
                                          static_cast<uint64_t*>(_d_var_rec), _d_scratch, _scratch_bytes, _s),
                   "srpc_frames_gather_var");
        run_var_unpack(m, k, 1, m.min_in);
        run_var_pack(m, k, 1);
        check_srpc(srpc_frames_scatter_var(m.resp_wire, m.resp_rec, static_cast<const uint32_t*>(_d_index), 1,
                                           static_cast<const uint64_t*>(_d_out_off), static_cast<uint8_t*>(_d_out), _s),
                   "srpc_frames_scatter_var");
    }
    /// unpack_var -> handler over n gathered requests (_d_gather, index
    /// _d_var_rec, at most wire_len bytes) of method k, then the first and last
    /// offsets of every response string field to m.h_ends (checked against the
    /// columns' sizes before anything reads the chars: run_var_pack).
    void run_var_unpack(method_entry& m, size_t k, uint64_t n, uint64_t wire_len) {
        check_srpc(srpc_gpu_unpack_var(m.in->get(), static_cast<const uint8_t*>(_d_gather), wire_len, n,
                                       static_cast<const uint64_t*>(_d_var_rec), m.req_cols.data(), m.req_offs.data(),
                                       _d_status + k, _d_var_scratch, _var_scratch_bytes, _s),
                   "srpc_gpu_unpack_var");
        std::vector<const uint64_t*> req_offs(m.req_offs.begin(), m.req_offs.end());
        var_batch b;
        b.n = n;
        b.req_cols = m.req_cols.data();
        b.req_str_offs = req_offs.data();
        b.resp_cols = m.resp_cols.data();
        b.resp_str_offs = m.resp_offs.data();
        b.resp_cap = m.resp_bytes.data();
        check_srpc(m.vhandler(b, _s), "batch handler");
        for (size_t f = 0; f < m.resp_offs.size(); ++f) {
            if (!m.resp_offs[f]) continue;
            check(hipMemcpyAsync(m.h_ends + 2 * f, m.resp_offs[f], 8, hipMemcpyDeviceToHost, _s));
            check(hipMemcpyAsync(m.h_ends + 2 * f + 1, m.resp_offs[f] + n, 8, hipMemcpyDeviceToHost, _s));
        }
    }
    /// The handler's response strings of method k fit its columns: offs[0] <=
    /// offs[n] <= the column's bytes (m.h_ends, after a sync).  The handler
    /// contract (var_batch) asks for non-decreasing offsets within the column.
    bool var_responses_fit(method_entry const& m) const {
        for (size_t f = 0; f < m.resp_offs.size(); ++f) {
            if (!m.resp_offs[f]) continue;
            const uint64_t a = m.h_ends[2 * f], e = m.h_ends[2 * f + 1];
            if (a > e || e > m.resp_bytes[f]) return false;
        }
        return true;
    }
    void run_var_pack(method_entry& m, size_t k, uint64_t n) {
        std::vector<const uint64_t*> resp_offs(m.resp_offs.begin(), m.resp_offs.end());
        std::vector<const void*> resp_cols(m.resp_cols.begin(), m.resp_cols.end());
        check_srpc(srpc_gpu_pack_var(m.out->get(), resp_cols.data(), resp_offs.data(), n, m.resp_wire, m.resp_wire_cap,
                                     m.resp_rec, _d_status + _m.size() + k, _d_var_scratch, _var_scratch_bytes, _s),
                   "srpc_gpu_pack_var");
    }

    void release() {
        for (auto& m : _m)
            if (m->var) free_var(*m);
        for (void* p : {_d_var_rec, _d_var_scratch})
            if (p) (void)hipFree(p);
        if (_h_out_off) (void)hipHostFree(_h_out_off);
        _d_var_rec = _d_var_scratch = nullptr;
        _h_out_off = nullptr;
        for (void* p : {_d_in, _d_offs, _d_cls, _d_index, _d_counts, _d_out_off, _d_gather, _d_resp, _d_out,
                        static_cast<void*>(_d_status), _d_scratch})
            if (p) (void)hipFree(p);
        for (slot& z : _slots) {
            for (void* p : {static_cast<void*>(z.h_in), static_cast<void*>(z.h_offs), static_cast<void*>(z.h_out),
                            static_cast<void*>(z.h_cls), static_cast<void*>(z.h_status)})
                if (p) (void)hipHostFree(p);
            if (z.done) (void)hipEventDestroy(z.done);
            z = slot{};
        }
        _nslots = 0;
        if (_h_counts) (void)hipHostFree(_h_counts);
        _d_in = _d_offs = _d_cls = _d_index = _d_counts = _d_out_off = _d_gather = _d_resp = _d_out = _d_scratch =
            nullptr;
        _d_status = nullptr;
        _h_in = _h_out = _h_cls = nullptr;
        _h_offs = nullptr;
        _h_counts = nullptr;
        _h_status = nullptr;
    }

    /// A batch between process_begin and process_end.
    struct pending {
        bool valid = false;
        int slot = 0;
        uint64_t nf = 0, used = 0, unknown = 0, total = 0;
        bool any_var = false, mixed = false;
        double gpu_s = 0;  // host time spent on the batch's GPU work (enqueue, syncs, the final wait)
    };
    void use_slot(int i) {
        slot& z = _slots[i];
        _h_in = z.h_in;
        _h_offs = z.h_offs;
        _h_out = z.h_out;
        _h_cls = z.h_cls;
        _h_status = z.h_status;
    }

    /// The GPU path for the nf whole frames in _h_in[0, used): every copy and
    /// kernel enqueued (with the host syncs the batch's own decisions need:
    /// its bucket counts, a string method's response sizes), the last copy
    /// marked by the slot's event.  process_end answers it.
    pending process_begin(uint64_t nf, uint64_t used, batch_stats& st) {
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
        const bool var_methods = !_var_idx.empty();
        if (var_methods) check(hipMemcpyAsync(_h_cls, _d_cls, nf, hipMemcpyDeviceToHost, _s));
        mark("classify");
        check(hipStreamSynchronize(_s));
        mark("sync1");
        st.classify_seconds += secs(t0);
        uint64_t unknown = _h_counts[K + 1];
        bool mixed = false, any_var = false;
        for (int k = 0; k < K; ++k) any_var |= _m[static_cast<size_t>(k)]->var && _h_counts[k] > 0;
        uint64_t var_bytes[SRPC_FRAMES_MAX_PLANS] = {};  // payload bytes of each string method's frames
        if (any_var)
            for (uint64_t i = 0; i < nf; ++i) {
                const uint8_t c = _h_cls[i];
                if (c != SRPC_FRAME_UNKNOWN && _m[c]->var) var_bytes[c] += (i + 1 < nf ? _h_offs[i + 1] : used) - _h_offs[i] - 4;
            }
        check(hipMemsetAsync(_d_status, 0, 2 * static_cast<uint64_t>(K) * sizeof(srpc_unpack_status), _s));
        bool demoted[SRPC_FRAMES_MAX_PLANS] = {};  // string methods whose answers go to the CPU this batch
        if (any_var) {
            // string methods first: their responses' sizes place every answer.
            // unpack + handler, then the responses' sizes are checked on the
            // host BEFORE anything reads the response chars: a batch whose
            // answers do not fit the columns (max_response_chars) is answered
            // on the CPU server instead, in place (its frames become unknown)
            for (int k = 0; k < K; ++k) {
                method_entry& m = *_m[static_cast<size_t>(k)];
                const uint64_t n = _h_counts[k];
                if (!m.var || !n) continue;
                mixed |= n != nf;
                check_srpc(srpc_frames_gather_var(d_in, d_offs, d_idx + static_cast<uint64_t>(k) * nf, n,
                                                  static_cast<uint8_t*>(_d_gather), static_cast<uint64_t*>(_d_var_rec),
                                                  _d_scratch, _scratch_bytes, _s),
                           "srpc_frames_gather_var");
                run_var_unpack(m, static_cast<size_t>(k), n, var_bytes[k]);
                mark("var unpack");
            }
            check(hipStreamSynchronize(_s));  // the responses' sizes
            bool any_demoted = false;
            for (int k = 0; k < K; ++k) {
                method_entry& m = *_m[static_cast<size_t>(k)];
                if (!m.var || !_h_counts[k] || var_responses_fit(m)) continue;
                demoted[k] = any_demoted = true;
                st.overflow_batches += 1;
            }
            if (any_demoted) {
                for (uint64_t i = 0; i < nf; ++i)
                    if (_h_cls[i] != SRPC_FRAME_UNKNOWN && demoted[_h_cls[i]]) _h_cls[i] = SRPC_FRAME_UNKNOWN;
                for (int k = 0; k < K; ++k)
                    if (demoted[k]) {
                        unknown += _h_counts[k];
                        _h_counts[k] = 0;
                    }
                check(hipMemcpyAsync(_d_cls, _h_cls, nf, hipMemcpyHostToDevice, _s));
                check(hipMemcpyAsync(d_counts, _h_counts, 8 * static_cast<uint64_t>(K), hipMemcpyHostToDevice, _s));
                // the copies read pinned memory the next batch rewrites
                check(hipStreamSynchronize(_s));
            }
            for (int k = 0; k < K; ++k) {
                method_entry& m = *_m[static_cast<size_t>(k)];
                if (m.var && _h_counts[k]) run_var_pack(m, static_cast<size_t>(k), _h_counts[k]);
            }
            mark("var pack");
            check_srpc(srpc_frames_offsets(_in_plans.data(), _resp_bytes.data(), K, static_cast<const uint8_t*>(_d_cls),
                                           nf, d_idx, d_counts, _var_rec.data(), d_out_off, d_counts + K, _d_scratch,
                                           _scratch_bytes, _s),
                       "srpc_frames_offsets");
            check(hipMemcpyAsync(_h_counts + K, d_counts + K, 8, hipMemcpyDeviceToHost, _s));
        }
        for (int k = 0; k < K; ++k) {
            const uint64_t n = _h_counts[k];
            method_entry& m = *_m[static_cast<size_t>(k)];
            if (!n || m.var) continue;
            const bool whole = n == nf;  // every frame is method k: they already are its contiguous records
            mixed |= !whole;
            const uint8_t* src = d_in;
            if (!whole) {
                check_srpc(srpc_frames_gather(d_in, d_offs, d_idx + static_cast<uint64_t>(k) * nf, n,
                                              static_cast<uint32_t>(m.fin), static_cast<uint8_t*>(_d_gather), _s),
                           "srpc_frames_gather");
                src = static_cast<const uint8_t*>(_d_gather);
            }
            check_srpc(srpc_gpu_unpack(m.in->get(), src, n * m.fin, n, m.req_cols.data(), _d_status + k, _s),
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
        if (any_var) {
            for (int k = 0; k < K; ++k) {
                method_entry& m = *_m[static_cast<size_t>(k)];
                const uint64_t n = _h_counts[k];
                if (m.var && n)
                    check_srpc(srpc_frames_scatter_var(m.resp_wire, m.resp_rec, d_idx + static_cast<uint64_t>(k) * nf,
                                                       n, d_out_off, static_cast<uint8_t*>(_d_out), _s),
                               "srpc_frames_scatter_var");
            }
            if (unknown) check(hipMemcpyAsync(_h_out_off, d_out_off, 8 * (nf + 1), hipMemcpyDeviceToHost, _s));
            check(hipStreamSynchronize(_s));  // the reply stream's size
            mark("sync_var");
        }
        const uint64_t total = _h_counts[K];
        if (total) check(hipMemcpyAsync(_h_out, _d_out, total, hipMemcpyDeviceToHost, _s));
        mark("d2h_out");
        if (unknown && !var_methods) check(hipMemcpyAsync(_h_cls, _d_cls, nf, hipMemcpyDeviceToHost, _s));
        check(hipMemcpyAsync(_h_status, _d_status, 2 * static_cast<uint64_t>(K) * sizeof(srpc_unpack_status),
                             hipMemcpyDeviceToHost, _s));
        mark("d2h");
        pending pd;
        for (int i = 0; i < _nslots; ++i)
            if (_slots[i].h_in == _h_in) pd.slot = i;
        check(hipEventRecord(_slots[pd.slot].done, _s));
        pd.valid = true;
        pd.nf = nf;
        pd.used = used;
        pd.unknown = unknown;
        pd.total = total;
        pd.any_var = any_var;
        pd.mixed = mixed;
        pd.gpu_s = secs(t0);
        return pd;
    }

    /// Wait for a batch's last copy (its slot's buffers in use), check its
    /// statuses and send its answers: the GPU's in runs, the CPU's in their
    /// places.
    void process_end(int fd, pending const& pd, batch_stats& st) {
        const int K = static_cast<int>(_m.size());
        const uint64_t nf = pd.nf, used = pd.used, unknown = pd.unknown, total = pd.total;
        const bool any_var = pd.any_var, mixed = pd.mixed, var_methods = !_var_idx.empty();
        auto t0 = clock::now();
        check(hipEventSynchronize(_slots[pd.slot].done));
        if (_trace)
            std::fprintf(stderr, "batch %llu nf %llu wait       %.3f ms\n", (unsigned long long)st.gpu_batches,
                         (unsigned long long)nf, 1e3 * secs(t0));
        // classification already matched every prefix and length (and walked
        // string records to their frame's end), and string responses were
        // checked against their columns before packing: a status here means
        // the buckets and the plans disagree (an internal invariant)
        for (int k = 0; k < 2 * K; ++k)
            if (_h_status[k].flags)
                throw plan_error(k < K ? "batch_server: classified frame failed to unpack"
                                       : "batch_server: string responses overran a sized wire",
                                 SRPC_E_INVALID);
        const double dt = pd.gpu_s + secs(t0);
        if (st.gpu_batches == 0 && st.fallback_requests == 0) st.first_batch_seconds = dt;
        st.gpu_seconds += dt;
        st.h2d_bytes += used + 4 * nf;
        st.d2h_bytes += total + (unknown || var_methods ? nf : 0) + (unknown && any_var ? 8 * (nf + 1) : 0);
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
                run = any_var ? _h_out_off[i + 1] : run + _m[c]->fout;  // the end of frame i's answer
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
    // the staging slot in use (the pinned buffers of _slots[i], use_slot)
    uint8_t* _h_in = nullptr;
    uint32_t* _h_offs = nullptr;
    uint8_t* _h_out = nullptr;
    uint8_t* _h_cls = nullptr;
    uint64_t* _h_counts = nullptr;
    srpc_unpack_status* _h_status = nullptr;
    struct slot {
        uint8_t* h_in = nullptr;
        uint32_t* h_offs = nullptr;
        uint8_t* h_out = nullptr;
        uint8_t* h_cls = nullptr;
        srpc_unpack_status* h_status = nullptr;
        hipEvent_t done = nullptr;  // the batch's last copy
    };
    slot _slots[2];
    int _nslots = 0;
    void *_d_in = nullptr, *_d_offs = nullptr, *_d_cls = nullptr, *_d_index = nullptr, *_d_counts = nullptr,
         *_d_out_off = nullptr, *_d_gather = nullptr, *_d_resp = nullptr, *_d_out = nullptr, *_d_scratch = nullptr;
    srpc_unpack_status* _d_status = nullptr;
    // string methods
    std::vector<const uint64_t*> _var_rec;  // per method: its response index (nullptr: fixed)
    std::vector<size_t> _var_idx;           // the string methods' slots
    void* _d_var_rec = nullptr;             // the request index of the bucket being served
    void* _d_var_scratch = nullptr;
    uint64_t _var_scratch_bytes = 0;
    uint64_t* _h_out_off = nullptr;
};

}  // namespace srpc::gpu
