// e2e_square: BASELINE.json configs[4] -- Calculator.square end to end over
// loopback, 1M requests, server-side GPU-batched unpack -> square -> pack --
// and the same server under mixed traffic.
//
// One process, two threads talking over 127.0.0.1:
//   client: the frames Calculator_stub sends (calculator_srpc.cpp:58-134:
//           pack_request("Calculator_servicer::<m>", Number | TwoNumbers) +
//           u32 BE length), all N pipelined on one connection by a sender
//           thread, responses read back and checked against the method's
//           result and (optionally) written out so their SHA-256 can be
//           compared with the reference digest;
//   server: --mode gpu: srpc::gpu::batch_server (include/srpc/gpu_server.hpp)
//                       with square (and with --gpu-methods all: add, subtract,
//                       multiply) on the GPU, the rest on the CPU server;
//           --mode cpu: the scalar srpc::server (include/srpc/server.hpp),
//                       the reference's per-request dispatch path.
// Traffic: num = splitmix64(0x5EED) % 46341 for square;
//   --mix F      a fraction F of add / subtract / multiply requests (TwoNumbers);
//   --foreign F  a fraction F of divide requests (a method the GPU server does
//                not have: answered by the CPU server in their places);
//   --poison i[,j..]   requests with an unknown method name (NOT_REGISTERED);
//   --poison-method    the name used (another length moves every later frame);
//   --oversize i       request i has a method name longer than the batch buffer;
//   --echo F     a fraction F of Echo_servicer::echo requests (multiple_primitives
//                with a 0..40-byte string, tests/cpp/echo_records.hpp): a
//                string-bodied method, on the GPU with --gpu-methods ...,echo
//                (register_var_method), else on the CPU server; --echo 1
//                --dump writes the unframed responses for the reference
//                digest (tests/golden/manifest.json echo_responses).
// Prints one JSON line.
#include <hip/hip_runtime.h>
#include <srpc/gpu_server.hpp>
#include <srpc/server.hpp>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../tests/cpp/echo_records.hpp"

struct Number : public srpc::message_base {
    int32_t num;
    static constexpr const char* name = "Number";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(Number, num, "Number::num"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> num;
    }
};

struct TwoNumbers : public srpc::message_base {
    int32_t left;
    int32_t right;
    static constexpr const char* name = "TwoNumbers";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(TwoNumbers, left, "TwoNumbers::left"),
                                                   STRUCT_MEMBER(TwoNumbers, right, "TwoNumbers::right"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> left;
        p >> right;
    }
};

// The reference packer test's message with a string (packer_test.cpp:26-45).
struct multiple_primitives : public srpc::message_base {
    int8_t arg1;
    char arg2;
    int64_t arg3;
    std::string arg4;
    static constexpr const char* name = "multiple_primitives";
    static constexpr auto fields =
        std::make_tuple(STRUCT_MEMBER(multiple_primitives, arg1, "multiple_primitives::arg1"),
                        STRUCT_MEMBER(multiple_primitives, arg2, "multiple_primitives::arg2"),
                        STRUCT_MEMBER(multiple_primitives, arg3, "multiple_primitives::arg3"),
                        STRUCT_MEMBER(multiple_primitives, arg4, "multiple_primitives::arg4"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> arg1;
        p >> arg2;
        p >> arg3;
        p >> arg4;
    }
};

struct Echo_servicer : srpc::servicer_base {
    virtual multiple_primitives echo(multiple_primitives&) { throw std::runtime_error("Method not implemented!"); }
    static constexpr const char* name = "Echo";
    static constexpr auto methods = std::make_tuple(STRUCT_MEMBER(Echo_servicer, echo, "Echo_servicer::echo"));
};
struct EchoImpl : Echo_servicer {
    multiple_primitives echo(multiple_primitives& q) override { return echo_fixture::answer(q); }
};

enum Op : int { SQUARE = 0, ADD = 1, SUB = 2, MUL = 3, DIV = 4, POISON = 5, OVERSIZE = 6, ECHO = 7 };

static int32_t expect(int op, int32_t l, int32_t r) {
    const uint32_t a = static_cast<uint32_t>(l), b = static_cast<uint32_t>(r);
    switch (op) {
        case SQUARE: return static_cast<int32_t>(a * a);
        case ADD: return static_cast<int32_t>(a + b);
        case SUB: return static_cast<int32_t>(a - b);
        case MUL: return static_cast<int32_t>(a * b);
        default: return l / r;
    }
}

struct Calculator_servicer : srpc::servicer_base {
    virtual Number add(TwoNumbers&) { throw std::runtime_error("Method not implemented!"); }
    virtual Number subtract(TwoNumbers&) { throw std::runtime_error("Method not implemented!"); }
    virtual Number multiply(TwoNumbers&) { throw std::runtime_error("Method not implemented!"); }
    virtual Number divide(TwoNumbers&) { throw std::runtime_error("Method not implemented!"); }
    virtual Number square(Number&) { throw std::runtime_error("Method not implemented!"); }
    static constexpr const char* name = "Calculator";
    static constexpr auto methods =
        std::make_tuple(STRUCT_MEMBER(Calculator_servicer, add, "Calculator_servicer::add"),
                        STRUCT_MEMBER(Calculator_servicer, subtract, "Calculator_servicer::subtract"),
                        STRUCT_MEMBER(Calculator_servicer, multiply, "Calculator_servicer::multiply"),
                        STRUCT_MEMBER(Calculator_servicer, divide, "Calculator_servicer::divide"),
                        STRUCT_MEMBER(Calculator_servicer, square, "Calculator_servicer::square"));
};

struct Calculator : Calculator_servicer {
    static Number num(int32_t v) {
        Number r;
        r.num = v;
        return r;
    }
    Number add(TwoNumbers& q) override { return num(expect(ADD, q.left, q.right)); }
    Number subtract(TwoNumbers& q) override { return num(expect(SUB, q.left, q.right)); }
    Number multiply(TwoNumbers& q) override { return num(expect(MUL, q.left, q.right)); }
    Number divide(TwoNumbers& q) override { return num(expect(DIV, q.left, q.right)); }
    Number square(Number& q) override { return num(expect(SQUARE, q.num, 0)); }
};

// The batched methods on the device: int32 columns in, one out.
__global__ void k_square(const int32_t* __restrict__ in, int32_t* __restrict__ out, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t v = static_cast<uint32_t>(in[i]);
        out[i] = static_cast<int32_t>(v * v);
    }
}

template <int OP>
__global__ void k_binop(const int32_t* __restrict__ l, const int32_t* __restrict__ r, int32_t* __restrict__ out,
                        uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t a = static_cast<uint32_t>(l[i]), b = static_cast<uint32_t>(r[i]);
        out[i] = static_cast<int32_t>(OP == ADD ? a + b : OP == SUB ? a - b : a * b);
    }
}

static int square_batch(void* const* req, void* const* resp, uint64_t n, hipStream_t s) {
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_square, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s,
                       static_cast<const int32_t*>(req[0]), static_cast<int32_t*>(resp[0]), n);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int OP>
static int binop_batch(void* const* req, void* const* resp, uint64_t n, hipStream_t s) {
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_binop<OP>, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s,
                       static_cast<const int32_t*>(req[0]), static_cast<const int32_t*>(req[1]),
                       static_cast<int32_t*>(resp[0]), n);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Echo on the device: ints + 1, each string with "!" appended (response
// string i starts at req_offs[i] - req_offs[0] + i).  A thread per record.
__global__ void k_echo(const int8_t* a1, const int8_t* a2, const int64_t* a3, const uint8_t* chars,
                       const uint64_t* offs, int8_t* r1, int8_t* r2, int64_t* r3, uint8_t* rchars, uint64_t* roffs,
                       uint64_t n, uint64_t cap) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i > n) return;
    const uint64_t o0 = offs[0];
    roffs[i] = offs[i] - o0 + i;
    if (i == n) return;
    r1[i] = static_cast<int8_t>(static_cast<uint8_t>(a1[i]) + 1u);
    r2[i] = static_cast<int8_t>(static_cast<uint8_t>(a2[i]) + 1u);
    r3[i] = static_cast<int64_t>(static_cast<uint64_t>(a3[i]) + 1u);
    const uint64_t b = offs[i], e = offs[i + 1], d = offs[i] - o0 + i;
    if (d + (e - b) + 1 > cap) return;  // past the response column: pack_var reports it
    for (uint64_t k = 0; k < e - b; ++k) rchars[d + k] = chars[b + k];
    rchars[d + (e - b)] = '!';
}

static int echo_batch(srpc::gpu::var_batch const& b, hipStream_t s) {
    const uint64_t blocks = (b.n + 1 + 255) / 256;
    hipLaunchKernelGGL(k_echo, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s,
                       static_cast<const int8_t*>(b.req_cols[0]), static_cast<const int8_t*>(b.req_cols[1]),
                       static_cast<const int64_t*>(b.req_cols[2]), static_cast<const uint8_t*>(b.req_cols[3]),
                       b.req_str_offs[3], static_cast<int8_t*>(b.resp_cols[0]), static_cast<int8_t*>(b.resp_cols[1]),
                       static_cast<int64_t*>(b.resp_cols[2]), static_cast<uint8_t*>(b.resp_cols[3]), b.resp_str_offs[3],
                       b.n, b.resp_cap[3]);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

static uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <typename T>
static void append_frame(std::vector<uint8_t>& frames, std::string const& method, T&& v) {
    srpc::packer pr;
    srpc::request_t<std::decay_t<T>> req;
    req.set_method_name(method);
    req.set_value(std::forward<T>(v));
    pr.pack_request(req);
    const uint32_t len = htonl(static_cast<uint32_t>(pr.size()));
    const uint8_t* lb = reinterpret_cast<const uint8_t*>(&len);
    frames.insert(frames.end(), lb, lb + 4);
    frames.insert(frames.end(), pr.data(), pr.data() + pr.size());
}

int main(int argc, char** argv) {
    uint64_t n = 1u << 20;
    uint64_t batch = 1u << 18;
    std::string mode = "gpu", port = "18090", dump, gpu_methods = "square";
    std::set<uint64_t> poison;
    std::string poison_method = "Calculator_servicer::squarX";  // same frame length as square's
    int64_t oversize = -1;
    double mix = 0, foreign = 0, echo = 0;
    int watchdog_s = 60;
    uint64_t max_resp_chars = 0;  // 0: var_limits' default
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&] { return std::string(i + 1 < argc ? argv[++i] : ""); };
        if (a == "--n") n = std::stoull(next());
        else if (a == "--batch") batch = std::stoull(next());
        else if (a == "--mode") mode = next();
        else if (a == "--port") port = next();
        else if (a == "--dump") dump = next();
        else if (a == "--poison") {
            std::stringstream ss(next());
            for (std::string t; std::getline(ss, t, ',');) poison.insert(std::stoull(t));
        } else if (a == "--poison-method") poison_method = next();
        else if (a == "--oversize") oversize = std::stoll(next());
        else if (a == "--mix") mix = std::stod(next());
        else if (a == "--foreign") foreign = std::stod(next());
        else if (a == "--echo") echo = std::stod(next());
        else if (a == "--gpu-methods") gpu_methods = next();
        else if (a == "--watchdog") watchdog_s = std::stoi(next());
        else if (a == "--max-resp-chars") max_resp_chars = std::stoull(next());
    }
    srpc::message_registry["Number"] = []() -> std::unique_ptr<Number> { return std::make_unique<Number>(); };
    srpc::message_registry["TwoNumbers"] = []() -> std::unique_ptr<TwoNumbers> {
        return std::make_unique<TwoNumbers>();
    };
    srpc::message_registry["multiple_primitives"] = []() -> std::unique_ptr<multiple_primitives> {
        return std::make_unique<multiple_primitives>();
    };

    // ---- server ------------------------------------------------------------
    Calculator calc;
    EchoImpl echo_svc;
    srpc::server cpu_server;
    cpu_server.register_service(calc);
    cpu_server.register_service(echo_svc);
    std::unique_ptr<srpc::gpu::batch_server> gsrv;
    uint64_t buffer_bytes = 0;
    if (mode == "gpu") {
        gsrv = srpc::gpu::batch_server::single<Number, Number>("Calculator_servicer::square", square_batch, batch, 0,
                                                               &cpu_server);
        if (gpu_methods.find("echo") != std::string::npos) {
            srpc::gpu::var_limits lim;
            if (max_resp_chars) lim.max_response_chars = max_resp_chars;
            gsrv->register_var_method<multiple_primitives, multiple_primitives>(echo_fixture::kMethod, echo_batch, lim);
        }
        if (gpu_methods.find("all") != std::string::npos) {
            gsrv->register_method<TwoNumbers, Number>("Calculator_servicer::add", binop_batch<ADD>);
            gsrv->register_method<TwoNumbers, Number>("Calculator_servicer::subtract", binop_batch<SUB>);
            gsrv->register_method<TwoNumbers, Number>("Calculator_servicer::multiply", binop_batch<MUL>);
        }
        buffer_bytes = gsrv->buffer_bytes();
    }

    // ---- client-side request frames, exactly as the stub builds them -------
    std::vector<int32_t> lhs(n), rhs(n);
    std::vector<uint8_t> ops(n);
    uint64_t st = 0x5EED, st2 = 0xF00D;
    for (uint64_t i = 0; i < n; ++i) {
        const int32_t v = static_cast<int32_t>(static_cast<uint32_t>(splitmix(&st)));
        lhs[i] = v % 46341;
        const double u = static_cast<double>(splitmix(&st2) >> 11) * 0x1.0p-53;
        const uint64_t w = splitmix(&st2);
        ops[i] = u < foreign ? DIV : u < foreign + mix ? static_cast<uint8_t>(ADD + w % 3)
                 : u < foreign + mix + echo ? ECHO : SQUARE;
        rhs[i] = ops[i] == DIV ? static_cast<int32_t>(w >> 40) % 1000 + 1 : static_cast<int32_t>(w >> 32);
        if (poison.count(i)) ops[i] = POISON;
        if (static_cast<int64_t>(i) == oversize) ops[i] = OVERSIZE;
    }
    static const char* kName[] = {"Calculator_servicer::square", "Calculator_servicer::add",
                                  "Calculator_servicer::subtract", "Calculator_servicer::multiply",
                                  "Calculator_servicer::divide"};
    std::vector<uint8_t> frames;
    frames.reserve(n * 62);
    uint64_t counts[8] = {};
    uint64_t resp_total = 0;
    std::vector<uint8_t> echo_resp;      // the expected echo answers, framed, in request order
    std::vector<uint64_t> echo_at(n, 0);  // where request i's answer starts in echo_resp
    for (uint64_t i = 0; i < n; ++i) {
        const int op = ops[i];
        counts[op] += 1;
        if (op == ECHO) {
            multiple_primitives q;
            echo_fixture::fill_request(q, i);
            srpc::packer pr;
            srpc::response_t<multiple_primitives> r;
            r.set_value(echo_fixture::answer(q));
            pr.pack_response(r);
            const uint32_t len = htonl(static_cast<uint32_t>(pr.size()));
            const uint8_t* lb = reinterpret_cast<const uint8_t*>(&len);
            echo_at[i] = echo_resp.size();
            echo_resp.insert(echo_resp.end(), lb, lb + 4);
            echo_resp.insert(echo_resp.end(), pr.data(), pr.data() + pr.size());
            resp_total += 4 + pr.size();
            append_frame(frames, echo_fixture::kMethod, std::move(q));
            continue;
        }
        if (op == SQUARE || op == POISON) {
            Number v;
            v.num = lhs[i];
            append_frame(frames, op == POISON ? poison_method : kName[SQUARE], std::move(v));
        } else if (op == OVERSIZE) {
            Number v;
            v.num = lhs[i];
            append_frame(frames, std::string(std::max<uint64_t>(buffer_bytes, 4096) + 1000, 'Z'), std::move(v));
        } else {
            TwoNumbers v;
            v.left = lhs[i];
            v.right = rhs[i];
            append_frame(frames, kName[op], std::move(v));
        }
        // an unknown method is answered with the one status byte RPC_ERR_FUNCTION_NOT_REGISTERED
        resp_total += op == POISON || op == OVERSIZE ? 5 : 23;
    }

    const int lfd = srpc::transport::create_server_socket(port);
    if (lfd < 0) return 3;
    srpc::gpu::batch_stats stats;
    size_t cpu_served = 0;
    std::thread server_thread([&] {
        sockaddr_storage a{};
        socklen_t al = sizeof(a);
        int fd = accept(lfd, reinterpret_cast<sockaddr*>(&a), &al);
        int big = 8 << 20;
        setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
        setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
        try {
            if (gsrv) stats = gsrv->serve_connection(fd);
            else cpu_served = cpu_server.serve_connection(fd);
        } catch (std::exception const& e) {
            std::fprintf(stderr, "server: %s\n", e.what());
            std::fflush(stderr);
            std::_Exit(6);
        }
        close(fd);
    });

    // ---- client ------------------------------------------------------------
    const int fd = srpc::transport::create_client_socket("127.0.0.1", port);
    if (fd < 0) return 4;
    int big = 8 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
    std::vector<uint8_t> resp(resp_total);
    auto t0 = std::chrono::steady_clock::now();
    std::atomic<uint64_t> sent{0}, got{0};
    std::atomic<bool> done{false};
    std::thread sender([&] {
        for (uint64_t o = 0; o < frames.size();) {  // send_all, with progress for the watchdog
            const uint64_t k = std::min<uint64_t>(frames.size() - o, 1u << 20);
            if (!srpc::transport::send_all(fd, frames.data() + o, k)) break;
            o += k;
            sent = o;
        }
    });
    // a run that stalls says where it stalled instead of hanging until killed
    std::thread watchdog([&] {
        for (int i = 0; i < watchdog_s * 10 && !done; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
        if (done) return;
        std::fprintf(stderr, "WATCHDOG: %d s: client sent %llu of %zu request bytes, received %llu of %llu response bytes\n",
                     watchdog_s, (unsigned long long)sent.load(), frames.size(), (unsigned long long)got.load(),
                     (unsigned long long)resp_total);
        std::fflush(stderr);
        std::_Exit(5);
    });
    bool got_all = true;
    for (uint64_t o = 0; o < resp.size();) {
        const uint64_t k = std::min<uint64_t>(resp.size() - o, 1u << 20);
        if (!srpc::transport::recv_all(fd, resp.data() + o, k)) {
            got_all = false;
            break;
        }
        o += k;
        got = o;
    }
    auto t1 = std::chrono::steady_clock::now();
    done = true;
    watchdog.join();
    sender.join();
    shutdown(fd, SHUT_WR);
    close(fd);
    server_thread.join();
    close(lfd);
    const double secs = std::chrono::duration<double>(t1 - t0).count();

    // ---- check every response (client-side unpack_response<Number>) --------
    uint64_t bad = 0;
    const uint8_t* f = resp.data();
    for (uint64_t i = 0; got_all && i < n; ++i) {
        const uint32_t len = (uint32_t(f[0]) << 24) | (uint32_t(f[1]) << 16) | (uint32_t(f[2]) << 8) | f[3];
        if (ops[i] == ECHO) {  // byte for byte the scalar packer's framed answer
            const uint8_t* e = echo_resp.data() + echo_at[i];
            const uint64_t el = 4 + ((uint64_t(e[0]) << 24) | (uint64_t(e[1]) << 16) | (uint64_t(e[2]) << 8) | e[3]);
            if (std::memcmp(f, e, el) != 0) {
                ++bad;
                break;
            }
            f += el;
            continue;
        }
        if (ops[i] == POISON || ops[i] == OVERSIZE) {
            if (len != 1 || f[4] != srpc::RPC_ERR_FUNCTION_NOT_REGISTERED) ++bad;
            f += 5;
            continue;
        }
        if (len != 19) {
            ++bad;
            break;  // the stream is out of step from here on
        }
        srpc::packer rpr(f + 4, len);
        f += 4 + len;
        srpc::response_t<Number> m = rpr.unpack_response<Number>();
        if (m.code() != srpc::RPC_SUCCESS || m.value().num != expect(ops[i], lhs[i], rhs[i])) ++bad;
    }
    const bool pure = poison.empty() && oversize < 0 && (counts[SQUARE] == n || counts[ECHO] == n);
    if (!dump.empty() && got_all && pure) {  // unframed responses, for the reference digest
        FILE* fp = std::fopen(dump.c_str(), "wb");
        const uint8_t* q = resp.data();
        for (uint64_t i = 0; fp && i < n; ++i) {
            const uint32_t len = (uint32_t(q[0]) << 24) | (uint32_t(q[1]) << 16) | (uint32_t(q[2]) << 8) | q[3];
            std::fwrite(q + 4, 1, len, fp);
            q += 4 + len;
        }
        if (fp) std::fclose(fp);
    }
    std::printf(
        "{\"workload\": \"Calculator e2e over 127.0.0.1, one connection, pipelined\", \"mode\": \"%s\", "
        "\"requests\": %llu, \"ok\": %s, \"bad\": %llu, \"seconds\": %.6f, \"requests_per_s\": %.1f, "
        "\"request_bytes\": %zu, \"wire_in_MBps\": %.1f, "
        "\"traffic\": {\"square\": %llu, \"add\": %llu, \"subtract\": %llu, \"multiply\": %llu, \"divide\": %llu, "
        "\"poison\": %llu, \"oversize\": %llu, \"echo\": %llu, \"mix\": %.4f, \"foreign\": %.4f, \"gpu_methods\": \"%s\"}, "
        "\"gpu\": {\"batches\": %llu, \"mixed_batches\": %llu, \"batch_frames\": %llu, \"buffer_bytes\": %llu, "
        "\"gpu_requests\": %llu, \"fallback_requests\": %llu, \"oversize_requests\": %llu, \"overflow_batches\": %llu, "
        "\"gpu_seconds\": %.6f, \"classify_seconds\": %.6f, \"first_batch_seconds\": %.6f, \"fallback_seconds\": %.6f, \"h2d_bytes\": %llu, \"d2h_bytes\": %llu, "
        "\"recv_seconds\": %.6f, \"send_seconds\": %.6f, \"gpu_requests_per_s\": %.1f}, \"cpu_served\": %zu}\n",
        mode.c_str(), (unsigned long long)n, (got_all && bad == 0) ? "true" : "false", (unsigned long long)bad, secs,
        n / secs, frames.size(), frames.size() / secs / 1e6, (unsigned long long)counts[SQUARE],
        (unsigned long long)counts[ADD], (unsigned long long)counts[SUB], (unsigned long long)counts[MUL],
        (unsigned long long)counts[DIV], (unsigned long long)counts[POISON], (unsigned long long)counts[OVERSIZE],
        (unsigned long long)counts[ECHO], mix,
        foreign, gpu_methods.c_str(), (unsigned long long)stats.gpu_batches, (unsigned long long)stats.mixed_batches,
        (unsigned long long)batch, (unsigned long long)buffer_bytes, (unsigned long long)stats.gpu_requests,
        (unsigned long long)stats.fallback_requests, (unsigned long long)stats.oversize_requests,
        (unsigned long long)stats.overflow_batches, stats.gpu_seconds,
        stats.classify_seconds, stats.first_batch_seconds, stats.fallback_seconds, (unsigned long long)stats.h2d_bytes, (unsigned long long)stats.d2h_bytes,
        stats.recv_seconds, stats.send_seconds,
        stats.gpu_seconds > 0 ? stats.gpu_requests / stats.gpu_seconds : 0.0, cpu_served);
    return (got_all && bad == 0) ? 0 : 1;
}
