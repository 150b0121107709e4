// e2e_square: BASELINE.json configs[4] -- Calculator.square end to end over
// loopback, 1M requests, server-side GPU-batched unpack -> square -> pack.
//
// One process, two threads talking over 127.0.0.1:
//   client: the frames Calculator_stub::square sends (calculator_srpc.cpp:120-134:
//           pack_request("Calculator_servicer::square", Number) + u32 BE length),
//           all N pipelined on one connection by a sender thread, responses
//           read back and checked against num^2 and (optionally) written out
//           so their SHA-256 can be compared with the reference digest;
//   server: --mode gpu: srpc::gpu::batch_server (include/srpc/gpu_server.hpp)
//           --mode cpu: the scalar srpc::server (include/srpc/server.hpp),
//                       the reference's per-request dispatch path.
// Inputs: num = splitmix64(0x5EED) % 46341.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <srpc/gpu_server.hpp>
#include <srpc/server.hpp>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

struct Number : public srpc::message_base {
    int32_t num;
    static constexpr const char* name = "Number";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(Number, num, "Number::num"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> num;
    }
};

struct Calculator_servicer : srpc::servicer_base {
    virtual Number square(Number&) { throw std::runtime_error("Method not implemented!"); }
    static constexpr const char* name = "Calculator";
    static constexpr auto methods =
        std::make_tuple(STRUCT_MEMBER(Calculator_servicer, square, "Calculator_servicer::square"));
};

struct Calculator : Calculator_servicer {
    Number square(Number& req) override {
        Number r;
        r.num = static_cast<int32_t>(static_cast<uint32_t>(req.num) * static_cast<uint32_t>(req.num));
        return r;
    }
};

// The batched method on the device: one int32 column in, one out.
__global__ void k_square(const int32_t* __restrict__ in, int32_t* __restrict__ out, uint64_t n) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t v = static_cast<uint32_t>(in[i]);
        out[i] = static_cast<int32_t>(v * v);
    }
}

static int square_batch(void* const* req, void* const* resp, uint64_t n, hipStream_t s) {
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(k_square, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s,
                       static_cast<const int32_t*>(req[0]), static_cast<int32_t*>(resp[0]), n);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

static uint64_t splitmix(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char** argv) {
    uint64_t n = 1u << 20;
    uint64_t batch = 1u << 18;
    std::string mode = "gpu", port = "18090", dump;
    int64_t poison = -1;  // request index sent with an unknown method (exercises the CPU fallback)
    std::string poison_method = "Calculator_servicer::squarX";  // same frame length as the real one
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&] { return std::string(i + 1 < argc ? argv[++i] : ""); };
        if (a == "--n") n = std::stoull(next());
        else if (a == "--batch") batch = std::stoull(next());
        else if (a == "--mode") mode = next();
        else if (a == "--port") port = next();
        else if (a == "--dump") dump = next();
        else if (a == "--poison") poison = std::stoll(next());
        else if (a == "--poison-method") poison_method = next();  // another length shifts every later frame
    }
    srpc::message_registry["Number"] = []() -> std::unique_ptr<Number> { return std::make_unique<Number>(); };

    // ---- client-side request frames, exactly as the stub builds them -------
    std::vector<int32_t> nums(n);
    uint64_t st = 0x5EED;
    for (uint64_t i = 0; i < n; ++i) {
        const int32_t v = static_cast<int32_t>(static_cast<uint32_t>(splitmix(&st)));
        nums[i] = v % 46341;
    }
    std::vector<uint8_t> frames;
    frames.reserve(n * 57);
    for (uint64_t i = 0; i < n; ++i) {
        srpc::packer pr;
        srpc::request_t<Number> req;
        req.set_method_name(static_cast<int64_t>(i) == poison ? poison_method : "Calculator_servicer::square");
        Number v;
        v.num = nums[i];
        req.set_value(std::move(v));
        pr.pack_request(req);
        const uint32_t len = htonl(static_cast<uint32_t>(pr.size()));
        const uint8_t* lb = reinterpret_cast<const uint8_t*>(&len);
        frames.insert(frames.end(), lb, lb + 4);
        frames.insert(frames.end(), pr.data(), pr.data() + pr.size());
    }
    const uint64_t resp_frame = 4 + 19;

    // ---- server ------------------------------------------------------------
    Calculator calc;
    srpc::server cpu_server;
    cpu_server.register_service(calc);
    std::unique_ptr<srpc::gpu::batch_server<Number, Number>> gsrv;
    if (mode == "gpu") {
        gsrv = std::make_unique<srpc::gpu::batch_server<Number, Number>>("Calculator_servicer::square", square_batch,
                                                                         batch, 0, &cpu_server);
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
        if (gsrv) stats = gsrv->serve_connection(fd);
        else cpu_served = cpu_server.serve_connection(fd);
        close(fd);
    });

    // ---- client ------------------------------------------------------------
    const int fd = srpc::transport::create_client_socket("127.0.0.1", port);
    if (fd < 0) return 4;
    int big = 8 << 20;
    setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &big, sizeof(big));
    setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &big, sizeof(big));
    // an unknown method is answered with the one status byte RPC_ERR_FUNCTION_NOT_REGISTERED
    const uint64_t resp_total = n * resp_frame - (poison >= 0 && static_cast<uint64_t>(poison) < n ? 18 : 0);
    std::vector<uint8_t> resp(resp_total);
    auto t0 = std::chrono::steady_clock::now();
    std::thread sender([&] { srpc::transport::send_all(fd, frames.data(), frames.size()); });
    const bool got_all = srpc::transport::recv_all(fd, resp.data(), resp.size());
    auto t1 = std::chrono::steady_clock::now();
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
        if (static_cast<int64_t>(i) == poison) {
            if (len != 1 || f[4] != srpc::RPC_ERR_FUNCTION_NOT_REGISTERED) ++bad;
            f += 5;
            continue;
        }
        srpc::packer rpr(f + 4, len);
        f += 4 + len;
        srpc::response_t<Number> m = rpr.unpack_response<Number>();
        if (len != 19 || m.code() != srpc::RPC_SUCCESS ||
            m.value().num != static_cast<int32_t>(static_cast<uint32_t>(nums[i]) * static_cast<uint32_t>(nums[i])))
            ++bad;
    }
    if (!dump.empty() && got_all && poison < 0) {  // unframed responses, for the reference digest
        FILE* fp = std::fopen(dump.c_str(), "wb");
        for (uint64_t i = 0; fp && i < n; ++i) std::fwrite(resp.data() + i * resp_frame + 4, 1, 19, fp);
        if (fp) std::fclose(fp);
    }
    std::printf(
        "{\"workload\": \"Calculator.square e2e over 127.0.0.1, one connection, pipelined\", \"mode\": \"%s\", "
        "\"requests\": %llu, \"ok\": %s, \"bad\": %llu, \"seconds\": %.6f, \"requests_per_s\": %.1f, "
        "\"request_frame_bytes\": 57, \"response_frame_bytes\": 23, \"wire_in_MBps\": %.1f, "
        "\"gpu\": {\"batches\": %llu, \"batch_frames\": %llu, \"fallback_requests\": %llu, "
        "\"gpu_seconds\": %.6f, \"h2d_bytes\": %llu, \"d2h_bytes\": %llu, \"recv_seconds\": %.6f, "
        "\"send_seconds\": %.6f, \"gpu_requests_per_s\": %.1f}, \"cpu_served\": %zu}\n",
        mode.c_str(), (unsigned long long)n, (got_all && bad == 0) ? "true" : "false", (unsigned long long)bad, secs,
        n / secs, n * 57.0 / secs / 1e6, (unsigned long long)stats.gpu_batches, (unsigned long long)batch,
        (unsigned long long)stats.fallback_requests, stats.gpu_seconds, (unsigned long long)stats.h2d_bytes,
        (unsigned long long)stats.d2h_bytes, stats.recv_seconds, stats.send_seconds,
        stats.gpu_seconds > 0 ? stats.requests / stats.gpu_seconds : 0.0, cpu_served);
    return (got_all && bad == 0) ? 0 : 1;
}
