// needs: reference
// The reference's GENERATED code (examples/calculator_srpc.cpp, included by
// path from /root/reference -- not copied) compiled unchanged against this
// repository's headers, then driven end to end over a real 127.0.0.1 socket:
// Calculator_stub -> transport frames -> srpc::server -> Calculator servicer.
#include <srpc/server.hpp>

#include <chrono>
#include <cstdio>
#include <thread>

#include "calculator_srpc.cpp"

struct Calculator : public Calculator_servicer {
    Number add(TwoNumbers& req) override {
        Number r;
        r.num = req.left + req.right;
        return r;
    }
    Number square(Number& req) override {
        Number r;
        r.num = req.num * req.num;
        return r;
    }
};

int main() {
    const std::string port = "18082";
    srpc::server s;
    Calculator calc;
    s.register_service(calc);
    std::thread th([&] {
        int lfd = srpc::transport::create_server_socket(port);
        sockaddr_storage a{};
        socklen_t al = sizeof(a);
        int fd = accept(lfd, reinterpret_cast<sockaddr*>(&a), &al);
        s.serve_connection(fd);
        close(fd);
        close(lfd);
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(100));
    int fails = 0;
    {
        Calculator_stub stub;
        stub.register_insecure_channel("127.0.0.1", port);
        for (int x : {2, -9, 46340}) {
            Number n;
            n.num = x;
            Number r = stub.square(n);
            if (r.num != x * x) { std::fprintf(stderr, "square(%d) = %d\n", x, r.num); ++fails; }
        }
        TwoNumbers t;
        t.left = 40;
        t.right = 2;
        Number r = stub.add(t);
        if (r.num != 42) { std::fprintf(stderr, "add = %d\n", r.num); ++fails; }
        // stub keeps its socket; closing it ends the server's connection loop
        stub.register_insecure_channel("127.0.0.1", "1");  // closes the old socket (connect fails)
    }
    th.join();
    std::printf("calculator_compat_test: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
