// host_columns_bench: what a C++ caller holding std::vector<T> pays on the
// host before / after the GPU runs (include/srpc/gpu.hpp host_columns), set
// beside the scalar packer loop it replaces (`packer p; for (r : recs) p << r`,
// reference packer.hpp:73) and a plain memcpy of the same bytes.
//   g++ -O2 -std=c++20 -I include tools/host_columns_bench.cpp -o /tmp/hcb && /tmp/hcb [n]
// Prints one JSON line per message type: ns per record for each leg.
#include <srpc/gpu.hpp>
#include <srpc/packer.hpp>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

struct Quad : public srpc::message_base {
    int32_t a, b, c, d;
    static constexpr const char* name = "Quad";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(Quad, a, "Quad::a"), STRUCT_MEMBER(Quad, b, "Quad::b"),
                                                   STRUCT_MEMBER(Quad, c, "Quad::c"), STRUCT_MEMBER(Quad, d, "Quad::d"));
    void unpack(srpc::buffer::ptr) override {}
};

struct multiple_primitives : public srpc::message_base {
    int8_t arg1;
    char arg2;
    int64_t arg3;
    std::string arg4;
    static constexpr const char* name = "multiple_primitives";
    static constexpr auto fields = std::make_tuple(
        STRUCT_MEMBER(multiple_primitives, arg1, "a1"), STRUCT_MEMBER(multiple_primitives, arg2, "a2"),
        STRUCT_MEMBER(multiple_primitives, arg3, "a3"), STRUCT_MEMBER(multiple_primitives, arg4, "a4"));
    void unpack(srpc::buffer::ptr) override {}
};

using clk = std::chrono::steady_clock;
static double secs(clk::time_point t0) { return std::chrono::duration<double>(clk::now() - t0).count(); }

template <typename T, typename Fill>
static void run(const char* label, size_t n, Fill fill) {
    std::vector<T> recs(n);
    for (size_t i = 0; i < n; ++i) fill(recs[i], i);
    srpc::gpu::host_columns<T> hc;  // reused across the repetitions, as a caller's would be
    double best_sc = 1e9, best_ga = 1e9, best_pk = 1e9, best_mc = 1e9;
    uint64_t col_bytes = 0, wire_bytes = 0;
    std::vector<T> back;
    for (int rep = 0; rep < 3; ++rep) {
        auto t0 = clk::now();
        hc.scatter(recs);
        best_sc = std::min(best_sc, secs(t0));
        col_bytes = 0;
        for (auto const& c : hc.col) col_bytes += c.size();
        for (auto const& o : hc.offs) col_bytes += 8 * o.size();
        t0 = clk::now();
        hc.gather(back);
        best_ga = std::min(best_ga, secs(t0));
        t0 = clk::now();
        srpc::packer p;
        for (auto const& r : recs) p << r;
        best_pk = std::min(best_pk, secs(t0));
        wire_bytes = p.size();
        std::vector<uint8_t> dst(col_bytes);
        std::vector<uint8_t> src(col_bytes, 1);
        t0 = clk::now();
        std::memcpy(dst.data(), src.data(), col_bytes);
        best_mc = std::min(best_mc, secs(t0));
        if (dst[col_bytes / 2] != 1) std::printf("?");
    }
    std::printf(
        "{\"type\": \"%s\", \"records\": %zu, \"column_bytes\": %llu, \"wire_bytes\": %llu, "
        "\"ns_per_record\": {\"host_columns_scatter\": %.2f, \"host_columns_gather\": %.2f, "
        "\"scalar_packer_loop\": %.2f, \"memcpy_of_column_bytes\": %.2f}}\n",
        label, n, (unsigned long long)col_bytes, (unsigned long long)wire_bytes, 1e9 * best_sc / n, 1e9 * best_ga / n,
        1e9 * best_pk / n, 1e9 * best_mc / n);
}

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? std::stoull(argv[1]) : (1u << 22);
    run<Quad>("Quad", n, [](Quad& q, size_t i) {
        q.a = static_cast<int32_t>(i);
        q.b = static_cast<int32_t>(i * 3);
        q.c = static_cast<int32_t>(i * 5);
        q.d = static_cast<int32_t>(i * 7);
    });
    run<multiple_primitives>("multiple_primitives (string 0-64 B)", n, [](multiple_primitives& m, size_t i) {
        m.arg1 = static_cast<int8_t>(i);
        m.arg2 = static_cast<char>(i * 3);
        m.arg3 = static_cast<int64_t>(i) * 1000003;
        m.arg4.assign((i * 2654435761u) % 65, 'x');
    });
    return 0;
}
