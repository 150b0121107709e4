// aos_bench: a C++ caller holding std::vector<Quad> (the reference's caller
// shape: `packer p; for (r : recs) p << r;`, packer.hpp:73) gets the batch's
// wire bytes into device memory, three ways, host clock around each:
//   scalar      the reference loop on the host, then one H2D of the wire;
//   columns     host_columns<T>::scatter (host transpose, reused buffers),
//               H2D of the columns, batch_packer<T>::pack;
//   records     H2D of the vector's raw bytes, batch_packer<T>::pack_records.
// The three wires are compared byte for byte.  Prints one JSON line.
#include <hip/hip_runtime.h>
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

#define HIPCHECK(x)                                                                                     \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess) {                                                                         \
            std::fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__);                    \
            return 2;                                                                                   \
        }                                                                                               \
    } while (0)

using clk = std::chrono::steady_clock;
static double ms(clk::time_point t0) { return 1e3 * std::chrono::duration<double>(clk::now() - t0).count(); }

int main(int argc, char** argv) {
    const size_t n = argc > 1 ? std::stoull(argv[1]) : (1u << 24);
    std::vector<Quad> recs(n);
    uint64_t s = 0x5EED;
    for (auto& r : recs) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        r.a = static_cast<int32_t>(s >> 32);
        r.b = static_cast<int32_t>(s);
        r.c = static_cast<int32_t>(s >> 16);
        r.d = static_cast<int32_t>(s >> 8);
    }
    srpc::gpu::batch_packer<Quad> bp;
    const uint64_t wb = n * bp.record_bytes();
    uint8_t *dw = nullptr, *dw2 = nullptr, *dw3 = nullptr;
    Quad* drecs = nullptr;
    std::vector<void*> dcols(4);
    HIPCHECK(hipMalloc(&dw, wb + 16));
    HIPCHECK(hipMalloc(&dw2, wb + 16));
    HIPCHECK(hipMalloc(&dw3, wb + 16));
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&drecs), n * sizeof(Quad) + 16));
    for (auto& c : dcols) HIPCHECK(hipMalloc(&c, 4 * n + 16));
    srpc::gpu::host_columns<Quad> hc;
    double best[3] = {1e30, 1e30, 1e30};
    std::vector<uint8_t> a(wb), b(wb), c(wb);
    for (int rep = 0; rep < 4; ++rep) {
        auto t0 = clk::now();
        srpc::packer p;
        for (auto const& r : recs) p << r;
        HIPCHECK(hipMemcpy(dw, p.data(), p.size(), hipMemcpyHostToDevice));
        best[0] = std::min(best[0], ms(t0));
        t0 = clk::now();
        hc.scatter(recs);
        for (int f = 0; f < 4; ++f) HIPCHECK(hipMemcpy(dcols[f], hc.col[f].data(), 4 * n, hipMemcpyHostToDevice));
        if (bp.pack(dcols.data(), n, dw2, wb) != SRPC_OK) return 3;
        HIPCHECK(hipDeviceSynchronize());
        best[1] = std::min(best[1], ms(t0));
        t0 = clk::now();
        HIPCHECK(hipMemcpy(drecs, recs.data(), n * sizeof(Quad), hipMemcpyHostToDevice));
        if (bp.pack_records(drecs, n, dw3, wb) != SRPC_OK) return 4;
        HIPCHECK(hipDeviceSynchronize());
        best[2] = std::min(best[2], ms(t0));
    }
    HIPCHECK(hipMemcpy(a.data(), dw, wb, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(b.data(), dw2, wb, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(c.data(), dw3, wb, hipMemcpyDeviceToHost));
    const bool same = a == b && a == c;
    std::printf(
        "{\"workload\": \"std::vector<Quad> on the host -> wire in HBM\", \"records\": %zu, \"struct_bytes\": %zu, "
        "\"ms\": {\"scalar_packer_then_h2d\": %.2f, \"host_columns_h2d_pack\": %.2f, \"h2d_records_pack_records\": %.2f}, "
        "\"identical\": %s}\n",
        n, sizeof(Quad), best[0], best[1], best[2], same ? "true" : "false");
    return same ? 0 : 1;
}
