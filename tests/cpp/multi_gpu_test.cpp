// needs: gpu
// srpc::gpu::sharded_packer / comm (include/srpc/gpu_multi.hpp) on every
// visible device: a Quad batch sharded with srpc_shard_range, each shard
// generated and packed on its own device, gathered to device 0 over RCCL,
// must equal the single-device pack of the whole batch byte for byte (the
// reference packer appends: core.hpp:34).  With one device this runs the
// group machinery end to end with the root's own shard only; the 8-GPU
// exchange itself is measured by bench.py at N > 1.
#include <hip/hip_runtime_api.h>
#include <srpc/gpu_multi.hpp>

#include <cstdio>
#include <vector>

static int g_fail = 0, g_pass = 0;
#define CHECK(c)                                                                                  \
    do {                                                                                          \
        if (c) ++g_pass;                                                                          \
        else { ++g_fail; std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); }      \
    } while (0)
#define HIPCHECK(x)                                                                               \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) { std::fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 2; } \
    } while (0)

struct Quad : public srpc::message_base {
    int32_t a, b, c, d;
    static constexpr const char* name = "Quad";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(Quad, a, "Quad::a"), STRUCT_MEMBER(Quad, b, "Quad::b"),
                                                   STRUCT_MEMBER(Quad, c, "Quad::c"), STRUCT_MEMBER(Quad, d, "Quad::d"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> a >> b >> c >> d;
    }
};

int main() {
    int G = 0;
    HIPCHECK(hipGetDeviceCount(&G));
    if (G > 8) G = 8;
    std::vector<int> devs;
    for (int g = 0; g < G; ++g) devs.push_back(g);
    const uint64_t n = (1u << 20) + 37;
    // the whole batch on device 0: the reference layout
    HIPCHECK(hipSetDevice(0));
    std::vector<int32_t*> full(4);
    for (auto& c : full) HIPCHECK(hipMalloc(&c, n * 4 + 16));
    CHECK(srpc_gpu_fill_splitmix_i32(full.data(), 4, n, 0x5EED, 0, nullptr) == SRPC_OK);
    srpc::gpu::batch_packer<Quad> one(0);
    uint8_t* want = nullptr;
    HIPCHECK(hipMalloc(&want, n * 16));
    const void* fc[4] = {full[0], full[1], full[2], full[3]};
    CHECK(one.pack(fc, n, want, n * 16) == SRPC_OK);
    HIPCHECK(hipDeviceSynchronize());

    // sharded: shard g generated and packed on device g, gathered to device 0
    srpc::gpu::sharded_packer<Quad> sp(devs);
    CHECK(sp.size() == G && sp.record_bytes() == 16);
    std::vector<std::vector<int32_t*>> cols(static_cast<size_t>(G), std::vector<int32_t*>(4));
    std::vector<const void* const*> dcols(static_cast<size_t>(G));
    std::vector<std::vector<const void*>> colptr(static_cast<size_t>(G));
    std::vector<uint8_t*> shard_wire(static_cast<size_t>(G));
    std::vector<void*> streams(static_cast<size_t>(G));
    uint64_t covered = 0;
    for (int g = 0; g < G; ++g) {
        auto [lo, hi] = sp.shard(n, g);
        CHECK(lo == covered && lo % SRPC_SHARD_ALIGN_RECORDS == 0);
        covered = hi;
        HIPCHECK(hipSetDevice(g));
        hipStream_t s;
        HIPCHECK(hipStreamCreate(&s));
        streams[static_cast<size_t>(g)] = s;
        for (auto& c : cols[static_cast<size_t>(g)]) HIPCHECK(hipMalloc(&c, (hi - lo) * 4 + 16));
        CHECK(srpc_gpu_fill_splitmix_i32(cols[static_cast<size_t>(g)].data(), 4, hi - lo, 0x5EED, lo, s) == SRPC_OK);
        for (auto* c : cols[static_cast<size_t>(g)]) colptr[static_cast<size_t>(g)].push_back(c);
        dcols[static_cast<size_t>(g)] = colptr[static_cast<size_t>(g)].data();
        HIPCHECK(hipMalloc(&shard_wire[static_cast<size_t>(g)], (hi - lo) * 16 + 16));
    }
    CHECK(covered == n);
    HIPCHECK(hipSetDevice(0));
    uint8_t* root = nullptr;
    HIPCHECK(hipMalloc(&root, n * 16));
    HIPCHECK(hipMemset(root, 0xA5, n * 16));
    CHECK(sp.pack_gather(dcols, n, shard_wire, root, n * 16, 0, streams) == SRPC_OK);
    for (int g = 0; g < G; ++g) {
        HIPCHECK(hipSetDevice(g));
        HIPCHECK(hipStreamSynchronize(static_cast<hipStream_t>(streams[static_cast<size_t>(g)])));
    }
    HIPCHECK(hipSetDevice(0));
    std::vector<uint8_t> a(n * 16), b(n * 16);
    HIPCHECK(hipMemcpy(a.data(), want, n * 16, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(b.data(), root, n * 16, hipMemcpyDeviceToHost));
    CHECK(a == b);

    // one process per GPU form, here with one rank: id, init, gather (the root's own shard)
    {
        const srpc::gpu::comm_id id = srpc::gpu::comm::unique_id();
        srpc::gpu::comm c(id, 1, 0, 0);
        CHECK(c.rank() == 0 && c.nranks() == 1);
        HIPCHECK(hipMemset(root, 0, n * 16));
        CHECK(c.gather_wire(want, n * 16, root, n * 16, {n * 16}, 0, nullptr) == SRPC_OK);
        CHECK(c.gather_wire(want, n * 16, root, n * 16 - 1, {n * 16}, 0, nullptr) == SRPC_E_CAPACITY);
        HIPCHECK(hipDeviceSynchronize());
        HIPCHECK(hipMemcpy(b.data(), root, n * 16, hipMemcpyDeviceToHost));
        CHECK(a == b);
    }
    std::printf("multi_gpu_test (%d devices): %d passed, %d failed\n", G, g_pass, g_fail);
    return g_fail ? 1 : 0;
}
