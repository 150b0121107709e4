// needs: gpu
// Compile-and-link check of the multi-GPU C++ API (include/srpc/gpu_multi.hpp)
// without a GPU: every member template of sharded_packer<T>, comm and
// device_group is instantiated (their addresses taken), so a signature that
// cannot compile -- e.g. sharded_packer<T>::request returning a group that
// cannot be moved -- fails here, in the CPU suite.  Nothing is called.
#include <cstdio>
#include <type_traits>

#include "srpc/gpu_multi.hpp"

struct Quad : public srpc::message_base {
    int32_t a = 0, b = 0, c = 0, d = 0;
    static constexpr const char* name = "Quad";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(Quad, a, "Quad::a"), STRUCT_MEMBER(Quad, b, "Quad::b"),
                                                   STRUCT_MEMBER(Quad, c, "Quad::c"), STRUCT_MEMBER(Quad, d, "Quad::d"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> a >> b >> c >> d;
    }
};

static_assert(std::is_move_constructible_v<srpc::gpu::device_group>);
static_assert(std::is_move_assignable_v<srpc::gpu::device_group>);
static_assert(std::is_move_constructible_v<srpc::gpu::sharded_packer<Quad>>);
static_assert(std::is_move_constructible_v<srpc::gpu::comm>);
static_assert(!std::is_copy_constructible_v<srpc::gpu::device_group>);

int main(int argc, char**) {
    auto req = &srpc::gpu::sharded_packer<Quad>::request;
    auto pg = &srpc::gpu::sharded_packer<Quad>::pack_gather;
    auto sh = &srpc::gpu::sharded_packer<Quad>::shard;
    auto gw = &srpc::gpu::comm::gather_wire;
    volatile bool never = argc > 1000;  // keep the calls out of the run, in the build
    if (never) {
        auto s = req({0}, "Svc_servicer::m");
        (void)pg;
        (void)(s.*sh)(1, 0);
        (void)gw;
    }
    std::printf("ok\n");
    return 0;
}
