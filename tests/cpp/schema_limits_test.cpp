// needs: gpu
// The schema limits of this build (include/srpc_gpu.h: SRPC_MAX_FIELDS leaf
// fields, SRPC_MAX_PREFIX envelope bytes) as a C++ caller meets them:
// srpc::gpu::batch_packer<T> throws srpc::gpu::plan_error carrying
// SRPC_E_UNSUPPORTED, raised by srpc_plan_create before any device work -- so
// this program runs without a GPU.  The reference's pack_struct
// (packer.hpp:172-178) has no such limits; the refusal is documented, not silent.
#include <srpc/gpu.hpp>
#include <srpc/packer.hpp>

#include <cstdio>
#include <string>

static int g_fail = 0, g_pass = 0;
#define CHECK(c)                                                                    \
    do {                                                                            \
        if (c) ++g_pass;                                                            \
        else { ++g_fail; std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); } \
    } while (0)

// 11 int8 leaves
struct Eleven : public srpc::message_base {
    int8_t a0, a1, a2, a3, a4, a5, a6, a7, a8, a9, a10;
    static constexpr const char* name = "Eleven";
    static constexpr auto fields = std::make_tuple(
        STRUCT_MEMBER(Eleven, a0, "a0"), STRUCT_MEMBER(Eleven, a1, "a1"), STRUCT_MEMBER(Eleven, a2, "a2"),
        STRUCT_MEMBER(Eleven, a3, "a3"), STRUCT_MEMBER(Eleven, a4, "a4"), STRUCT_MEMBER(Eleven, a5, "a5"),
        STRUCT_MEMBER(Eleven, a6, "a6"), STRUCT_MEMBER(Eleven, a7, "a7"), STRUCT_MEMBER(Eleven, a8, "a8"),
        STRUCT_MEMBER(Eleven, a9, "a9"), STRUCT_MEMBER(Eleven, a10, "a10"));
    void unpack(srpc::buffer::ptr) override {}
};

// 3 x 11 = 33 leaves after flattening: one past SRPC_MAX_FIELDS
struct ThirtyThree : public srpc::message_base {
    Eleven x, y, z;
    static constexpr const char* name = "ThirtyThree";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(ThirtyThree, x, "x"), STRUCT_MEMBER(ThirtyThree, y, "y"),
                                                   STRUCT_MEMBER(ThirtyThree, z, "z"));
    void unpack(srpc::buffer::ptr) override {}
};

template <typename Fn>
static int code_of(Fn&& fn) {
    try {
        fn();
    } catch (srpc::gpu::plan_error const& e) {
        std::printf("refused: %s (code %d)\n", e.what(), e.code);
        return e.code;
    } catch (...) {
        return 999;
    }
    return 0;
}

int main() {
    static_assert(SRPC_MAX_FIELDS == 32 && SRPC_MAX_PREFIX == 1024);
    CHECK(srpc::gpu::flat_kinds<ThirtyThree>().size() == 33);
    CHECK(code_of([] { srpc::gpu::batch_packer<ThirtyThree> p(0); }) == SRPC_E_UNSUPPORTED);
    // request envelope u64 | method | u64 | "Eleven": a 1003-byte method name
    // makes 1025 bytes, one past SRPC_MAX_PREFIX
    CHECK(srpc::gpu::request_prefix<Eleven>(std::string(1003, 'm')).size() == 1025);
    CHECK(code_of([] { (void)srpc::gpu::batch_packer<Eleven>::request(std::string(1003, 'm'), 0); }) ==
          SRPC_E_UNSUPPORTED);
    // the C ABI itself: limits before validation of anything device-side
    int32_t kinds[33];
    for (int32_t& k : kinds) k = SRPC_KIND_INT64;
    srpc_plan* p = nullptr;
    srpc_schema_desc d{33, kinds, nullptr, 0};
    CHECK(srpc_plan_create(&d, 0, &p) == SRPC_E_UNSUPPORTED && p == nullptr);
    uint8_t pre[1025] = {};
    srpc_schema_desc e{1, kinds, pre, 1025};
    CHECK(srpc_plan_create(&e, 0, &p) == SRPC_E_UNSUPPORTED && p == nullptr);
    srpc_schema_desc z{0, kinds, nullptr, 0};
    CHECK(srpc_plan_create(&z, 0, &p) == SRPC_E_INVALID);
    int32_t bad_kind = 42;
    srpc_schema_desc b{1, &bad_kind, nullptr, 0};
    CHECK(code_of([&] {
              if (int rc = srpc_plan_create(&b, 0, &p); rc != SRPC_OK) throw srpc::gpu::plan_error("create", rc);
          }) == SRPC_E_INVALID);
    std::printf("%d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
