// needs: batchgen
// The message structs srpc_amd.batchgen emits (--messages) against the scalar
// packer: a nested, string-carrying record packs to the bytes of its fields in
// declaration order and unpacks back through the generated unpack (nested
// messages share the buffer cursor), and the batch view's schema constants
// agree with what srpc::gpu derives from T::fields.
#include <batchgen_example_batch.hpp>

#include <cstdio>
#include <cstring>
#include <vector>

static int g_fail = 0, g_pass = 0;
#define CHECK(c)                                                                                  \
    do {                                                                                          \
        if (c) ++g_pass;                                                                          \
        else { ++g_fail; std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); }      \
    } while (0)

template <typename B>
static bool kinds_match() {
    const std::vector<int32_t> k = srpc::gpu::flat_kinds<typename B::message_type>();
    return k.size() == B::nfields && std::memcmp(k.data(), B::kinds, sizeof(B::kinds)) == 0;
}

int main() {
    CHECK(kinds_match<Inner_batch>());
    CHECK(kinds_match<Point_batch>());
    CHECK(kinds_match<Number_batch>());
    CHECK(kinds_match<Record_batch>());
    CHECK(Record_batch::nfields == 9 && Record_batch::has_strings && Record_batch::fixed_bytes == 37);
    CHECK(std::strcmp(Record_batch::paths[1], "in_tag") == 0 && std::strcmp(Record_batch::paths[7], "p_y") == 0);
    CHECK(std::strcmp(Geo_batch::square_method, "Geo_servicer::square") == 0);

    Record r;
    r.id = -7;
    r.in.tag = 3;
    r.in.small = -300;
    r.flag = true;
    r.label = "hello";
    r.c = 'z';
    r.p.x = 11;
    r.p.y = -12;
    r.note = "";
    srpc::packer p;
    p << r;
    std::vector<uint8_t> want;
    auto put = [&](const void* v, size_t k) {
        const uint8_t* b = static_cast<const uint8_t*>(v);
        want.insert(want.end(), b, b + k);
    };
    const uint64_t l5 = 5, l0 = 0;
    put(&r.id, 8);
    put(&r.in.tag, 1);
    put(&r.in.small, 2);
    put(&r.flag, 1);
    put(&l5, 8);
    put("hello", 5);
    put(&r.c, 1);
    put(&r.p.x, 4);
    put(&r.p.y, 4);
    put(&l0, 8);
    CHECK(std::vector<uint8_t>(*p.buf()) == want);
    CHECK(want.size() == Record_batch::fixed_bytes + 5);

    Record back;
    srpc::packer q(want.data(), want.size());
    back.unpack(q.buf());
    CHECK(back.id == r.id && back.in.tag == r.in.tag && back.in.small == r.in.small && back.flag == r.flag);
    CHECK(back.label == r.label && back.c == r.c && back.p.x == r.p.x && back.p.y == r.p.y && back.note.empty());
    CHECK(q.buf()->offset() == want.size());

    std::printf("%d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
