// needs: gpu
// srpc::gpu::batch_packer<T> (include/srpc/gpu.hpp) against the scalar
// packer of the same headers: for generated-style message types, the bytes of
// one GPU launch over N records must equal `packer p; for r: p << r;` (and the
// pack_request / pack_response loops), and GPU unpack must give the records back.
#include <hip/hip_runtime_api.h>
#include <srpc/gpu.hpp>
#include <srpc/packer.hpp>

#include <cstdio>
#include <algorithm>
#include <cstring>
#include <random>
#include <type_traits>
#include <vector>

static int g_fail = 0, g_pass = 0;
#define CHECK(c)                                                                    \
    do {                                                                            \
        if (c) ++g_pass;                                                            \
        else { ++g_fail; std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); } \
    } while (0)
#define HIPCHECK(x)                                                                 \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) { std::fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 2; } \
    } while (0)

struct Number : public srpc::message_base {
    int32_t num;
    static constexpr const char* name = "Number";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(Number, num, "Number::num"));
    void unpack(srpc::buffer::ptr bp) override { srpc::packer p(bp); p >> num; }
};

struct Inner : public srpc::message_base {
    int8_t tag;
    int16_t small;
    static constexpr const char* name = "Inner";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(Inner, tag, "Inner::tag"),
                                                   STRUCT_MEMBER(Inner, small, "Inner::small"));
};

struct Outer : public srpc::message_base {
    int64_t id;
    Inner in;
    bool flag;
    char c;
    int32_t v;
    static constexpr const char* name = "Outer";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(Outer, id, "Outer::id"), STRUCT_MEMBER(Outer, in, "Outer::in"),
                                                   STRUCT_MEMBER(Outer, flag, "Outer::flag"), STRUCT_MEMBER(Outer, c, "Outer::c"),
                                                   STRUCT_MEMBER(Outer, v, "Outer::v"));
};

template <typename T, typename Fill, typename Eq, typename Emit>
static int run(srpc::gpu::batch_packer<T>& bp, size_t n, Fill fill, Eq eq, Emit emit_scalar) {
    std::vector<T> recs(n);
    for (size_t i = 0; i < n; ++i) fill(recs[i], i);
    srpc::packer ref;
    for (auto& r : recs) emit_scalar(ref, r);
    std::vector<uint8_t> want(*ref.buf());
    CHECK(want.size() == n * bp.record_bytes());

    srpc::gpu::host_columns<T> hc;
    hc.scatter(recs);
    std::vector<void*> dcols(hc.col.size()), dback(hc.col.size());
    for (size_t f = 0; f < hc.col.size(); ++f) {
        HIPCHECK(hipMalloc(&dcols[f], hc.col[f].size() + 16));
        HIPCHECK(hipMalloc(&dback[f], hc.col[f].size() + 16));
        HIPCHECK(hipMemcpy(dcols[f], hc.col[f].data(), hc.col[f].size(), hipMemcpyHostToDevice));
    }
    uint8_t* dw = nullptr;
    HIPCHECK(hipMalloc(&dw, want.size() + 16));
    CHECK(bp.pack(dcols.data(), n, dw, want.size()) == SRPC_OK);
    std::vector<uint8_t> got(want.size());
    HIPCHECK(hipMemcpy(got.data(), dw, got.size(), hipMemcpyDeviceToHost));
    CHECK(got == want);
    srpc_unpack_status* st = nullptr;
    HIPCHECK(hipMalloc(&st, sizeof(*st)));
    CHECK(bp.unpack(dw, want.size(), n, dback.data(), st) == SRPC_OK);
    srpc_unpack_status hs{};
    HIPCHECK(hipMemcpy(&hs, st, sizeof(hs), hipMemcpyDeviceToHost));
    CHECK(hs.flags == 0);
    srpc::gpu::host_columns<T> back = hc;
    for (size_t f = 0; f < hc.col.size(); ++f)
        HIPCHECK(hipMemcpy(back.col[f].data(), dback[f], hc.col[f].size(), hipMemcpyDeviceToHost));
    std::vector<T> out;
    back.gather(out);
    bool same = out.size() == recs.size();
    for (size_t i = 0; same && i < n; ++i) same = eq(out[i], recs[i]);
    CHECK(same);
    // the same records straight from / into the raw bytes of the std::vector<T>
    // (pack_records / unpack_records: no host transpose)
    T* drecs = nullptr;
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&drecs), n * sizeof(T) + 16));
    HIPCHECK(hipMemcpy(drecs, recs.data(), n * sizeof(T), hipMemcpyHostToDevice));
    HIPCHECK(hipMemset(dw, 0, want.size()));
    CHECK(bp.pack_records(drecs, n, dw, want.size()) == SRPC_OK);
    HIPCHECK(hipMemcpy(got.data(), dw, got.size(), hipMemcpyDeviceToHost));
    CHECK(got == want);
    std::vector<T> out2(n);  // default objects: their vtable pointers travel to the device and back
    HIPCHECK(hipMemcpy(drecs, out2.data(), n * sizeof(T), hipMemcpyHostToDevice));
    CHECK(bp.unpack_records(dw, want.size(), n, drecs, st) == SRPC_OK);
    HIPCHECK(hipMemcpy(static_cast<void*>(out2.data()), drecs, n * sizeof(T), hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(&hs, st, sizeof(hs), hipMemcpyDeviceToHost));
    CHECK(hs.flags == 0);
    same = true;
    for (size_t i = 0; same && i < n; ++i) same = eq(out2[i], recs[i]);
    CHECK(same);
    // into fresh objects: the device array holds garbage, every non-field
    // byte (the vtable pointer) comes from a T{} (unpack_records_fresh)
    if (sizeof(T) <= 256) {
        HIPCHECK(hipMemset(drecs, 0xA5, n * sizeof(T)));
        std::vector<T> out3(n);
        const T proto{};
        CHECK(bp.unpack_records_fresh(dw, want.size(), n, drecs, proto, st) == SRPC_OK);
        HIPCHECK(hipMemcpy(static_cast<void*>(out3.data()), drecs, n * sizeof(T), hipMemcpyDeviceToHost));
        same = true;
        for (size_t i = 0; same && i < n; ++i)
            same = eq(out3[i], recs[i]) &&
                   (!std::is_polymorphic_v<T> || std::memcmp(static_cast<const void*>(&out3[i]),
                                                             static_cast<const void*>(&proto), sizeof(void*)) == 0);
        CHECK(same);
    }
    // host-terminated (ABI 7): pinned host columns -> host wire and back,
    // direct (kernels on the mapped buffers) and through a 2-slot ring of
    // 7-record chunks
    {
        std::vector<void*> hcols(hc.col.size()), hback(hc.col.size());
        for (size_t f = 0; f < hc.col.size(); ++f) {
            HIPCHECK(hipHostMalloc(&hcols[f], hc.col[f].size() + 16, hipHostMallocDefault));
            HIPCHECK(hipHostMalloc(&hback[f], hc.col[f].size() + 16, hipHostMallocDefault));
            std::memcpy(hcols[f], hc.col[f].data(), hc.col[f].size());
        }
        uint8_t* hw = nullptr;
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&hw), want.size() + 16, hipHostMallocDefault));
        const uint64_t sb = bp.host_scratch_bytes(7, 2);
        void* scratch = nullptr;
        HIPCHECK(hipMalloc(&scratch, sb));
        for (uint64_t chunk : {uint64_t{0}, uint64_t{7}}) {
            std::memset(hw, 0, want.size());
            CHECK(bp.pack_host(hcols.data(), n, hw, want.size(), chunk, 2, scratch, sb) == SRPC_OK);
            HIPCHECK(hipDeviceSynchronize());
            CHECK(std::memcmp(hw, want.data(), want.size()) == 0);
            for (size_t f = 0; f < hc.col.size(); ++f) std::memset(hback[f], 0, hc.col[f].size());
            CHECK(bp.unpack_host(hw, want.size(), n, hback.data(), st, chunk, 2, scratch, sb) == SRPC_OK);
            HIPCHECK(hipDeviceSynchronize());
            HIPCHECK(hipMemcpy(&hs, st, sizeof(hs), hipMemcpyDeviceToHost));
            CHECK(hs.flags == 0);
            bool eqc = true;
            for (size_t f = 0; f < hc.col.size(); ++f)
                eqc = eqc && std::memcmp(hback[f], hc.col[f].data(), hc.col[f].size()) == 0;
            CHECK(eqc);
        }
        (void)hipFree(scratch);
        (void)hipHostFree(hw);
        for (size_t f = 0; f < hc.col.size(); ++f) { (void)hipHostFree(hcols[f]); (void)hipHostFree(hback[f]); }
    }
    (void)hipFree(drecs);
    for (size_t f = 0; f < hc.col.size(); ++f) { (void)hipFree(dcols[f]); (void)hipFree(dback[f]); }
    (void)hipFree(dw);
    (void)hipFree(st);
    return 0;
}

struct Text : public srpc::message_base {
    int8_t a;
    std::string s;
    int64_t b;
    Inner in;
    std::string t;
    static constexpr const char* name = "Text";
    static constexpr auto fields = std::make_tuple(STRUCT_MEMBER(Text, a, "Text::a"), STRUCT_MEMBER(Text, s, "Text::s"),
                                                   STRUCT_MEMBER(Text, b, "Text::b"), STRUCT_MEMBER(Text, in, "Text::in"),
                                                   STRUCT_MEMBER(Text, t, "Text::t"));
};

// String schemas: batch_packer<T>::pack_var / unpack_var against `p << r`.
static int run_var(srpc::gpu::batch_packer<Text>& bp, size_t n, std::mt19937_64& rng) {
    std::vector<Text> recs(n);
    for (size_t i = 0; i < n; ++i) {
        recs[i].a = static_cast<int8_t>(rng());
        recs[i].b = static_cast<int64_t>(rng());
        recs[i].in.tag = static_cast<int8_t>(rng());
        recs[i].in.small = static_cast<int16_t>(rng());
        recs[i].s.assign(rng() % 70, 'x');
        for (auto& c : recs[i].s) c = static_cast<char>(rng());
        recs[i].t.assign(rng() % 3 == 0 ? 0 : rng() % 500, 'y');
    }
    srpc::packer ref;
    for (auto& r : recs) ref << r;
    std::vector<uint8_t> want(*ref.buf());
    srpc::gpu::host_columns<Text> hc;
    hc.scatter(recs);
    const size_t F = hc.col.size();
    std::vector<void*> dcols(F), dback(F);
    std::vector<uint64_t*> doffs(F, nullptr), dboffs(F, nullptr);
    for (size_t f = 0; f < F; ++f) {
        HIPCHECK(hipMalloc(&dcols[f], hc.col[f].size() + 16));
        HIPCHECK(hipMemcpy(dcols[f], hc.col[f].data(), hc.col[f].size(), hipMemcpyHostToDevice));
        HIPCHECK(hipMalloc(&dback[f], std::max(hc.col[f].size(), want.size()) + 16));
        if (!hc.offs[f].empty()) {
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&doffs[f]), 8 * (n + 1)));
            HIPCHECK(hipMemcpy(doffs[f], hc.offs[f].data(), 8 * (n + 1), hipMemcpyHostToDevice));
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&dboffs[f]), 8 * (n + 1)));
        }
    }
    uint8_t* dw = nullptr;
    uint64_t* drec = nullptr;
    void* scratch = nullptr;
    const uint64_t sb = bp.scratch_bytes(n, want.size());
    HIPCHECK(hipMalloc(&dw, want.size() + 16));
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&drec), 8 * (n + 1)));
    HIPCHECK(hipMalloc(&scratch, sb + 16));
    std::vector<const uint64_t*> coffs(doffs.begin(), doffs.end());
    CHECK(bp.pack_var(dcols.data(), coffs.data(), n, dw, want.size(), drec, scratch, sb) == SRPC_OK);
    std::vector<uint8_t> got(want.size());
    HIPCHECK(hipMemcpy(got.data(), dw, got.size(), hipMemcpyDeviceToHost));
    CHECK(got == want);
    srpc_unpack_status* st = nullptr;
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&st), sizeof(*st)));
    CHECK(bp.unpack_var(dw, want.size(), n, drec, dback.data(), dboffs.data(), scratch, sb, st) == SRPC_OK);
    srpc_unpack_status hs{};
    HIPCHECK(hipMemcpy(&hs, st, sizeof(hs), hipMemcpyDeviceToHost));
    CHECK(hs.flags == 0);
    srpc::gpu::host_columns<Text> back = hc;
    for (size_t f = 0; f < F; ++f) {
        if (!hc.offs[f].empty())
            HIPCHECK(hipMemcpy(back.offs[f].data(), dboffs[f], 8 * (n + 1), hipMemcpyDeviceToHost));
        back.col[f].resize(hc.offs[f].empty() ? hc.col[f].size() : back.offs[f][n]);
        HIPCHECK(hipMemcpy(back.col[f].data(), dback[f], back.col[f].size(), hipMemcpyDeviceToHost));
    }
    std::vector<Text> out;
    back.gather(out);
    bool same = true;
    for (size_t i = 0; same && i < n; ++i)
        same = out[i].a == recs[i].a && out[i].s == recs[i].s && out[i].b == recs[i].b && out[i].in.tag == recs[i].in.tag &&
               out[i].in.small == recs[i].in.small && out[i].t == recs[i].t;
    CHECK(same);
    for (size_t f = 0; f < F; ++f) {
        (void)hipFree(dcols[f]);
        (void)hipFree(dback[f]);
        if (doffs[f]) (void)hipFree(doffs[f]);
        if (dboffs[f]) (void)hipFree(dboffs[f]);
    }
    (void)hipFree(dw);
    (void)hipFree(drec);
    (void)hipFree(scratch);
    (void)hipFree(st);
    return 0;
}

int main() {
    std::mt19937_64 rng(42);
    using srpc::gpu::batch_packer;
    const std::vector<int32_t> kinds = srpc::gpu::flat_kinds<Outer>();
    CHECK((kinds == std::vector<int32_t>{SRPC_KIND_INT64, SRPC_KIND_INT8, SRPC_KIND_INT16, SRPC_KIND_BOOL,
                                          SRPC_KIND_CHAR, SRPC_KIND_INT32}));
    for (size_t n : {1ul, 100ul, 4099ul, 1ul << 20}) {
        batch_packer<Number> body;
        auto fillN = [&](Number& r, size_t) { r.num = static_cast<int32_t>(rng()); };
        auto eqN = [](const Number& a, const Number& b) { return a.num == b.num; };
        if (run(body, n, fillN, eqN, [](srpc::packer& p, const Number& r) { p << r; })) return 2;
        auto req = batch_packer<Number>::request("Calculator_servicer::square");
        CHECK(req.record_bytes() == 53);
        if (run(req, n, fillN, eqN, [](srpc::packer& p, const Number& r) {
                srpc::request_t<Number> q;
                q.set_method_name("Calculator_servicer::square");
                q.set_value(r);
                p.pack_request(q);
            })) return 2;
        auto resp = batch_packer<Number>::response(srpc::RPC_SUCCESS);
        CHECK(resp.record_bytes() == 19);
        if (run(resp, n, fillN, eqN, [](srpc::packer& p, const Number& r) {
                srpc::response_t<Number> q;
                q.set_value(r);
                p.pack_response(q);
            })) return 2;
        batch_packer<Outer> outer;
        CHECK(outer.record_bytes() == 8 + 1 + 2 + 1 + 1 + 4);
        if (run(outer, n,
                [&](Outer& r, size_t) {
                    r.id = static_cast<int64_t>(rng());
                    r.in.tag = static_cast<int8_t>(rng());
                    r.in.small = static_cast<int16_t>(rng());
                    r.flag = rng() & 1;
                    r.c = static_cast<char>(rng());
                    r.v = static_cast<int32_t>(rng());
                },
                [](const Outer& a, const Outer& b) {
                    return a.id == b.id && a.in.tag == b.in.tag && a.in.small == b.in.small && a.flag == b.flag &&
                           a.c == b.c && a.v == b.v;
                },
                [](srpc::packer& p, const Outer& r) { p << r; })) return 2;
    }
    {
        batch_packer<Text> text;
        CHECK(text.has_strings());
        for (size_t n : {1ul, 1000ul, 70001ul})
            if (run_var(text, n, rng)) return 2;
    }
    std::printf("gpu_batch_test: %d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
