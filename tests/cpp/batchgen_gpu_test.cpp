// needs: gpu, batchgen
// Generated batch views (srpc_amd.batchgen) driving the GPU batch path: a
// Record_batch (nested + strings) packed as Geo.locate responses and a
// Point_batch packed as Geo.locate requests must equal the scalar packer's
// pack_response / pack_request loops, and unpack must give the columns back.
#include <hip/hip_runtime_api.h>
#include <batchgen_example_batch.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
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

// Device copy of a host SoA image into a generated batch view.
template <typename B>
static int upload(const srpc::gpu::host_columns<typename B::message_type>& hc, B& b) {
    b.n = hc.n;
    for (uint32_t f = 0; f < B::nfields; ++f) {
        HIPCHECK(hipMalloc(&b.cols[f], hc.col[f].size() + 16));
        HIPCHECK(hipMemcpy(b.cols[f], hc.col[f].data(), hc.col[f].size(), hipMemcpyHostToDevice));
        if (!hc.offs[f].empty()) {
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&b.offs[f]), 8 * (hc.n + 1)));
            HIPCHECK(hipMemcpy(b.offs[f], hc.offs[f].data(), 8 * (hc.n + 1), hipMemcpyHostToDevice));
        }
    }
    return 0;
}

template <typename B>
static void release(B& b) {
    for (uint32_t f = 0; f < B::nfields; ++f) {
        if (b.cols[f]) (void)hipFree(b.cols[f]);
        if (b.offs[f]) (void)hipFree(b.offs[f]);
    }
}

int main() {
    std::mt19937_64 rng(7);
    const size_t n = 20000;
    // ---- Geo.locate responses: Record (nested + two strings), variable-size path
    std::vector<Record> recs(n);
    for (auto& r : recs) {
        r.id = static_cast<int64_t>(rng());
        r.in.tag = static_cast<int8_t>(rng());
        r.in.small = static_cast<int16_t>(rng());
        r.flag = rng() & 1;
        r.label.assign(rng() % 40, 'a');
        for (auto& ch : r.label) ch = static_cast<char>('a' + rng() % 26);
        r.c = static_cast<char>(rng());
        r.p.x = static_cast<int32_t>(rng());
        r.p.y = static_cast<int32_t>(rng());
        r.note.assign(rng() % 5 == 0 ? rng() % 300 : 0, 'n');
    }
    srpc::packer ref;
    for (auto& r : recs) {
        srpc::response_t<Record> resp;
        resp.set_value(Record(r));
        ref.pack_response(resp);
    }
    const std::vector<uint8_t> want(*ref.buf());
    srpc::gpu::host_columns<Record> hc;
    hc.scatter(recs);
    Record_batch rb;
    if (upload(hc, rb)) return 2;
    auto resp = Geo_batch::locate_response();
    CHECK(resp.has_strings());
    uint8_t* dw = nullptr;
    uint64_t* drec = nullptr;
    void* scratch = nullptr;
    const uint64_t sb = resp.scratch_bytes(n, want.size());
    HIPCHECK(hipMalloc(&dw, want.size() + 16));
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&drec), 8 * (n + 1)));
    HIPCHECK(hipMalloc(&scratch, sb + 16));
    CHECK(resp.pack_var(rb.columns(), rb.str_offsets(), n, dw, want.size(), drec, scratch, sb) == SRPC_OK);
    std::vector<uint8_t> got(want.size());
    HIPCHECK(hipMemcpy(got.data(), dw, got.size(), hipMemcpyDeviceToHost));
    CHECK(got == want);
    // unpack into a second batch view and compare the columns
    Record_batch back;
    back.n = n;
    for (uint32_t f = 0; f < Record_batch::nfields; ++f) {
        HIPCHECK(hipMalloc(&back.cols[f], std::max(hc.col[f].size(), want.size()) + 16));
        if (!hc.offs[f].empty()) HIPCHECK(hipMalloc(reinterpret_cast<void**>(&back.offs[f]), 8 * (n + 1)));
    }
    CHECK(resp.unpack_var(dw, want.size(), n, drec, back.columns(), back.str_offsets(), scratch, sb) == SRPC_OK);
    bool same = true;
    for (uint32_t f = 0; f < Record_batch::nfields && same; ++f) {
        std::vector<uint8_t> col(hc.col[f].size());
        HIPCHECK(hipMemcpy(col.data(), back.cols[f], col.size(), hipMemcpyDeviceToHost));
        same = col == hc.col[f];
        if (!hc.offs[f].empty()) {
            std::vector<uint64_t> o(n + 1);
            HIPCHECK(hipMemcpy(o.data(), back.offs[f], 8 * (n + 1), hipMemcpyDeviceToHost));
            same = same && o == hc.offs[f];
        }
    }
    CHECK(same);
    release(rb);
    release(back);
    (void)hipFree(dw);
    (void)hipFree(drec);
    (void)hipFree(scratch);

    // ---- Geo.locate requests: Point, fixed-size path
    std::vector<Point> pts(n);
    for (auto& p : pts) {
        p.x = static_cast<int32_t>(rng());
        p.y = static_cast<int32_t>(rng());
    }
    srpc::packer pref;
    for (auto& p : pts) {
        srpc::request_t<Point> q;
        q.set_method_name(Geo_batch::locate_method);
        q.set_value(Point(p));
        pref.pack_request(q);
    }
    const std::vector<uint8_t> pwant(*pref.buf());
    srpc::gpu::host_columns<Point> phc;
    phc.scatter(pts);
    Point_batch pb;
    if (upload(phc, pb)) return 2;
    auto req = Geo_batch::locate_request();
    CHECK(req.record_bytes() * n == pwant.size());
    HIPCHECK(hipMalloc(&dw, pwant.size() + 16));
    CHECK(req.pack(pb.columns(), n, dw, pwant.size()) == SRPC_OK);
    std::vector<uint8_t> pgot(pwant.size());
    HIPCHECK(hipMemcpy(pgot.data(), dw, pgot.size(), hipMemcpyDeviceToHost));
    CHECK(pgot == pwant);
    release(pb);
    (void)hipFree(dw);

    std::printf("%d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
