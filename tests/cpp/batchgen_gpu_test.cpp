// needs: gpu, batchgen
// Generated batch views (srpc_amd.batchgen) driving the GPU batch
// path, pinned to the REFERENCE packer: the Geo.locate records of
// tests/cpp/geo_records.hpp are packed on the GPU as Record responses (nested
// + two strings, VAR path) and as Point requests (TILE path), and the bytes are
// written to <out_dir>/geo_locate_{responses,requests}.bin.
// tests/test_batchgen.py hashes them against the digests the reference
// produced from the same records (tests/golden/manifest.json "batchgen",
// oracle/ref_shim.cpp ref_geo_locate_*).  Unpack must give the columns back.
#include <hip/hip_runtime_api.h>
#include <batchgen_example_batch.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "geo_records.hpp"

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

static bool write_file(const std::string& path, const std::vector<uint8_t>& b) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const bool ok = std::fwrite(b.data(), 1, b.size(), f) == b.size();
    return std::fclose(f) == 0 && ok;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <out_dir>\n", argv[0]);
        return 2;
    }
    const std::string out_dir = argv[1];
    const size_t n = geo_fixture::kRecords;
    uint64_t seed = geo_fixture::kSeed;
    // ---- Geo.locate responses: Record (nested + two strings), variable-size path
    std::vector<Record> recs(n);
    uint64_t chars = 0;
    for (auto& r : recs) {
        geo_fixture::fill_record(r, seed);
        chars += r.label.size() + r.note.size();
    }
    srpc::gpu::host_columns<Record> hc;
    hc.scatter(recs);
    Record_batch rb;
    if (upload(hc, rb)) return 2;
    auto resp = Geo_batch::locate_response();
    CHECK(resp.has_strings());
    uint8_t* dw = nullptr;
    uint64_t* drec = nullptr;
    void* scratch = nullptr;
    const uint64_t cap = n * 128 + chars;  // > prefix + fixed fields + lengths per record, plus the chars
    const uint64_t sb = resp.scratch_bytes(n, cap);
    HIPCHECK(hipMalloc(&dw, cap + 16));
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&drec), 8 * (n + 1)));
    HIPCHECK(hipMalloc(&scratch, sb + 16));
    CHECK(resp.pack_var(rb.columns(), rb.str_offsets(), n, dw, cap, drec, scratch, sb) == SRPC_OK);
    uint64_t total = 0;
    HIPCHECK(hipMemcpy(&total, drec + n, 8, hipMemcpyDeviceToHost));
    CHECK(total > 0 && total <= cap);
    std::vector<uint8_t> got(std::min(total, cap));
    HIPCHECK(hipMemcpy(got.data(), dw, got.size(), hipMemcpyDeviceToHost));
    CHECK(write_file(out_dir + "/geo_locate_responses.bin", got));
    const std::vector<uint8_t>& want = got;
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
    seed = geo_fixture::kSeed;  // the reference draws the request stream from the seed again
    for (auto& p : pts) geo_fixture::fill_point(p, seed);
    srpc::gpu::host_columns<Point> phc;
    phc.scatter(pts);
    Point_batch pb;
    if (upload(phc, pb)) return 2;
    auto req = Geo_batch::locate_request();
    const uint64_t pbytes = req.record_bytes() * n;
    HIPCHECK(hipMalloc(&dw, pbytes + 16));
    CHECK(req.pack(pb.columns(), n, dw, pbytes) == SRPC_OK);
    std::vector<uint8_t> pgot(pbytes);
    HIPCHECK(hipMemcpy(pgot.data(), dw, pgot.size(), hipMemcpyDeviceToHost));
    CHECK(write_file(out_dir + "/geo_locate_requests.bin", pgot));
    release(pb);
    (void)hipFree(dw);

    std::printf("%d passed, %d failed\n", g_pass, g_fail);
    return g_fail ? 1 : 0;
}
