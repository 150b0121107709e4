// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Thin extern "C" wrappers that drive the *reference* sRPC packer, compiled
// from the unmodified headers where they lie under /root/reference (see
// oracle/Makefile for the exact compiler flags and why they are needed).
// The resulting library, oracle/_ref/libsrpc_ref.so, is used for two things:
//   1. generating golden fixtures (tests/golden/make_golden.py), so the C
//      restatement in packer_oracle.c is pinned to the reference's own bytes;
//   2. the "reference" CPU baseline in bench.py (the real packer, timed on the
//      GPU box's host cores, using the reference's own usage pattern:
//      one packer, `p << r` per record; `r.unpack(bp)` per record).
// No reference source is copied into this repository; this file only
// #includes it by path at build time.  The message structs below are written
// the way the reference code generator emits them
// (include/srpc/generator.hpp:100-134, examples/calculator_srpc.cpp:11-40).
#include <srpc/core.hpp>
#include <srpc/packer.hpp>
#include <srpc/server.hpp>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

// Number / TwoNumbers / Calculator_stub / Calculator_servicer, as generated
// by the reference tool from examples/calculator.contract.
#include "calculator_srpc.cpp"

// deterministic Geo records shared with tests/cpp/batchgen_gpu_test.cpp
#include "../tests/cpp/geo_records.hpp"
// deterministic Echo requests shared with tools/e2e_square.hip --echo
#include "../tests/cpp/echo_records.hpp"

namespace {

// Synthetic schema of configs 3/4: message Quad { int32 a,b,c,d; }
struct Quad : public srpc::message_base {
    int32_t a;
    int32_t b;
    int32_t c;
    int32_t d;
    static constexpr const char* name = "Quad";
    static constexpr auto fields = std::make_tuple(
        STRUCT_MEMBER(Quad, a, "Quad::a"), STRUCT_MEMBER(Quad, b, "Quad::b"),
        STRUCT_MEMBER(Quad, c, "Quad::c"), STRUCT_MEMBER(Quad, d, "Quad::d"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> a;
        p >> b;
        p >> c;
        p >> d;
    }
};

// The three messages of the reference's packer test (tests/packer_test.cpp:11-89).
struct single_primitive : public srpc::message_base {
    int8_t arg1;
    static constexpr const char* name = "single_primitive";
    static constexpr auto fields =
        std::make_tuple(STRUCT_MEMBER(single_primitive, arg1, "single_primitive::arg1"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> arg1;
    }
};

struct multiple_primitives : public srpc::message_base {
    int8_t arg1;
    char arg2;
    int64_t arg3;
    std::string arg4;
    static constexpr const char* name = "multiple_primitives";
    static constexpr auto fields =
        std::make_tuple(STRUCT_MEMBER(multiple_primitives, arg1, "multiple_primitives::arg1"),
                        STRUCT_MEMBER(multiple_primitives, arg2, "multiple_primitives::arg2"),
                        STRUCT_MEMBER(multiple_primitives, arg3, "multiple_primitives::arg3"),
                        STRUCT_MEMBER(multiple_primitives, arg4, "multiple_primitives::arg4"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> arg1;
        p >> arg2;
        p >> arg3;
        p >> arg4;
    }
};

struct nested_message : public srpc::message_base {
    int64_t arg1;
    single_primitive arg2;
    multiple_primitives arg3;
    static constexpr const char* name = "nested_message";
    static constexpr auto fields =
        std::make_tuple(STRUCT_MEMBER(nested_message, arg1, "nested_message::arg1"),
                        STRUCT_MEMBER(nested_message, arg2, "nested_message::arg2"),
                        STRUCT_MEMBER(nested_message, arg3, "nested_message::arg3"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> arg1;
        single_primitive a2;
        a2.unpack(bp);
        arg2 = std::move(a2);
        multiple_primitives a3;
        a3.unpack(bp);
        arg3 = std::move(a3);
    }
};

// Every fixed-size IDL kind once (parser.hpp:253-274).
struct all_kinds : public srpc::message_base {
    bool k_bool;
    int8_t k_i8;
    char k_char;
    int16_t k_i16;
    int32_t k_i32;
    int64_t k_i64;
    static constexpr const char* name = "all_kinds";
    static constexpr auto fields = std::make_tuple(
        STRUCT_MEMBER(all_kinds, k_bool, "all_kinds::k_bool"),
        STRUCT_MEMBER(all_kinds, k_i8, "all_kinds::k_i8"),
        STRUCT_MEMBER(all_kinds, k_char, "all_kinds::k_char"),
        STRUCT_MEMBER(all_kinds, k_i16, "all_kinds::k_i16"),
        STRUCT_MEMBER(all_kinds, k_i32, "all_kinds::k_i32"),
        STRUCT_MEMBER(all_kinds, k_i64, "all_kinds::k_i64"));
    void unpack(srpc::buffer::ptr bp) override {
        srpc::packer p(bp);
        p >> k_bool;
        p >> k_i8;
        p >> k_char;
        p >> k_i16;
        p >> k_i32;
        p >> k_i64;
    }
};

// The messages of tests/cpp/batchgen_example.contract (the f3 pin), written
// the way the reference generator emits a message (generator.hpp:100-134:
// fields in declaration order, one STRUCT_MEMBER each, nested messages as
// members).  Only packing is used: the generator's nested unpack does not
// compile (generator.hpp:127), so these structs have no nested unpack.
namespace geo_ref {
struct Inner : public srpc::message_base {
    int8_t tag;
    int16_t small;
    static constexpr const char* name = "Inner";
    static constexpr auto fields =
        std::make_tuple(STRUCT_MEMBER(Inner, tag, "Inner::tag"), STRUCT_MEMBER(Inner, small, "Inner::small"));
    void unpack(srpc::buffer::ptr) override {}
};
struct Point : public srpc::message_base {
    int32_t x;
    int32_t y;
    static constexpr const char* name = "Point";
    static constexpr auto fields =
        std::make_tuple(STRUCT_MEMBER(Point, x, "Point::x"), STRUCT_MEMBER(Point, y, "Point::y"));
    void unpack(srpc::buffer::ptr) override {}
};
struct Record : public srpc::message_base {
    int64_t id;
    Inner in;
    bool flag;
    std::string label;
    char c;
    Point p;
    std::string note;
    static constexpr const char* name = "Record";
    static constexpr auto fields = std::make_tuple(
        STRUCT_MEMBER(Record, id, "Record::id"), STRUCT_MEMBER(Record, in, "Record::in"),
        STRUCT_MEMBER(Record, flag, "Record::flag"), STRUCT_MEMBER(Record, label, "Record::label"),
        STRUCT_MEMBER(Record, c, "Record::c"), STRUCT_MEMBER(Record, p, "Record::p"),
        STRUCT_MEMBER(Record, note, "Record::note"));
    void unpack(srpc::buffer::ptr) override {}
};
}  // namespace geo_ref

// A service with a string-bodied method, declared the way the reference
// generator emits a servicer (generator.hpp, calculator_srpc.cpp:63-83).
struct Echo_servicer : srpc::servicer_base {
    virtual multiple_primitives echo(multiple_primitives&) { throw std::runtime_error("Method not implemented!"); }
    static constexpr const char* name = "Echo";
    static constexpr auto methods = std::make_tuple(STRUCT_MEMBER(Echo_servicer, echo, "Echo_servicer::echo"));
};
struct EchoImpl : Echo_servicer {
    multiple_primitives echo(multiple_primitives& q) override { return echo_fixture::answer(q); }
};

struct Calc : public Calculator_servicer {
    Number square(Number& req) override {
        Number r;
        r.num = req.num * req.num;
        return r;
    }
};

uint64_t copy_out(srpc::packer& p, uint8_t* out, uint64_t cap) {
    auto& v = *p.buf();
    if (v.size() > cap) return UINT64_MAX;
    std::memcpy(out, v.data(), v.size());
    return v.size();
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

void register_all() {
    srpc::message_registry["single_primitive"] = []() -> std::unique_ptr<single_primitive> {
        return std::make_unique<single_primitive>();
    };
    srpc::message_registry["multiple_primitives"] = []() -> std::unique_ptr<multiple_primitives> {
        return std::make_unique<multiple_primitives>();
    };
    srpc::message_registry["nested_message"] = []() -> std::unique_ptr<nested_message> {
        return std::make_unique<nested_message>();
    };
    srpc::message_registry["Number"] = []() -> std::unique_ptr<Number> {
        return std::make_unique<Number>();
    };
    srpc::message_registry["Quad"] = []() -> std::unique_ptr<Quad> {
        return std::make_unique<Quad>();
    };
}

single_primitive make_sp() {
    single_primitive sp;
    sp.arg1 = 5;
    return sp;
}
multiple_primitives make_mp() {
    multiple_primitives mp;
    mp.arg1 = 22;
    mp.arg2 = 'z';
    mp.arg3 = INT64_MAX;
    mp.arg4 = "testing_string";
    return mp;
}
nested_message make_nm() {
    nested_message nm;
    nm.arg1 = INT64_MAX;
    nm.arg2 = make_sp();
    nm.arg3 = make_mp();
    return nm;
}

}  // namespace

extern "C" {

// The six "pack" sections of tests/packer_test.cpp, produced by the reference:
// which = 0..2 -> pack_request {single, multiple, nested} with method "test"
//         3..5 -> pack_response {single (code 0), multiple (2), nested (1)}
uint64_t ref_packer_test_vector(int which, uint8_t* out, uint64_t cap) {
    srpc::packer pr;
    switch (which) {
    case 0: { srpc::request_t<single_primitive> r; r.set_value(make_sp()); r.set_method_name("test"); pr.pack_request(r); break; }
    case 1: { srpc::request_t<multiple_primitives> r; r.set_value(make_mp()); r.set_method_name("test"); pr.pack_request(r); break; }
    case 2: { srpc::request_t<nested_message> r; r.set_value(make_nm()); r.set_method_name("test"); pr.pack_request(r); break; }
    case 3: { srpc::response_t<single_primitive> r; r.set_value(make_sp()); r.set_code(srpc::RPC_SUCCESS); pr.pack_response(r); break; }
    case 4: { srpc::response_t<multiple_primitives> r; r.set_value(make_mp()); r.set_code(srpc::RPC_ERR_RECV_TIMEOUT); pr.pack_response(r); break; }
    case 5: { srpc::response_t<nested_message> r; r.set_value(make_nm()); r.set_code(srpc::RPC_ERR_FUNCTION_NOT_REGISTERED); pr.pack_response(r); break; }
    default: return UINT64_MAX;
    }
    return copy_out(pr, out, cap);
}

// Reference decode of a request/response of the packer-test messages.  The
// decoded value is re-emitted as a bare body (`p << value`) and the method
// name / status code is returned, so the caller can compare field by field.
// kind: 0 single, 1 multiple, 2 nested; is_response selects unpack_response.
uint64_t ref_packer_test_decode(int kind, int is_response, const uint8_t* in, uint64_t len,
                                uint8_t* body_out, uint64_t cap, char* method_out,
                                int* code_out) {
    register_all();
    srpc::packer pr(in, len);
    srpc::packer body;
    auto emit = [&](auto const& v) { body << v; };
    if (!is_response) {
        std::string m;
        switch (kind) {
        case 0: { auto r = pr.unpack_request<single_primitive>(); emit(r.value()); m = r.method_name(); break; }
        case 1: { auto r = pr.unpack_request<multiple_primitives>(); emit(r.value()); m = r.method_name(); break; }
        case 2: { auto r = pr.unpack_request<nested_message>(); emit(r.value()); m = r.method_name(); break; }
        default: return UINT64_MAX;
        }
        std::memcpy(method_out, m.c_str(), m.size() + 1);
    } else {
        switch (kind) {
        case 0: { auto r = pr.unpack_response<single_primitive>(); emit(r.value()); *code_out = r.code(); break; }
        case 1: { auto r = pr.unpack_response<multiple_primitives>(); emit(r.value()); *code_out = r.code(); break; }
        case 2: { auto r = pr.unpack_response<nested_message>(); emit(r.value()); *code_out = r.code(); break; }
        default: return UINT64_MAX;
        }
    }
    return copy_out(body, body_out, cap);
}

// ---- bodies: `packer p; for r: p << r;` (packer.hpp:73) -------------------

uint64_t ref_pack_number(const int32_t* num, uint64_t n, uint8_t* out, uint64_t cap) {
    srpc::packer p;
    for (uint64_t i = 0; i < n; ++i) {
        Number r;
        r.num = num[i];
        p << r;
    }
    return copy_out(p, out, cap);
}

uint64_t ref_pack_two_numbers(const int32_t* l, const int32_t* r_, uint64_t n, uint8_t* out,
                              uint64_t cap) {
    srpc::packer p;
    for (uint64_t i = 0; i < n; ++i) {
        TwoNumbers r;
        r.left = l[i];
        r.right = r_[i];
        p << r;
    }
    return copy_out(p, out, cap);
}

uint64_t ref_pack_all_kinds(const uint8_t* kb, const int8_t* k8, const char* kc, const int16_t* k16,
                            const int32_t* k32, const int64_t* k64, uint64_t n, uint8_t* out,
                            uint64_t cap) {
    srpc::packer p;
    for (uint64_t i = 0; i < n; ++i) {
        all_kinds r;
        r.k_bool = kb[i] != 0;
        r.k_i8 = k8[i];
        r.k_char = kc[i];
        r.k_i16 = k16[i];
        r.k_i32 = k32[i];
        r.k_i64 = k64[i];
        p << r;
    }
    return copy_out(p, out, cap);
}

// multiple_primitives records with variable-length strings: chars + n+1 offsets.
uint64_t ref_pack_multiple(const int8_t* a1, const char* a2, const int64_t* a3, const char* chars,
                           const uint64_t* offs, uint64_t n, uint8_t* out, uint64_t cap) {
    srpc::packer p;
    for (uint64_t i = 0; i < n; ++i) {
        multiple_primitives r;
        r.arg1 = a1[i];
        r.arg2 = a2[i];
        r.arg3 = a3[i];
        r.arg4.assign(chars + offs[i], chars + offs[i + 1]);
        p << r;
    }
    return copy_out(p, out, cap);
}

// Unpack n multiple_primitives bodies with the generated per-record unpack;
// strings are written back-to-back into chars_out with n+1 offsets.
int ref_unpack_multiple(const uint8_t* wire, uint64_t len, uint64_t n, int8_t* a1, char* a2,
                        int64_t* a3, char* chars_out, uint64_t* offs_out) {
    srpc::packer p(wire, len);
    offs_out[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        multiple_primitives r;
        r.unpack(p.buf());
        a1[i] = r.arg1;
        a2[i] = r.arg2;
        a3[i] = r.arg3;
        std::memcpy(chars_out + offs_out[i], r.arg4.data(), r.arg4.size());
        offs_out[i + 1] = offs_out[i] + r.arg4.size();
    }
    return p.size() == 0 ? 0 : 1;
}

// Unpack all_kinds bodies.
int ref_unpack_all_kinds(const uint8_t* wire, uint64_t len, uint64_t n, uint8_t* kb, int8_t* k8,
                         char* kc, int16_t* k16, int32_t* k32, int64_t* k64) {
    srpc::packer p(wire, len);
    for (uint64_t i = 0; i < n; ++i) {
        all_kinds r;
        r.unpack(p.buf());
        kb[i] = r.k_bool ? 1 : 0;
        k8[i] = r.k_i8;
        kc[i] = r.k_char;
        k16[i] = r.k_i16;
        k32[i] = r.k_i32;
        k64[i] = r.k_i64;
    }
    return p.size() == 0 ? 0 : 1;
}

// ---- Quad: the bench workload -----------------------------------------------

// Pack n Quads into out; *secs = time of the `p << r` loop only.
uint64_t ref_pack_quad(const int32_t* a, const int32_t* b, const int32_t* c, const int32_t* d,
                       uint64_t n, uint8_t* out, uint64_t cap, double* secs) {
    srpc::packer p;
    double t0 = now_s();
    for (uint64_t i = 0; i < n; ++i) {
        Quad r;
        r.a = a[i];
        r.b = b[i];
        r.c = c[i];
        r.d = d[i];
        p << r;
    }
    double t1 = now_s();
    if (secs) *secs = t1 - t0;
    return out ? copy_out(p, out, cap) : p.size();
}

// Unpack n Quads with the generated per-record unpack; *secs = loop time.
int ref_unpack_quad(const uint8_t* wire, uint64_t len, uint64_t n, int32_t* a, int32_t* b,
                    int32_t* c, int32_t* d, double* secs) {
    srpc::packer p(wire, len);
    srpc::buffer::ptr bp = p.buf();
    double t0 = now_s();
    for (uint64_t i = 0; i < n; ++i) {
        Quad r;
        r.unpack(bp);
        a[i] = r.a;
        b[i] = r.b;
        c[i] = r.c;
        d[i] = r.d;
    }
    double t1 = now_s();
    if (secs) *secs = t1 - t0;
    return p.size() == 0 ? 0 : 1;
}

// Multi-threaded variant: one independent packer per contiguous shard, the
// shard's bytes then copied to out at the shard's offset (16 B per Quad).
// *secs covers pack (and copy-out) of all shards, threads started inside.
uint64_t ref_pack_quad_mt(const int32_t* a, const int32_t* b, const int32_t* c, const int32_t* d,
                          uint64_t n, uint8_t* out, int nthreads, double* secs) {
    if (nthreads < 1) nthreads = 1;
    double t0 = now_s();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        uint64_t lo = n * t / nthreads, hi = n * (t + 1) / nthreads;
        th.emplace_back([=]() {
            srpc::packer p;
            for (uint64_t i = lo; i < hi; ++i) {
                Quad r;
                r.a = a[i];
                r.b = b[i];
                r.c = c[i];
                r.d = d[i];
                p << r;
            }
            std::memcpy(out + lo * 16, p.buf()->data(), p.buf()->size());
        });
    }
    for (auto& x : th) x.join();
    if (secs) *secs = now_s() - t0;
    return n * 16;
}

int ref_unpack_quad_mt(const uint8_t* wire, uint64_t n, int32_t* a, int32_t* b, int32_t* c,
                       int32_t* d, int nthreads, double* secs) {
    if (nthreads < 1) nthreads = 1;
    double t0 = now_s();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        uint64_t lo = n * t / nthreads, hi = n * (t + 1) / nthreads;
        th.emplace_back([=]() {
            srpc::packer p(wire + lo * 16, (hi - lo) * 16);
            srpc::buffer::ptr bp = p.buf();
            for (uint64_t i = lo; i < hi; ++i) {
                Quad r;
                r.unpack(bp);
                a[i] = r.a;
                b[i] = r.b;
                c[i] = r.c;
                d[i] = r.d;
            }
        });
    }
    for (auto& x : th) x.join();
    if (secs) *secs = now_s() - t0;
    return 0;
}

// ---- Calculator.square envelopes (configs 2 and 5) --------------------------

// n requests `pack_request("Calculator_servicer::square", Number{num[i]})`,
// concatenated unframed (what the stub sends, calculator_srpc.cpp:120-126).
uint64_t ref_pack_square_requests(const int32_t* num, uint64_t n, uint8_t* out, uint64_t cap,
                                  double* secs) {
    uint64_t o = 0;
    double t0 = now_s();
    for (uint64_t i = 0; i < n; ++i) {
        srpc::packer pr;
        srpc::request_t<Number> req;
        req.set_method_name("Calculator_servicer::square");
        Number v;
        v.num = num[i];
        req.set_value(std::move(v));
        pr.pack_request(req);
        auto& b = *pr.buf();
        if (o + b.size() > cap) return UINT64_MAX;
        std::memcpy(out + o, b.data(), b.size());
        o += b.size();
    }
    if (secs) *secs = now_s() - t0;
    return o;
}

// The server path of config 5 for each fixed-size request of req_size bytes:
// `>> funcname`, `call` -> getv -> square -> pack_response (server.hpp:58-69,
// 17-30, 106-115), responses concatenated unframed.
uint64_t ref_server_square(const uint8_t* reqs, uint64_t req_size, uint64_t n, uint8_t* out,
                           uint64_t cap, double* secs) {
    register_all();
    srpc::server s;
    Calc calc;
    s.register_service(calc);
    uint64_t o = 0;
    double t0 = now_s();
    for (uint64_t i = 0; i < n; ++i) {
        srpc::packer::ptr p = std::make_shared<srpc::packer>(reqs + i * req_size, req_size);
        std::string funcname;
        (*p) >> funcname;
        srpc::packer::ptr r = s.call(funcname, p);
        if (o + r->size() > cap) return UINT64_MAX;
        std::memcpy(out + o, r->data(), r->size());
        o += r->size();
    }
    if (secs) *secs = now_s() - t0;
    return o;
}

// n Echo requests (echo_fixture::fill_request, pack_request with method
// "Echo_servicer::echo") through the reference server one at a time, as
// ref_server_square; *req_bytes = the request stream's bytes (unframed),
// returns the response stream's bytes (unframed), written to out.
uint64_t ref_server_echo(uint64_t n, uint8_t* out, uint64_t cap, uint64_t* req_bytes) {
    register_all();
    srpc::server s;
    EchoImpl svc;
    s.register_service(svc);
    uint64_t o = 0, rq = 0;
    for (uint64_t i = 0; i < n; ++i) {
        multiple_primitives m;
        echo_fixture::fill_request(m, i);
        srpc::packer pr;
        srpc::request_t<multiple_primitives> req;
        req.set_method_name(echo_fixture::kMethod);
        req.set_value(std::move(m));
        pr.pack_request(req);
        rq += pr.size();
        srpc::packer::ptr p = std::make_shared<srpc::packer>(pr.data(), pr.size());
        std::string funcname;
        (*p) >> funcname;
        srpc::packer::ptr r = s.call(funcname, p);
        if (o + r->size() > cap) return UINT64_MAX;
        std::memcpy(out + o, r->data(), r->size());
        o += r->size();
    }
    if (req_bytes) *req_bytes = rq;
    return o;
}

// Client-side decode of n fixed-size responses (unpack_response<Number>,
// calculator_srpc.cpp:127-131); num_out[i] = value, code_out[i] = status.
int ref_unpack_square_responses(const uint8_t* resp, uint64_t resp_size, uint64_t n,
                                int32_t* num_out, uint8_t* code_out) {
    register_all();
    for (uint64_t i = 0; i < n; ++i) {
        srpc::packer rpr(resp + i * resp_size, resp_size);
        srpc::response_t<Number> m = rpr.unpack_response<Number>();
        num_out[i] = m.value().num;
        code_out[i] = m.code();
    }
    return 0;
}

// ---- generated-message batches --------------------------------
// n Geo.locate responses (pack_response<Record>, code RPC_SUCCESS) and n
// Geo.locate requests (pack_request<Point>, method "Geo_servicer::locate", the
// name generator.hpp:84 gives it), records drawn by geo_fixture from `seed`,
// each stream concatenated in one packer as a server / client appends them.
uint64_t ref_geo_locate_responses(uint64_t n, uint64_t seed, uint8_t* out, uint64_t cap) {
    srpc::packer p;
    uint64_t s = seed;
    for (uint64_t i = 0; i < n; ++i) {
        geo_ref::Record r;
        geo_fixture::fill_record(r, s);
        srpc::response_t<geo_ref::Record> resp;
        resp.set_value(r);
        p.pack_response(resp);
    }
    return copy_out(p, out, cap);
}

uint64_t ref_geo_locate_requests(uint64_t n, uint64_t seed, uint8_t* out, uint64_t cap) {
    srpc::packer p;
    uint64_t s = seed;
    for (uint64_t i = 0; i < n; ++i) {
        geo_ref::Point pt;
        geo_fixture::fill_point(pt, s);
        srpc::request_t<geo_ref::Point> req;
        req.set_method_name("Geo_servicer::locate");
        req.set_value(std::move(pt));
        p.pack_request(req);
    }
    return copy_out(p, out, cap);
}

}  // extern "C"
