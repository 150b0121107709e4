// srpc/gpu.hpp -- batched GPU packing for sRPC messages (host C++ over the C ABI).
//
// srpc::gpu::batch_packer<T> packs / unpacks N records of a generated message
// type T in one launch on an MI355X, producing exactly the bytes of
//     srpc::packer p; for (auto& r : batch) p << r;                   (body)
//     for (auto& r : batch) p.pack_request(request_t<T>{method, r});  (request)
//     for (auto& r : batch) p.pack_response(response_t<T>{code, r});  (response)
// The field list comes from T::fields at compile time (nested messages are
// flattened, as pack_struct inlines them: reference packer.hpp:172-178,
// 183-186), so no hand-written schema is needed.
//
// Records live on the device as one column per flattened field (SoA), the
// wire bytes as one contiguous buffer.  All pointers are device pointers; the
// stream is a hipStream_t passed as void*.  Link with -lsrpc_gpu
// (srpc_amd/libsrpc_gpu.so).
#pragma once

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "../srpc_gpu.h"
#include "core.hpp"
#include "packer.hpp"

namespace srpc::gpu {

template <typename T, typename M>
using member_t = std::remove_cvref_t<decltype(std::declval<T const&>().*std::declval<M>())>;

/// srpc_kind of one C++ field type (the IDL table, parser.hpp:253-290).
template <typename F>
constexpr int32_t kind_of() {
    if constexpr (std::is_same_v<F, bool>) return SRPC_KIND_BOOL;
    else if constexpr (std::is_same_v<F, char>) return SRPC_KIND_CHAR;
    else if constexpr (std::is_same_v<F, std::string>) return SRPC_KIND_STRING;
    else if constexpr (std::is_integral_v<F> || std::is_enum_v<F>) {
        static_assert(sizeof(F) == 1 || sizeof(F) == 2 || sizeof(F) == 4 || sizeof(F) == 8);
        if constexpr (sizeof(F) == 1) return SRPC_KIND_INT8;
        else if constexpr (sizeof(F) == 2) return SRPC_KIND_INT16;
        else if constexpr (sizeof(F) == 4) return SRPC_KIND_INT32;
        else return SRPC_KIND_INT64;
    } else {
        static_assert(sizeof(F) == 0, "srpc::gpu: unsupported field type");
        return 0;
    }
}

/// Visit every leaf field of T (nested messages flattened) in wire order:
/// fn(const Leaf& value_in_record) for a const record, or with a mutable one.
template <typename T, typename Rec, typename Fn>
void for_each_leaf(Rec& rec, Fn&& fn) {
    std::apply(
        [&](const auto&... m) {
            (
                [&] {
                    auto& v = rec.*(std::get<MEMBER_ADDR>(m));
                    using F = std::remove_cvref_t<decltype(v)>;
                    if constexpr (std::is_base_of_v<message_base, F>) for_each_leaf<F>(v, fn);
                    else fn(v);
                }(),
                ...);
        },
        T::fields);
}

template <SrpcMessage T>
std::vector<int32_t> flat_kinds() {
    std::vector<int32_t> k;
    T probe{};
    for_each_leaf<T>(probe, [&](const auto& v) { k.push_back(kind_of<std::remove_cvref_t<decltype(v)>>()); });
    return k;
}

/// The constant header that pack_request / pack_response emit before a body
/// of T -- produced by the scalar packer itself, so the bytes cannot differ.
template <SrpcMessage T>
std::vector<uint8_t> request_prefix(std::string const& method) {
    packer p;
    p << method << T::name;
    return std::vector<uint8_t>(p.data(), p.data() + p.size());
}

template <SrpcMessage T>
std::vector<uint8_t> response_prefix(rpc_status_code code) {
    packer p;
    p << code << T::name;
    return std::vector<uint8_t>(p.data(), p.data() + p.size());
}

/// Host-side SoA image of a batch: one column per flattened field.  A fixed
/// field is n little-endian values; a string field is its chars back to back
/// plus n+1 u64 offsets (the layout srpc_gpu_pack_var / _unpack_var use).
template <SrpcMessage T>
struct host_columns {
    std::vector<std::vector<uint8_t>> col;   // fixed: values; string: chars
    std::vector<std::vector<uint64_t>> offs; // string: n+1 offsets; fixed: empty
    uint64_t n = 0;

    void scatter(std::vector<T> const& recs) {
        n = recs.size();
        // the columns are reused from call to call: fresh ones cost a page
        // fault per 4 KiB on first touch, twice the copy itself (Quad: 12.5
        // ns per record with new vectors, ~4.5 reused, profiles/r02_host_columns.log)
        T probe{};
        size_t nf = 0;
        for_each_leaf<T>(probe, [&](const auto&) { ++nf; });
        col.resize(nf);
        offs.resize(nf);
        size_t g = 0;
        for_each_leaf<T>(probe, [&](const auto& v) {
            using F = std::remove_cvref_t<decltype(v)>;
            if constexpr (std::is_same_v<F, std::string>) {
                col[g].clear();
                offs[g].assign(1, 0);
                offs[g].reserve(n + 1);
            } else {
                col[g].resize(n * sizeof(F));
                offs[g].clear();
            }
            ++g;
        });
        uint8_t* dst[kMaxLeaves] = {};
        for (size_t f = 0; f < col.size() && f < kMaxLeaves; ++f) dst[f] = col[f].data();
        for (uint64_t i = 0; i < n; ++i) {
            size_t f = 0;
            for_each_leaf<T>(recs[i], [&](const auto& v) {
                using F = std::remove_cvref_t<decltype(v)>;
                if constexpr (std::is_same_v<F, std::string>) {
                    col[f].insert(col[f].end(), v.begin(), v.end());
                    offs[f].push_back(col[f].size());
                } else {
                    std::memcpy(dst[f] + i * sizeof(F), &v, sizeof(F));
                }
                ++f;
            });
        }
    }

    void gather(std::vector<T>& recs) const {
        recs.resize(n);
        const uint8_t* src[kMaxLeaves] = {};
        for (size_t f = 0; f < col.size() && f < kMaxLeaves; ++f) src[f] = col[f].data();
        for (uint64_t i = 0; i < n; ++i) {
            size_t f = 0;
            for_each_leaf<T>(recs[i], [&](auto& v) {
                using F = std::remove_cvref_t<decltype(v)>;
                if constexpr (std::is_same_v<F, std::string>) {
                    v.assign(reinterpret_cast<const char*>(col[f].data()) + offs[f][i], offs[f][i + 1] - offs[f][i]);
                } else {
                    std::memcpy(&v, src[f] + i * sizeof(F), sizeof(F));
                }
                ++f;
            });
        }
    }

private:
    static constexpr size_t kMaxLeaves = SRPC_MAX_FIELDS;
};

/// Byte offset of each leaf field of T inside a T object (T::fields order,
/// nested messages flattened) -- the field_offsets of srpc_gpu_pack_aos.
template <SrpcMessage T>
std::vector<uint32_t> leaf_offsets() {
    std::vector<uint32_t> o;
    T probe{};
    const auto* base = reinterpret_cast<const unsigned char*>(&probe);
    for_each_leaf<T>(probe, [&](const auto& v) {
        o.push_back(static_cast<uint32_t>(reinterpret_cast<const unsigned char*>(&v) - base));
    });
    return o;
}

class plan_error : public std::runtime_error {
public:
    plan_error(const char* what, int code)
        : std::runtime_error(std::string(what) + ": " + srpc_status_string(code)), code(code) {}
    int code;
};

/// One plan per (message type, envelope, device).
template <SrpcMessage T>
class batch_packer {
public:
    explicit batch_packer(int device = 0) : batch_packer(std::vector<uint8_t>{}, device) {}

    static batch_packer request(std::string const& method, int device = 0) {
        return batch_packer(request_prefix<T>(method), device);
    }
    static batch_packer response(rpc_status_code code = RPC_SUCCESS, int device = 0) {
        return batch_packer(response_prefix<T>(code), device);
    }

    batch_packer(batch_packer&& o) noexcept
        : _plan(o._plan), _nfields(o._nfields), _rb(o._rb), _offs(std::move(o._offs)) {
        o._plan = nullptr;
    }
    batch_packer(batch_packer const&) = delete;
    batch_packer& operator=(batch_packer const&) = delete;
    ~batch_packer() {
        if (_plan) srpc_plan_destroy(_plan);
    }

    /// Fixed wire bytes per record; 0 when T has string fields (use the *_var calls).
    uint64_t record_bytes() const { return _rb; }
    bool has_strings() const { return _rb == 0; }
    uint32_t nfields() const { return _nfields; }
    srpc_plan* plan() const { return _plan; }

    /// d_cols: nfields() device column pointers.  Returns an srpc status.
    int pack(const void* const* d_cols, uint64_t n, uint8_t* d_wire, uint64_t wire_cap,
             void* stream = nullptr) const {
        return srpc_gpu_pack(_plan, d_cols, n, d_wire, wire_cap, stream);
    }
    int unpack(const uint8_t* d_wire, uint64_t wire_len, uint64_t n, void* const* d_cols,
               srpc_unpack_status* d_status = nullptr, void* stream = nullptr) const {
        return srpc_gpu_unpack(_plan, d_wire, wire_len, n, d_cols, d_status, stream);
    }

    /// Host-terminated batches (ABI 7): host columns <-> host wire bytes.
    /// chunk_records = 0 runs the kernels on the host buffers in place (they
    /// must be page-locked and device-mapped, e.g. hipHostMalloc; no scratch);
    /// otherwise the batch is pipelined in chunks through `depth` device
    /// buffers in d_scratch (host_scratch_bytes).
    uint64_t host_scratch_bytes(uint64_t chunk_records, uint32_t depth = 3) const {
        uint64_t b = 0;
        srpc_plan_host_scratch_bytes(_plan, chunk_records, depth, &b);
        return b;
    }
    int pack_host(const void* const* h_cols, uint64_t n, uint8_t* h_wire, uint64_t wire_cap,
                  uint64_t chunk_records = 0, uint32_t depth = 3, void* d_scratch = nullptr,
                  uint64_t scratch_bytes = 0, void* stream = nullptr) const {
        return srpc_gpu_pack_host(_plan, h_cols, n, h_wire, wire_cap, chunk_records, depth, d_scratch,
                                  scratch_bytes, stream);
    }
    int unpack_host(const uint8_t* h_wire, uint64_t wire_len, uint64_t n, void* const* h_cols,
                    srpc_unpack_status* d_status = nullptr, uint64_t chunk_records = 0, uint32_t depth = 3,
                    void* d_scratch = nullptr, uint64_t scratch_bytes = 0, void* stream = nullptr) const {
        return srpc_gpu_unpack_host(_plan, h_wire, wire_len, n, h_cols, chunk_records, depth, d_scratch,
                                    scratch_bytes, d_status, stream);
    }

    /// Fixed-size T: n records straight from / into a device copy of a T
    /// array (the raw bytes of a std::vector<T>, one hipMemcpy), no host
    /// transpose into columns.  unpack_records writes only the leaf fields.
    int pack_records(const T* d_records, uint64_t n, uint8_t* d_wire, uint64_t wire_cap,
                     void* stream = nullptr) const {
        return srpc_gpu_pack_aos(_plan, d_records, sizeof(T), _offs.data(), n, d_wire, wire_cap, stream);
    }
    int unpack_records(const uint8_t* d_wire, uint64_t wire_len, uint64_t n, T* d_records,
                       srpc_unpack_status* d_status = nullptr, void* stream = nullptr) const {
        return srpc_gpu_unpack_aos(_plan, d_wire, wire_len, n, d_records, sizeof(T), _offs.data(), d_status, stream);
    }
    /// Into fresh objects: every byte no leaf field covers comes from `proto`
    /// (default: a T{}), so the old array is not read (T trivially copyable
    /// apart from its vtable pointer, sizeof(T) <= 256).
    int unpack_records_fresh(const uint8_t* d_wire, uint64_t wire_len, uint64_t n, T* d_records,
                             const T& proto = T{}, srpc_unpack_status* d_status = nullptr,
                             void* stream = nullptr) const {
        return srpc_gpu_unpack_aos_fill(_plan, d_wire, wire_len, n, d_records, sizeof(T), _offs.data(),
                                        static_cast<const void*>(&proto), d_status, stream);
    }

    /// String schemas: device scratch needed by pack_var / unpack_var for n
    /// records and wire_bytes of wire (pack: wire_cap, unpack: wire_len).
    uint64_t scratch_bytes(uint64_t n, uint64_t wire_bytes) const {
        uint64_t b = 0;
        srpc_plan_var_scratch_bytes(_plan, n, wire_bytes, &b);
        return b;
    }
    int pack_var(const void* const* d_cols, const uint64_t* const* d_str_offs, uint64_t n, uint8_t* d_wire,
                 uint64_t wire_cap, uint64_t* d_rec_offs, void* d_scratch, uint64_t scratch_bytes,
                 srpc_unpack_status* d_status = nullptr, void* stream = nullptr) const {
        return srpc_gpu_pack_var(_plan, d_cols, d_str_offs, n, d_wire, wire_cap, d_rec_offs, d_status, d_scratch,
                                 scratch_bytes, stream);
    }
    int unpack_var(const uint8_t* d_wire, uint64_t wire_len, uint64_t n, const uint64_t* d_rec_offs,
                   void* const* d_cols, uint64_t* const* d_str_offs, void* d_scratch, uint64_t scratch_bytes,
                   srpc_unpack_status* d_status = nullptr, void* stream = nullptr) const {
        return srpc_gpu_unpack_var(_plan, d_wire, wire_len, n, d_rec_offs, d_cols, d_str_offs, d_status, d_scratch,
                                   scratch_bytes, stream);
    }

private:
    batch_packer(std::vector<uint8_t> const& prefix, int device) {
        const std::vector<int32_t> kinds = flat_kinds<T>();
        srpc_schema_desc d{static_cast<uint32_t>(kinds.size()), kinds.data(), prefix.empty() ? nullptr : prefix.data(),
                           static_cast<uint32_t>(prefix.size())};
        if (int rc = srpc_plan_create(&d, device, &_plan); rc != SRPC_OK) throw plan_error("srpc_plan_create", rc);
        _nfields = static_cast<uint32_t>(kinds.size());
        srpc_plan_record_bytes(_plan, &_rb);
        _offs = leaf_offsets<T>();
    }

    srpc_plan* _plan = nullptr;
    uint32_t _nfields = 0;
    uint64_t _rb = 0;
    std::vector<uint32_t> _offs;
};

}  // namespace srpc::gpu
