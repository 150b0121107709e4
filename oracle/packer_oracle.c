/*
 * packer_oracle.c -- TEST INFRASTRUCTURE ONLY (see packer_oracle.h).
 *
 * CPU restatement of the sRPC packer, one record at a time, following the
 * reference exactly:
 *   - fixed fields: raw host (little-endian) bytes, no padding, no tags
 *       pack_arg<T> generic          include/srpc/packer.hpp:183-191
 *       buffer::append               include/srpc/core.hpp:34-35
 *   - strings: u64 length then the bytes, no NUL
 *       pack_arg<std::string>        include/srpc/packer.hpp:193-198
 *       pack_arg<const char*>        include/srpc/packer.hpp:203-208
 *   - message bodies: fields in T::fields order, nested messages inlined
 *       pack_struct                  include/srpc/packer.hpp:172-178
 *   - envelopes
 *       pack_request                 include/srpc/packer.hpp:77-82
 *       pack_response                include/srpc/packer.hpp:86-91
 *   - decode with a shared cursor and bounds check
 *       pipe_output<T>               include/srpc/packer.hpp:210-214
 *       pipe_output<std::string>     include/srpc/packer.hpp:216-222
 *       buffer::increment            include/srpc/core.hpp:28-33
 * The reference throws inside noexcept (=> std::terminate) on a bounds
 * error; the oracle returns ORC_ERR_BOUNDS instead.
 */
#include "packer_oracle.h"

#include <string.h>

int orc_kind_size(int kind) {
    switch (kind) {
    case ORC_BOOL:
    case ORC_INT8:
    case ORC_CHAR: return 1;
    case ORC_INT16: return 2;
    case ORC_INT32: return 4;
    case ORC_INT64: return 8;
    case ORC_STRING: return 0;
    default: return -1;
    }
}

uint64_t orc_fixed_record_size(const int* kinds, int nfields, uint64_t prefix_len) {
    uint64_t s = prefix_len;
    for (int f = 0; f < nfields; ++f) {
        int k = orc_kind_size(kinds[f]);
        if (k <= 0) return 0;
        s += (uint64_t)k;
    }
    return s;
}

/* pack_arg<size_t>: sizeof(size_t)=8 raw bytes (packer.hpp:195-196, 205-206) */
static void put_u64(uint8_t* out, uint64_t v) { memcpy(out, &v, 8); }

uint64_t orc_request_prefix(const char* method, const char* name, uint8_t* out) {
    uint64_t lm = strlen(method), ln = strlen(name), o = 0;
    put_u64(out + o, lm); o += 8;
    memcpy(out + o, method, lm); o += lm;
    put_u64(out + o, ln); o += 8;
    memcpy(out + o, name, ln); o += ln;
    return o;
}

uint64_t orc_response_prefix(uint8_t code, const char* name, uint8_t* out) {
    uint64_t ln = strlen(name), o = 0;
    out[o++] = code; /* rpc_status_code is uint8_t (packer.hpp:16) */
    put_u64(out + o, ln); o += 8;
    memcpy(out + o, name, ln); o += ln;
    return o;
}

uint64_t orc_pack(const int* kinds, int nfields, const uint8_t* prefix,
                  uint64_t prefix_len, const void* const* cols,
                  const uint64_t* const* str_offs, uint64_t n, uint8_t* out,
                  uint64_t out_cap) {
    uint64_t o = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (o + prefix_len > out_cap) return UINT64_MAX;
        if (prefix_len) memcpy(out + o, prefix, prefix_len);
        o += prefix_len;
        for (int f = 0; f < nfields; ++f) {
            int sz = orc_kind_size(kinds[f]);
            if (sz > 0) {
                if (o + (uint64_t)sz > out_cap) return UINT64_MAX;
                memcpy(out + o, (const uint8_t*)cols[f] + i * (uint64_t)sz, (size_t)sz);
                o += (uint64_t)sz;
            } else if (sz == 0) {
                uint64_t b = str_offs[f][i], e = str_offs[f][i + 1], len = e - b;
                if (o + 8 + len > out_cap) return UINT64_MAX;
                put_u64(out + o, len);
                o += 8;
                memcpy(out + o, (const uint8_t*)cols[f] + b, len);
                o += len;
            } else {
                return UINT64_MAX;
            }
        }
    }
    return o;
}

int orc_unpack(const int* kinds, int nfields, const uint8_t* prefix,
               uint64_t prefix_len, const uint8_t* wire, uint64_t wire_len,
               uint64_t n, void* const* cols, uint64_t* const* str_offs,
               uint64_t* consumed, uint64_t* err_record) {
    uint64_t cur = 0; /* buffer::_offset (core.hpp:39) */
    uint64_t* char_pos = NULL;
    uint64_t char_pos_store[64];
    if (nfields > 64) return ORC_ERR_ARG;
    char_pos = char_pos_store;
    for (int f = 0; f < nfields; ++f) {
        char_pos[f] = 0;
        if (kinds[f] == ORC_STRING && str_offs && str_offs[f]) str_offs[f][0] = 0;
    }
    for (uint64_t i = 0; i < n; ++i) {
        if (prefix_len) {
            if (cur + prefix_len > wire_len) goto bounds;
            if (memcmp(wire + cur, prefix, prefix_len) != 0) {
                if (consumed) *consumed = cur;
                if (err_record) *err_record = i;
                return ORC_ERR_PREFIX;
            }
            cur += prefix_len;
        }
        for (int f = 0; f < nfields; ++f) {
            int sz = orc_kind_size(kinds[f]);
            if (sz > 0) {
                if (cur + (uint64_t)sz > wire_len) goto bounds;
                memcpy((uint8_t*)cols[f] + i * (uint64_t)sz, wire + cur, (size_t)sz);
                cur += (uint64_t)sz;
            } else if (sz == 0) {
                int64_t len;
                if (cur + 8 > wire_len) goto bounds;
                memcpy(&len, wire + cur, 8);
                cur += 8;
                if (len < 0 || (uint64_t)len > wire_len - cur) goto bounds;
                memcpy((uint8_t*)cols[f] + char_pos[f], wire + cur, (size_t)len);
                char_pos[f] += (uint64_t)len;
                str_offs[f][i + 1] = char_pos[f];
                cur += (uint64_t)len;
            } else {
                return ORC_ERR_ARG;
            }
        }
        continue;
    bounds:
        if (consumed) *consumed = cur;
        if (err_record) *err_record = i;
        return ORC_ERR_BOUNDS;
    }
    if (consumed) *consumed = cur;
    if (err_record) *err_record = n;
    return ORC_OK;
}

static inline uint64_t splitmix_next(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void orc_splitmix_i32(uint64_t* state, int32_t* out, uint64_t count) {
    for (uint64_t i = 0; i < count; ++i) {
        uint32_t lo = (uint32_t)(splitmix_next(state) & 0xffffffffULL);
        memcpy(&out[i], &lo, 4);
    }
}

void orc_splitmix_columns_i32(uint64_t* state, int32_t* const* cols, int nfields,
                              uint64_t n) {
    for (uint64_t i = 0; i < n; ++i)
        for (int f = 0; f < nfields; ++f) {
            uint32_t lo = (uint32_t)(splitmix_next(state) & 0xffffffffULL);
            memcpy(&cols[f][i], &lo, 4);
        }
}
