/*
 * packer_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the sRPC packer wire format
 * (reference: include/srpc/packer.hpp + include/srpc/core.hpp).  It is the
 * checker for the HIP path: only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  Nothing in srpc_amd/ links it.
 *
 * Parity pinning: every function here is checked against (a) the 12 literal
 * byte vectors of the reference's tests/packer_test.cpp and (b) fixtures and
 * SHA-256 digests produced by the reference headers themselves, compiled
 * unmodified by oracle/Makefile into oracle/_ref/ (see tests/golden/).
 */
#ifndef SRPC_PACKER_ORACLE_H
#define SRPC_PACKER_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Field kinds: the IDL type table of the reference parser
 * (include/srpc/parser.hpp:253-290).  Values match include/srpc_gpu.h. */
enum {
    ORC_BOOL = 1,
    ORC_INT8 = 2,
    ORC_CHAR = 3,
    ORC_INT16 = 4,
    ORC_INT32 = 5,
    ORC_INT64 = 6,
    ORC_STRING = 7
};

/* Unpack status codes (the reference throws/terminates instead: core.hpp:28-33). */
enum {
    ORC_OK = 0,
    ORC_ERR_BOUNDS = 1,  /* read past end of wire (core.hpp:29-31)            */
    ORC_ERR_PREFIX = 2,  /* envelope prefix != expected method/name header     */
    ORC_ERR_ARG = 4
};

/* Byte size of a fixed-size kind, 0 for ORC_STRING, -1 for unknown. */
int orc_kind_size(int kind);

/* Wire size of one record of an all-fixed schema with a constant prefix,
 * 0 if the schema contains a string field. */
uint64_t orc_fixed_record_size(const int* kinds, int nfields, uint64_t prefix_len);

/* pack_request header (packer.hpp:77-82): u64 len(method) | method |
 * u64 len(name) | name.  Returns bytes written (needs 16+lm+ln). */
uint64_t orc_request_prefix(const char* method, const char* name, uint8_t* out);

/* pack_response header (packer.hpp:86-91): u8 code | u64 len(name) | name. */
uint64_t orc_response_prefix(uint8_t code, const char* name, uint8_t* out);

/* Pack n records (column-major input) into wire bytes, record after record:
 * prefix bytes, then every field in declaration order (packer.hpp:172-178,
 * 183-198).  cols[f] points at n elements of the field's C type; for a
 * string field cols[f] is the character buffer and str_offs[f] holds n+1
 * byte offsets into it.  Returns bytes written, or UINT64_MAX if out_cap
 * is too small. */
uint64_t orc_pack(const int* kinds, int nfields, const uint8_t* prefix,
                  uint64_t prefix_len, const void* const* cols,
                  const uint64_t* const* str_offs, uint64_t n, uint8_t* out,
                  uint64_t out_cap);

/* Unpack n records with the reference's shared-cursor semantics
 * (packer.hpp:70,210-222; core.hpp:28-33): each record must start with the
 * prefix, then each field is read and the cursor advanced.  Fixed fields
 * are written to cols[f][i]; string fields write their bytes to
 * cols[f] + str_offs[f][i] and str_offs[f][i+1] (caller sizes chars by
 * wire_len).  Returns ORC_OK or the first error; *consumed = cursor. */
int orc_unpack(const int* kinds, int nfields, const uint8_t* prefix,
               uint64_t prefix_len, const uint8_t* wire, uint64_t wire_len,
               uint64_t n, void* const* cols, uint64_t* const* str_offs,
               uint64_t* consumed, uint64_t* err_record);

/* splitmix64 stream (SURVEY.md §8c synthetic-input definition): state
 * advances by 0x9E3779B97F4A7C15 per draw; out[i] = (int32)(z & 0xffffffff). */
void orc_splitmix_i32(uint64_t* state, int32_t* out, uint64_t count);

/* Fill F int32 columns record-major from one splitmix stream:
 * record i, field f gets draw number i*F+f (records in order, fields in
 * declaration order). */
void orc_splitmix_columns_i32(uint64_t* state, int32_t* const* cols, int nfields,
                              uint64_t n);

#ifdef __cplusplus
}
#endif

#endif
