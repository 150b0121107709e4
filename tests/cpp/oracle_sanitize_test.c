/* oracle_sanitize_test.c -- TEST INFRASTRUCTURE ONLY (SURVEY §5 "host
 * ASan/UBSan build of the CPU restatement").
 *
 * Built with -fsanitize=address,undefined by tests/test_sanitizers.py and
 * linked with oracle/packer_oracle.c.  Feeds orc_unpack the inputs that the
 * reference reads before it checks (packer.hpp:212-213 vs core.hpp:29-31):
 *   - a valid multi-string stream cut at EVERY length (each copy in its own
 *     exactly-sized heap block, so one byte of over-read is an ASan error);
 *   - string lengths that are oversized (remaining + 1, 2^31, 2^63, 2^64 - 1);
 *   - envelope prefixes that differ;
 *   - more records asked for than the stream holds.
 * Every case must return the documented status and never touch a byte
 * outside the inputs and outputs it was given. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/packer_oracle.h"

static int fails = 0, passes = 0;
#define CHECK(c)                                                       \
    do {                                                               \
        if (c) ++passes;                                               \
        else { ++fails; fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); } \
    } while (0)

enum { N = 40, NF = 5 };
static const int kinds[NF] = {ORC_INT8, ORC_STRING, ORC_INT64, ORC_STRING, ORC_INT16};

/* Unpack `len` bytes copied into a fresh exactly-sized heap block. */
static int unpack_copy(const uint8_t* wire, uint64_t len, uint64_t n, const uint8_t* prefix, uint64_t plen,
                       uint64_t* consumed, uint64_t* err) {
    uint8_t* w = (uint8_t*)malloc(len ? len : 1);
    if (len) memcpy(w, wire, len);
    int8_t* c0 = (int8_t*)malloc(n ? n : 1);
    int64_t* c2 = (int64_t*)malloc(8 * (n ? n : 1));
    int16_t* c4 = (int16_t*)malloc(2 * (n ? n : 1));
    uint8_t* s1 = (uint8_t*)malloc(len ? len : 1);
    uint8_t* s3 = (uint8_t*)malloc(len ? len : 1);
    uint64_t* o1 = (uint64_t*)malloc(8 * (n + 1));
    uint64_t* o3 = (uint64_t*)malloc(8 * (n + 1));
    void* cols[NF] = {c0, s1, c2, s3, c4};
    uint64_t* offs[NF] = {NULL, o1, NULL, o3, NULL};
    int rc = orc_unpack(kinds, NF, prefix, plen, w, len, n, cols, offs, consumed, err);
    free(w); free(c0); free(c2); free(c4); free(s1); free(s3); free(o1); free(o3);
    return rc;
}

int main(void) {
    /* a valid stream: N records, strings of 0..N-1 and (3 i) % 17 bytes */
    int8_t a[N]; int64_t b[N]; int16_t c[N];
    uint64_t o1[N + 1], o3[N + 1];
    uint8_t chars1[4096], chars3[4096];
    o1[0] = o3[0] = 0;
    for (int i = 0; i < N; ++i) {
        a[i] = (int8_t)(i * 7); b[i] = (int64_t)i * -123456789; c[i] = (int16_t)(i * 311);
        o1[i + 1] = o1[i] + (uint64_t)i;
        o3[i + 1] = o3[i] + (uint64_t)((3 * i) % 17);
    }
    for (int i = 0; i < 4096; ++i) { chars1[i] = (uint8_t)(i * 13); chars3[i] = (uint8_t)(255 - i); }
    uint8_t prefix[64];
    uint64_t plen = orc_request_prefix("Svc_servicer::m", "Msg", prefix);
    const void* cols[NF] = {a, chars1, b, chars3, c};
    const uint64_t* offs[NF] = {NULL, o1, NULL, o3, NULL};
    static uint8_t wire[65536];
    uint64_t len = orc_pack(kinds, NF, prefix, plen, cols, offs, N, wire, sizeof wire);
    CHECK(len != UINT64_MAX && len > 0);
    /* record starts, to know which record a cut falls in */
    uint64_t start[N + 1];
    start[0] = 0;
    for (int i = 0; i < N; ++i) start[i + 1] = start[i] + plen + 1 + 8 + (o1[i + 1] - o1[i]) + 8 + 8 + (o3[i + 1] - o3[i]) + 2;
    CHECK(start[N] == len);

    uint64_t consumed = 0, err = 0;
    CHECK(unpack_copy(wire, len, N, prefix, plen, &consumed, &err) == ORC_OK && consumed == len && err == N);
    /* 1. every truncation */
    for (uint64_t cut = 0; cut < len; ++cut) {
        int rc = unpack_copy(wire, cut, N, prefix, plen, &consumed, &err);
        uint64_t r = 0;
        while (start[r + 1] <= cut) ++r;  /* the record the cut falls in */
        if (!(rc == ORC_ERR_BOUNDS && err == r && consumed <= cut)) {
            CHECK(0);
            fprintf(stderr, "  cut %llu: rc %d err %llu (record %llu)\n", (unsigned long long)cut, rc,
                    (unsigned long long)err, (unsigned long long)r);
            break;
        }
    }
    ++passes;
    /* 2. oversized string lengths in record 7's first string */
    const uint64_t bigs[] = {0, UINT64_C(1) << 31, UINT64_C(1) << 63, UINT64_MAX};
    for (int k = 0; k < 4; ++k) {
        static uint8_t w2[65536];
        memcpy(w2, wire, len);
        uint64_t at = start[7] + plen + 1;
        uint64_t v = k == 0 ? len - (at + 8) + 1 : bigs[k];
        memcpy(w2 + at, &v, 8);
        CHECK(unpack_copy(w2, len, N, prefix, plen, &consumed, &err) == ORC_ERR_BOUNDS && err == 7);
    }
    /* 3. a prefix that differs in record 11 */
    {
        static uint8_t w3[65536];
        memcpy(w3, wire, len);
        w3[start[11] + 9] ^= 0x20;
        CHECK(unpack_copy(w3, len, N, prefix, plen, &consumed, &err) == ORC_ERR_PREFIX && err == 11 &&
              consumed == start[11]);
    }
    /* 4. more records than the stream holds */
    CHECK(unpack_copy(wire, len, N + 5, prefix, plen, &consumed, &err) == ORC_ERR_BOUNDS && err == N);
    /* 5. pack into too small a buffer at every capacity */
    for (uint64_t cap = 0; cap < len; cap += 7) {
        uint8_t* out = (uint8_t*)malloc(cap ? cap : 1);
        uint64_t got = orc_pack(kinds, NF, prefix, plen, cols, offs, N, out, cap);
        free(out);
        if (got != UINT64_MAX) { CHECK(0); break; }
    }
    ++passes;
    printf("%d passed, %d failed\n", passes, fails);
    return fails ? 1 : 0;
}
