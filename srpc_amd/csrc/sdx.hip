// sdx.hip -- srpc_gpu_unpack_var_stream: decode a concatenated record stream
// with NO record index, in three phases with no device-side waiting.
//
// The reference decodes a batch with ONE shared cursor (buffer::_offset,
// core.hpp:28-39): every pipe_output advances it (packer.hpp:210-222; nested
// unpack sharing the buffer as in tests/packer_test.cpp:77-88), so where a
// record starts is known only once every record before it was read.  Here:
//
// 1. k_sx_spec, a workgroup per 8 KiB block of the wire (+ a 1.5 KiB margin),
//    staged in LDS by LDS-DMA.  A lane per 32-byte chunk speculates the
//    chunk's first record start (a filter over its 32 positions from register
//    windows of the stage, then whole records must parse; of the plausible
//    starts within a length field's 8 bytes the one with the smallest first
//    string length) and walks the records starting in the chunk.  Chunks
//    whose start is their predecessor's exit form segments (scans give any
//    segment suffix in O(1)).  Then the block's TABLE: for every plausible
//    position of its first 64 bytes (else the first speculated start), the
//    chain of records from it to the block end -- exit, records, chars per
//    string field, stop -- a transfer function from "where the cursor enters"
//    to "where it leaves".  The speculated start of every chunk goes to
//    scratch (one byte) for phase 3.  The wire is read once here.
// 2. the scan of those tables, three small launches:
//    k_sx_groups  a wave per group of 64 blocks: the group's own table, one
//                 chain per slot of its first block through its 64 blocks;
//    k_sx_top     one wave: the groups in order (a group's table entry for the
//                 cursor's position, held in registers 64 groups at a time),
//                 every group's entry state; the stream's end: record T where
//                 it stopped, the status (first bad record, PREFIX / BOUNDS);
//    k_sx_blocks  a wave per group: every block's entry state (position,
//                 records before it, chars before it per string field).
//    A position found in no table (a "miss": the cursor enters a block where
//    the block did not speculate) is walked record by record from global
//    memory right there, so the scan is exact on any input and its work is
//    bounded by the records of the blocks it walks.
// 3. k_sx_decode, a workgroup per block: the block again (its speculated
//    chunk starts from scratch, the chunks walked again from LDS), the chain
//    from the block's exact entry (whole segments jumped), and the block's
//    records written: rec_offs, fixed columns, str_offs, and the chars (a
//    lane per record, straight from the stage: aligned 16-byte stores between
//    byte / dword edges; a string of 8 KiB or more by the whole block).  Each block's output bases come
//    from phase 2: no look-back, no wait.
//
// Error semantics are orc_unpack's (oracle/packer_oracle.c): the first record
// that does not parse stops the stream; it is reported (PREFIX or BOUNDS) as
// the first bad record, every later record BOUNDS; rec_offs[T] = where the
// stream stopped, rec_offs[T + 1 .. n] = wire_len.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdint>
#include <cstring>

#include "plan.h"
#include "srpc_gpu.h"

namespace srpc_impl {
namespace {

constexpr uint32_t kSB = 8192;                   // wire bytes per block (one workgroup)
constexpr uint32_t kSC = kSB / kBlock;           // 32: wire bytes per speculating lane
static_assert(kSC % 16 == 0 && kSC <= 64, "16-byte window reads; a chunk's positions fit one 64-bit mask");
constexpr uint32_t kMargin = 1536;               // staged bytes past the block
// Landing slots (round 5): the table also holds a slot at the end of every
// record that starts in the kPre bytes before the block (its premargin) and
// ends in the block past the window -- the true entry of a record that
// straddles the block's start by up to kPre bytes, whatever the speculation
// made of the block.  Wave 1 finds them alone (land_slots), from the
// premargin staged with the block, while wave 0 builds the window table (no
// barrier, nothing read from global memory; a whole-workgroup scan with
// barriers cost every random row 25-30 %, a wave-0 scan after the table
// 10-28 %, this one 2-9 %: profiles/r05_sdx_ab.log).  A/B build
// SRPC_SX_NOLAND leaves them out.
#ifndef SRPC_SX_NOLAND
constexpr uint32_t kPre = 1024;                  // premargin: bytes before the block scanned for landings
#else
constexpr uint32_t kPre = 0;
#endif
constexpr uint32_t kStage = kSB + kMargin + 32;  // + 16-byte alignment slack on both sides
constexpr uint32_t kStageS = kPre + kStage;      // phase 1's stage: the premargin, the block, the margin
constexpr uint32_t kWin = 64;                    // entry window of a block's table (a lane per position)
#ifndef SRPC_SX_NOLAND
constexpr uint32_t kX = 128;                     // landing slots per block
#else
constexpr uint32_t kX = 0;
#endif
// Exit slots (round 6, the repair pass): the live exits of every chain from
// every position of the block before (and from longer records of blocks
// further back), so the cursor's entry into a block is always a slot -- see
// k_sx_repair.
constexpr uint32_t kE = 255;                     // exit slots per block (header word 5 counts them in 8 bits)
constexpr uint32_t kXS = kX + kE;                // a wave's LDS copy of a block's landing + exit slots
constexpr uint32_t kEnt = kWin + 1 + kX + kE;    // table entries per block: the window's, the extra slot,
                                                 // the landing slots, then the exit slots
constexpr uint32_t kHdr = 8;                     // header words per block
constexpr uint32_t kRepairMin = 16;              // segments past which k_sx_spec repairs its chunks
constexpr uint32_t kRepairMax = 16;              // repair passes at most
constexpr uint32_t kGroup = 64;                  // blocks per group of the scan (a lane per block)
constexpr int kMaxNC = 3;                        // chars values carried per state (string fields 0..ns-2)
constexpr uint32_t kMaxRec = kSB / 8;            // records starting in a block (each >= 8 bytes)
constexpr uint32_t kHugeLog2 = 13;               // strings from 8 KiB: copied by the whole block
constexpr uint16_t kFar = 0xFFFF;
constexpr uint32_t kWaveCopyAvg = 128;  // chars per record from which the decode copies a wave per record
constexpr uint32_t kFarList = 32;       // records of a block whose chars the decode copies from global memory
constexpr uint32_t kPlausPrefixed = 1, kPlausBare = 2;
constexpr uint16_t kNoStart = 0xFFFF;
constexpr uint8_t kNoSpec = 0xFF;
constexpr int kKeep = 4;                         // table entries per block the scans hold in registers
constexpr uint64_t kCnt40 = (1ull << 40) - 1;
constexpr uint32_t kNoPrim = 0xFF;
constexpr uint32_t kListCap = 4;                 // record starts a 32-byte chunk holds (records >= 8 bytes apart)
static_assert(kSB / 32 == kBlock && kListCap == 4, "a wave's part of the chunk lists holds 128 u16 landing slots");
constexpr uint32_t kDead = 0x81;                 // stop bits of a group-table chain given up (k_sx_groups)

// control words (scratch; k_sx_spec block 0 zeroes them each call)
constexpr uint32_t kCtlMiss = 0;     // entries found in no table (walked from global memory)
constexpr uint32_t kCtlOff = 1;      // entries that were not a block's primary slot
constexpr uint32_t kCtlTailOn = 2;   // the stream stopped before record n: the tail fill runs
constexpr uint32_t kCtlT = 3;        // ... from record T
constexpr uint32_t kCtlTot = 4;      // ... str_offs value per string ordinal (kMaxNC + 1 words)
constexpr uint32_t kCtlRepair = 8;   // the first scan met a position no table holds: repair, scan again
constexpr uint32_t kCtlOver = 9;     // blocks whose exit slots overflowed (diagnostics)
constexpr uint32_t kCtlDone = 10;    // k_sx_groups workgroups done, per pass (2 words): the last runs the scan
constexpr uint32_t kCtlWords = 16;

// stop bits: bit 0 = the chain stopped, bits 1-2 = why (SRPC_STATUS_PREFIX / _BOUNDS)

// Per-phase clock (A/B diagnostics, compiled only with -DSRPC_SX_PHASES):
// thread 0 of every block of k_sx_spec (words 0-7) and k_sx_decode (words
// 8-15) adds the clock64() cycles between its phase marks into 16 words of
// its own; srpc_debug_sx_phases points them at a caller's buffer.
#ifdef SRPC_SX_PHASES
__device__ unsigned long long* g_sxph = nullptr;
__device__ unsigned long long g_sxph_blocks = 0;
#define SXP_BEGIN uint64_t sxp_last_ = clock64();
#define SXP(i)                                                                                     \
    do {                                                                                           \
        if (threadIdx.x == 0 && blockIdx.x < g_sxph_blocks) {                                      \
            const uint64_t now_ = clock64();                                                       \
            g_sxph[static_cast<uint64_t>(blockIdx.x) * 16 + (i)] += now_ - sxp_last_;              \
            sxp_last_ = now_;                                                                      \
        }                                                                                          \
    } while (0)
#define SXP_FLAG(i)                                                                                \
    do {                                                                                           \
        if (threadIdx.x == 0 && blockIdx.x < g_sxph_blocks) g_sxph[static_cast<uint64_t>(blockIdx.x) * 16 + (i)] = 1; \
    } while (0)
#define SXP_SET(i, v)                                                                              \
    do {                                                                                           \
        if (blockIdx.x < g_sxph_blocks) g_sxph[static_cast<uint64_t>(blockIdx.x) * 16 + (i)] = (v);    \
    } while (0)
#define SXP_ADD(i, v)                                                                              \
    do {                                                                                           \
        if (blockIdx.x < g_sxph_blocks) atomicAdd(g_sxph + static_cast<uint64_t>(blockIdx.x) * 16 + (i), \
                                                  static_cast<unsigned long long>(v));              \
    } while (0)
#else
#define SXP_BEGIN
#define SXP(i)
#define SXP_FLAG(i)
#define SXP_SET(i, v)
#define SXP_ADD(i, v)
#endif

typedef const uint8_t __attribute__((address_space(1))) global_u8;
typedef uint8_t __attribute__((address_space(3))) lds_u8;
typedef const uint8_t __attribute__((address_space(3))) lds_u8c;
typedef const uint32_t __attribute__((address_space(3))) lds_u32c;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct SxArgs {
    uint32_t size[kMaxFields];   // fixed field bytes, 0 = string
    uint32_t sord[kMaxFields];   // string ordinal of a string field
    uint8_t* col[kMaxFields];    // fixed: column; string: chars
    uint64_t* soff[kMaxFields];  // string: n + 1 chars offsets
    const uint8_t* prefix;       // device copy (16 zero bytes past the end)
    uint64_t* rec_offs;
    uint64_t n, W;
    uint64_t pre8;               // the prefix's first 8 bytes (zero padded)
    uint32_t nfields, nstrings, prefix_len, fixed_bytes;
    uint32_t first_len_at;       // byte offset of the first string's u64 length in a record
    uint32_t plaus;              // records that must parse from a candidate
    uint32_t cap;                // record starts a chunk can hold: 1 + kSC / fixed_bytes
    uint32_t nb, ng;             // blocks, groups
    uint32_t gap[kMaxFields + 1];  // fixed bytes before string ordinal 0 (prefix included), between
                                   // strings k - 1 and k, after the last string (the parse's program)
    uint32_t mode;               // test hooks: 1 = tables hold only the first speculated start, 2 = empty
                                 // tables, 4 = the exact filter at every position (A/B), 8 = no repair
                                 // pass (a position no table holds is walked, as before round 6)
};

struct SxScratch {
    uint8_t* spec;   // per chunk: its speculated start minus its first byte, or kNoSpec
    uint64_t* hdr;   // per block: window mask, first speculated start, slots | primary << 8, 0
    uint64_t* ent;   // per block, per slot (compact, window order): the chain's E words
    uint64_t* gent;  // per group, per slot of its first block: the chain to the group's end
    uint64_t* gp;    // per group: its first block's header words 0-2, then its primary slot's gent entry
    uint64_t* gin;   // per group: the cursor's state where the group starts (E words)
    uint64_t* bst;   // per block: the cursor's state where the block starts (E words)
    uint64_t* ctl;   // kCtlWords
    uint16_t* rl;    // per block, kMaxRec slots: its chunks' record starts in order (offsets from the block)
    uint16_t* xp;    // per block, kX slots: its landing slots' positions (offsets from the block, ascending)
    uint16_t* ep;    // per block, kE slots: its exit slots' positions (offsets from the block, ascending)
};

// A chain's result / the cursor's state: position (exit, or the next record
// start), records, chars of string fields 0..NC-1, stop bits.  Stored as
// E = 2 + NC words: x, cnt | stop << 40, chars.
template <int NC>
struct St {
    uint64_t x, cnt;
    uint64_t ch[kMaxNC + 1];
    uint32_t stop;
};
template <int NC>
constexpr uint32_t ew() { return 2 + NC; }

template <int NC>
__device__ __forceinline__ void st_store(uint64_t* p, const St<NC>& s) {
    p[0] = s.x;
    p[1] = (s.cnt & kCnt40) | (static_cast<uint64_t>(s.stop) << 40);
#pragma unroll
    for (int k = 0; k < NC; ++k) p[2 + k] = s.ch[k];
}
template <int NC>
__device__ __forceinline__ St<NC> st_load(const uint64_t* p) {
    St<NC> s{};
    s.x = p[0];
    const uint64_t c = p[1];
    s.cnt = c & kCnt40;
    s.stop = static_cast<uint32_t>(c >> 40);
#pragma unroll
    for (int k = 0; k < NC; ++k) s.ch[k] = p[2 + k];
    return s;
}
// the cursor moves through a block along one of its chains
template <int NC>
__device__ __forceinline__ void st_add(St<NC>& s, const St<NC>& e) {
    s.x = e.x;
    s.cnt += e.cnt;
#pragma unroll
    for (int k = 0; k < NC; ++k) s.ch[k] += e.ch[k];
    s.stop = e.stop;
}
// nothing after this state counts: a record failed, or the wire ended
template <int NC>
__device__ __forceinline__ bool st_done(const St<NC>& s, uint64_t W) {
    return (s.stop & 1) || s.x >= W;
}

__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), l);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), l);
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// ---- wire readers --------------------------------------------------------------
struct GlobalRd {
    const uint8_t* w;
    const uint8_t* pre;  // the prefix (device copy)
    __device__ __forceinline__ uint64_t u64(uint64_t p) const {
        uint64_t v;
        __builtin_memcpy(&v, w + p, 8);
        return v;
    }
    __device__ __forceinline__ uint8_t u8(uint64_t p) const { return w[p]; }
    __device__ __forceinline__ uint64_t pre64(uint32_t i) const {
        uint64_t v;
        __builtin_memcpy(&v, pre + i, 8);
        return v;
    }
    __device__ __forceinline__ uint8_t pre8(uint32_t i) const { return pre[i]; }
};
// A workgroup's LDS copy of wire bytes [lo, hi) (lds[x] = byte base + x), global
// memory past it (records that run past the margin).
struct StagedRd {
    global_u8* w;
    lds_u8c* lds;
    uint64_t base, lo, hi;
    lds_u8c* pre;  // LDS copy of the prefix, 16-aligned
    __device__ __forceinline__ uint64_t u64(uint64_t p) const {
        if (p >= lo && p + 8 <= hi) return u64_lds(p);
        uint64_t v;
        __builtin_memcpy(&v, (const uint8_t*)(w + p), 8);
        return v;
    }
    __device__ __forceinline__ uint8_t u8(uint64_t p) const { return p >= lo && p < hi ? lds[p - base] : w[p]; }
    // the sz (1, 2, 4, 8) bytes of a fixed field at p, never a byte past them in global memory
    __device__ __forceinline__ uint64_t field(uint64_t p, uint32_t sz) const {
        if (p >= lo && p + sz <= hi) return u64_lds(p);  // the LDS stage has slack past hi
        switch (sz) {
        case 1: return w[p];
        case 2: { uint16_t v; __builtin_memcpy(&v, (const uint8_t*)(w + p), 2); return v; }
        case 4: { uint32_t v; __builtin_memcpy(&v, (const uint8_t*)(w + p), 4); return v; }
        default: { uint64_t v; __builtin_memcpy(&v, (const uint8_t*)(w + p), 8); return v; }
        }
    }
    __device__ __forceinline__ uint64_t u64_lds(uint64_t p) const {
        const uint32_t off = static_cast<uint32_t>(p - base);
        lds_u32c* q = reinterpret_cast<lds_u32c*>(lds + (off & ~3u));
        const uint32_t sh = off & 3, w0 = q[0], w1 = q[1], w2 = q[2];
        return (static_cast<uint64_t>(__builtin_amdgcn_alignbyte(w2, w1, sh)) << 32) |
               __builtin_amdgcn_alignbyte(w1, w0, sh);
    }
    __device__ __forceinline__ uint64_t pre64(uint32_t i) const {
        lds_u32c* q = reinterpret_cast<lds_u32c*>(pre + i);
        return (static_cast<uint64_t>(q[1]) << 32) | q[0];
    }
    __device__ __forceinline__ uint8_t pre8(uint32_t i) const { return pre[i]; }
    __device__ __forceinline__ bool staged(uint64_t p, uint64_t e) const { return p >= lo && e <= hi && p <= e; }
};
// The staged bytes only, for speculation: a read past them yields ~0 (no
// length fits, no prefix matches), so a candidate whose records run past the
// stage is not plausible -- a start one byte early whose length reads as
// len * 256 + a char would otherwise send lanes to global memory.
struct StageOnlyRd {
    StagedRd s;
    __device__ __forceinline__ uint64_t u64(uint64_t p) const { return p >= s.lo && p + 8 <= s.hi ? s.u64_lds(p) : ~0ull; }
    __device__ __forceinline__ uint8_t u8(uint64_t p) const {
        return p >= s.lo && p < s.hi ? s.lds[p - s.base] : static_cast<uint8_t>(~s.pre[0]);
    }
    __device__ __forceinline__ uint64_t pre64(uint32_t i) const { return s.pre64(i); }
    __device__ __forceinline__ uint8_t pre8(uint32_t i) const { return s.pre8(i); }
};

// orc_unpack's cursor over one record at p: the position after it, or p with
// *err set (SRPC_STATUS_PREFIX / _BOUNDS); chars of string fields 0..NC-1
// added to ch[].  Every loop runs a uniform number of times with the error
// as a predicate (no early exit): its counter stays wave-uniform, so the
// schema words it indexes (a.gap[k]) are scalar loads -- an index made
// divergent by an early return turns each of them into a vector load from
// the kernel-argument segment, a memory round trip per field per parse.
template <int NC, class Rd>
__device__ __forceinline__ uint64_t parse_rd(const SxArgs& a, const Rd& r, uint64_t p, uint32_t* err,
                                             uint64_t (&ch)[kMaxNC + 1]) {
    const uint64_t W = a.W;
    uint32_t e = 0;
    if (a.prefix_len) {
        if (a.prefix_len > W - p) {
            e = SRPC_STATUS_BOUNDS;
        } else {
            uint64_t diff = 0;
            uint32_t i = 0;
            for (; i + 8 <= a.prefix_len; i += 8) diff |= r.u64(p + i) ^ r.pre64(i);
            for (; i < a.prefix_len; ++i) diff |= r.u8(p + i) ^ r.pre8(i);
            if (diff) e = SRPC_STATUS_PREFIX;
        }
    }
    // the fields as a program of runs: fixed bytes, then a string, ..., then
    // the fixed bytes after the last string (a read past the wire anywhere in
    // a run is the same BOUNDS error the field-by-field cursor meets there)
    uint64_t q = p;
    uint64_t add[kMaxNC + 1] = {};
    for (uint32_t k = 0; k < a.nstrings; ++k) {
        const uint32_t g = a.gap[k] + 8;  // the fixed run and the string's u64 length
        if (!e) {
            if (g > W - q) {
                e = SRPC_STATUS_BOUNDS;
            } else {
                q += g;
                const uint64_t len = r.u64(q - 8);
                if (len > W - q) {
                    e = SRPC_STATUS_BOUNDS;
                } else {
                    q += len;
#pragma unroll
                    for (int j = 0; j < NC; ++j) add[j] += k == static_cast<uint32_t>(j) ? len : 0;
                }
            }
        }
    }
    const uint32_t gl = a.gap[a.nstrings];
    if (!e && gl > W - q) e = SRPC_STATUS_BOUNDS;
    *err = e;
    if (e) return p;
    q += gl;
#pragma unroll
    for (int j = 0; j < NC; ++j) ch[j] += add[j];
    return q;
}

// Necessary for a record to parse at p: the prefix's first (up to 8) bytes
// match and the first string's length fits the wire.
template <class Rd>
__device__ __forceinline__ bool filter(const SxArgs& a, const Rd& r, uint64_t p) {
    const uint64_t W = a.W;
    if (p > W || a.first_len_at + 8 > W - p) return false;
    if (a.prefix_len) {
        const uint32_t k = a.prefix_len < 8 ? a.prefix_len : 8;
        const uint64_t mask = k == 8 ? ~0ull : (1ull << (8 * k)) - 1;
        uint64_t v = 0;
        if (8 <= W - p) v = r.u64(p);
        else
            for (uint32_t i = 0; i < k; ++i) v |= static_cast<uint64_t>(r.u8(p + i)) << (8 * i);
        if (((v ^ a.pre8) & mask) != 0) return false;
    }
    return r.u64(p + a.first_len_at) <= W - (p + a.first_len_at + 8);
}

template <class Rd>
__device__ __forceinline__ bool plausible(const SxArgs& a, const Rd& r, uint64_t p) {
    uint64_t ch[kMaxNC + 1];
    for (uint32_t k = 0; k < a.plaus; ++k) {
        if (p == a.W) return k > 0;  // the stream may end right after a record
        uint32_t err;
        const uint64_t q = parse_rd<0>(a, r, p, &err, ch);
        if (err) return false;
        p = q;
    }
    return true;
}

// The N dwords at LDS byte offset o & ~3 of the stage, in 16-byte reads (o
// mod 16 is the same for every lane: chunks are a multiple of 16 bytes
// apart, so the dword shift is a uniform switch).
template <int N>
__device__ __forceinline__ void lds_window(const uint8_t* st, uint32_t o, uint32_t (&d)[N]) {
    constexpr int NQ = (N + 3 + 3) / 4;
    uint32_t w[4 * NQ];
    typedef const u32x4 __attribute__((address_space(3))) lds_u32x4c;
    lds_u32x4c* q = reinterpret_cast<lds_u32x4c*>((lds_u8c*)st + (o & ~15u));
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const u32x4 v = q[i];
        w[4 * i] = v.x;
        w[4 * i + 1] = v.y;
        w[4 * i + 2] = v.z;
        w[4 * i + 3] = v.w;
    }
    switch (__builtin_amdgcn_readfirstlane((o >> 2) & 3)) {
    case 0:
#pragma unroll
        for (int k = 0; k < N; ++k) d[k] = w[k];
        break;
    case 1:
#pragma unroll
        for (int k = 0; k < N; ++k) d[k] = w[k + 1];
        break;
    case 2:
#pragma unroll
        for (int k = 0; k < N; ++k) d[k] = w[k + 2];
        break;
    default:
#pragma unroll
        for (int k = 0; k < N; ++k) d[k] = w[k + 3];
        break;
    }
}

// Positions of a chunk (LDS offset `at`, wire offset clo, up to chi) that pass
// the filter, as a mask: the first string's length at p + first_len_at fits
// the wire, the prefix's first 8 bytes match -- all positions at once from
// register windows of the stage.
__device__ __forceinline__ uint64_t chunk_mask(const SxArgs& a, const uint8_t* st, uint32_t at, uint64_t clo,
                                               uint64_t chi) {
    const uint64_t W = a.W;
    uint64_t mask = 0;
    {
        uint32_t d[kSC / 4 + 3];
        const uint32_t o = at + a.first_len_at, sh = o & 3;
        lds_window(st, o, d);
#pragma unroll
        for (int k = 0; k < static_cast<int>(kSC / 4 + 2); ++k) d[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        // position j passes when len + j <= lim0 = W - (clo + first_len_at + 8)
        // (a wrapped sum only adds a candidate: the filter stays necessary)
        const uint64_t need = clo + a.first_len_at + 8;
        const uint64_t lim0 = need <= W ? W - need : 0;
#pragma unroll
        for (int j = 0; j < static_cast<int>(kSC); ++j) {
            const int k = j >> 2, s8 = j & 3;
            const uint32_t lo32 = s8 ? __builtin_amdgcn_alignbyte(d[k + 1], d[k], s8) : d[k];
            const uint32_t hi32 = s8 ? __builtin_amdgcn_alignbyte(d[k + 2], d[k + 1], s8) : d[k + 1];
            const uint64_t len = (static_cast<uint64_t>(hi32) << 32) | lo32;
            mask |= static_cast<uint64_t>(len + j <= lim0) << j;
        }
        // positions inside the chunk whose length field lies inside the wire
        const uint64_t jmax = need <= W ? min<uint64_t>(chi - clo, W - need + 1) : 0;
        mask &= jmax >= 64 ? ~0ull : (1ull << jmax) - 1;
    }
    if (a.prefix_len && mask) {
        uint32_t d[kSC / 4 + 3];
        const uint32_t sh = at & 3;
        lds_window(st, at, d);
#pragma unroll
        for (int k = 0; k < static_cast<int>(kSC / 4 + 2); ++k) d[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        const uint32_t k8 = a.prefix_len < 8 ? a.prefix_len : 8;
        const uint64_t pm = k8 == 8 ? ~0ull : (1ull << (8 * k8)) - 1;
        uint64_t keep = 0;
#pragma unroll
        for (int j = 0; j < static_cast<int>(kSC); ++j) {
            const int k = j >> 2, s8 = j & 3;
            const uint32_t lo32 = s8 ? __builtin_amdgcn_alignbyte(d[k + 1], d[k], s8) : d[k];
            const uint32_t hi32 = s8 ? __builtin_amdgcn_alignbyte(d[k + 2], d[k + 1], s8) : d[k + 1];
            const uint64_t v = (static_cast<uint64_t>(hi32) << 32) | lo32;
            keep |= static_cast<uint64_t>(((v ^ a.pre8) & pm) == 0) << j;
        }
        mask &= keep;
    }
    return mask;
}

// chunk_mask for wires under 4 GiB: a length that fits has its four high
// bytes zero, so only positions whose length field has them zero are
// candidates (a zero-byte mask of the window: ~5 VALU per dword instead of ~8
// per position), and each candidate is then tested exactly (its length, the
// prefix's first 8 bytes) from LDS.  The same mask as chunk_mask.
__device__ __forceinline__ uint64_t chunk_mask_z(const SxArgs& a, const uint8_t* st, uint32_t at, uint64_t clo,
                                                 uint64_t chi, uint32_t* pick) {
    const uint64_t W = a.W;
    const uint64_t need = clo + a.first_len_at + 8;
    *pick = ~0u;
    if (need > W) return 0;
    const uint64_t lim0 = W - need;
    const uint64_t jmax = min<uint64_t>(chi - clo, W - need + 1);
    uint32_t d[kSC / 4 + 3];
    const uint32_t o = at + a.first_len_at, sh = o & 3;
    lds_window(st, o, d);
    // z bit i: byte i of the window (wire offset clo + first_len_at + i) is zero
    uint64_t z = 0;
#pragma unroll
    for (int k = 0; k < static_cast<int>(kSC / 4 + 2); ++k) {
        const uint32_t v = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
        const uint32_t nz = ((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v;  // bit 7 of each nonzero byte
        const uint32_t zb = (~nz >> 7) & 0x01010101u;              // bit 0 of each zero byte
        z |= static_cast<uint64_t>(((zb * 0x00204081u) >> 21) & 0xFu) << (4 * k);
    }
    uint64_t cand = (z >> 4) & (z >> 5) & (z >> 6) & (z >> 7);  // bytes 4..7 of the length at j
    cand &= jmax >= 64 ? ~0ull : (1ull << jmax) - 1;
    uint64_t mask = 0;
    const uint32_t k8 = a.prefix_len < 8 ? a.prefix_len : 8;
    const uint64_t pm = k8 == 8 ? ~0ull : (1ull << (8 * k8)) - 1;
    const lds_u8c* sl = (lds_u8c*)st;
    auto u64_at = [&](uint32_t off) -> uint64_t {
        lds_u32c* q = reinterpret_cast<lds_u32c*>(sl + (off & ~3u));
        const uint32_t s3 = off & 3, w0 = q[0], w1 = q[1], w2 = q[2];
        return (static_cast<uint64_t>(__builtin_amdgcn_alignbyte(w2, w1, s3)) << 32) |
               __builtin_amdgcn_alignbyte(w1, w0, s3);
    };
    uint32_t j0 = ~0u;
    uint64_t best = ~0ull;
    while (cand) {
        const uint32_t j = __builtin_ctzll(cand);
        cand &= cand - 1;
        const uint64_t len = u64_at(o + j);
        if (len + j > lim0) continue;
        if (a.prefix_len && ((u64_at(at + j) ^ a.pre8) & pm)) continue;
        mask |= 1ull << j;
        // the first cluster's pick (k_sx_spec): of the passing positions
        // within 8 bytes of the first, the smallest first string length
        if (j0 == ~0u) j0 = j;
        if (j < j0 + 8 && len < best) {
            best = len;
            *pick = j;
        }
    }
    return mask;
}

// Exclusive scan of one value per thread over the workgroup (*total = sum).
__device__ __forceinline__ uint64_t block_xscan(uint64_t x, uint64_t* total, uint64_t* ws) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        before += w < wave ? ws[w] : 0;
        all += ws[w];
    }
    __syncthreads();
    *total = all;
    return before + inc - x;
}

// First set bit at index >= i of a 256-bit mask (4 words in LDS), or 256.
__device__ __forceinline__ uint32_t next_bit(const uint64_t* m, uint32_t i) {
    if (i >= 256) return 256;
    uint32_t w = i >> 6;
    uint64_t v = m[w] & (~0ull << (i & 63));
    while (!v && ++w < 4) v = m[w];
    return w < 4 ? 64 * w + __builtin_ctzll(v) : 256;
}

// Last set bit at index <= i of a 256-bit mask (4 words in LDS), or 256.
__device__ __forceinline__ uint32_t prev_bit(const uint64_t* m, uint32_t i) {
    int w = static_cast<int>(i >> 6);
    uint64_t v = m[w] & ((i & 63) == 63 ? ~0ull : ((2ull << (i & 63)) - 1));
    while (!v && --w >= 0) v = m[w];
    return w >= 0 ? 64 * w + 63 - __builtin_clzll(v) : 256;
}

// A block's chunks in LDS (both the speculation and the decode keep them):
// per chunk its first start (offset from the block, or none), the position
// after its records, stop bits, the exclusive scans of records and chars, and
// 256-bit masks: chunks with a start, segment tails, chunks a chain jumped.
template <int NC>
struct ChunkChars {
    uint64_t pch[NC][kBlock + 1];
};
template <>
struct ChunkChars<0> {  // no chars scans (never indexed: loops over k < NC)
    uint64_t pch[1][1];
};
template <int NC>
struct Chunks : ChunkChars<NC> {
    uint64_t exit[kBlock];
    uint32_t pcnt[kBlock + 1];
    uint16_t start[kBlock];
    uint8_t stop[kBlock];
    uint64_t has[4], tail[4], jump[4];
    uint64_t ws[kBlock / 64];
};

// The zero map of a zero-heavy block (round 6; built only where k_sx_spec
// repaired the speculation, header word 2 bit 17): bit j = bytes [b0 + 32 j,
// b0 + 32 j + 32) hold a nonzero byte or lie past the stage.  A chain that
// meets a run of zero bytes off the speculation crosses it in one step: with
// no prefix, a record of Z = fixed_bytes zero bytes (every string empty)
// parses at every position of the run, so from q the next k = (run end - q) / Z
// records are zero records (no chars) -- the round-5 walk parsed them one by
// one (all-zero multiple_primitives 6.5x its random row).  Random blocks never
// build or read it: their chains take walk_chain<..., ZM = false>.
constexpr uint32_t kZC = (kSB + kMargin) / 32;  // chunks the map covers
constexpr uint32_t kZW = (kZC + 63) / 64;       // its words
// Every thread of the workgroup takes part; a barrier at the end.
__device__ __forceinline__ void build_zmap(const StagedRd& rd, uint64_t b0, uint64_t* zm) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    for (uint32_t j0 = tid & ~63u; j0 < kZW * 64; j0 += kBlock) {
        const uint32_t j = j0 + lane;
        const uint64_t lo = b0 + 32ull * j;
        bool nz = true;
        if (j < kZC && lo >= rd.lo && lo + 32 <= rd.hi) {
            lds_u32c* q = reinterpret_cast<lds_u32c*>(rd.lds + (lo - rd.base));  // (b0 - base: a multiple of 16)
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) v |= q[k];
            nz = v != 0;
        }
        const uint64_t m = __ballot(nz);
        if (lane == 0) zm[j0 >> 6] = m;
    }
    __syncthreads();
}
// A bit per byte of the 32 bytes at cl (a chunk of the map): the byte is
// nonzero, or lies past the stage (8 aligned dword reads).
template <class Rd>
__device__ __forceinline__ uint32_t chunk_nz(const Rd& rd, uint64_t cl) {
    if (cl < rd.lo || cl + 32 > rd.hi) return ~0u;
    lds_u32c* q = reinterpret_cast<lds_u32c*>(rd.lds + (cl - rd.base));  // (16-aligned: b0 - base is)
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t d = q[k];
        // 0x80 in each byte of d that is nonzero
        const uint32_t h = (((d & 0x7f7f7f7fu) + 0x7f7f7f7fu) | d) & 0x80808080u;
        // bits 7, 15, 23, 31 -> bits 0..3 of this dword's nibble
        const uint32_t nib = ((h >> 7) & 1u) | ((h >> 14) & 2u) | ((h >> 21) & 4u) | ((h >> 28) & 8u);
        m |= nib << (4 * k);
    }
    return m;
}

// The first nonzero byte at or after q (q >= b0), or the end of what the map
// covers: bytes [q, result) are zero.
template <class Rd>
__device__ __forceinline__ uint64_t zero_run_end(const Rd& rd, const uint64_t* zm, uint64_t b0, uint64_t q) {
    uint32_t j = static_cast<uint32_t>((q - b0) >> 5);
    if (j >= kZC) return q;
    if ((zm[j >> 6] >> (j & 63)) & 1) {  // q's chunk: its nonzero bytes at or after q
        const uint32_t m = chunk_nz(rd, b0 + 32ull * j) & (~0u << ((q - b0) & 31));
        if (m) return b0 + 32ull * j + __builtin_ctz(m);
        ++j;
    }
    // the next chunk with a nonzero byte
    for (; j < kZC; j = (j | 63) + 1) {
        const uint64_t w = zm[j >> 6] >> (j & 63);
        if (w) {
            j += __builtin_ctzll(w);
            break;
        }
    }
    if (j >= kZC) return b0 + 32ull * kZC;
    const uint32_t m = chunk_nz(rd, b0 + 32ull * j);
    return b0 + 32ull * j + (m ? __builtin_ctz(m) : 32);
}

// The chain from x (x >= the block start): explicit records are parsed until
// the walk meets a speculated chunk start, whose segment is then taken whole
// from the scans (O(1)), and so on.  REC: the explicit starts go to xl (u16
// offsets from the block, ascending) and jumped chunks to the jump mask.
// ZM: runs of zero bytes crossed in one step (the zero map zm, above).
template <int NC, bool REC, bool ZM = false, class Rd>
__device__ St<NC> walk_chain(const SxArgs& a, const Rd& rd, Chunks<NC>& L, uint64_t b0, uint64_t b1, uint64_t x,
                             uint16_t* xl, uint32_t* nx, const uint64_t* zm = nullptr) {
    St<NC> g{};
    uint64_t q = x;
    uint32_t ne = 0;
    while (q < b1) {
        const uint32_t c = static_cast<uint32_t>((q - b0) / kSC);
        const uint16_t sc = L.start[c];
        if (sc != kNoStart && b0 + sc == q) {  // on a speculated segment: jump to its end
            const uint32_t e = next_bit(L.tail, c);  // the segment's last chunk (always a tail)
            g.cnt += L.pcnt[e + 1] - L.pcnt[c];
#pragma unroll
            for (int k = 0; k < NC; ++k) g.ch[k] += L.pch[k][e + 1] - L.pch[k][c];
            if (REC) {
                for (uint32_t j = c; j <= e;) {  // chunks c..e into the jump mask
                    const uint32_t wi = j >> 6, lo = j & 63, hi = min<uint32_t>(63, e - 64 * wi);
                    L.jump[wi] |= (hi == 63 ? ~0ull : ((2ull << hi) - 1)) & (~0ull << lo);
                    j = 64 * (wi + 1);
                }
            }
            q = L.exit[e];
            if (L.stop[e]) {
                g.stop = L.stop[e];
                break;
            }
            continue;
        }
        if constexpr (ZM) {
            const uint32_t Z = a.fixed_bytes;
            if (!a.prefix_len) {
                const uint64_t re = zero_run_end(rd, zm, b0, q);
                if (re >= q + Z && re <= a.W) {
                    // records q, q + Z, ... while they lie in the run, the last one
                    // the first to start at or past b1 at most
                    const uint64_t k = min<uint64_t>((re - q) / Z, (b1 - q + Z - 1) / Z);
                    if (REC)
                        for (uint64_t i = 0; i < k; ++i) xl[ne + i] = static_cast<uint16_t>(q + i * Z - b0);
                    ne += static_cast<uint32_t>(k);
                    g.cnt += k;
                    q += k * Z;
                    continue;
                }
            }
        }
        uint32_t err;
        const uint64_t q2 = parse_rd<NC>(a, rd, q, &err, g.ch);
        if (err) {
            g.stop = 1 | (err << 1);
            break;
        }
        if (REC) xl[ne] = static_cast<uint16_t>(q - b0);
        ++ne;
        ++g.cnt;
        q = q2;
    }
    g.x = q;
    if (REC) *nx = ne;
    return g;
}

// A wave's private LDS copy of a block (+ margin) for the scan's walks: the
// wire bytes [lo, hi) at stage offset (wire offset - base), the prefix read
// from global memory (it stays in the caches).
struct WaveRd {
    global_u8* w;
    lds_u8c* lds;
    uint64_t base, lo, hi;
    const uint8_t* pre;
    __device__ __forceinline__ uint64_t u64(uint64_t p) const {
        if (p >= lo && p + 8 <= hi) {
            const uint32_t off = static_cast<uint32_t>(p - base);
            lds_u32c* q = reinterpret_cast<lds_u32c*>(lds + (off & ~3u));
            const uint32_t sh = off & 3, w0 = q[0], w1 = q[1], w2 = q[2];
            return (static_cast<uint64_t>(__builtin_amdgcn_alignbyte(w2, w1, sh)) << 32) |
                   __builtin_amdgcn_alignbyte(w1, w0, sh);
        }
        uint64_t v;
        __builtin_memcpy(&v, (const uint8_t*)(w + p), 8);
        return v;
    }
    __device__ __forceinline__ uint8_t u8(uint64_t p) const { return p >= lo && p < hi ? lds[p - base] : w[p]; }
    __device__ __forceinline__ uint64_t pre64(uint32_t i) const {
        uint64_t v;
        __builtin_memcpy(&v, pre + i, 8);
        return v;
    }
    __device__ __forceinline__ uint8_t pre8(uint32_t i) const { return pre[i]; }
};
constexpr uint32_t kWaveStage = kSB + kMargin + 32;  // one block + margin, 16-byte aligned either side

// A wave's copy of block [b0, min(b1 + kMargin, W)) into its LDS stage
// (16-byte loads, all in flight at once); every lane of the wave takes part.
__device__ __forceinline__ WaveRd stage_wave(const SxArgs& a, const uint8_t* w, uint8_t* stage, uint64_t b0,
                                             uint64_t b1) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t hi = min<uint64_t>(b1 + kMargin, a.W);
    const uint64_t A = (reinterpret_cast<uint64_t>(w) + b0) & ~15ull;
    const uint32_t ng = static_cast<uint32_t>((reinterpret_cast<uint64_t>(w) + hi - A + 15) >> 4);
    constexpr uint32_t kPer = (kWaveStage / 16 + 63) / 64;
    u32x4 v[kPer];
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t gi = lane + 64 * k;
        if (gi < ng) v[k] = *reinterpret_cast<const u32x4*>(A + 16ull * gi);
    }
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k) {
        const uint32_t gi = lane + 64 * k;
        if (gi < ng) *reinterpret_cast<u32x4*>(stage + 16 * gi) = v[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // the wave's LDS writes before its reads
    return WaveRd{(global_u8*)w, (lds_u8c*)stage, A - reinterpret_cast<uint64_t>(w), b0, hi, a.prefix};
}

template <int NC>
__device__ St<NC> walk_global(const SxArgs& a, const uint8_t* w, uint64_t x, uint64_t b1) {
    const GlobalRd rd{w, a.prefix};
    St<NC> g{};
    uint64_t q = x;
    while (q < b1) {
        uint32_t err;
        const uint64_t q2 = parse_rd<NC>(a, rd, q, &err, g.ch);
        if (err) {
            g.stop = 1 | (err << 1);
            break;
        }
        ++g.cnt;
        q = q2;
    }
    g.x = q;
    return g;
}

// Slot of position x in a block's table (header words h0 = window mask, h1 =
// the first speculated start, h3 = the first speculated start past the
// window): its compact index (kWin for the extra slot), or -1 (not one of
// these; the landing slots are looked up by find_slot).
__device__ __forceinline__ int slot_of(uint64_t h0, uint64_t h1, uint64_t h3, uint32_t nslots, uint64_t b0,
                                       uint64_t x) {
    const uint64_t off = x - b0;
    if (h0 && off < kWin) return ((h0 >> off) & 1) ? __builtin_popcountll(h0 & ((1ull << off) - 1)) : -1;
    if (!h0 && nslots && x == h1) return 0;
    return x == h3 ? static_cast<int>(kWin) : -1;
}

// Header word 4: landing slots, their overflow, the block's first nonzero byte.
__device__ __forceinline__ uint32_t h4_nx(uint64_t h4) { return static_cast<uint32_t>(h4 & 0xff); }
__device__ __forceinline__ uint32_t h4_zr(uint64_t h4) { return static_cast<uint32_t>((h4 >> 16) & 0xffff); }
__device__ __forceinline__ uint32_t h4_za(uint64_t h4) { return static_cast<uint32_t>((h4 >> 32) & 0xff); }
// Header word 5: exit slots (0 until a repair pass gives the block some).
__device__ __forceinline__ uint32_t h5_ne(uint64_t h5) { return static_cast<uint32_t>(h5 & 0xff); }
// The landing slots a lookup uses (none in the test-hook table modes).
__device__ __forceinline__ uint32_t nx_used(const SxArgs& a, uint64_t h4) { return (a.mode & 3) ? 0 : h4_nx(h4); }

// First index in xs[0, n) whose value is >= v (xs ascending).
__device__ __forceinline__ uint32_t lower16(const uint16_t* xs, uint32_t n, uint32_t v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if (xs[m] < v) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// Where the cursor at x goes through block blk: the table entry `idx` (its
// chain to the block's end), minus `sub` zero records (below), or idx < 0 (a
// miss).  Beyond slot_of:
// - the landing slots (xs[0, nx): the block's ascending offsets, staged in
//   LDS by the caller; a binary search per lane);
// - a run of zero bytes: when the block's bytes [za, x) are all zero (za:
//   just past the window's last nonzero byte, header word 4), the schema has
//   no prefix and its all-zero record (fixed_bytes = Z long, every string
//   empty) is at most kWin bytes, the window position w = za + (x - za) mod Z
//   parses as zero records up to x -- so w's chain passes through x and the
//   chain from x is w's without its first (x - w) / Z records (no chars).  A
//   record whose chars are zeros and that straddles the block's start ends
//   there, whatever its length (its length field may lie in the window);
// - the exit slots (xs[kX, kX + ne), after a repair pass; in every mode).
struct Slot {
    int idx;
    uint32_t sub;
};
__device__ __forceinline__ Slot find_slot(const SxArgs& a, uint64_t h0, uint64_t h1, uint64_t h3, uint32_t meta,
                                          uint64_t h4, uint64_t h5, const uint16_t* xs, uint64_t b0, uint64_t x) {
    Slot r{slot_of(h0, h1, h3, meta & 0xff, b0, x), 0};
    if (r.idx >= 0) return r;
    const uint64_t off = x - b0;
    if (!(a.mode & 3)) {
        const uint32_t nx = kX ? h4_nx(h4) : 0;
        if (kX && nx && off < kSB) {
            const uint32_t lo = lower16(xs, nx, static_cast<uint32_t>(off));
            if (lo < nx && xs[lo] == off) {
                r.idx = static_cast<int>(kWin + 1 + lo);
                return r;
            }
        }
        const uint32_t Z = a.fixed_bytes, za = h4_za(h4);
        if (!a.prefix_len && Z <= kWin && off >= za && off <= h4_zr(h4)) {
            const uint32_t wo = za + static_cast<uint32_t>((off - za) % Z);
            if (wo < kWin && ((h0 >> wo) & 1)) {
                r.idx = __builtin_popcountll(h0 & ((1ull << wo) - 1));
                r.sub = static_cast<uint32_t>((off - wo) / Z);
                return r;
            }
        }
    }
    const uint32_t ne = h5_ne(h5);
    if (ne && off < kSB) {
        const uint32_t lo = lower16(xs + kX, ne, static_cast<uint32_t>(off));
        if (lo < ne && xs[kX + lo] == off) r.idx = static_cast<int>(kWin + 1 + kX + lo);
    }
    return r;
}

// The wave's LDS copy of block blk's landing slots (xs[0, nx)) and exit slots
// (xs[kX, kX + ne)); wave-uniform blk; every lane takes part.
__device__ __forceinline__ void stage_xs(const SxScratch& S, uint64_t blk, uint32_t nx, uint32_t ne, uint16_t* xs) {
    if (!nx && !ne) return;
    const uint32_t lane = threadIdx.x & 63;
    if constexpr (kX > 0)
        for (uint32_t i = lane; i < nx; i += 64) xs[i] = S.xp[blk * kX + i];
    for (uint32_t i = lane; i < ne; i += 64) xs[kX + i] = S.ep[blk * kE + i];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

// Prologue shared by the speculation and the decode: the prefix and the
// block's bytes [b0 - pre, min(b1 + kMargin, W)) in LDS (LDS-DMA), then a barrier.
__device__ __forceinline__ StagedRd stage_block(const SxArgs& a, const uint8_t* w, uint8_t* st, uint8_t* pre,
                                                uint64_t b0, uint64_t b1, uint32_t before = 0) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    for (uint32_t i = tid; i < a.prefix_len + 16; i += kBlock) pre[i] = i < a.prefix_len ? a.prefix[i] : 0;
    const uint64_t lo = b0 > before ? b0 - before : 0;
    const uint64_t hi = min<uint64_t>(b1 + kMargin, a.W);
    const uint64_t A = (reinterpret_cast<uint64_t>(w) + lo) & ~15ull;
    const uint32_t ng = static_cast<uint32_t>((reinterpret_cast<uint64_t>(w) + hi - A + 15) >> 4);
    for (uint32_t w0 = tid & ~63u; w0 < ng; w0 += kBlock) {
        const uint32_t gi = w0 + lane;
        if (gi < ng) {
            const uint32_t wb = __builtin_amdgcn_readfirstlane(w0);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<global_u8*>(A + 16ull * gi), (lds_u8*)(st + 16 * wb), 16,
                                             0, 0);
        }
    }
    __syncthreads();  // waits for the LDS-DMA and publishes the stage
    return StagedRd{(global_u8*)w, (lds_u8c*)st, A - reinterpret_cast<uint64_t>(w), lo, hi, (lds_u8c*)pre};
}

// Chunk tid's records from its start sp (or none): count, the position after
// them, chars, stop bits, their starts (up to cap, offsets in the chunk).
template <int NC, class Rd>
__device__ __forceinline__ void walk_chunk(const SxArgs& a, const Rd& rd, uint64_t sp, uint64_t chi,
                                           uint32_t* cnt, uint64_t* exit, uint64_t (&ch)[kMaxNC + 1], uint32_t* stop,
                                           uint8_t* list) {
    *cnt = 0;
    *stop = 0;
    *exit = ~0ull;
    if (sp == ~0ull) return;
    uint64_t p = sp;
    uint32_t k = 0;
    while (p < chi) {
        uint32_t err;
        const uint64_t q = parse_rd<NC>(a, rd, p, &err, ch);
        if (err) {
            *stop = 1 | (err << 1);
            break;
        }
        if (list && k < a.cap) list[k] = static_cast<uint8_t>(p % kSC);
        ++k;
        p = q;
    }
    *cnt = k;
    *exit = p;
}

// The chunks' segments: chunk c continues its predecessor's segment when that
// chunk's exit is c's start (and it did not stop); tails end segments.  Fills
// L.tail, L.pcnt and L.pch (exclusive scans, totals at [kBlock]).
template <int NC>
__device__ __forceinline__ void link_chunks(Chunks<NC>& L, uint64_t b0, uint64_t sp, uint64_t cexit, uint32_t cstop,
                                            uint32_t ccnt, const uint64_t (&cch)[kMaxNC + 1]) {
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    bool tail = false;
    if (sp != ~0ull) {
        const uint32_t nxt = next_bit(L.has, tid + 1);
        tail = cstop || nxt >= kBlock || cexit != b0 + L.start[nxt];
    }
    const uint64_t tm = __ballot(tail);
    if (lane == 0) L.tail[tid >> 6] = tm;
    uint64_t tot;
    const uint64_t x = block_xscan(ccnt, &tot, L.ws);
    L.pcnt[tid] = static_cast<uint32_t>(x);
    if (tid == 0) L.pcnt[kBlock] = static_cast<uint32_t>(tot);
    if constexpr (NC > 0) {
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            const uint64_t y = block_xscan(cch[k], &tot, L.ws);
            L.pch[k][tid] = y;
            if (tid == 0) L.pch[k][kBlock] = tot;
        }
    }
    __syncthreads();
}

// The cursor's way through a block from x when x is in none of its table's
// slots (a miss), by one wave (every lane calls it; lanes with !mine get
// nothing): the block is staged in the wave's LDS, its 256 chunks are walked
// again from phase 1's speculated starts -- four a lane, as k_sx_decode walks
// them -- and linked into segments (wave scans), then each missing lane's
// chain crosses the block in segment jumps, parsing records only where it is
// off the speculation.  A record-by-record walk of a block by one lane cost
// ~250 ns a record (8 KiB of 19-byte records: ~0.1 ms, serial in k_sx_top).
template <int NC>
__device__ St<NC> walk_miss(const SxArgs& a, const uint8_t* w, const SxScratch& S, uint64_t blk, uint8_t* stage,
                            Chunks<NC>& C, uint64_t b0, uint64_t b1, uint64_t x, bool mine) {
    const uint32_t lane = threadIdx.x & 63;
    const WaveRd rd = stage_wave(a, w, stage, b0, b1);
    if (lane < 4) {
        C.has[lane] = 0;
        C.tail[lane] = 0;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll 1
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t c = 4 * lane + q;
        const uint64_t clo = b0 + static_cast<uint64_t>(c) * kSC, chi = min<uint64_t>(clo + kSC, b1);
        const uint8_t sb = clo < b1 ? S.spec[blk * kBlock + c] : kNoSpec;
        const uint64_t sp = sb == kNoSpec ? ~0ull : clo + sb;
        uint64_t ch[kMaxNC + 1] = {};
        uint32_t cnt, cstop;
        uint64_t cexit;
        walk_chunk<NC>(a, rd, sp, chi, &cnt, &cexit, ch, &cstop, nullptr);
        C.start[c] = sp == ~0ull ? kNoStart : static_cast<uint16_t>(sp - b0);
        C.exit[c] = cexit;
        C.stop[c] = static_cast<uint8_t>(cstop);
        C.pcnt[c] = cnt;
        if constexpr (NC > 0) {
#pragma unroll
            for (int k = 0; k < NC; ++k) C.pch[k][c] = ch[k];
        }
        if (sp != ~0ull) atomicOr(reinterpret_cast<unsigned long long*>(&C.has[c >> 6]), 1ull << (c & 63));
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // segment tails (as link_chunks), then exclusive scans of the records and
    // chars over the chunks: a lane's four in order, the lanes by a wave scan
    uint64_t tot = 0, totc[kMaxNC + 1] = {};
#pragma unroll 1
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t c = 4 * lane + q;
        if (C.start[c] != kNoStart) {
            const uint32_t nxt = next_bit(C.has, c + 1);
            if (C.stop[c] || nxt >= kBlock || C.exit[c] != b0 + C.start[nxt])
                atomicOr(reinterpret_cast<unsigned long long*>(&C.tail[c >> 6]), 1ull << (c & 63));
        }
        tot += C.pcnt[c];
        if constexpr (NC > 0) {
#pragma unroll
            for (int k = 0; k < NC; ++k) totc[k] += C.pch[k][c];
        }
    }
    uint64_t inc = tot, incc[kMaxNC + 1];
#pragma unroll
    for (int k = 0; k < NC; ++k) incc[k] = totc[k];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(inc, d, 64);
        if (lane >= static_cast<uint32_t>(d)) inc += y;
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            const uint64_t z = __shfl_up(incc[k], d, 64);
            if (lane >= static_cast<uint32_t>(d)) incc[k] += z;
        }
    }
    uint64_t run = inc - tot, runc[kMaxNC + 1];
#pragma unroll
    for (int k = 0; k < NC; ++k) runc[k] = incc[k] - totc[k];
#pragma unroll 1
    for (uint32_t q = 0; q < 4; ++q) {
        const uint32_t c = 4 * lane + q;
        const uint32_t v = C.pcnt[c];
        C.pcnt[c] = static_cast<uint32_t>(run);
        run += v;
        if constexpr (NC > 0) {
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                const uint64_t y = C.pch[k][c];
                C.pch[k][c] = runc[k];
                runc[k] += y;
            }
        }
    }
    if (lane == 63) {
        C.pcnt[kBlock] = static_cast<uint32_t>(run);
        if constexpr (NC > 0) {
#pragma unroll
            for (int k = 0; k < NC; ++k) C.pch[k][kBlock] = runc[k];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (!mine) return St<NC>{};
    return walk_chain<NC, false>(a, rd, C, b0, b1, x, nullptr, nullptr);
}

// Workgroup i -> block.  Dispatch order by default; with SRPC_SX_XCD the
// dispatcher's round robin over the 8 XCDs (i mod 8, each with its own L2)
// gives XCD x one contiguous run of blocks, so the bytes a block stages past
// its end (and the next one's premargin) would be found in that XCD's L2 the
// second time -- measured 1-3 % slower on every random row (the kernels are
// not bound by those re-reads: profiles/r05_sdx_ab.log), so not the default.
__device__ __forceinline__ uint64_t xcd_block(uint32_t i, uint32_t G) {
#ifndef SRPC_SX_XCD
    return i;
#endif
    const uint32_t x = i & 7, k = i >> 3, q = G >> 3, r = G & 7;
    return static_cast<uint64_t>(x) * q + min(x, r) + k;
}

// ---- phase 1: speculation and the block tables ----------------------------------
template <int NC>
struct SpecLds {
    alignas(16) uint8_t st[kStageS + 16];  // wire bytes [base, base + kStageS)
    alignas(16) uint8_t pre[kMaxPrefix + 16];
    Chunks<NC> c;
    // per chunk: its records' starts (offsets in the chunk); then wave 0's
    // part (the record list written out) holds the landing slots
    alignas(4) uint8_t list[kBlock * kListCap];
    uint32_t s_nx;  // landings found (wave 1's counter)
    uint64_t zm[kZW];  // the zero map (zero-heavy blocks only)
};
static_assert(64 * kListCap >= 2 * kX, "the landing slots fit wave 0's part of the chunk lists");

// Wave 1 of k_sx_spec: the block's zero run and landing slots (their chains
// to the block's end and their positions), header word 4.
template <int NC>
__device__ __forceinline__ void land_slots(const SxArgs& a, const StagedRd& rd, const StageOnlyRd& so,
                                           const SxScratch& S, SpecLds<NC>& L, Chunks<NC>& C, uint64_t b,
                                           uint64_t b0, uint64_t b1, uint64_t sF2, bool zflag) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = a.W;
    // The zero run the window ends in (find_slot's zero-run rule, for schemas
    // with no prefix whose all-zero record is at most kWin bytes): za = just
    // past the window's last nonzero byte, zr = the first nonzero byte from
    // there on -- bytes [za, zr) of the block are zero.
    uint32_t za = 0, zr = 0;
    if (!(a.mode & 3) && b > 0 && !a.prefix_len && a.fixed_bytes <= kWin) {
        const uint32_t wofs = static_cast<uint32_t>(b0 - rd.base), blen = static_cast<uint32_t>(b1 - b0);
        const uint64_t nz = __ballot(lane < blen && L.st[wofs + lane] != 0);
        za = nz ? 64 - __builtin_clzll(nz) : 0;
        zr = za;
        if (za + a.fixed_bytes <= kWin) {  // a congruent window position can lie in the run
            zr = blen;
            for (uint32_t o = kWin; o < blen; o += 256) {  // a dword per lane from o on
                const uint32_t p4 = o + 4 * lane;
                uint32_t v = 0;
                if (p4 < blen) {
                    lds_u32c* q = reinterpret_cast<lds_u32c*>((lds_u8c*)L.st + ((wofs + p4) & ~3u));
                    const uint32_t sh = (wofs + p4) & 3;
                    v = sh ? __builtin_amdgcn_alignbyte(q[1], q[0], sh) : q[0];
                    if (blen - p4 < 4) v &= (1u << (8 * (blen - p4))) - 1;
                }
                const uint64_t m = __ballot(v != 0);
                if (m) {
                    const uint32_t l0 = __builtin_ctzll(m);
                    const uint32_t v0 = __builtin_amdgcn_readlane(v, l0);
                    zr = o + 4 * l0 + (__builtin_ctz(v0) >> 3);
                    break;
                }
            }
        }
    }
    // The landing slots: the end q of every record that parses at a position
    // p of the premargin [b0 - kPre, b0) and ends in the block past the
    // window, where a record parses too (not at sF2, the extra slot).  Lane l
    // takes positions p0 .. p0 + 15.  On a wire under 4 GiB a length that
    // fits has its four high bytes zero: the lane's first string lengths come
    // from one window of stage dwords and only those positions are tested (as
    // chunk_mask_z).  Wave 1's part of the chunk lists (read above) holds the
    // ends, then sorted (a rank per entry; duplicates are harmless).
    uint32_t nx = 0, xover = 0;
    uint16_t* xl = reinterpret_cast<uint16_t*>(L.list + 64 * kListCap);  // wave 1's part
#ifdef SRPC_SX_NOSCAN
    if (false) {  // (A/B: the slots' layout and the premargin's staging without the scan)
#else
    if (kX && !(a.mode & 3) && b > 0) {
#endif
        const uint64_t p0 = b0 - kPre + 16 * lane;
        uint32_t cand = 0xffff;
        if (W < (1ull << 32) && a.first_len_at + 64 <= kMargin) {  // (the window's dwords lie in the stage)
            const uint32_t o = static_cast<uint32_t>(p0 + a.first_len_at - rd.base);
            lds_u32c* q = reinterpret_cast<lds_u32c*>((lds_u8c*)L.st + (o & ~3u));
            uint32_t d[7];
#pragma unroll
            for (uint32_t k = 0; k < 7; ++k) d[k] = q[k];
            const uint32_t sh = o & 3;  // (the same for every lane)
#pragma unroll
            for (uint32_t k = 0; k < 6; ++k) d[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
            // and, from the same window, the record's end where it is fixed
            // by the first length (one string, no prefix): in the block past
            // the window; otherwise at least not past the block's end
            const bool one = a.nstrings == 1 && !a.prefix_len;
            const uint32_t rest = one ? a.fixed_bytes : a.first_len_at + 8;
            const uint32_t off0 = kPre - 16 * lane, blen = static_cast<uint32_t>(b1 - b0);  // b0 - p0
            cand = 0;
#pragma unroll
            for (uint32_t i = 0; i < 16; ++i) {  // bytes i + 4 .. i + 7 of the window zero
                const uint32_t k = (i + 4) >> 2, s8 = (i + 4) & 3;
                const uint32_t hi32 = s8 ? __builtin_amdgcn_alignbyte(d[k + 1], d[k], s8) : d[k];
                const uint32_t k0 = i >> 2, s0 = i & 3;
                const uint32_t lo32 = s0 ? __builtin_amdgcn_alignbyte(d[k0 + 1], d[k0], s0) : d[k0];
                // the end q - b0 = len + rest - (off0 - i) (a length of 2^24 or
                // more ends past any block: clamped there, 32-bit arithmetic)
                const int32_t e = static_cast<int32_t>(min(lo32, 1u << 24) + rest) - static_cast<int32_t>(off0 - i);
                const bool ok = hi32 == 0 && e < static_cast<int32_t>(blen) && (!one || e >= static_cast<int32_t>(kWin));
                cand |= (ok ? 1u : 0u) << i;
            }
            if (a.prefix_len) {  // the prefix's first (up to 4) bytes at p
                const uint32_t po = static_cast<uint32_t>(p0 - rd.base);
                lds_u32c* r = reinterpret_cast<lds_u32c*>((lds_u8c*)L.st + (po & ~3u));
                uint32_t e5[6];
#pragma unroll
                for (uint32_t k = 0; k < 6; ++k) e5[k] = r[k];
                const uint32_t sp = po & 3;  // (the same for every lane)
#pragma unroll
                for (uint32_t k = 0; k < 5; ++k) e5[k] = __builtin_amdgcn_alignbyte(e5[k + 1], e5[k], sp);
                const uint32_t pk = a.prefix_len < 4 ? a.prefix_len : 4;
                const uint32_t pm = pk == 4 ? ~0u : (1u << (8 * pk)) - 1, pv = static_cast<uint32_t>(a.pre8) & pm;
                uint32_t mp = 0;
#pragma unroll
                for (uint32_t i = 0; i < 16; ++i) {
                    const uint32_t k = i >> 2, s8 = i & 3;
                    const uint32_t v = s8 ? __builtin_amdgcn_alignbyte(e5[k + 1], e5[k], s8) : e5[k];
                    mp |= ((v & pm) == pv ? 1u : 0u) << i;
                }
                cand &= mp;
            }
        }
        SXP_ADD(5, __builtin_popcount(cand));
        while (cand) {
            const uint32_t i = __builtin_ctz(cand);
            cand &= cand - 1;
            const uint64_t p = p0 + i;
            if (!filter(a, rd, p)) continue;
            uint64_t qe;
            if (a.nstrings == 1 && !a.prefix_len) {
                qe = p + a.fixed_bytes + rd.u64(p + a.first_len_at);
            } else {
                uint32_t err;
                uint64_t t[kMaxNC + 1];
                qe = parse_rd<0>(a, rd, p, &err, t);
                if (err) continue;
            }
            SXP_ADD(6, qe >= b0 + kWin && qe < b1 && qe != sF2 ? 1 : 0);
            if (qe >= b0 + kWin && qe < b1 && qe != sF2 && filter(a, so, qe) && plausible(a, rd, qe)) {
                const uint32_t j = atomicAdd(&L.s_nx, 1u);
                if (j < kX) xl[j] = static_cast<uint16_t>(qe - b0);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const uint32_t tot = __builtin_amdgcn_readfirstlane(__atomic_load_n(&L.s_nx, __ATOMIC_RELAXED));
        SXP_SET(7, tot);

        nx = min(tot, kX);
        xover = tot > kX ? 1u : 0u;
        if (nx > 1) {
            const uint32_t v0 = lane < nx ? xl[lane] : 0xffffu, v1 = lane + 64 < nx ? xl[lane + 64] : 0xffffu;
            uint32_t r0 = 0, r1 = 0;
            for (uint32_t k = 0; k < nx; ++k) {
                const uint32_t v = xl[k];
                r0 += v < v0 || (v == v0 && k < lane);
                r1 += v < v1 || (v == v1 && k < lane + 64);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // every read before the writes
            if (lane < nx) xl[r0] = static_cast<uint16_t>(v0);
            if (lane + 64 < nx) xl[r1] = static_cast<uint16_t>(v1);
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
    }
    for (uint32_t j = lane; j < nx; j += 64) {
        const uint32_t o = xl[j];
        st_store<NC>(S.ent + (b * kEnt + kWin + 1 + j) * ew<NC>(),
                     zflag ? walk_chain<NC, false, true>(a, rd, C, b0, b1, b0 + o, nullptr, nullptr, L.zm)
                           : walk_chain<NC, false>(a, rd, C, b0, b1, b0 + o, nullptr, nullptr));
        S.xp[b * kX + j] = static_cast<uint16_t>(o);
    }
    if (lane == 0)
        S.hdr[kHdr * b + 4] = nx | (xover << 8) | (static_cast<uint64_t>(zr) << 16) | (static_cast<uint64_t>(za) << 32);
}

// k_sx_spec held to the registers of 8 waves per SIMD (56 VGPRs, no spill):
// left to itself the compiler takes 64-68 and the kernel drops to 7 waves per
// SIMD, 8 % slower on the random rows (profiles/r05_sdx_ab.log).  A/B builds
// set SRPC_SX_WPE (0 = no hint).
#ifndef SRPC_SX_WPE
#define SRPC_SX_WPE 8
#endif
#if SRPC_SX_WPE
// (the three-chars-states instance is held to 7 by its LDS: the hint stays a hint)
#pragma clang diagnostic ignored "-Wpass-failed"
#define SX_SPEC_ATTR __attribute__((amdgpu_waves_per_eu(SRPC_SX_WPE, SRPC_SX_WPE)))
#else
#define SX_SPEC_ATTR
#endif
template <int NC>
__global__ __launch_bounds__(kBlock) SX_SPEC_ATTR void k_sx_spec(SxArgs a, const uint8_t* __restrict__ w, SxScratch S) {
    __shared__ SpecLds<NC> L;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint64_t b = xcd_block(blockIdx.x, gridDim.x);
    const uint64_t W = a.W;
    const uint64_t b0 = b * kSB, b1 = min<uint64_t>(b0 + kSB, W);
    SXP_BEGIN
    if (b == 0 && tid < kCtlWords) S.ctl[tid] = 0;  // this call's counters (read by the later launches)
    if (tid == 0) L.s_nx = 0;
    const StagedRd rd = stage_block(a, w, L.st, L.pre, b0, b1, kPre);
    const StageOnlyRd so{rd};
    SXP(0);

    // speculation: chunk c = tid
    const uint64_t clo = b0 + static_cast<uint64_t>(tid) * kSC, chi = min<uint64_t>(clo + kSC, b1);
    uint64_t sp = ~0ull;   // the chunk's first plausible start
    uint64_t sq1 = ~0ull;  // the end of its first record, when the speculation parsed it
    uint64_t sch1[kMaxNC + 1] = {};
    if (clo < b1) {
        if (clo == 0) {
            sp = 0;  // the stream starts at 0: no speculation
        } else {
            const uint32_t at = static_cast<uint32_t>(clo - rd.base);
            uint32_t pj = ~0u;
            const bool zf = W < (1ull << 32) && !(a.mode & 4);
            uint64_t mask = zf ? chunk_mask_z(a, L.st, at, clo, chi, &pj) : chunk_mask(a, L.st, at, clo, chi);
            bool tried = false;  // the first cluster's pick was tested
            // the first cluster of passing positions (8 bytes from the first):
            // its smallest first string length is the true start (a start
            // 1-3 bytes early reads the true length shifted up), tested first
            // -- one plausibility test per chunk on random data
            if (mask) {
                uint64_t pick = pj != ~0u ? clo + pj : ~0ull;
                if (!zf) {
                    const uint32_t j0 = __builtin_ctzll(mask);
                    uint64_t cl = (mask >> j0) & 0xff;
                    uint64_t best = ~0ull;
                    while (cl) {
                        const uint64_t q = clo + j0 + __builtin_ctzll(cl);
                        cl &= cl - 1;
                        const uint64_t l = so.u64(q + a.first_len_at);
                        if (l < best) {
                            best = l;
                            pick = q;
                        }
                    }
                }
                uint32_t err = SRPC_STATUS_BOUNDS;
                uint64_t tmp[kMaxNC + 1] = {};
                tried = pick != ~0ull;
                const uint64_t q1 = pick != ~0ull ? parse_rd<NC>(a, so, pick, &err, tmp) : 0;
                bool ok = !err;
                if (ok && a.plaus > 1 && q1 != W) {
                    uint64_t t2[kMaxNC + 1];
                    (void)parse_rd<0>(a, so, q1, &err, t2);
                    ok = !err;
                }
                if (ok) {
                    sp = pick;
                    sq1 = q1;
#pragma unroll
                    for (int k = 0; k < NC; ++k) sch1[k] = tmp[k];
                }
            }
            SXP_ADD(4, sp == ~0ull && mask ? 1 : 0);
            if (sp == ~0ull && __builtin_popcountll(mask) <= 16) {
                // otherwise, in a chunk where few positions pass: cluster by
                // cluster (8 bytes from a cluster's first passing position),
                // its smallest first length tested for plausibility (the first
                // cluster's was, above).  A chunk of a schema whose later
                // string lengths also have zero high bytes (zh4: int8, string,
                // int16, string) often starts with such a false cluster:
                // testing every position in order cost zh4 random ~130
                // fallbacks x ~8 plausibility tests a block (34 % of its
                // throughput, profiles/r05_sdx_ab.log).  (A start missed here
                // is only a slower chain, never a wrong one.)
                uint64_t m = mask;
                bool skip = tried;
                while (m) {
                    const uint32_t j0 = __builtin_ctzll(m);
                    uint64_t cl = (m >> j0) & 0xff;
                    m &= j0 + 8 < 64 ? ~0ull << (j0 + 8) : 0ull;
                    if (skip) {
                        skip = false;
                        continue;
                    }
                    uint64_t best = ~0ull, pk = clo + j0;
                    while (cl) {
                        const uint64_t q = clo + j0 + __builtin_ctzll(cl);
                        cl &= cl - 1;
                        const uint64_t l = so.u64(q + a.first_len_at);
                        if (l < best) {
                            best = l;
                            pk = q;
                        }
                    }
                    if (plausible(a, so, pk)) {
                        sp = pk;
                        break;
                    }
                }
            } else if (sp == ~0ull) {
                // where most positions pass (zero-heavy bytes): the first
                // plausible position, then of the plausible ones within 8
                // bytes the smallest first length
                const uint64_t passing = mask;
                while (mask) {
                    const uint32_t j = __builtin_ctzll(mask);
                    if (plausible(a, so, clo + j)) {
                        sp = clo + j;
                        break;
                    }
                    mask &= mask - 1;
                }
                if (sp != ~0ull) {
                    const uint32_t jb = static_cast<uint32_t>(sp - clo);
                    uint64_t cand = (passing >> (jb + 1)) & 0x7f;
                    uint64_t best = so.u64(sp + a.first_len_at), pick = sp;
                    while (cand) {
                        const uint64_t q = sp + 1 + __builtin_ctzll(cand);
                        cand &= cand - 1;
                        const uint64_t l = so.u64(q + a.first_len_at);
                        if (l < best && plausible(a, so, q)) {
                            best = l;
                            pick = q;
                        }
                    }
                    sp = pick;
                }
            }
        }
    }
    S.spec[b * kBlock + tid] = sp == ~0ull ? kNoSpec : static_cast<uint8_t>(sp - clo);
    uint64_t cch[kMaxNC + 1] = {};
    uint32_t ccnt, cstop;
    uint64_t cexit;
    if (sq1 != ~0ull) {  // the first record was parsed by the test above: walk on from its end
#pragma unroll
        for (int k = 0; k < NC; ++k) cch[k] = sch1[k];
        L.list[tid * kListCap] = static_cast<uint8_t>(sp - clo);
        walk_chunk<NC>(a, rd, sq1, chi, &ccnt, &cexit, cch, &cstop, L.list + tid * kListCap + 1);
        if (sq1 >= chi) {  // (the walk saw no record: cexit = ~0)
            ccnt = 0;
            cexit = sq1;
            cstop = 0;
        }
        ++ccnt;
    } else {
        walk_chunk<NC>(a, rd, sp, chi, &ccnt, &cexit, cch, &cstop, L.list + tid * kListCap);
    }
    Chunks<NC>& C = L.c;
    C.start[tid] = sp == ~0ull ? kNoStart : static_cast<uint16_t>(sp - b0);
    C.exit[tid] = cexit;
    C.stop[tid] = static_cast<uint8_t>(cstop);
    const uint64_t hm = __ballot(sp != ~0ull);
    if (lane == 0) C.has[tid >> 6] = hm;
    __syncthreads();
    SXP(1);
    link_chunks<NC>(C, b0, sp, cexit, cstop, ccnt, cch);
    // Repair, in blocks the speculation cut into many segments (zero-heavy
    // bytes, where most positions parse): each chunk whose predecessor's walk
    // exits inside it walks again from that exit (or has no start when the
    // exit is past it), all at once, until nothing changes or kRepairMax
    // passes.  A run of k wrong chunks after a right one is right after k
    // passes; the chains then cross the block in a few segment jumps instead
    // of record by record (here and in k_sx_decode, which walks its chunks
    // from the repaired starts).  A first pass that joins fewer than 4
    // segments ends the repair.  Random blocks have 1-4 segments: not taken.
    bool zflag = false;  // a zero-heavy block: its chains cross zero runs by the zero map
    {
        uint32_t ntail = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) ntail += __builtin_popcountll(C.tail[k]);
#ifdef SRPC_SX_NOREPAIR
        if (false) {  // (A/B)
#else
        if (__builtin_expect(ntail > kRepairMin, 0)) {
#endif
#ifndef SRPC_SX_NOZMAP
            zflag = !a.prefix_len && NC < 3;  // (four string fields: the walker's registers spill)
            if (zflag) {
                build_zmap(rd, b0, L.zm);
                // worth it where zero runs are long: at least half the block's
                // chunks all zero (zero-heavy chars with a nonzero byte every
                // ~20 make one-record runs: there the map costs more than it
                // saves)
                uint32_t zc = 0;
#pragma unroll
                for (uint32_t k = 0; k < kSB / 32 / 64; ++k) zc += 64 - __builtin_popcountll(L.zm[k]);
                zflag = 2 * zc >= kSB / 32;
            }
#endif
#pragma nounroll
            for (uint32_t pass = 0; pass < kRepairMax; ++pass) {
                const uint32_t pc = tid ? prev_bit(C.has, tid - 1) : 256;
                uint64_t nsp = sp;
                if (pc < 256 && !C.stop[pc] && clo < b1) {
                    const uint64_t e = C.exit[pc];
                    if (e >= chi) nsp = ~0ull;
                    else if (e >= clo) nsp = e;
                }
                const bool redo = nsp != sp;
                if (!__syncthreads_or(redo)) break;  // (every chunk read its predecessor's exit)
                if (redo) {
                    sp = nsp;
#pragma unroll
                    for (int k = 0; k <= kMaxNC; ++k) cch[k] = 0;
                    walk_chunk<NC>(a, rd, sp, chi, &ccnt, &cexit, cch, &cstop, L.list + tid * kListCap);
                    C.start[tid] = sp == ~0ull ? kNoStart : static_cast<uint16_t>(sp - b0);
                    C.exit[tid] = cexit;
                    C.stop[tid] = static_cast<uint8_t>(cstop);
                }
                const uint64_t hm2 = __ballot(sp != ~0ull);
                if (lane == 0) C.has[tid >> 6] = hm2;
                __syncthreads();
                // (the passes need only the starts, exits and stops: the
                // segments' scans are built once, after the last pass)
                if (pass == 0) {
                    // a first pass that joins few segments (long runs of
                    // wrong chunks, e.g. zero bytes read in the wrong
                    // alignment: one chunk a pass) is not repeated
                    bool tail = false;
                    if (sp != ~0ull) {
                        const uint32_t nxt = next_bit(C.has, tid + 1);
                        tail = cstop || nxt >= kBlock || cexit != b0 + C.start[nxt];
                    }
                    const uint32_t nt = static_cast<uint32_t>(__syncthreads_count(tail));
                    if (nt + 4 > ntail) break;
                }
            }
            link_chunks<NC>(C, b0, sp, cexit, cstop, ccnt, cch);
            if (clo < b1) S.spec[b * kBlock + tid] = sp == ~0ull ? kNoSpec : static_cast<uint8_t>(sp - clo);
        }
    }
    // the chunks' records in order (the block's whole record list when its
    // chunks form one segment: k_sx_decode's fast path takes it from here)
    {
        const uint32_t r0 = C.pcnt[tid];
        uint16_t* rl = S.rl + b * kMaxRec;
        for (uint32_t k = 0; k < ccnt && r0 + k < kMaxRec; ++k)
            rl[r0 + k] = static_cast<uint16_t>(tid * kSC + L.list[tid * kListCap + k]);
    }
    SXP(2);

    const uint32_t F2 = next_bit(C.has, kWin / kSC);
    const uint64_t sF2 = F2 < kBlock && b > 0 && !(a.mode & 3) ? b0 + C.start[F2] : ~0ull;

    // The table, three waves at once (the workgroup holds its LDS until the
    // last of them is done: work added to one wave's share lengthens every
    // block's life, and so the kernel, unless it overlaps another's).
    // - wave 0 (lane = window position): every plausible position of the
    //   block's first kWin bytes; a window with none holds the first
    //   speculated start (sF) alone.  The primary slot is sF's: the entry the
    //   speculation itself predicts.  Header words 0-2.
    // - wave 1: the zero run and the landing slots, header word 4.
    // - one lane of wave 3: the extra slot, the first speculated start past
    //   the window (a record longer than the window that ends where its chunk
    //   speculated: entered there, not walked), header word 3.
    if (tid >= 128) {
        if (tid == kBlock - 1) {
            if (sF2 != ~0ull)
                st_store<NC>(S.ent + (b * kEnt + kWin) * ew<NC>(),
                             zflag ? walk_chain<NC, false, true>(a, rd, C, b0, b1, sF2, nullptr, nullptr, L.zm)
                                   : walk_chain<NC, false>(a, rd, C, b0, b1, sF2, nullptr, nullptr));
            S.hdr[kHdr * b + 3] = sF2;
        }
        return;
    }
    if (tid >= 64) {
        land_slots<NC>(a, rd, so, S, L, C, b, b0, b1, sF2, zflag);
        return;
    }
    const uint32_t F = next_bit(C.has, 0);
    const uint64_t sF = F < kBlock ? b0 + C.start[F] : ~0ull;
    uint64_t mycand = ~0ull;
    if (b == 0) {
        if (lane == 0) mycand = 0;
    } else if (!(a.mode & 3)) {
        // (the records read through the stage or, for a record that runs past
        // it, global memory: a true entry whose next record starts beyond the
        // stage is a slot too, not a miss)
        const uint64_t p = b0 + lane;
        if (p < b1 && filter(a, so, p) && plausible(a, rd, p)) mycand = p;
    }
    uint64_t wmask = __ballot(mycand != ~0ull);
    if (!wmask && lane == 0 && sF != ~0ull && !(a.mode & 2)) mycand = sF;
    const uint64_t vmask = __ballot(mycand != ~0ull);
    const uint32_t nslots = __builtin_popcountll(vmask);
    uint32_t prim = kNoPrim;
    if (sF != ~0ull && nslots) {
        if (wmask) {
            const uint64_t off = sF - b0;  // sF lies in the window whenever the window has a slot
            if (off < kWin && ((wmask >> off) & 1)) prim = __builtin_popcountll(wmask & ((1ull << off) - 1));
        } else {
            prim = 0;
        }
    }
    St<NC> mine{};
    if (mycand != ~0ull) {
        mine = zflag ? walk_chain<NC, false, true>(a, rd, C, b0, b1, mycand, nullptr, nullptr, L.zm)
                     : walk_chain<NC, false>(a, rd, C, b0, b1, mycand, nullptr, nullptr);
        const uint32_t k = __builtin_popcountll(vmask & ((1ull << lane) - 1));
        st_store<NC>(S.ent + (b * kEnt + k) * ew<NC>(), mine);
    }
    if (lane == 0) {
        // one segment from sF to the block's end (a single tail, leaving the
        // block or stopping): a cursor entering at sF takes every chunk's
        // records as speculated (k_sx_decode skips the chain walk)
        uint32_t ntail = 0, lastc = 0;
        for (int k = 0; k < 4; ++k) {
            ntail += __builtin_popcountll(C.tail[k]);
            if (C.tail[k]) lastc = 64 * k + 63 - __builtin_clzll(C.tail[k]);
        }
        const bool one = sF != ~0ull && ntail == 1 && (C.stop[lastc] || C.exit[lastc] >= b1);
        SXP_SET(14, ntail);
        uint64_t* h = S.hdr + kHdr * b;
        h[0] = wmask;
        h[1] = sF;
        h[2] = nslots | (static_cast<uint64_t>(prim) << 8) | (one ? 1ull << 16 : 0ull) | (zflag ? 1ull << 17 : 0ull) |
               (static_cast<uint64_t>(min<uint32_t>(C.pcnt[kBlock], kMaxRec)) << 32);
        h[5] = 0;  // no exit slots (until a repair pass)
    }
    SXP(3);
}

// ---- the repair pass (round 6): exit slots -----------------------------------------
// Run only after the first scan met a position no table holds (ctl
// kCtlRepair; otherwise every workgroup reads one word and ends).  The
// reference's cursor enters block c at the end of the record that straddles
// c's start: a record that starts at a position of block c - 1 the cursor
// reaches.  k_sx_repair's workgroup for block c takes EVERY position p of
// block c - 1: the record at p, parsed in full (where one parses), links p to
// the next record start; pointer jumping over those links in LDS (in place,
// at most log2 of the records a block holds + 1 rounds) gives every p its
// exit from block c - 1 -- the first record start past its end -- or a stop.
// The distinct exits inside block c at which a record parses ("live": a
// cursor entering anywhere else stops right there, one parse) are every
// position the cursor can enter block c at from block c - 1, whatever the
// speculation made of either block's bytes.  Those block c's table does not
// already hold become its exit slots (at most kE, ascending): each one's
// chain through block c, like the table's other chains.  The second scan
// then meets a position no table holds only where block c had more possible
// entries than kE, where the record that enters c started two or more blocks
// back (longer than a block), or on a wire of 4 GiB or more (32-bit offsets):
// those are walked, as every miss was before round 6.  Cost: one parse per
// position (most stop at the first length) and the jumping, every block in
// parallel -- O(bytes), no serial chain of blocks.
constexpr uint32_t kJStop = 0xFFFFFFFFu;
static_assert(kSB / 32 == kBlock, "one bitmap word per thread");

template <int NC>
struct RepairLds {
    alignas(16) uint8_t st[kStage + 16];
    alignas(16) uint8_t pre[kMaxPrefix + 16];
    union {
        uint32_t J[kSB];  // block c - 1, per position: the next record start (< kSB: in the block), its exit, kJStop
        Chunks<NC> c;     // block c's chunks
    } u;
    uint32_t cand[kSB / 32];  // block c's positions: live exits of block c - 1, then those its table lacks
    uint16_t xs[kXS];         // block c's landing slots, then (kX on) its exit slots
    uint64_t ws[kBlock / 64];
    uint64_t zm[kZW];
};

// The end of the record at p when it parses and ends at most at `limit`;
// otherwise p with *far set when it would end past `limit` (its exit cannot
// be an entry of the next block: the repair ignores it, so a record whose
// first string alone runs past the limit costs no read of the far bytes its
// later fields would need) or *err set when it does not parse.
template <class Rd>
__device__ __forceinline__ uint64_t parse_near(const SxArgs& a, const Rd& r, uint64_t p, uint64_t limit, bool* bad) {
    const uint64_t W = a.W;
    bool e = false;
    if (a.prefix_len) {
        if (a.prefix_len > W - p) {
            e = true;
        } else {
            uint64_t diff = 0;
            uint32_t i = 0;
            for (; i + 8 <= a.prefix_len; i += 8) diff |= r.u64(p + i) ^ r.pre64(i);
            for (; i < a.prefix_len; ++i) diff |= r.u8(p + i) ^ r.pre8(i);
            e = diff != 0;
        }
    }
    uint64_t q = p;
    for (uint32_t k = 0; k < a.nstrings; ++k) {
        const uint32_t g = a.gap[k] + 8;
        if (!e) {
            if (g > W - q || q + g > limit) {
                e = true;
            } else {
                q += g;
                const uint64_t len = r.u64(q - 8);
                if (len > W - q || len > limit - q) e = true;
                else q += len;
            }
        }
    }
    const uint32_t gl = a.gap[a.nstrings];
    if (!e && (gl > W - q || q + gl > limit)) e = true;
    *bad = e;
    return e ? p : q + gl;
}

// A record parses at x (read through the stage where it holds x).
template <class Rd>
__device__ __forceinline__ bool live_at(const SxArgs& a, const Rd& rd, uint64_t x) {
    if (!filter(a, rd, x)) return false;
    uint32_t err;
    uint64_t t[kMaxNC + 1];
    (void)parse_rd<0>(a, rd, x, &err, t);
    return !err;
}

template <int NC>
__global__ __launch_bounds__(kBlock) void k_sx_repair(SxArgs a, const uint8_t* __restrict__ w, SxScratch S) {
    if (!S.ctl[kCtlRepair]) return;
    __shared__ RepairLds<NC> L;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    for (uint64_t c = 1 + blockIdx.x; c < a.nb; c += gridDim.x) {
        if (a.W >= kJStop) break;  // offsets in 32 bits: beyond, the second scan walks
        // ---- block c - 1: every position's exit
        const uint64_t p0 = (c - 1) * kSB, p1 = p0 + kSB;  // (a whole block: not the last)
        L.cand[tid] = 0;
        {
            const StagedRd rd = stage_block(a, w, L.st, L.pre, p0, p1);  // (ends in a barrier)
            // (a record that would end past block c: a stop here -- its exit
            // and those of the chains through it are not entries of block c)
            const uint64_t lim = min<uint64_t>(p1 + kSB, a.W);
            for (uint32_t i = tid; i < kSB; i += kBlock) {
                const uint64_t p = p0 + i;
                uint32_t v = kJStop;
                if (filter(a, rd, p)) {
                    bool bad;
                    const uint64_t q = parse_near(a, rd, p, lim, &bad);
                    if (!bad) v = static_cast<uint32_t>(q - p0);
                }
                L.u.J[i] = v;
            }
            __syncthreads();
            // pointer jumping: a link inside the block is replaced by its
            // target's (a concurrent reader sees either, both on one chain)
            for (uint32_t r = 0; r < 32; ++r) {
                bool more = false;
                for (uint32_t i = tid; i < kSB; i += kBlock) {
                    uint32_t v = L.u.J[i];
                    if (v < kSB) {
                        v = L.u.J[v];
                        L.u.J[i] = v;
                        more |= v < kSB;
                    }
                }
                if (!__syncthreads_or(more)) break;
            }
            // the distinct exits into block c, a bit per position.  Most
            // positions share a few exits (chains converge): the lanes of a
            // wave holding one value elect one of them, and a bit already set
            // is not set again (an atomic per position on one LDS word
            // serialised the whole block: ~1 ms a block on zero-heavy bytes)
            for (uint32_t i = tid; i < kSB; i += kBlock) {
                const uint32_t v0 = L.u.J[i];
                // an exit into block c, as its offset there + 1 (0: none)
                uint32_t v = v0 == kJStop || v0 < kSB || v0 >= 2 * kSB || p0 + v0 >= a.W ? 0u : v0 - kSB + 1;
                for (uint64_t act = __ballot(v != 0); act; act = __ballot(v != 0)) {
                    const uint32_t lv = __builtin_amdgcn_readlane(v, __builtin_ctzll(act));
                    const uint64_t mine = __ballot(v == lv);
                    if (v == lv && lane == static_cast<uint32_t>(__builtin_ctzll(mine))) {
                        const uint32_t o = lv - 1, wi = o >> 5, bit = 1u << (o & 31);
                        if (!(L.cand[wi] & bit)) atomicOr(&L.cand[wi], bit);
                    }
                    if (v == lv) v = 0;
                }
            }
            __syncthreads();
        }
        const uint32_t any = __syncthreads_or(L.cand[tid] != 0);  // (also: the stage is free)
        if (!any) {
            if (tid == 0) S.hdr[kHdr * c + 5] = 0;
            __syncthreads();
            continue;
        }
        // ---- block c: the candidates its table does not hold, their chains
        const uint64_t b0 = c * kSB, b1 = min<uint64_t>(b0 + kSB, a.W);
        const uint64_t* h = S.hdr + kHdr * c;
        const uint64_t h0 = h[0], h1 = h[1], h3 = h[3], h4 = h[4];
        const uint32_t meta = static_cast<uint32_t>(h[2]), nx = nx_used(a, h4);
        for (uint32_t i = tid; i < nx; i += kBlock) L.xs[i] = S.xp[c * kX + i];
        const StagedRd rd = stage_block(a, w, L.st, L.pre, b0, b1);  // (ends in a barrier)
        // the chunks from phase 1's (repaired) starts, linked into segments
        const uint64_t clo = b0 + static_cast<uint64_t>(tid) * kSC, chi = min<uint64_t>(clo + kSC, b1);
        const uint8_t sb = clo < b1 ? S.spec[c * kBlock + tid] : kNoSpec;
        const uint64_t sp = sb == kNoSpec ? ~0ull : clo + sb;
        uint64_t cch[kMaxNC + 1] = {};
        uint32_t ccnt, cstop;
        uint64_t cexit;
        walk_chunk<NC>(a, rd, sp, chi, &ccnt, &cexit, cch, &cstop, nullptr);
        Chunks<NC>& C = L.u.c;
        C.start[tid] = sp == ~0ull ? kNoStart : static_cast<uint16_t>(sp - b0);
        C.exit[tid] = cexit;
        C.stop[tid] = static_cast<uint8_t>(cstop);
        const uint64_t hm = __ballot(sp != ~0ull);
        if (lane == 0) C.has[tid >> 6] = hm;
        __syncthreads();
        link_chunks<NC>(C, b0, sp, cexit, cstop, ccnt, cch);  // (ends in a barrier)
        // the live exits (a record parses there: read from this block's
        // stage) its table does not hold
        uint32_t m = L.cand[tid], keep = 0;
        while (m) {
            const uint32_t bit = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t o = 32 * tid + bit;
            if (live_at(a, rd, b0 + o) && find_slot(a, h0, h1, h3, meta, h4, 0, L.xs, b0, b0 + o).idx < 0)
                keep |= 1u << bit;
        }
        uint64_t tot;
        uint64_t k = block_xscan(__builtin_popcount(keep), &tot, L.ws);
        while (keep) {
            const uint32_t bit = __builtin_ctz(keep);
            keep &= keep - 1;
            if (k < kE) L.xs[kX + k] = static_cast<uint16_t>(32 * tid + bit);
            ++k;
        }
        __syncthreads();
        const uint32_t nu = static_cast<uint32_t>(min<uint64_t>(tot, kE));
        const bool zf = ((meta >> 17) & 1) && NC < 3;  // a mostly-zero block: chains cross zero runs by its map
        if (zf) build_zmap(rd, b0, L.zm);
        for (uint32_t j = tid; j < nu; j += kBlock) {
            const uint32_t o = L.xs[kX + j];
            st_store<NC>(S.ent + (c * kEnt + kWin + 1 + kX + j) * ew<NC>(),
                         zf ? walk_chain<NC, false, true>(a, rd, C, b0, b1, b0 + o, nullptr, nullptr, L.zm)
                            : walk_chain<NC, false>(a, rd, C, b0, b1, b0 + o, nullptr, nullptr));
            S.ep[c * kE + j] = static_cast<uint16_t>(o);
        }
        if (tid == 0) {
            const bool over = tot > kE;
            S.hdr[kHdr * c + 5] = nu | (over ? 1u << 8 : 0u);
            if (over) atomicAdd(reinterpret_cast<unsigned long long*>(&S.ctl[kCtlOver]), 1ull);
        }
        __syncthreads();  // (the next block's stage overwrites this one's LDS)
    }
}

// ---- phase 2: the scan of the tables ----------------------------------------------
// A block's header and its first kKeep table entries, one block per lane;
// and the runs of primary links: lane j's primary chain (from its block's
// first speculated start h1) leaves the block exactly at block j + 1's, so a
// cursor entering block j at its primary crosses blocks j .. run[j] by adding
// the primary chains' records and chars (inclusive prefix sums over the lanes).
template <int NC>
struct Held {
    uint64_t h0, h1, h3, h4, h5;
    uint32_t meta;  // slots | primary << 8
    uint64_t e[kKeep][ew<NC>()];
    bool has_prim;
    St<NC> pe;                          // the primary slot's chain
    uint64_t icnt, ich[kMaxNC + 1];     // inclusive prefix over lanes of pe.cnt / pe.ch
    uint32_t run;                       // the last block of the run of primary links from this one
    __device__ __forceinline__ void load(const SxScratch& S, uint64_t blk, bool ok, uint32_t nbk) {
        const uint32_t lane = threadIdx.x & 63;
        h0 = h4 = h5 = 0;
        h1 = h3 = ~0ull;
        meta = 0;
        has_prim = false;
        pe = St<NC>{};
        if (ok) {
            const uint64_t* h = S.hdr + kHdr * blk;
            h0 = h[0];
            h1 = h[1];
            h3 = h[3];
            h4 = h[4];
            h5 = h[5];
            meta = static_cast<uint32_t>(h[2]);
            const uint32_t ns = meta & 0xff, prim = (meta >> 8) & 0xff;
#pragma unroll
            for (int k = 0; k < kKeep; ++k)
                if (static_cast<uint32_t>(k) < ns)
#pragma unroll
                    for (uint32_t j = 0; j < ew<NC>(); ++j) e[k][j] = S.ent[(blk * kEnt + k) * ew<NC>() + j];
            if (prim != kNoPrim) {
                has_prim = true;
                pe = st_load<NC>(S.ent + (blk * kEnt + prim) * ew<NC>());
            }
        }
        const uint64_t next_p = __shfl_down(h1, 1, 64);
        const uint32_t next_has = __shfl_down(static_cast<uint32_t>(has_prim), 1, 64);
        const bool link = has_prim && lane + 1 < nbk && next_has && !(pe.stop & 1) && pe.x == next_p;
        const uint64_t lmask = __ballot(link);
        const uint64_t rest = ~lmask & (~0ull << lane);
        run = min<uint32_t>(rest ? __builtin_ctzll(rest) : 63, nbk ? nbk - 1 : 0);
        icnt = has_prim ? pe.cnt : 0;
#pragma unroll
        for (int k = 0; k < NC; ++k) ich[k] = has_prim ? pe.ch[k] : 0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(icnt, d, 64);
            if (lane >= static_cast<uint32_t>(d)) icnt += y;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                const uint64_t z = __shfl_up(ich[k], d, 64);
                if (lane >= static_cast<uint32_t>(d)) ich[k] += z;
            }
        }
    }
    // A cursor entering block j (a uniform lane) at its primary start crosses
    // blocks j .. run[j] at once (per lane: `mine` says which lanes move).
    __device__ __forceinline__ void jump(uint32_t j, St<NC>& s, bool mine) const {
        if (!__ballot(mine)) return;
        const uint32_t m = __builtin_amdgcn_readlane(run, j);
        const uint64_t ex_cnt = rl64(icnt, j) - rl64(has_prim ? pe.cnt : 0, j);
        const uint64_t in_cnt = rl64(icnt, m);
        uint64_t dch[kMaxNC + 1];
#pragma unroll
        for (int k = 0; k < NC; ++k) dch[k] = rl64(ich[k], m) - (rl64(ich[k], j) - rl64(has_prim ? pe.ch[k] : 0, j));
        const uint64_t x = rl64(pe.x, m);
        const uint32_t stp = __builtin_amdgcn_readlane(pe.stop, m);
        if (mine) {
            s.cnt += in_cnt - ex_cnt;
#pragma unroll
            for (int k = 0; k < NC; ++k) s.ch[k] += dch[k];
            s.x = x;
            s.stop = stp;
        }
    }
};

// The cursor's state s through block blk (held in lane l of hv; uniform
// across the wave or per lane), or, past the held entries, from scratch;
// in no slot: walked from global memory.  *miss / *off count what happened.
// xs: the wave's LDS room for the block's landing slots.
template <int NC>
__device__ __forceinline__ void through_block(const SxArgs& a, const uint8_t* w, const SxScratch& S,
                                              const Held<NC>& hv, uint32_t l, uint64_t blk, St<NC>& s, bool* miss,
                                              bool* off, uint8_t* stage, Chunks<NC>* mc, uint16_t* xs,
                                              bool may_walk = true) {
    // the held words of lane l (uniform reads, every lane takes part)
    const uint64_t h0 = rl64(hv.h0, l), h1 = rl64(hv.h1, l), h3 = rl64(hv.h3, l), h4 = rl64(hv.h4, l);
    const uint64_t h5 = rl64(hv.h5, l);
    const uint32_t meta = __builtin_amdgcn_readlane(hv.meta, l);
    uint64_t e[kKeep][ew<NC>()];
#pragma unroll
    for (int k = 0; k < kKeep; ++k)
#pragma unroll
        for (uint32_t j = 0; j < ew<NC>(); ++j) e[k][j] = rl64(hv.e[k][j], l);
    const uint64_t b0 = blk * kSB, b1 = min<uint64_t>(b0 + kSB, a.W);
    // a block no record starts in (the cursor is past its end) passes the state on
    const bool act = !st_done(s, a.W) && s.x < b1;
    if (__ballot(act)) stage_xs(S, blk, nx_used(a, h4), h5_ne(h5), xs);
    const Slot sl = act ? find_slot(a, h0, h1, h3, meta, h4, h5, xs, b0, s.x) : Slot{0, 0};
    const bool walk = act && sl.idx < 0 && may_walk;
    // every lane of the wave takes part in the staging of walk_miss
    St<NC> mw{};
    if (__ballot(walk)) mw = walk_miss<NC>(a, w, S, blk, stage, *mc, b0, b1, s.x, walk);
    if (act && sl.idx < 0 && !may_walk) {  // a chain the caller gives up on instead of walking it
        s.stop = kDead;
        return;
    }
    if (!act) return;
    St<NC> t;
    if (sl.idx >= 0 && sl.idx < kKeep) {
        uint64_t v[ew<NC>()];
#pragma unroll
        for (uint32_t j = 0; j < ew<NC>(); ++j) {
            v[j] = e[0][j];
#pragma unroll
            for (int k = 1; k < kKeep; ++k) v[j] = sl.idx == k ? e[k][j] : v[j];
        }
        t = st_load<NC>(v);
        t.cnt -= sl.sub;
    } else if (sl.idx >= 0) {
        t = st_load<NC>(S.ent + (blk * kEnt + sl.idx) * ew<NC>());
        t.cnt -= sl.sub;
    } else {
        t = mw;
        *miss = true;
    }
    if (sl.idx != static_cast<int>((meta >> 8) & 0xff) || sl.sub) *off = true;
    st_add<NC>(s, t);
}

// A wave per group: for every slot of the group's first block -- window
// slots, the extra slot, landing slots, exit slots -- the chain through the
// group's blocks (the group's table, indexed like the first block's).  A
// chain that meets a position no table holds is given up (kDead): in the
// first scan (pass 0) every such chain -- the cursor that meets one sends the
// call through the repair pass, which makes such positions slots -- and in
// the second (pass 1, only after a repair) every chain but the primary
// slot's, which is walked (a start the block speculated wrongly that runs
// into positions no table holds would otherwise cost a walk in every later
// block, and the cursor enters a group there rarely: k_sx_top then takes
// that group block by block).  Test-hook mode 8 (no repair): pass 0 walks the
// primary chains, as pass 1 does.
// A wave's LDS for sx_group's shared continuations (below).
template <int NC>
struct GroupDedup {
    uint64_t ux[64];             // distinct positions the group's chains continue from after its first block
    uint64_t res[64][2 + kMaxNC];  // each one's chain through the rest of the group (St words)
    uint64_t prim;               // which of them the primary slot's chain continues from
    uint32_t nd;
};

// One wave: group g's table (k_sx_groups).  With more than 64 slots (a
// block the repair pass gave exit slots), the chains of the first block's
// slots mostly meet again where they leave it: their states after the first
// block go to the group table, the distinct positions they continue from are
// walked once each through the rest of the group (rounds of 64), and each
// slot's entry is its first-block state plus its continuation's -- instead of
// a batch of 64 chains walked through all 64 blocks per 64 slots (a group of
// 321 slots cost ~360 us).
template <int NC>
__device__ void sx_group(const SxArgs& a, const uint8_t* __restrict__ w, const SxScratch& S, uint32_t pass,
                         uint64_t g, uint8_t* stage, Chunks<NC>& mch, uint16_t* xs, GroupDedup<NC>& D) {
    const bool walk_prim = pass || (a.mode & 8);
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t bf = g * kGroup;
    const uint32_t nbk = static_cast<uint32_t>(min<uint64_t>(kGroup, a.nb - bf));
    Held<NC> hv;
    hv.load(S, bf + lane, lane < nbk, nbk);
    const uint32_t meta0 = __builtin_amdgcn_readlane(hv.meta, 0);
    const uint32_t ns0 = meta0 & 0xff, prim0 = (meta0 >> 8) & 0xff;
    const bool has3 = rl64(hv.h3, 0) != ~0ull;
    const uint32_t nx0 = nx_used(a, rl64(hv.h4, 0)), ne0 = h5_ne(rl64(hv.h5, 0));
    const uint32_t total = ns0 + (has3 ? 1 : 0) + nx0 + ne0;
    constexpr uint32_t E = ew<NC>();
    bool miss = false, off = false;
    uint64_t* q = S.gp + g * (kHdr + E);
    // lane -> slot index: window slots, the extra slot, the landing slots, the exit slots
    auto slot_idx = [&](uint32_t k) -> uint32_t {
        if (k < ns0) return k;
        const uint32_t r = k - ns0 - (has3 ? 1 : 0);  // (for k past the extra slot)
        return has3 && k == ns0 ? kWin : r < nx0 ? kWin + 1 + r : kWin + 1 + kX + (r - nx0);
    };
    // the chain state s through blocks 1 .. nbk - 1 of the group (per lane)
    auto through_rest = [&](St<NC>& s, bool act, bool may) {
        for (uint32_t j = 1; j < nbk; ++j) {
            // chains entering block j at its primary cross its whole run at once
            const bool hp = __builtin_amdgcn_readlane(static_cast<uint32_t>(hv.has_prim), j);
            if (hp) hv.jump(j, s, act && !st_done(s, a.W) && s.x == rl64(hv.h1, j));
            const uint64_t b1 = min<uint64_t>((bf + j + 1) * kSB, a.W);
            if (!__ballot(act && !st_done(s, a.W) && s.x < b1)) continue;  // every chain is past block j
            St<NC> t = s;
            through_block<NC>(a, w, S, hv, j, bf + j, t, &miss, &off, stage, &mch, xs, may);
            if (act) s = t;
        }
    };
    if (total <= 64) {
        const uint32_t k = lane;
        const bool act = k < total;
        const uint32_t idx = slot_idx(k);
        St<NC> s{};
        s.stop = 1;  // lanes past the slots stay put
        if (act) s = st_load<NC>(S.ent + (bf * kEnt + idx) * E);
        const bool primary = act && idx == prim0;
        through_rest(s, act, primary && walk_prim);
        if (act) st_store<NC>(S.gent + (g * kEnt + idx) * E, s);
        if (primary) st_store<NC>(q + kHdr, s);  // what the in-order pass reads first
    } else {
        const uint64_t gend = min<uint64_t>((bf + nbk) * kSB, a.W);
        auto pending = [&](const St<NC>& s) { return !st_done(s, a.W) && s.x < gend; };
        // every slot's state after the first block
        for (uint32_t k0 = 0; k0 < total; k0 += 64) {
            const uint32_t k = k0 + lane;
            if (k >= total) continue;
            const uint32_t idx = slot_idx(k);
            const St<NC> s = st_load<NC>(S.ent + (bf * kEnt + idx) * E);
            st_store<NC>(S.gent + (g * kEnt + idx) * E, s);
            if (idx == prim0 && !pending(s)) st_store<NC>(q + kHdr, s);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        for (;;) {
            // up to 64 distinct continuation positions of the slots still pending
            if (lane == 0) {
                D.nd = 0;
                D.prim = 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            bool any = false;
            for (uint32_t k0 = 0; k0 < total; k0 += 64) {
                const uint32_t k = k0 + lane;
                const uint32_t idx = slot_idx(k);
                St<NC> s{};
                bool pend = false;
                if (k < total) {
                    s = st_load<NC>(S.gent + (g * kEnt + idx) * E);
                    pend = pending(s);
                }
                any = any || __ballot(pend);
                uint64_t left = __ballot(pend);
                while (left) {
                    const uint64_t lx = rl64(s.x, __builtin_ctzll(left));
                    const uint64_t same = __ballot(pend && s.x == lx);
                    const uint32_t nd = D.nd;
                    uint32_t d = nd;
                    for (uint32_t i = 0; i < nd; ++i)
                        if (D.ux[i] == lx) d = i;
                    if (d == nd && nd < 64 && lane == 0) {
                        D.ux[nd] = lx;
                        D.nd = nd + 1;
                    }
                    if (d < 64 && __ballot(pend && s.x == lx && idx == prim0) && lane == 0) D.prim |= 1ull << d;
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
                    left &= ~same;
                }
            }
            if (!any) break;
            // each distinct position's chain through the rest of the group
            const uint32_t nd = D.nd;
            {
                const bool act = lane < nd;
                St<NC> r{};
                r.x = act ? D.ux[lane] : 0;
                r.stop = act ? 0u : 1u;
                through_rest(r, act, act && ((D.prim >> lane) & 1) && walk_prim);
                if (act) st_store<NC>(D.res[lane], r);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
            // every pending slot that continues from one of them: its state plus that chain
            for (uint32_t k0 = 0; k0 < total; k0 += 64) {
                const uint32_t k = k0 + lane;
                if (k >= total) continue;
                const uint32_t idx = slot_idx(k);
                St<NC> s = st_load<NC>(S.gent + (g * kEnt + idx) * E);
                if (!pending(s)) continue;
                uint32_t d = nd;
                for (uint32_t i = 0; i < nd; ++i)
                    if (D.ux[i] == s.x) d = i;
                if (d == nd) continue;  // (a later round)
                st_add<NC>(s, st_load<NC>(D.res[d]));
                st_store<NC>(S.gent + (g * kEnt + idx) * E, s);
                if (idx == prim0) st_store<NC>(q + kHdr, s);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        }
    }
    // the first block's header words, with the primary chain above: one record
    if (lane < 6) {
        const uint64_t hw[6] = {rl64(hv.h0, 0), rl64(hv.h1, 0), meta0, rl64(hv.h3, 0), rl64(hv.h4, 0), rl64(hv.h5, 0)};
        uint64_t v = hw[0];
#pragma unroll
        for (uint32_t i = 1; i < 6; ++i) v = lane == i ? hw[i] : v;
        q[lane] = v;
    }
}

// One wave: the groups in order.  Each group's entry state (the cursor where
// the group starts) goes to gin; the group's table entry for the cursor's
// position is taken from registers (its primary slot) or scratch; a position
// in no slot of the group's first block, or past that block, takes the group
// block by block.  Then the stream's end: T, rec_offs[T], str_offs[.][T], the
// status and the tail fill's parameters for k_sx_decode.
// Pass 0 walks nothing: at the first position no table holds (or a group
// chain given up there) it asks for the repair pass (ctl kCtlRepair) and
// ends, writing nothing; pass 1 runs only after a repair and walks what is
// still missing (a block whose exit slots overflowed).  Mode 8: pass 0 walks.
// Run by one wave: the last workgroup of k_sx_groups to finish (its wave 0,
// with that wave's LDS), or k_sx_top where there are no groups.
template <int NC, bool kDecode>
__device__ void sx_top(const SxArgs& a, const uint8_t* __restrict__ w, const SxScratch& S, srpc_unpack_status* st,
                       uint32_t pass, uint8_t* stage, Chunks<NC>& mch, uint16_t* xs) {
    const bool may_walk = pass || (a.mode & 8);
    constexpr uint32_t E = ew<NC>();
    constexpr uint32_t R = kHdr + E;  // words of a group's record in S.gp
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = a.W;
    St<NC> s{};
    bool miss = false, off = false;
    // lane l: group base + l -- its first block's header and the group's
    // primary entry (S.gp), the next batch's loaded while this one is walked
    uint64_t nq[R];
    auto fetch = [&](uint64_t base) {
        const uint64_t g = base + lane;
#pragma unroll
        for (uint32_t j = 0; j < R; ++j) nq[j] = g < a.ng && (j < 6 || j >= kHdr) ? S.gp[g * R + j] : 0;
    };
    fetch(0);
    for (uint64_t base = 0; base < a.ng; base += 64) {
        const uint32_t cnt = static_cast<uint32_t>(min<uint64_t>(64, a.ng - base));
        const uint64_t g = base + lane;
        const uint64_t h0 = nq[0], h1 = nq[1], h3 = nq[3], h4 = nq[4], h5 = nq[5];
        const uint32_t meta = static_cast<uint32_t>(nq[2]);
        St<NC> pe = st_load<NC>(nq + kHdr);  // the group's chain from its primary slot (its first block's sF = h1)
        fetch(base + 64);
        const bool has_prim = lane < cnt && ((meta >> 8) & 0xff) != kNoPrim;
        // link k -> k + 1: group k's primary chain enters group k + 1 at its primary
        const uint64_t next_p = __shfl_down(h1, 1, 64);
        const uint32_t next_has = __shfl_down(static_cast<uint32_t>(has_prim), 1, 64);
        const bool link = has_prim && lane + 1 < cnt && next_has && !(pe.stop & 1) && pe.x == next_p;
        const uint64_t lmask = __ballot(link);
        // inclusive prefix sums over the batch of the primary chains' records and chars
        uint64_t icnt = has_prim ? pe.cnt : 0, ich[kMaxNC + 1];
#pragma unroll
        for (int k = 0; k < NC; ++k) ich[k] = has_prim ? pe.ch[k] : 0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(icnt, d, 64);
            if (lane >= static_cast<uint32_t>(d)) icnt += y;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                const uint64_t z = __shfl_up(ich[k], d, 64);
                if (lane >= static_cast<uint32_t>(d)) ich[k] += z;
            }
        }
        uint64_t in[E];
        uint32_t l = 0;
        while (l < cnt) {
            const uint64_t gl = base + l;
            const uint64_t lh0 = rl64(h0, l), lh1 = rl64(h1, l), lh3 = rl64(h3, l), lh4 = rl64(h4, l);
            const uint64_t lh5 = rl64(h5, l);
            const uint32_t lmeta = __builtin_amdgcn_readlane(meta, l);
            const uint32_t lprim = (lmeta >> 8) & 0xff;
            if (!st_done(s, W) && lprim != kNoPrim && s.x == lh1) {
                // a run of groups entered at their primaries: l .. m, m the first
                // group whose primary chain does not lead to the next one's
                const uint64_t rest = ~lmask & (~0ull << l);
                const uint32_t m = min<uint32_t>(rest ? __builtin_ctzll(rest) : 63, cnt - 1);
                // group k in l..m starts at its primary with the records / chars
                // of the runs before it: s + (exclusive prefix at k - at l)
                const uint64_t ex_l_cnt = rl64(icnt, l) - rl64(has_prim ? pe.cnt : 0, l);
                uint64_t ex_l_ch[kMaxNC + 1];
#pragma unroll
                for (int k = 0; k < NC; ++k) ex_l_ch[k] = rl64(ich[k], l) - rl64(has_prim ? pe.ch[k] : 0, l);
                if (lane >= l && lane <= m) {
                    St<NC> v{};
                    v.x = h1;
                    v.cnt = s.cnt + (icnt - pe.cnt) - ex_l_cnt;
#pragma unroll
                    for (int k = 0; k < NC; ++k) v.ch[k] = s.ch[k] + (ich[k] - pe.ch[k]) - ex_l_ch[k];
                    v.stop = 0;
                    st_store<NC>(in, v);
                }
                St<NC> t{};
                t.x = rl64(pe.x, m);
                t.cnt = s.cnt + rl64(icnt, m) - ex_l_cnt;
#pragma unroll
                for (int k = 0; k < NC; ++k) t.ch[k] = s.ch[k] + rl64(ich[k], m) - ex_l_ch[k];
                t.stop = __builtin_amdgcn_readlane(pe.stop, m);
                s = t;
                l = m + 1;
                if (!may_walk && s.stop == kDead) {  // a primary chain given up: repair first
                    if (lane == 0) S.ctl[kCtlRepair] = 1;
                    return;
                }
                continue;
            }
            {
                uint64_t v[E];
                st_store<NC>(v, s);
#pragma unroll
                for (uint32_t j = 0; j < E; ++j) in[j] = lane == l ? v[j] : in[j];
            }
            ++l;
            if (st_done(s, W)) continue;
            const uint64_t bf = gl * kGroup;
            const uint64_t bend = min<uint64_t>(bf + kGroup, a.nb);
            if (s.x >= min<uint64_t>(bend * kSB, W)) continue;  // the whole group lies inside one record
            const uint64_t blk = s.x / kSB;
            if (blk == bf) {
                stage_xs(S, bf, nx_used(a, lh4), h5_ne(lh5), xs);
                const Slot sl = find_slot(a, lh0, lh1, lh3, lmeta, lh4, lh5, xs, bf * kSB, s.x);
                if (sl.idx >= 0) {
                    St<NC> e = st_load<NC>(S.gent + (gl * kEnt + sl.idx) * E);
                    if (e.stop != kDead) {  // (the primary slot's is taken above)
                        off = true;
                        e.cnt -= sl.sub;
                        st_add<NC>(s, e);
                        continue;
                    }
                }
            }
            // block by block from the cursor's block to the group's end
            for (uint64_t j = blk; j < bend && !st_done(s, W); ++j) {
                const uint64_t b0 = j * kSB, b1 = min<uint64_t>(b0 + kSB, W);
                if (s.x >= b1) continue;
                const uint64_t* h = S.hdr + kHdr * j;
                const uint64_t m = h[2], hj4 = h[4], hj5 = h[5];
                stage_xs(S, j, nx_used(a, hj4), h5_ne(hj5), xs);
                const Slot sl = find_slot(a, h[0], h[1], h[3], static_cast<uint32_t>(m), hj4, hj5, xs, b0, s.x);
                if (sl.idx != static_cast<int>((m >> 8) & 0xff) || sl.sub) off = true;
                if (sl.idx >= 0) {
                    St<NC> t = st_load<NC>(S.ent + (j * kEnt + sl.idx) * E);
                    t.cnt -= sl.sub;
                    st_add<NC>(s, t);
                } else {
                    if (!may_walk) {  // a position no table holds: repair first
                        if (lane == 0) S.ctl[kCtlRepair] = 1;
                        return;
                    }
                    st_add<NC>(s, walk_miss<NC>(a, w, S, j, stage, mch, b0, b1, s.x, true));
                    miss = true;
                }
            }
        }
        if (lane < cnt)
#pragma unroll
            for (uint32_t j = 0; j < E; ++j) S.gin[g * E + j] = in[j];
    }
    if (lane != 0) return;
    if (miss) atomicAdd(reinterpret_cast<unsigned long long*>(&S.ctl[kCtlMiss]), 1ull);
    if (off) atomicAdd(reinterpret_cast<unsigned long long*>(&S.ctl[kCtlOff]), 1ull);
    // the stream's end: s.cnt records decode; record T = s.cnt fails (or the wire ends)
    const uint64_t n = a.n, T = s.cnt;
    if (kDecode && st && T >= n) {
        st->flags = 0;
        st->first_bad_record = ~0ull;
    }
    if (T > n) return;  // record n starts in a block: k_sx_decode writes index n
    uint64_t tot[kMaxNC + 1];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        tot[k] = s.ch[k];
        sum += s.ch[k];
    }
    // the last string field: every byte before s.x is a fixed part or chars
    tot[NC] = s.x - T * a.fixed_bytes - sum;
    a.rec_offs[T] = s.x;
    if (kDecode)
        for (uint32_t f = 0; f < a.nfields; ++f) {
            if (a.size[f]) continue;
            const uint32_t si = a.sord[f];
            uint64_t v = 0;
#pragma unroll
            for (int k = 0; k <= NC; ++k) v = si == static_cast<uint32_t>(k) ? tot[k] : v;
            a.soff[f][T] = v;
            S.ctl[kCtlTot + si] = v;
        }
    if (T < n) {
        S.ctl[kCtlT] = T;
        S.ctl[kCtlTailOn] = 1;
        if (kDecode && st) {
            const uint32_t kind = (s.stop & 1) ? (s.stop >> 1) & 3 : 0;
            st->flags = (kind ? kind : SRPC_STATUS_BOUNDS) | (T + 1 < n ? SRPC_STATUS_BOUNDS : 0);
            st->first_bad_record = T;
        }
    }
}

template <int NC, bool kDecode>
__global__ __launch_bounds__(kBlock) void k_sx_groups(SxArgs a, const uint8_t* __restrict__ w, SxScratch S,
                                                      srpc_unpack_status* st, uint32_t pass) {
    if (pass && !S.ctl[kCtlRepair]) return;  // (the second scan runs only after a repair)
    __shared__ __attribute__((aligned(16))) uint8_t stages[kBlock / 64][kWaveStage + 16];
    __shared__ uint16_t xss[kBlock / 64][kXS];
    __shared__ Chunks<NC> mchs[kBlock / 64];  // walk_miss's chunks, one set per wave
    __shared__ GroupDedup<NC> dds[kBlock / 64];
    __shared__ uint32_t s_last;
    const uint64_t g = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + (threadIdx.x >> 6);
    if (g < a.ng) sx_group<NC>(a, w, S, pass, g, stages[threadIdx.x >> 6], mchs[threadIdx.x >> 6],
                               xss[threadIdx.x >> 6], dds[threadIdx.x >> 6]);
    // the last workgroup to finish runs the in-order scan (no waiting: the
    // others have ended; their tables are published by the fences)
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = atomicAdd(reinterpret_cast<unsigned long long*>(&S.ctl[kCtlDone + pass]), 1ull) == gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    if (threadIdx.x < 64) sx_top<NC, kDecode>(a, w, S, st, pass, stages[0], mchs[0], xss[0]);
}

template <int NC, bool kDecode>
__global__ __launch_bounds__(64) void k_sx_top(SxArgs a, const uint8_t* __restrict__ w, SxScratch S,
                                               srpc_unpack_status* st, uint32_t pass) {
    if (pass && !S.ctl[kCtlRepair]) return;
    __shared__ __attribute__((aligned(16))) uint8_t stage[kWaveStage + 16];
    __shared__ Chunks<NC> mch;  // walk_miss's chunks
    __shared__ uint16_t xs[kXS];
    sx_top<NC, kDecode>(a, w, S, st, pass, stage, mch, xs);
}

// One wave: every block's entry state of group g, from the group's.
template <int NC>
__device__ void sx_blocks_group(const SxArgs& a, const uint8_t* __restrict__ w, const SxScratch& S, uint64_t g,
                                uint8_t* stage, Chunks<NC>& mch, uint16_t* xs) {
    constexpr uint32_t E = ew<NC>();
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t bf = g * kGroup;
    const uint32_t nbk = static_cast<uint32_t>(min<uint64_t>(kGroup, a.nb - bf));
    Held<NC> hv;
    hv.load(S, bf + lane, lane < nbk, nbk);
    St<NC> s = st_load<NC>(S.gin + g * E);
    uint64_t out[E];
    bool miss = false, off = false;
    for (uint32_t j = 0; j < nbk;) {
        const bool hp = __builtin_amdgcn_readlane(static_cast<uint32_t>(hv.has_prim), j);
        if (hp && !st_done(s, a.W) && s.x == rl64(hv.h1, j)) {
            // entering block j at its primary: blocks j .. run[j] in one step,
            // each block k of the run entered at its primary with the records
            // and chars of the run's blocks before it
            const uint32_t m = __builtin_amdgcn_readlane(hv.run, j);
            const uint64_t ex_cnt = rl64(hv.icnt, j) - rl64(hv.has_prim ? hv.pe.cnt : 0, j);
            uint64_t ex_ch[kMaxNC + 1];
#pragma unroll
            for (int k = 0; k < NC; ++k) ex_ch[k] = rl64(hv.ich[k], j) - rl64(hv.has_prim ? hv.pe.ch[k] : 0, j);
            if (lane >= j && lane <= m) {
                St<NC> v{};
                v.x = hv.h1;
                v.cnt = s.cnt + (hv.icnt - hv.pe.cnt) - ex_cnt;
#pragma unroll
                for (int k = 0; k < NC; ++k) v.ch[k] = s.ch[k] + (hv.ich[k] - hv.pe.ch[k]) - ex_ch[k];
                v.stop = 0;
                st_store<NC>(out, v);
            }
            hv.jump(j, s, true);
            j = m + 1;
            continue;
        }
        uint64_t v[E];
        st_store<NC>(v, s);
#pragma unroll
        for (uint32_t k = 0; k < E; ++k) out[k] = lane == j ? v[k] : out[k];
        through_block<NC>(a, w, S, hv, j, bf + j, s, &miss, &off, stage, &mch, xs);
        ++j;
    }
    if (lane < nbk)
#pragma unroll
        for (uint32_t k = 0; k < E; ++k) S.bst[(bf + lane) * E + k] = out[k];
    if (lane == 0 && miss) atomicAdd(reinterpret_cast<unsigned long long*>(&S.ctl[kCtlMiss]), 1ull);
    if (lane == 0 && off) atomicAdd(reinterpret_cast<unsigned long long*>(&S.ctl[kCtlOff]), 1ull);
}

// A wave per group: every block's entry state (sx_blocks_group).
template <int NC>
__global__ __launch_bounds__(kBlock) void k_sx_blocks(SxArgs a, const uint8_t* __restrict__ w, SxScratch S) {
    __shared__ __attribute__((aligned(16))) uint8_t stages[kBlock / 64][kWaveStage + 16];
    __shared__ uint16_t xss[kBlock / 64][kXS];
    __shared__ Chunks<NC> mchs[kBlock / 64];  // walk_miss's chunks, one set per wave
    const uint32_t wv = threadIdx.x >> 6;
    const uint64_t g = static_cast<uint64_t>(blockIdx.x) * (kBlock / 64) + wv;
    if (g < a.ng) sx_blocks_group<NC>(a, w, S, g, stages[wv], mchs[wv], xss[wv]);
}

// ---- phase 3: the records of every block ----------------------------------------
// len bytes of the wire at p -> d, by `lanes` lanes (this one `lane`):
// aligned 16-byte stores built from aligned dword loads (funnel shifts), the
// unaligned head and tail of d byte by byte (lanes 0 and 1, or lane 0 alone);
// never a load past the wire's W bytes.
__device__ __forceinline__ void copy_global(uint8_t* d, const uint8_t* w, uint64_t p, uint64_t len, uint64_t W,
                                            uint32_t lane, uint32_t lanes) {
    const uint64_t a0 = min<uint64_t>(len, (16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15);
    const uint64_t n16 = (len - a0) >> 4, t0 = a0 + 16 * n16;
    if (lane == 0)
#pragma nounroll
        for (uint64_t x = 0; x < a0; ++x) d[x] = w[p + x];
    if (lane == (lanes > 1 ? 1u : 0u))
#pragma nounroll
        for (uint64_t x = t0; x < len; ++x) d[x] = w[p + x];
    const uintptr_t wend = reinterpret_cast<uintptr_t>(w + W);
    for (uint64_t c = lane; c < n16; c += lanes) {
        const uint8_t* px = w + p + a0 + 16 * c;
        const uintptr_t ax = reinterpret_cast<uintptr_t>(px) & ~uintptr_t{3};
        uint8_t* dx = d + a0 + 16 * c;
        if (ax + 20 <= wend) {
            const uint32_t* q = reinterpret_cast<const uint32_t*>(ax);
            const uint32_t s3 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(px) & 3);
            const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
            *reinterpret_cast<u32x4*>(dx) =
                u32x4{__builtin_amdgcn_alignbyte(w1, w0, s3), __builtin_amdgcn_alignbyte(w2, w1, s3),
                      __builtin_amdgcn_alignbyte(w3, w2, s3), __builtin_amdgcn_alignbyte(w4, w3, s3)};
        } else {
            for (uint32_t i = 0; i < 16; ++i) dx[i] = px[i];
        }
    }
}

template <int NC>
struct DecLds {
    alignas(16) uint8_t pre[kMaxPrefix + 16];
    alignas(16) uint8_t st[kStage + 16];
    union {
        struct {  // until the block's records are listed in tbl
            Chunks<0> c;
            uint8_t list[kBlock * kListCap];
            uint16_t xl[kMaxRec];  // the chain's explicit starts
        } w;
        struct {  // then, per local record of the string field being copied:
            uint32_t loff[kMaxRec + 1];  // its chars' offset in the block's run of chars
            uint16_t src[kMaxRec];       // where its chars are on the wire, from the block start
                                         // (kFar: 64 KiB or more, found again from the record)
        } s;
    } u;
    alignas(8) uint16_t tbl[kMaxRec + 4];  // the block's records in order: offset from the block
    uint64_t ws[kBlock / 64];
    uint64_t zm[kZW];  // the zero map (zero-heavy blocks only)
    uint32_t far[kFarList];  // lane-per-record copies whose chars run past the stage (a wave each)
    uint32_t s_nexp, nfar;
};

template <int NC, bool kDecode>
__global__ __launch_bounds__(kBlock, 8) void k_sx_decode(SxArgs a, const uint8_t* __restrict__ w, SxScratch S,
                                                      srpc_unpack_status* st) {
    __shared__ DecLds<NC> L;
    constexpr uint32_t E = ew<NC>();
    const uint32_t tid = threadIdx.x;
    const uint64_t b = xcd_block(blockIdx.x, gridDim.x);
    const uint64_t W = a.W, n = a.n;
    // the tail: records T + 1 .. n when the stream stopped before record n
    if (S.ctl[kCtlTailOn]) {
        const uint64_t T = S.ctl[kCtlT];
        const uint64_t gs = static_cast<uint64_t>(gridDim.x) * kBlock;
        for (uint64_t r = T + 1 + b * kBlock + tid; r <= n; r += gs) {
            a.rec_offs[r] = W;
            if (kDecode)
                for (uint32_t f = 0; f < a.nfields; ++f)
                    if (!a.size[f]) a.soff[f][r] = S.ctl[kCtlTot + a.sord[f]];
        }
    }
    if (b == 0 && tid == 0 && st && kDecode) {  // diagnostics (srpc_unpack_status.reserved)
        const uint64_t miss = S.ctl[kCtlMiss], off = S.ctl[kCtlOff], rep = S.ctl[kCtlRepair], ov = S.ctl[kCtlOver];
        st->reserved = (off ? 1u : 0u) | (miss ? 2u : 0u) | (rep ? 4u : 0u) | (ov ? 8u : 0u) |
                       (static_cast<uint32_t>(min<uint64_t>(miss, 0xffffff)) << 8);
    }
    if (b >= a.nb) return;
    const uint64_t b0 = b * kSB, b1 = min<uint64_t>(b0 + kSB, W);
    // the block's state, its chunks' speculated starts and its bytes all in
    // flight at once (a block no record of the batch starts in wastes its stage)
    SXP_BEGIN
    const St<NC> s = st_load<NC>(S.bst + b * E);
    const uint64_t hsF = S.hdr[kHdr * b + 1], hmeta = S.hdr[kHdr * b + 2];
    const uint64_t clo = b0 + static_cast<uint64_t>(tid) * kSC, chi = min<uint64_t>(clo + kSC, b1);
    const uint8_t sb = clo < b1 ? S.spec[b * kBlock + tid] : kNoSpec;
    // the record list's first 256 entries (the fast path's, read before it is
    // known to be taken: one round trip instead of two)
    const uint64_t* rl = reinterpret_cast<const uint64_t*>(S.rl + b * kMaxRec);
    const uint64_t rl0 = tid < 64 ? rl[tid] : 0;
    const StagedRd rd = stage_block(a, w, L.st, L.pre, b0, b1);
    SXP(8);
    const uint64_t x = s.x, R = s.cnt;
    if ((s.stop & 1) || x >= b1 || R > n) return;  // no record of the batch starts here
    Chunks<0>& C = L.u.w.c;
    uint32_t nrec;
    if (((hmeta >> 16) & 1) && x == hsF) {
        // entered at the first speculated start of a block whose chunks form
        // one segment: every chunk's records, in order, are the block's --
        // phase 1 listed them
        nrec = static_cast<uint32_t>((hmeta >> 32) & 0xFFFF);
        if (tid < 64 && 4 * tid < nrec) reinterpret_cast<uint64_t*>(L.tbl)[tid] = rl0;
        for (uint32_t k = 64 + tid; 4 * k < nrec; k += kBlock) reinterpret_cast<uint64_t*>(L.tbl)[k] = rl[k];
        __syncthreads();
        SXP_FLAG(15);
        SXP(9);
        SXP(10);
    } else {
    // every chunk again from its speculated start (phase 1's byte)
    const uint64_t sp = sb == kNoSpec ? ~0ull : clo + sb;
    uint64_t cch[kMaxNC + 1] = {};
    uint32_t ccnt, cstop;
    uint64_t cexit;
    walk_chunk<0>(a, rd, sp, chi, &ccnt, &cexit, cch, &cstop, L.u.w.list + tid * kListCap);
    C.start[tid] = sp == ~0ull ? kNoStart : static_cast<uint16_t>(sp - b0);
    C.exit[tid] = cexit;
    C.stop[tid] = static_cast<uint8_t>(cstop);
    const uint64_t hm = __ballot(sp != ~0ull);
    if ((tid & 63) == 0) C.has[tid >> 6] = hm;
    if (tid < 4) C.jump[tid] = 0;
    __syncthreads();
    SXP(9);
    link_chunks<0>(C, b0, sp, cexit, cstop, ccnt, cch);
    SXP(10);

    // the chain from the block's entry: explicit starts (xl, until the table is
    // built) and the chunks it jumped
    uint16_t* xl = L.u.w.xl;
    const bool zf = (hmeta >> 17) & 1;  // a zero-heavy block (k_sx_spec built its zero map too)
    if (zf) build_zmap(rd, b0, L.zm);
    if (tid == 0) {
        uint32_t ne = 0;
        if (zf) (void)walk_chain<0, true, true>(a, rd, C, b0, b1, x, xl, &ne, L.zm);
        else (void)walk_chain<0, true>(a, rd, C, b0, b1, x, xl, &ne);
        L.s_nexp = ne;
    }
    __syncthreads();
    const uint32_t ne = L.s_nexp;
    // chunk tid: explicit starts inside it (binary search in the ascending
    // list), then its speculated starts if the chain jumped it
    uint32_t e0 = 0, e1 = 0;
    if (ne) {
        const uint32_t lo16 = tid * kSC, hi16 = lo16 + kSC;
        uint32_t l = 0, h = ne;
        while (l < h) {
            const uint32_t m = (l + h) >> 1;
            if (xl[m] < lo16) l = m + 1;
            else h = m;
        }
        e0 = l;
        h = ne;
        while (l < h) {
            const uint32_t m = (l + h) >> 1;
            if (xl[m] < hi16) l = m + 1;
            else h = m;
        }
        e1 = l;
    }
    const bool jumped = (C.jump[tid >> 6] >> (tid & 63)) & 1;
    const uint32_t fc = (e1 - e0) + (jumped ? ccnt : 0);
    uint64_t tot;
    const uint32_t fb = static_cast<uint32_t>(block_xscan(fc, &tot, L.ws));
    for (uint32_t k = e0; k < e1; ++k) L.tbl[fb + (k - e0)] = xl[k];
    if (jumped)
        for (uint32_t k = 0; k < ccnt; ++k)
            L.tbl[fb + (e1 - e0) + k] = static_cast<uint16_t>(tid * kSC + L.u.w.list[tid * kListCap + k]);
    __syncthreads();
    nrec = static_cast<uint32_t>(min<uint64_t>(tot, kMaxRec));
    }
    SXP(11);

    // records r = R + k of the batch, up to index n (record n's start); the
    // first string field's lengths and chars positions on the way (the
    // strings pass below takes them from here)
    uint32_t huge0 = 0;
    for (uint32_t k = tid; k < nrec; k += kBlock) {
        const uint64_t r = R + k;
        if (kDecode && r >= n) L.u.s.loff[k] = 0;  // (no chars: not a record of the batch)
        if (r > n) continue;
        const uint64_t sr = b0 + L.tbl[k];
        a.rec_offs[r] = sr;
        if (!kDecode || r == n) continue;
        uint64_t pos = sr + a.prefix_len;
        for (uint32_t f = 0; f < a.nfields; ++f) {
            const uint32_t sz = a.size[f];
            const uint64_t v = sz ? rd.field(pos, sz) : rd.u64(pos);
            if (sz) {
                uint8_t* dst = a.col[f] + r * sz;
                switch (sz) {
                case 1: dst[0] = static_cast<uint8_t>(v); break;
                case 2: *reinterpret_cast<uint16_t*>(dst) = static_cast<uint16_t>(v); break;
                case 4: *reinterpret_cast<uint32_t*>(dst) = static_cast<uint32_t>(v); break;
                default: *reinterpret_cast<uint64_t*>(dst) = v; break;
                }
                pos += sz;
            } else {
                if (a.sord[f] == 0) {
                    huge0 |= (v >> kHugeLog2) | ((pos + 8 - b0) >> 31) ? 1u : 0u;
                    L.u.s.loff[k] = static_cast<uint32_t>(v);
                    L.u.s.src[k] = static_cast<uint16_t>(min<uint64_t>(pos + 8 - b0, kFar));
                }
                pos += 8 + v;
            }
        }
    }
    SXP(12);
    if constexpr (kDecode) {
        // per string field: local offsets (a scan over the block's records),
        // str_offs, each record's chars copied from the stage by its lane
        uint64_t Pbase[kMaxNC + 1];
        {
            uint64_t sum = 0;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                Pbase[k] = s.ch[k];
                sum += Pbase[k];
            }
            // the last string field: every byte of a record is its fixed part or chars
            Pbase[NC] = x - R * a.fixed_bytes - sum;
        }
        const uint32_t nw = static_cast<uint32_t>(min<uint64_t>(nrec, n - R));  // records written (r < n)
        const uint32_t per = (nrec + kBlock - 1) / kBlock;                    // contiguous records per lane
        for (uint32_t f = 0; f < a.nfields; ++f) {
            if (a.size[f]) continue;
            const uint32_t si = a.sord[f];
            uint64_t P = 0;
#pragma unroll
            for (int k = 0; k <= NC; ++k) P = si == static_cast<uint32_t>(k) ? Pbase[k] : P;
            // this field's length and where its chars are, lane per record
            // (string ordinal 0: from the fixed-field pass)
            uint32_t huge = si == 0 ? huge0 : 0;
            for (uint32_t k = tid; k < nrec && si != 0; k += kBlock) {
                uint64_t pos = b0 + L.tbl[k] + a.prefix_len, len = 0;
                for (uint32_t g = 0; g <= f; ++g) {
                    const uint32_t sz = a.size[g];
                    if (sz) {
                        pos += sz;
                        continue;
                    }
                    len = rd.u64(pos);
                    pos += 8 + (g < f ? len : 0);
                }
                len = k < nw ? len : 0;
                huge |= (len >> kHugeLog2) | ((pos - b0) >> 31) ? 1u : 0u;
                L.u.s.loff[k] = static_cast<uint32_t>(len);
                L.u.s.src[k] = static_cast<uint16_t>(min<uint64_t>(pos - b0, kFar));
            }
            uint64_t* so = a.soff[f];
            uint8_t* chars = a.col[f];
            if (__syncthreads_or(huge)) {
                // a string of 8 KiB or more: the records one at a time (64-bit
                // offsets, the whole block copying each one's chars)
                uint64_t off = 0;
                for (uint32_t k = 0; k < nrec; ++k) {
                    uint64_t pos = b0 + L.tbl[k] + a.prefix_len, len = 0;
                    for (uint32_t g = 0; g <= f; ++g) {
                        const uint32_t sz = a.size[g];
                        if (sz) {
                            pos += sz;
                            continue;
                        }
                        len = rd.u64(pos);
                        pos += 8 + (g < f ? len : 0);
                    }
                    len = k < nw ? len : 0;
                    if (tid == 0 && R + k <= n) so[R + k] = P + off;
                    copy_global(chars + P + off, w, pos, len, W, tid, kBlock);
                    off += len;
                }
                __syncthreads();
                continue;
            }
            // contiguous per lane: serial sums, then the block scan
            uint64_t mysum = 0;
            const uint32_t k0 = min(tid * per, nrec), k1 = min(k0 + per, nrec);
            for (uint32_t k = k0; k < k1; ++k) mysum += L.u.s.loff[k];
            uint64_t ftot;
            uint64_t run = block_xscan(mysum, &ftot, L.ws);
            for (uint32_t k = k0; k < k1; ++k) {
                const uint32_t len = L.u.s.loff[k];
                L.u.s.loff[k] = static_cast<uint32_t>(run);
                run += len;
            }
            if (tid == 0) {
                L.u.s.loff[nrec] = static_cast<uint32_t>(ftot);
                L.nfar = 0;
            }
            __syncthreads();
            for (uint32_t k = tid; k < nrec && R + k <= n; k += kBlock) so[R + k] = P + L.u.s.loff[k];
            // len chars from stage offset so to d: bytes up to a 4-byte
            // boundary of d, dwords up to a 16-byte one, aligned 16-byte
            // stores, then dwords and bytes
            auto copy_run = [&](uint8_t* d, uint32_t so, uint32_t len) {
                const uint32_t head = min<uint32_t>(len, (4 - (reinterpret_cast<uintptr_t>(d) & 3)) & 3);
                uint32_t i = 0;
#pragma nounroll
                for (; i < head; ++i) d[i] = rd.lds[so + i];
                const uint32_t sa = (so + i) & 3;
                lds_u32c* sw = reinterpret_cast<lds_u32c*>(rd.lds + ((so + i) & ~3u));
                uint32_t* dw = reinterpret_cast<uint32_t*>(d + i);
                const uint32_t nd = (len - i) >> 2;
                uint32_t w0 = sw[0], j = 0;
                const uint32_t pre = min<uint32_t>(nd, ((16 - (reinterpret_cast<uintptr_t>(dw) & 15)) & 15) >> 2);
#pragma nounroll
                for (; j < pre; ++j) {
                    const uint32_t w1 = sw[j + 1];
                    dw[j] = __builtin_amdgcn_alignbyte(w1, w0, sa);
                    w0 = w1;
                }
#pragma nounroll
                for (; j + 4 <= nd; j += 4) {
                    const uint32_t w1 = sw[j + 1], w2 = sw[j + 2], w3 = sw[j + 3], w4 = sw[j + 4];
                    *reinterpret_cast<u32x4*>(dw + j) =
                        u32x4{__builtin_amdgcn_alignbyte(w1, w0, sa), __builtin_amdgcn_alignbyte(w2, w1, sa),
                              __builtin_amdgcn_alignbyte(w3, w2, sa), __builtin_amdgcn_alignbyte(w4, w3, sa)};
                    w0 = w4;
                }
#pragma nounroll
                for (; j < nd; ++j) {
                    const uint32_t w1 = sw[j + 1];
                    dw[j] = __builtin_amdgcn_alignbyte(w1, w0, sa);
                    w0 = w1;
                }
#pragma nounroll
                for (i += 4 * nd; i < len; ++i) d[i] = rd.lds[so + i];
            };
            // where record k's chars are on the wire
            auto chars_at = [&](uint32_t k) -> uint64_t {
                if (L.u.s.src[k] != kFar) return b0 + L.u.s.src[k];
                uint64_t sp = b0 + L.tbl[k] + a.prefix_len;
                for (uint32_t g = 0; g < f; ++g) sp += a.size[g] ? a.size[g] : 8 + rd.u64(sp);
                return sp + 8;
            };
            if (ftot >= static_cast<uint64_t>(kWaveCopyAvg) * nw) {
                // long strings (few records a block): a wave per record, a lane
                // per aligned 16-byte piece of its chars; its unaligned head and
                // tail (< 16 bytes each) byte by byte by lanes 0 and 1
                const uint32_t lane = tid & 63;
                for (uint32_t k = tid >> 6; k < nw; k += kBlock / 64) {
                    const uint32_t o = L.u.s.loff[k], len = L.u.s.loff[k + 1] - o;
                    if (!len) continue;
                    const uint64_t sp = chars_at(k);
                    uint8_t* d = chars + P + o;
                    const uint32_t a0 = min<uint32_t>(len, (16 - (reinterpret_cast<uintptr_t>(d) & 15)) & 15);
                    const uint32_t n16 = (len - a0) >> 4, t0 = a0 + 16 * n16;
                    if (!rd.staged(sp, sp + len)) {
                        // chars past the stage (a record that runs past the
                        // block): the same aligned 16-byte stores, from aligned
                        // dword loads of global memory (byte copies took 10 of
                        // the 15 ms of 410 MiB of zero-filled straddlers)
                        copy_global(d, w, sp, len, W, lane, 64);
                        continue;
                    }
                    const uint32_t so = static_cast<uint32_t>(sp - rd.base);
                    if (lane < 2) {  // lane 0 the head, lane 1 the tail (byte stores)
                        const uint32_t x0 = lane ? t0 : 0, x1 = lane ? len : a0;
#pragma nounroll
                        for (uint32_t x = x0; x < x1; ++x) d[x] = rd.lds[so + x];
                    }
                    for (uint32_t c = lane; c < n16; c += 64) {
                        const uint32_t x = so + a0 + 16 * c;
                        lds_u32c* q = reinterpret_cast<lds_u32c*>(rd.lds + (x & ~3u));
                        const uint32_t s3 = x & 3, w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3], w4 = q[4];
                        *reinterpret_cast<u32x4*>(d + a0 + 16 * c) =
                            u32x4{__builtin_amdgcn_alignbyte(w1, w0, s3), __builtin_amdgcn_alignbyte(w2, w1, s3),
                                  __builtin_amdgcn_alignbyte(w3, w2, s3), __builtin_amdgcn_alignbyte(w4, w3, s3)};
                    }
                }
            } else {
                // lane per record; chars that run past the stage (a record
                // straddling the block's end) are listed and copied a wave
                // per record below -- a lane's byte loop from global memory
                // took 670K of a zero-filled straddler block's 760K cycles
                for (uint32_t k = tid; k < nw; k += kBlock) {
                    const uint32_t o = L.u.s.loff[k], len = L.u.s.loff[k + 1] - o;
                    if (!len) continue;
                    const uint64_t sp = chars_at(k);
                    uint8_t* d = chars + P + o;
                    if (!rd.staged(sp, sp + len)) {
                        const uint32_t j = atomicAdd(&L.nfar, 1u);
                        if (j < kFarList) L.far[j] = k;
                        else copy_global(d, w, sp, len, W, 0, 1);
                        continue;
                    }
                    copy_run(d, static_cast<uint32_t>(sp - rd.base), len);
                }
                __syncthreads();
                const uint32_t nf = min(L.nfar, kFarList);
                for (uint32_t j = tid >> 6; j < nf; j += kBlock / 64) {
                    const uint32_t k = L.far[j], o = L.u.s.loff[k], len = L.u.s.loff[k + 1] - o;
                    copy_global(chars + P + o, w, chars_at(k), len, W, tid & 63, 64);
                }
            }
            __syncthreads();
        }
    }
    SXP(13);
}

__global__ void k_zero_ctl(uint64_t* ctl) {
    if (threadIdx.x < kCtlWords) ctl[threadIdx.x] = 0;
}

uint64_t r256(uint64_t b) { return (b + 255) & ~255ull; }

struct SxLayout {
    uint64_t nb, ng, spec, hdr, ent, gent, gp, gin, bst, ctl, rl, xp, ep, total;
};

SxLayout sx_layout(uint64_t wire_len, uint32_t nc) {
    SxLayout L{};
    L.nb = (wire_len + kSB - 1) / kSB;
    L.ng = (L.nb + kGroup - 1) / kGroup;
    const uint64_t E = 2 + nc;
    uint64_t o = 0;
    L.spec = o;
    o += r256(L.nb * kBlock);
    L.hdr = o;
    o += r256(8 * kHdr * L.nb);
    L.ent = o;
    o += r256(8 * E * kEnt * L.nb);
    L.gent = o;
    o += r256(8 * E * kEnt * L.ng);
    L.gp = o;
    o += r256(8 * (kHdr + E) * L.ng);
    L.gin = o;
    o += r256(8 * E * L.ng);
    L.bst = o;
    o += r256(8 * E * L.nb);
    L.ctl = o;
    o += r256(8 * kCtlWords);
    L.rl = o;
    o += r256(2 * kMaxRec * L.nb);
    L.xp = o;
    o += r256(2 * kX * L.nb);
    L.ep = o;
    o += r256(2 * kE * L.nb);
    L.total = o;
    return L;
}

std::atomic<uint32_t> g_sx_mode{0};

bool sx_decodes(const srpc_plan* p) { return p->nstrings <= kMaxNC + 1; }

template <int NC, bool kDecode>
void launch_sx(const SxArgs& a, const uint8_t* wire, const SxScratch& S, srpc_unpack_status* st, hipStream_t s) {
    // test hook 16: wait for each kernel and name the first that fails
    bool ok = true;
    auto done = [&](const char* k) {
        if (!(a.mode & 16) || !ok) return;
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            ok = false;
            std::fprintf(stderr, "srpc sdx: %s<%d>: %s\n", k, NC, hipGetErrorString(e));
        }
    };
    if (a.nb) launch(k_sx_spec<NC>, dim3(a.nb), dim3(kBlock), 0, s, a, wire, S);
    else hipLaunchKernelGGL(k_zero_ctl, dim3(1), dim3(64), 0, s, S.ctl);
    done("spec");
    const uint32_t gw = (a.ng + kBlock / 64 - 1) / (kBlock / 64);
    // the groups' tables, then (their last workgroup) the in-order scan
    if (a.ng) launch(k_sx_groups<NC, kDecode>, dim3(gw), dim3(kBlock), 0, s, a, wire, S, st, 0u);
    else launch(k_sx_top<NC, kDecode>, dim3(1), dim3(64), 0, s, a, wire, S, st, 0u);
    done("groups0");
    // the repair pass and the second scan: each workgroup reads one control
    // word and ends unless the first scan asked for them (the repair from a
    // bounded grid); then every block's state
    if (a.nb > 1)
        launch(k_sx_repair<NC>, dim3(static_cast<uint32_t>(std::min<uint64_t>(a.nb - 1, 1024))), dim3(kBlock), 0, s, a,
               wire, S);
    done("repair");
    if (a.ng) launch(k_sx_groups<NC, kDecode>, dim3(gw), dim3(kBlock), 0, s, a, wire, S, st, 1u);
    done("groups1");
    if (a.ng) launch(k_sx_blocks<NC>, dim3(gw), dim3(kBlock), 0, s, a, wire, S);
    done("blocks");
    const uint32_t g = static_cast<uint32_t>(std::max<uint64_t>(a.nb, 1));
    launch(k_sx_decode<NC, kDecode>, dim3(g), dim3(kBlock), 0, s, a, wire, S, st);
    done("decode");
}

}  // namespace
}  // namespace srpc_impl

using namespace srpc_impl;

extern "C" {

int srpc_plan_var_stream_scratch_bytes(const srpc_plan* p, uint64_t n, uint64_t wire_len, uint64_t* out) {
    if (!p || !out || !p->has_string) return SRPC_E_INVALID;
    uint64_t var = 0;
    if (int rc = srpc_plan_var_scratch_bytes(p, n, wire_len, &var)) return rc;
    *out = (sx_decodes(p) ? 0 : r256(var)) + sx_layout(wire_len, sx_decodes(p) ? p->nstrings - 1 : 0).total;
    return SRPC_OK;
}

int srpc_gpu_unpack_var_stream(const srpc_plan* p, const uint8_t* wire, uint64_t wire_len, uint64_t n,
                               uint64_t* rec_offs, void* const* cols, uint64_t* const* str_offs,
                               srpc_unpack_status* st, void* scratch, uint64_t scratch_bytes, void* stream) {
    const TimedCall timed;
    if (!p || !p->has_string || !rec_offs || !scratch || !cols || !str_offs) return SRPC_E_INVALID;
    if (wire_len && !wire) return SRPC_E_INVALID;
    if (!aligned(rec_offs, 8) || !aligned(scratch, 256)) return SRPC_E_ALIGN;
    uint64_t need = 0;
    if (int rc = srpc_plan_var_stream_scratch_bytes(p, n, wire_len, &need)) return rc;
    if (scratch_bytes < need) return SRPC_E_CAPACITY;
    const bool decode = sx_decodes(p);
    for (uint32_t f = 0; f < p->nfields && decode; ++f) {
        if (!cols[f]) return SRPC_E_INVALID;
        if (p->size[f] && !aligned(cols[f], p->size[f])) return SRPC_E_ALIGN;
        if (p->size[f] == 0 && (!str_offs[f] || !aligned(str_offs[f], 8) || !aligned(cols[f], 16))) return SRPC_E_ALIGN;
    }
    const uint32_t nc = decode ? p->nstrings - 1 : 0;
    const SxLayout SL = sx_layout(wire_len, nc);
    // counts travel in 40 bits; positions and chars in full words
    if (SL.nb > 0x7fffffffull || wire_len >= (1ull << 40) || p->fixed_bytes < 8) return SRPC_E_UNSUPPORTED;
    uint64_t var = 0;
    srpc_plan_var_scratch_bytes(p, n, wire_len, &var);
    auto* base = static_cast<uint8_t*>(scratch) + (decode ? 0 : r256(var));
    SxScratch S{base + SL.spec,
                reinterpret_cast<uint64_t*>(base + SL.hdr),
                reinterpret_cast<uint64_t*>(base + SL.ent),
                reinterpret_cast<uint64_t*>(base + SL.gent),
                reinterpret_cast<uint64_t*>(base + SL.gp),
                reinterpret_cast<uint64_t*>(base + SL.gin),
                reinterpret_cast<uint64_t*>(base + SL.bst),
                reinterpret_cast<uint64_t*>(base + SL.ctl),
                reinterpret_cast<uint16_t*>(base + SL.rl),
                reinterpret_cast<uint16_t*>(base + SL.xp),
                reinterpret_cast<uint16_t*>(base + SL.ep)};
    SxArgs a{};
    uint32_t si = 0;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        a.size[f] = p->size[f];
        a.sord[f] = p->size[f] ? 0 : si++;
        a.col[f] = decode ? static_cast<uint8_t*>(cols[f]) : nullptr;
        a.soff[f] = decode && !p->size[f] ? str_offs[f] : nullptr;
    }
    a.prefix = p->d_prefix;
    a.rec_offs = rec_offs;
    a.n = n;
    a.W = wire_len;
    a.nfields = p->nfields;
    a.nstrings = p->nstrings;
    a.prefix_len = p->prefix_len;
    a.fixed_bytes = p->fixed_bytes;
    a.first_len_at = p->prefix_len;
    for (uint32_t f = 0; f < p->nfields && p->size[f]; ++f) a.first_len_at += p->size[f];
    a.plaus = p->prefix_len >= 8 ? kPlausPrefixed : kPlausBare;
    for (uint32_t i = 0; i < 8 && i < p->prefix_len; ++i) a.pre8 |= static_cast<uint64_t>(p->h_prefix[i]) << (8 * i);
    a.cap = (kSC + p->fixed_bytes - 1) / p->fixed_bytes;  // <= kListCap (fixed_bytes >= 8)
    {
        uint32_t k = 0, run = p->prefix_len;
        for (uint32_t f = 0; f < p->nfields; ++f) {
            if (p->size[f]) {
                run += p->size[f];
                continue;
            }
            a.gap[k++] = run;
            run = 0;
        }
        a.gap[k] = run;
    }
    a.nb = static_cast<uint32_t>(SL.nb);
    a.ng = static_cast<uint32_t>(SL.ng);
    a.mode = g_sx_mode.load(std::memory_order_relaxed);
    auto s = static_cast<hipStream_t>(stream);
    if (!decode) launch_sx<0, false>(a, wire, S, st, s);
    else if (nc == 0) launch_sx<0, true>(a, wire, S, st, s);
    else if (nc == 1) launch_sx<1, true>(a, wire, S, st, s);
    else if (nc == 2) launch_sx<2, true>(a, wire, S, st, s);
    else launch_sx<3, true>(a, wire, S, st, s);
    if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
    if (!decode)  // more string fields than a state carries: the indexed decode over the index just built
        return srpc_gpu_unpack_var(p, wire, wire_len, n, rec_offs, cols, str_offs, st, scratch, var, stream);
    return SRPC_OK;
}

}  // extern "C"

// Test hook (not part of the C ABI in include/), bits: 1 = block tables hold
// only the first speculated start (every other entry needs the repair pass's
// exit slots, or a walk), 2 = empty tables (every block entered needs them),
// 4 = the speculation's exact filter at every position instead of zero-byte
// candidates, 8 = no repair pass (a position no table holds is walked, the
// round-5 path), 16 = wait for each kernel and name the first that fails on
// stderr; 0 = normal.  Returns the previous setting.
#ifdef SRPC_SX_PHASES
extern "C" int srpc_debug_sx_phases(void* d_buf, uint64_t nblocks) {
    unsigned long long* p = static_cast<unsigned long long*>(d_buf);
    unsigned long long nb = nblocks;
    if (hipMemcpyToSymbol(HIP_SYMBOL(srpc_impl::g_sxph), &p, sizeof(p)) != hipSuccess) return SRPC_E_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(srpc_impl::g_sxph_blocks), &nb, sizeof(nb)) != hipSuccess) return SRPC_E_HIP;
    return SRPC_OK;
}
#endif

extern "C" __attribute__((visibility("default"))) int srpc_debug_stream_tables(int mode) {
    return static_cast<int>(srpc_impl::g_sx_mode.exchange(static_cast<uint32_t>(mode < 0 ? 0 : mode > 31 ? 31 : mode)));
}
