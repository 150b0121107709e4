// stream1.hip -- decode a concatenated record stream with no index in ONE
// pass over the wire: the bounded decode of srpc_gpu_unpack_var_stream
// (stream.hip), run when the speculative chunk pipeline's parallel repair
// rounds do not settle (data on which a wrong record start parses too).
//
// The reference decodes a batch with ONE shared cursor (buffer::_offset,
// core.hpp:39): each pipe_output advances it (packer.hpp:210-222; nested
// unpack sharing the buffer as in tests/packer_test.cpp:77-88), so where a
// record starts is only known once every record before it was read.
//
// Here the wire is cut into blocks of kSB bytes, one workgroup each, in one
// launch (k_stream_decode).  A block's state at its start is the cursor's:
// the position of the first record start at or after the block (its entry),
// the records before it and, per string field, the chars before it.  Every
// block:
//  1. stages its bytes (+ kMargin) in LDS by LDS-DMA;
//  2. speculates, a lane per kSC-byte chunk: the chunk's first plausible
//     record start (a filter over all its positions at once from register
//     windows, then whole records must parse; of the plausible starts within
//     a length field's 8 bytes the one with the smallest first length), and
//     walks the records that start in the chunk: their starts, count, chars
//     per string field, the position after them (exit) and whether a record
//     failed (stop);
//  3. links the chunks: a chunk whose start is its predecessor's exit
//     continues its segment; exclusive scans of counts and chars give every
//     segment's totals from any of its chunks in O(1);
//  4. candidates for its entry -- every plausible position in its first kWin
//     bytes, else the first speculated start -- and, per candidate, the chain
//     of records from it to the block end (walk_chain: records are parsed
//     one by one until the walk meets a speculated start, then whole segments
//     are jumped): exit, records, chars, stop.  This table is published
//     (AGG) before the block knows its entry;
//  5. looks back (decoupled look-back over the tables): from the nearest
//     block whose inclusive state is published (INC), the tables of the
//     blocks between are composed -- a block's entry is its predecessor's
//     exit; an entry found in that block's table moves the state on, one past
//     its end passes the block through; an entry in no table (the cursor
//     enters the block where no candidate was) waits for that block's own INC;
//  6. publishes its INC and writes its records: rec_offs, fixed fields,
//     str_offs and chars (an LDS image per string field, aligned 16-byte
//     stores), every record parsed once more from the stage.
// Wire bytes are read from HBM once (the stage); the margin re-reads <= 25 %
// of a block from L2 / the Infinity Cache.  Zero-heavy data, where a wrong
// start parses too (every phase of a periodic record is plausible), costs a
// longer walk per candidate, not more rounds: tables hold one entry per
// plausible position of the window, and the look-back composes them in one
// pass.  An entry that is in no table -- a record longer than the window
// whose end is not where the block speculated -- costs one look-back hop.
// Error semantics are the cursor's (oracle/packer_oracle.c orc_unpack): the
// first record that does not parse stops the stream; it is reported
// (PREFIX or BOUNDS) as the first bad record, every later record BOUNDS;
// rec_offs[T] = where the stream stopped, later entries wire_len.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <unistd.h>

#include "plan.h"
#include "srpc_gpu.h"

#include "stream1.h"

namespace srpc_impl {
namespace {

#ifndef SRPC_STREAM_NOLOOK  // A/B timing only (wrong results): no look-back, an estimated state
#define SRPC_STREAM_NOLOOK 0
#endif
#ifndef SRPC_STREAM_NOOUT  // A/B timing only: no outputs
#define SRPC_STREAM_NOOUT 0
#endif
// Per-phase clock (A/B diagnostics, compiled only with -DSRPC_STREAM_PHASES):
// thread 0 of every block adds the clock64() cycles between its phase marks,
// plus look-back counters; srpc_debug_stream_phases reads them.
// Per-phase clock (A/B diagnostics, compiled only with -DSRPC_STREAM_PHASES):
// thread 0 of every block stores the clock64() cycles between its phase
// marks, and look-back counters, in 16 words of its own (plain stores: global
// atomics from every block distorted the timing); see srpc_debug_stream_phases.
#ifdef SRPC_STREAM_PHASES
__device__ unsigned long long* g_sph = nullptr;
__device__ unsigned long long g_sph_blocks = 0;
#define SP_BEGIN uint64_t sp_last_ = clock64();
#define SP_SLOT(i) g_sph[static_cast<uint64_t>(blockIdx.x) * 16 + (i)]
#define SP(i)                                                                 \
    do {                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < g_sph_blocks) {                  \
            const uint64_t now_ = clock64();                                  \
            SP_SLOT(i) += now_ - sp_last_;                                    \
            sp_last_ = now_;                                                  \
        }                                                                     \
    } while (0)
#define SP_ADD(i, v)                                                          \
    do {                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < g_sph_blocks) SP_SLOT(i) += (v); \
    } while (0)
#else
#define SP_BEGIN
#define SP(i)
#define SP_ADD(i, v)
#endif
constexpr uint32_t kSB = 8192;                  // wire bytes per block (one workgroup)
constexpr uint32_t kSC = kSB / kBlock;          // 32: wire bytes per speculating lane
static_assert(kSC % 16 == 0 && kSC <= 64, "16-byte window reads; a chunk's positions fit one 64-bit mask");
constexpr uint32_t kMargin = 2048;              // staged bytes past the block
constexpr uint32_t kStage = kSB + kMargin + 32; // + 16-byte alignment slack on both sides
constexpr uint32_t kWin = 64;                   // candidate window (one lane of wave 0 per position)
constexpr int kMaxNC = 3;                       // chars values carried per state (string fields 0..ns-2)
constexpr uint32_t kMaxRec = kSB / 8;           // records starting in a block (each >= 8 bytes)
constexpr uint32_t kImage = kSB + kMargin + 64; // chars image of one string field
constexpr uint32_t kPlausPrefixed = 1, kPlausBare = 2;
constexpr uint16_t kNoStart = 0xFFFF;
#ifndef SRPC_STREAM_SPIN
#define SRPC_STREAM_SPIN (1u << 18)
#endif
constexpr uint32_t kSpinMax = SRPC_STREAM_SPIN;  // polls of one wait: then STALLED (reported, never a hang)
constexpr uint32_t kAgg = 1, kInc = 2;          // flag states
// stop bits: bit 0 = the chain stopped, bits 1-2 = why (SRPC_STATUS_PREFIX /
// _BOUNDS; 0 = not an error: the block is past record n, nothing after counts)

typedef const uint8_t __attribute__((address_space(1))) global_u8;
typedef uint8_t __attribute__((address_space(3))) lds_u8;
typedef const uint8_t __attribute__((address_space(3))) lds_u8c;
typedef const uint32_t __attribute__((address_space(3))) lds_u32c;
typedef const uint64_t __attribute__((address_space(3))) lds_u64c;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct StreamArgs {
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
    uint32_t nb;                 // blocks
    uint32_t epoch;              // this call's tag in the flag words
};

struct Scratch {
    uint64_t* flag;  // per block: epoch << 32 | state << 8 | primary slot
    uint64_t* inc;   // per block: exit, count | stop << 61, chars[NC]
    uint64_t* agg;   // per block: its table, word k of slot s at k * kWin + s
    uint64_t* pri;   // per block: its primary entry, slot 0's position, slot mask (two halves)
    uint32_t* ctl;   // [0] first block past record n, [1] diagnostics, [2] blocks that missed, [3] stalled
};

template <int NC>
constexpr uint32_t inc_words() { return 2 + NC; }
template <int NC>
constexpr uint32_t agg_words() { return 2 + NC; }  // per slot: exit, count | stop << 40, chars[NC]
// a block's table: word k of slot s at k * kWin + s (a word of every slot contiguous)
template <int NC>
constexpr uint32_t agg_block_words() { return agg_words<NC>() * kWin; }
template <int NC>
constexpr uint32_t pri_words() { return 5 + NC; }
constexpr uint32_t kNoPrim = 0xff;

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- wire readers --------------------------------------------------------------
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
    __device__ __forceinline__ uint64_t u64(uint64_t p) const { return p >= s.lo && p + 8 <= s.hi ? s.u64(p) : ~0ull; }
    __device__ __forceinline__ uint8_t u8(uint64_t p) const {
        return p >= s.lo && p < s.hi ? s.lds[p - s.base] : static_cast<uint8_t>(~s.pre[0]);
    }
    __device__ __forceinline__ uint64_t pre64(uint32_t i) const { return s.pre64(i); }
    __device__ __forceinline__ uint8_t pre8(uint32_t i) const { return s.pre8(i); }
};

// orc_unpack's cursor over one record at p: the position after it, or p with
// *err set (SRPC_STATUS_PREFIX / _BOUNDS); chars of string fields 0..NC-1
// added to ch[].
template <int NC, class Rd>
__device__ __forceinline__ uint64_t parse_rd(const StreamArgs& a, const Rd& r, uint64_t p, uint32_t* err,
                                             uint64_t (&ch)[kMaxNC + 1]) {
    const uint64_t W = a.W;
    *err = 0;
    if (a.prefix_len) {
        if (a.prefix_len > W - p) {
            *err = SRPC_STATUS_BOUNDS;
            return p;
        }
        uint32_t i = 0;
        for (; i + 8 <= a.prefix_len; i += 8)
            if (r.u64(p + i) != r.pre64(i)) {
                *err = SRPC_STATUS_PREFIX;
                return p;
            }
        for (; i < a.prefix_len; ++i)
            if (r.u8(p + i) != r.pre8(i)) {
                *err = SRPC_STATUS_PREFIX;
                return p;
            }
    }
    uint64_t q = p + a.prefix_len;
    uint64_t add[kMaxNC + 1] = {};
    uint32_t si = 0;
    for (uint32_t f = 0; f < a.nfields; ++f) {
        const uint32_t sz = a.size[f];
        if (sz) {
            if (sz > W - q) {
                *err = SRPC_STATUS_BOUNDS;
                return p;
            }
            q += sz;
            continue;
        }
        if (8 > W - q) {
            *err = SRPC_STATUS_BOUNDS;
            return p;
        }
        const uint64_t len = r.u64(q);
        q += 8;
        if (len > W - q) {
            *err = SRPC_STATUS_BOUNDS;
            return p;
        }
        q += len;
#pragma unroll
        for (int k = 0; k < NC; ++k) add[k] += si == static_cast<uint32_t>(k) ? len : 0;
        ++si;
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) ch[k] += add[k];
    return q;
}

// Necessary for a record to parse at p: the prefix's first (up to 8) bytes
// match and the first string's length fits the wire.
template <class Rd>
__device__ __forceinline__ bool filter(const StreamArgs& a, const Rd& r, uint64_t p) {
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
__device__ __forceinline__ bool plausible(const StreamArgs& a, const Rd& r, uint64_t p) {
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
// apart, so the dword shift is a uniform switch).  Dword reads of lanes'
// windows sat on the same banks (82 % of LDS cycles conflicted,
// profiles/r02_stream_window_ab.log).
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

// Positions of a chunk (LDS offset `at`, wire offset clo, up to `jmax`) that
// pass the filter, as a mask: the first string's length at p + first_len_at
// fits the wire, the prefix's first 8 bytes match -- all positions at once
// from register windows of the stage.
__device__ __forceinline__ uint64_t chunk_mask(const StreamArgs& a, const uint8_t* st, uint32_t at, uint64_t clo,
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

// A block's chain from an entry: what the cursor does from `x` until the first
// record start at or past the block end (exit), or a record that fails (stop).
template <int NC>
struct Agg {
    uint64_t exit, cnt;
    uint64_t ch[kMaxNC + 1];
    uint32_t stop;  // 0, or 1 | kind << 1
};

// The block's LDS (static; k_stream_decode).
template <int NC>
struct BlockLds {
    alignas(16) uint8_t st[kStage + 16];             // wire bytes [base, base + kStage)
    alignas(16) uint8_t pre[kMaxPrefix + 16];
    alignas(16) uint8_t img[kImage + 32];            // chars image; the explicit start list while walking
    uint64_t exit[kBlock];                           // per chunk: position after its records
    uint64_t pch[NC ? NC : 1][kBlock + 1];           // per chunk, then exclusive scan: chars of fields 0..NC-1
    uint32_t pcnt[kBlock + 1];                       // per chunk, then exclusive scan: records
    uint32_t loff[kMaxRec + 1];                      // per local record: chars offset (field being copied)
    uint16_t start[kBlock];                          // per chunk: first start (offset from the block), or none
    uint16_t tbl[kMaxRec + 1];                       // the block's records in order: offset from the block
    uint8_t list[kBlock * 5];                        // per chunk: its starts minus the chunk's first byte
    uint8_t stop[kBlock];                            // per chunk: 0, or 1 | kind << 1
    uint64_t has[4], tail[4], jump[4];               // 256-bit masks over chunks
    uint64_t ws[kBlock / 64];
    // the block's state (from the look-back) and its own chain
    uint64_t s_cnt, s_ch[kMaxNC + 1], s_x;
    uint32_t s_nexp;
};

// The chain from x (x >= the block start): explicit records are parsed until
// the walk meets a speculated chunk start, whose segment is then taken whole
// from the scans (O(1)), and so on.  REC: the explicit starts go to the list
// (LDS u16 offsets, ascending) and jumped chunks to the jump mask.
template <int NC, bool REC>
__device__ Agg<NC> walk_chain(const StreamArgs& a, const StagedRd& rd, BlockLds<NC>& L, uint64_t b0, uint64_t b1,
                              uint64_t x, uint16_t* xl, uint32_t* nx) {
    Agg<NC> g{};
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
    g.exit = q;
    if (REC) *nx = ne;
    return g;
}

template <int NC>
__device__ __forceinline__ void add_agg(uint64_t& exit, uint64_t& cnt, uint64_t (&ch)[kMaxNC + 1], uint32_t& stop,
                                        const Agg<NC>& g) {
    exit = g.exit;
    cnt += g.cnt;
#pragma unroll
    for (int k = 0; k < NC; ++k) ch[k] += g.ch[k];
    stop = g.stop;
}

// Wave-uniform sleep-and-count: false once the spin budget is spent.
// Polls read a flag word only (a waiting block's data loads come once its
// flags say ready): pollers next to a stream cost chip bandwidth
// (MI355X_MICROARCH.md "polling-cost").
__device__ __forceinline__ bool spin(uint32_t* n) {
    if (++*n >= kSpinMax) return false;
    __builtin_amdgcn_s_sleep(8);
    return true;
}

// ---- look-back words --------------------------------------------------------
// Every published word carries the call's 21-bit tag over a 43-bit value, so
// no word needs a fence or a drain before the flag that announces it: a
// reader that finds a stale tag reads again (handoff by tagged 8-byte
// granules, MI355X_MICROARCH.md "handoff-1to1").  Counts are 40 bits, with the
// stop bits above them.
constexpr uint64_t kValMask = (1ull << 43) - 1;
constexpr uint64_t kTagMax = (1ull << 21) - 1;
constexpr uint64_t kCnt40 = (1ull << 40) - 1;
__device__ __forceinline__ uint64_t tg(uint64_t v, uint64_t t21) { return (v & kValMask) | (t21 << 43); }
__device__ __forceinline__ bool tag_ok(uint64_t w, uint64_t t21) { return (w >> 43) == t21; }
// A flag word's state for this call (0: not published yet)
__device__ __forceinline__ uint32_t flag_state(uint64_t f, uint32_t epoch) {
    return (f >> 32) == epoch ? static_cast<uint32_t>((f >> 8) & 0xff) : 0;
}

// The cursor's state at a block boundary: position of the next record start,
// records before it, chars of string fields 0..NC-1 before it, stop bits.
template <int NC>
struct St {
    uint64_t ex, cn;
    uint64_t ch[kMaxNC + 1];
    uint32_t stp;
};

template <int NC>
__device__ __forceinline__ void publish_inc(const Scratch& S, uint64_t b, const St<NC>& s, uint64_t flag,
                                            uint64_t t21) {
    uint64_t* iw = S.inc + b * inc_words<NC>();
    st_sc1(iw, tg(s.ex, t21));
    st_sc1(iw + 1, tg((s.cn & kCnt40) | (static_cast<uint64_t>(s.stp) << 40), t21));
#pragma unroll
    for (int k = 0; k < NC; ++k) st_sc1(iw + 2 + k, tg(s.ch[k], t21));
    st_sc1(S.flag + b, flag);
}

__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), l);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), l);
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// One block per lane of the look-back wave: its flag, its INC words (when
// published and whole), its primary entry, slot 0's position and slot mask.
template <int NC>
struct Win {
    int64_t idx;            // the lane's block (< 0 or past b - 1: none)
    uint32_t prim;          // primary slot (kNoPrim: none)
    bool inc_ok, pri_ok;    // INC / table published (flag of this call, every word's tag)
    uint64_t iex, icn, ich[kMaxNC + 1];  // INC
    uint32_t istp;
    uint64_t pX, pC, pCH[kMaxNC + 1];    // primary entry
    uint32_t pST;
    uint64_t candp, pos0, mask;
    __device__ __forceinline__ void load(const Scratch& S, const StreamArgs& a, int64_t j, uint64_t b) {
        idx = j;
        inc_ok = pri_ok = false;
        prim = kNoPrim;
        candp = ~0ull;
        mask = 0;
        if (j < 0 || static_cast<uint64_t>(j) >= b) {
            idx = -1;
            return;
        }
        const uint64_t t21 = a.epoch & kTagMax;
        const uint64_t f = ld_sc1(S.flag + j);
        const uint64_t* iw = S.inc + j * inc_words<NC>();
        const uint64_t* q = S.pri + j * pri_words<NC>();
        uint64_t w[2 + kMaxNC], v[5 + kMaxNC];
#pragma unroll
        for (int k = 0; k < 2 + NC; ++k) w[k] = ld_sc1(iw + k);
#pragma unroll
        for (int k = 0; k < 5 + NC; ++k) v[k] = ld_sc1(q + k);
        const uint32_t stt = flag_state(f, a.epoch);
        prim = stt ? static_cast<uint32_t>(f & 0xff) : kNoPrim;
        bool ok = stt == kInc;
#pragma unroll
        for (int k = 0; k < 2 + NC; ++k) ok = ok && tag_ok(w[k], t21);
        inc_ok = ok;
        iex = w[0] & kValMask;
        icn = w[1] & kCnt40;
        istp = static_cast<uint32_t>((w[1] >> 40) & 7);
#pragma unroll
        for (int k = 0; k < NC; ++k) ich[k] = w[2 + k] & kValMask;
        // the table: the slot map words always, the primary's when there is one
        bool tok = stt >= kAgg && j > 0;
#pragma unroll
        for (int k = 2 + NC; k < 5 + NC; ++k) tok = tok && tag_ok(v[k], t21);
        if (prim != kNoPrim)
#pragma unroll
            for (int k = 0; k < 2 + NC; ++k) tok = tok && tag_ok(v[k], t21);
        pri_ok = tok || inc_ok;
        pX = v[0] & kValMask;
        pC = v[1] & kCnt40;
        pST = static_cast<uint32_t>((v[1] >> 40) & 7);
#pragma unroll
        for (int k = 0; k < NC; ++k) pCH[k] = v[2 + k] & kValMask;
        pos0 = v[2 + NC] & kValMask;
        mask = (v[3 + NC] & 0xffffffffull) | ((v[4 + NC] & 0xffffffffull) << 32);
        if (!tok) mask = 0;
        if (tok && prim != kNoPrim) candp = prim == 0 ? pos0 : static_cast<uint64_t>(j) * kSB + prim;
    }
    __device__ __forceinline__ St<NC> inc_state(uint32_t l) const {
        St<NC> s;
        s.ex = rl64(iex, l);
        s.cn = rl64(icn, l);
#pragma unroll
        for (int k = 0; k < NC; ++k) s.ch[k] = rl64(ich[k], l);
        s.stp = __builtin_amdgcn_readlane(istp, l);
        return s;
    }
};

// Fold the window's blocks [lo, lo + cnt) (lane l = block lo + l, its words
// in wv) into the state s.  Each lane's primary entry leads to the block its
// exit lands in; pointer jumping gives every lane its path's result to where
// the path leaves the window, or to a block whose INC is published (an exact
// state, not a sum), and whether every link on the way entered the next block
// at its primary.  The wave then follows the chain in scalar registers: a
// whole valid path at once, one block where a path leaves the primaries, and
// an entry off every primary from that block's slot map (one load) or, in no
// slot, from that block's own INC.  The window's last block then gets its
// inclusive state published (later look-backs stop there).
template <int NC>
__device__ void fold(const Scratch& S, const StreamArgs& a, const Win<NC>& wv, St<NC>& s, uint64_t lo, uint32_t cnt,
                     uint64_t tag, uint64_t t21, uint32_t* spins, bool* stalled) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = a.W;
    const bool mine_ok = lane < cnt && wv.idx >= 0;
    // the lane's own step: INC (absolute) or the primary entry (a sum)
    const bool isabs = mine_ok && wv.inc_ok;
    const bool hasp = mine_ok && !isabs && wv.candp != ~0ull;
    uint64_t X = isabs ? wv.iex : wv.pX, C = isabs ? wv.icn : wv.pC;
    uint64_t CH[kMaxNC + 1];
#pragma unroll
    for (int k = 0; k < NC; ++k) CH[k] = isabs ? wv.ich[k] : wv.pCH[k];
    uint32_t ST = isabs ? wv.istp : wv.pST;
    uint32_t A = isabs;  // the result is an absolute state
    uint32_t N = 64;     // next lane on the path
    if ((isabs || hasp) && !(ST & 1) && X < W) {
        const uint64_t m = X / kSB;
        if (m >= lo && m < lo + cnt) N = static_cast<uint32_t>(m - lo);
    }
    const uint64_t cand_n = __shfl(wv.candp, N & 63, 64);
    const uint32_t abs_n = __shfl(static_cast<uint32_t>(isabs), N & 63, 64);
    uint32_t V = N == 64 || abs_n || cand_n == X;  // enters the next block at its primary (or its INC)
    const uint64_t X1 = X, C1 = C;
    uint64_t CH1[kMaxNC + 1];
#pragma unroll
    for (int k = 0; k < NC; ++k) CH1[k] = CH[k];
    const uint32_t ST1 = ST, A1 = A;
    for (int d = 0; d < 6; ++d) {
        const uint32_t n2 = N & 63;
        const uint32_t nN = __shfl(N, n2, 64), nV = __shfl(V, n2, 64), nST = __shfl(ST, n2, 64),
                       nA = __shfl(A, n2, 64);
        const uint64_t nX = __shfl(X, n2, 64), nC = __shfl(C, n2, 64);
        uint64_t nCH[kMaxNC + 1];
#pragma unroll
        for (int k = 0; k < NC; ++k) nCH[k] = __shfl(CH[k], n2, 64);
        if (N < 64) {
            C = nA ? nC : C + nC;
#pragma unroll
            for (int k = 0; k < NC; ++k) CH[k] = nA ? nCH[k] : CH[k] + nCH[k];
            A |= nA;
            X = nX;
            ST = nST;
            V &= nV;
            N = nN;
        }
    }
    while (!(s.stp & 1) && s.ex < W) {
        const uint64_t kb = s.ex / kSB;
        if (kb < lo || kb >= lo + cnt) {  // leaves the window (behind it: never expected -- reported)
            if (kb < lo) *stalled = true;
            break;
        }
        const uint64_t ex_before = s.ex;
        const uint32_t l = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(kb - lo));
        const bool labs = __builtin_amdgcn_readlane(static_cast<uint32_t>(isabs), l);
        if (labs || rl64(wv.candp, l) == s.ex) {
            const bool whole = __builtin_amdgcn_readlane(V, l);
            const uint32_t a_ = __builtin_amdgcn_readlane(whole ? A : A1, l);
            const uint64_t cx = rl64(whole ? C : C1, l);
            s.cn = a_ ? cx : s.cn + cx;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                const uint64_t v = rl64(whole ? CH[k] : CH1[k], l);
                s.ch[k] = a_ ? v : s.ch[k] + v;
            }
            s.ex = rl64(whole ? X : X1, l);
            s.stp = __builtin_amdgcn_readlane(whole ? ST : ST1, l);
        } else {
            SP_ADD(12, 1);
            const uint64_t mk = rl64(wv.mask, l), p0 = rl64(wv.pos0, l);
            const uint64_t off = s.ex - kb * kSB;
            int slot = -1;
            if (off < kWin && ((mk >> off) & 1) && (off || p0 == s.ex)) slot = static_cast<int>(off);
            else if ((mk & 1) && p0 == s.ex) slot = 0;
            if (slot >= 0) {
                const uint64_t* e = S.agg + kb * agg_block_words<NC>() + slot;
                uint64_t w[2 + kMaxNC];
                bool ok;
                do {
#pragma unroll
                    for (int k = 0; k < 2 + NC; ++k) w[k] = ld_sc1(e + k * kWin);
                    ok = true;
#pragma unroll
                    for (int k = 0; k < 2 + NC; ++k) ok = ok && tag_ok(w[k], t21);
                } while (!ok && spin(spins));
                if (!ok) {
                    *stalled = true;
                    return;
                }
                s.ex = w[0] & kValMask;
                s.cn += w[1] & kCnt40;
                s.stp = static_cast<uint32_t>((w[1] >> 40) & 7);
#pragma unroll
                for (int k = 0; k < NC; ++k) s.ch[k] += w[2 + k] & kValMask;
            } else {  // in no slot: that block's own INC (poll its flag, then its words)
                Win<NC> one;
                while (true) {
                    if (flag_state(ld_sc1(S.flag + kb), a.epoch) == kInc) {
                        one.load(S, a, static_cast<int64_t>(kb), kb + 1);
                        if (__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(one.inc_ok))) break;
                    }
                    if (!spin(spins)) {
                        *stalled = true;
                        return;
                    }
                }
                s = one.inc_state(__builtin_amdgcn_readfirstlane(lane));
            }
        }
        if (!(s.stp & 1) && s.ex <= ex_before) {  // no progress: never expected -- reported
            *stalled = true;
            return;
        }
    }
    // help: the state after the window is its last block's inclusive state
    const uint32_t last = cnt - 1;
    const uint32_t last_inc = __shfl(static_cast<uint32_t>(wv.inc_ok), last, 64);
    const uint32_t last_pr = __shfl(wv.prim, last, 64);
    if (!*stalled && !last_inc && lane == 0)
        publish_inc<NC>(S, lo + last, s, tag | (kInc << 8) | last_pr, t21);
}



// One launch decodes the whole stream; see the file comment.  kDecode =
// false: the record index only (rec_offs), for schemas with more string
// fields than a state carries (the indexed decode follows).
template <int NC, bool kDecode>
__global__ __launch_bounds__(kBlock) void k_stream_decode(StreamArgs a, const uint8_t* __restrict__ w, Scratch S,
                                                          const uint32_t* gate) {
    if (gate && !*gate) return;  // the chunk pipeline settled: nothing to do
    __shared__ BlockLds<NC> L;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint64_t b = blockIdx.x;
    const uint64_t W = a.W;
    const uint64_t b0 = b * kSB, b1 = min<uint64_t>(b0 + kSB, W);
    const uint64_t tag = static_cast<uint64_t>(a.epoch) << 32;

    // a block past the one that holds record n has nothing to do: it passes a
    // stopped state on (nothing after it counts either)
    if (b > 0 && b > __hip_atomic_load(&S.ctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        if (tid == 0) {
            St<NC> st{};
            st.ex = W;
            st.cn = a.n + 1;
            st.stp = 1;
            publish_inc<NC>(S, b, st, tag | (kInc << 8) | kNoPrim, a.epoch & kTagMax);
        }
        return;
    }

    SP_BEGIN
    SP_ADD(10, 1);
    // 1. prefix and stage (LDS-DMA)
    for (uint32_t i = tid; i < a.prefix_len + 16; i += kBlock) L.pre[i] = i < a.prefix_len ? a.prefix[i] : 0;
    const uint64_t hi = min<uint64_t>(b1 + kMargin, W);
    const uint64_t A = (reinterpret_cast<uint64_t>(w) + b0) & ~15ull;
    const uint32_t ng = static_cast<uint32_t>((reinterpret_cast<uint64_t>(w) + hi - A + 15) >> 4);
    for (uint32_t w0 = tid & ~63u; w0 < ng; w0 += kBlock) {
        const uint32_t gi = w0 + lane;
        if (gi < ng) {
            const uint32_t wb = __builtin_amdgcn_readfirstlane(w0);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<global_u8*>(A + 16ull * gi), (lds_u8*)(L.st + 16 * wb),
                                             16, 0, 0);
        }
    }
    if (tid < 4) L.jump[tid] = 0;
    __syncthreads();  // waits for the LDS-DMA and publishes the stage
    const StagedRd rd{(global_u8*)w, (lds_u8c*)L.st, A - reinterpret_cast<uint64_t>(w), b0, hi, (lds_u8c*)L.pre};
    const StageOnlyRd so{rd};
    SP(0);

    // 2. speculation: chunk c = tid
    const uint64_t clo = b0 + static_cast<uint64_t>(tid) * kSC, chi = min<uint64_t>(clo + kSC, b1);
    uint64_t sp = ~0ull;  // the chunk's first plausible start
    if (clo < b1) {
        if (clo == 0) {
            sp = 0;  // the stream starts at 0: no speculation
        } else {
            uint64_t mask = chunk_mask(a, L.st, static_cast<uint32_t>(clo - rd.base), clo, chi);
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
                // plausible candidates sp .. sp + 7 inside the chunk: the one
                // with the smallest first string length (a start 1-3 bytes
                // early reads the true length shifted up)
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
    uint64_t cch[kMaxNC + 1] = {};
    uint32_t ccnt = 0, cstop = 0;
    uint64_t cexit = ~0ull;
    if (sp != ~0ull) {  // walk the chunk's records
        uint64_t p = sp;
        while (p < chi) {
            uint32_t err;
            const uint64_t q = parse_rd<NC>(a, rd, p, &err, cch);
            if (err) {
                cstop = 1 | (err << 1);
                break;
            }
            if (ccnt < a.cap) L.list[tid * 5 + ccnt] = static_cast<uint8_t>(p - clo);
            ++ccnt;
            p = q;
        }
        cexit = p;
    }
    L.start[tid] = sp == ~0ull ? kNoStart : static_cast<uint16_t>(sp - b0);
    L.exit[tid] = cexit;
    L.stop[tid] = static_cast<uint8_t>(cstop);
    const uint64_t hm = __ballot(sp != ~0ull);
    if (lane == 0) L.has[tid >> 6] = hm;
    __syncthreads();
    SP(1);

    // 3. segments: chunk c continues its predecessor's segment when that
    // chunk's exit is c's start (and it did not stop); tails end segments
    bool tail = false;
    if (sp != ~0ull) {
        const uint32_t nxt = next_bit(L.has, tid + 1);
        tail = cstop || nxt >= kBlock || cexit != b0 + L.start[nxt];
    }
    const uint64_t tm = __ballot(tail);
    if (lane == 0) L.tail[tid >> 6] = tm;
    {
        uint64_t tot;
        const uint64_t x = block_xscan(ccnt, &tot, L.ws);
        L.pcnt[tid] = static_cast<uint32_t>(x);
        if (tid == 0) L.pcnt[kBlock] = static_cast<uint32_t>(tot);
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            const uint64_t y = block_xscan(cch[k], &tot, L.ws);
            L.pch[k][tid] = y;
            if (tid == 0) L.pch[k][kBlock] = tot;
        }
    }
    __syncthreads();

    SP(2);
    // 4. candidates (wave 0, lane = slot): position b0 + lane when plausible;
    // a window with none puts the first speculated start (sF) in slot 0.  The
    // primary slot is sF's: the entry the speculation itself predicts.
    const uint32_t F = next_bit(L.has, 0);
    const uint64_t sF = F < kBlock ? b0 + L.start[F] : ~0ull;
    if (tid < 64) {
        uint64_t mycand = ~0ull;
        if (b == 0) {
            if (lane == 0) mycand = 0;
        } else {
            const uint64_t p = b0 + lane;
            if (p < b1 && filter(a, so, p) && plausible(a, so, p)) mycand = p;
            if (!__ballot(mycand != ~0ull) && lane == 0 && sF != ~0ull) mycand = sF;
        }
        const uint64_t vmask = __ballot(mycand != ~0ull);
        const uint64_t pos0 = __shfl(mycand, 0, 64);  // slot 0's position (b0, sF, or none)
        uint32_t prim = kNoPrim;
        if (b == 0) prim = 0;
        else if (sF != ~0ull) prim = sF - b0 < kWin ? static_cast<uint32_t>(sF - b0) : 0;
        Agg<NC> mine{};
        if (mycand != ~0ull) mine = walk_chain<NC, false>(a, rd, L, b0, b1, mycand, nullptr, nullptr);
        const uint64_t t21 = a.epoch & kTagMax;
        if (b > 0) {  // publish the table (block 0 publishes its INC at once)
            uint64_t* t = S.agg + b * agg_block_words<NC>();
            if (mycand != ~0ull) {
                uint64_t* e = t + lane;
                st_sc1(e, tg(mine.exit, t21));
                st_sc1(e + kWin, tg(mine.cnt | (static_cast<uint64_t>(mine.stop) << 40), t21));
#pragma unroll
                for (int j = 0; j < NC; ++j) st_sc1(e + (2 + j) * kWin, tg(mine.ch[j], t21));
                if (lane == prim) {  // the primary entry again, beside the slot map
                    uint64_t* q = S.pri + b * pri_words<NC>();
                    st_sc1(q, tg(mine.exit, t21));
                    st_sc1(q + 1, tg(mine.cnt | (static_cast<uint64_t>(mine.stop) << 40), t21));
#pragma unroll
                    for (int j = 0; j < NC; ++j) st_sc1(q + 2 + j, tg(mine.ch[j], t21));
                }
            }
            if (lane == 0) {
                uint64_t* q = S.pri + b * pri_words<NC>() + 2 + NC;
                st_sc1(q, tg(pos0 == ~0ull ? kValMask : pos0, t21));
                st_sc1(q + 1, tg(vmask & 0xffffffffull, t21));
                st_sc1(q + 2, tg(vmask >> 32, t21));
                st_sc1(S.flag + b, tag | (kAgg << 8) | prim);  // every word above carries the tag
            }
        }

        SP(3);
        // 5. look-back: the inclusive state before this block
        St<NC> s{};
        uint32_t spins = 0;
        bool stalled = false;
        if (SRPC_STREAM_NOLOOK && b > 0) {
            s.ex = sF == ~0ull ? b1 : sF;
            s.cn = b * (a.n / a.nb);
        } else if (b > 0) {
            // (a) back, 64 flags per round trip, to the nearest block whose
            // INC is published; the blocks after it must have their tables
            int64_t top = static_cast<int64_t>(b) - 1, base = -1;
            while (true) {
                const int64_t j = top - static_cast<int64_t>(lane);
                const uint32_t stt = j >= 0 ? flag_state(ld_sc1(S.flag + j), a.epoch) : 0;
                const uint64_t incf = __ballot(stt == kInc);
                const uint32_t lim = incf ? __builtin_ctzll(incf) : 64;
                if (__ballot(j >= 0 && lane < lim && stt < kAgg)) {  // tables still to come
                    if (!spin(&spins)) {
                        stalled = true;
                        break;
                    }
                    continue;
                }
                if (incf) {
                    base = top - lim;
                    break;
                }
                top -= 64;  // 64 blocks with tables only: further back
                if (top < 0) {  // cannot happen (block 0 publishes an INC); never hang
                    stalled = true;
                    break;
                }
            }
            SP(4);
            SP_ADD(13, static_cast<uint64_t>(static_cast<int64_t>(b) - 1 - base));
            // (b) the INC of `base`, then the windows of blocks base + 1 .. b - 1,
            // one round trip each (words whose tag is not visible yet: again)
            bool have = false;
            for (uint64_t lo = static_cast<uint64_t>(base) + 1; !stalled && !(have && (s.stp & 1)); lo += 64) {
                const uint32_t cnt = lo < b ? static_cast<uint32_t>(min<uint64_t>(64, b - lo)) : 0;
                Win<NC> wv, bw;
                while (true) {
                    wv.load(S, a, lane < cnt ? static_cast<int64_t>(lo + lane) : -1, b);
                    if (!have) bw.load(S, a, base, b);
                    const bool need = (lane < cnt && !wv.pri_ok && !wv.inc_ok) || (!have && !bw.inc_ok);
                    if (!__ballot(need)) break;
                    if (!spin(&spins)) {
                        stalled = true;
                        break;
                    }
                }
                if (stalled) break;
                if (!have) {
                    s = bw.inc_state(__builtin_amdgcn_readfirstlane(lane));
                    have = true;
                }
                if (!cnt) break;
                SP_ADD(11, 1);
                fold<NC>(S, a, wv, s, lo, cnt, tag, t21, &spins, &stalled);
            }
        }
        if (stalled) s.stp = 1;  // reported; the result is not valid
        SP(5);

        // 6. this block's own chain from its entry: its slot, else a walk
        uint64_t x = ~0ull;
        const St<NC> s0 = s;
        if (!(s.stp & 1) && s.ex < b1) {
            x = s.ex;
            const uint64_t hit = __ballot(mycand == x);
            Agg<NC> g;
            if (hit) {
                const uint32_t hl = __builtin_ctzll(hit);
                g.exit = __shfl(mine.exit, hl, 64);
                g.cnt = __shfl(mine.cnt, hl, 64);
#pragma unroll
                for (int k = 0; k < NC; ++k) g.ch[k] = __shfl(mine.ch[k], hl, 64);
                g.stop = __shfl(mine.stop, hl, 64);
            } else {  // no candidate: walk from the entry (all lanes, same result)
                g = walk_chain<NC, false>(a, rd, L, b0, b1, x, nullptr, nullptr);
                if (lane == 0) {
                    atomicOr(&S.ctl[1], 2u);
                    atomicAdd(&S.ctl[2], 1u);
                }
            }
            s.ex = g.exit;
            s.cn += g.cnt;
#pragma unroll
            for (int k = 0; k < NC; ++k) s.ch[k] += g.ch[k];
            s.stp = g.stop;
        }
        if (lane == 0) {
            publish_inc<NC>(S, b, s, tag | (kInc << 8) | prim, t21);
            if (s.cn > a.n) atomicMin(&S.ctl[0], static_cast<uint32_t>(min<uint64_t>(b, 0xfffffffeull)));
            if (stalled) atomicOr(&S.ctl[3], 1u);
            L.s_x = x;
            L.s_cnt = s0.cn;
#pragma unroll
            for (int k = 0; k < NC; ++k) L.s_ch[k] = s0.ch[k];
        }
    }
    __syncthreads();
    const uint64_t x = L.s_x;
    const uint64_t R = L.s_cnt;
    SP(6);
    if (x == ~0ull || R > a.n || SRPC_STREAM_NOOUT) return;  // no record starts here (or all are past record n)
    SP_ADD(15, 1);

    // 7. the chain's records in order: walk again recording explicit starts
    // (the list lives in the image area until the table is built)
    uint16_t* xl = reinterpret_cast<uint16_t*>(L.img);
    if (tid == 0) {
        uint32_t ne = 0;
        (void)walk_chain<NC, true>(a, rd, L, b0, b1, x, xl, &ne);
        L.s_nexp = ne;
        if (ne || x != sF) atomicOr(&S.ctl[1], 1u);  // the chain left the block's speculation
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
    const bool jumped = (L.jump[tid >> 6] >> (tid & 63)) & 1;
    const uint32_t ccount = L.pcnt[tid + 1] - L.pcnt[tid];
    const uint32_t fc = (e1 - e0) + (jumped ? ccount : 0);
    uint64_t tot;
    const uint32_t fb = static_cast<uint32_t>(block_xscan(fc, &tot, L.ws));
    for (uint32_t k = e0; k < e1; ++k) L.tbl[fb + (k - e0)] = xl[k];
    if (jumped)
        for (uint32_t k = 0; k < ccount; ++k)
            L.tbl[fb + (e1 - e0) + k] = static_cast<uint16_t>(tid * kSC + L.list[tid * 5 + k]);
    __syncthreads();
    const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(tot, kMaxRec));

    SP(7);
    // 8. outputs: record r = R + k of the batch (up to index n)
    const uint64_t n = a.n;
    for (uint32_t k = tid; k < nrec; k += kBlock) {
        const uint64_t r = R + k;
        if (r > n) break;
        const uint64_t s = b0 + L.tbl[k];
        a.rec_offs[r] = s;
        if (!kDecode || r == n) continue;
        uint64_t pos = s + a.prefix_len;
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
                pos += 8 + v;
            }
        }
    }
    SP(8);
    if constexpr (kDecode) {
        // per string field: local offsets (a scan over the block's records),
        // str_offs, the chars image, aligned stores
        uint64_t Pbase[kMaxNC + 1];
        {
            uint64_t sum = 0;
#pragma unroll
            for (int k = 0; k < NC; ++k) {
                Pbase[k] = L.s_ch[k];
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
            // lengths of this field (strided: lane per record)
            for (uint32_t k = tid; k < nrec; k += kBlock) {
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
                L.loff[k] = k < nw ? static_cast<uint32_t>(len) : 0;
            }
            __syncthreads();
            // contiguous per lane: serial sums, then the block scan
            uint64_t mysum = 0;
            const uint32_t k0 = min(tid * per, nrec), k1 = min(k0 + per, nrec);
            for (uint32_t k = k0; k < k1; ++k) mysum += L.loff[k];
            uint64_t ftot;
            uint64_t run = block_xscan(mysum, &ftot, L.ws);
            for (uint32_t k = k0; k < k1; ++k) {
                const uint32_t len = L.loff[k];
                L.loff[k] = static_cast<uint32_t>(run);
                run += len;
            }
            if (tid == 0) L.loff[nrec] = static_cast<uint32_t>(ftot);
            __syncthreads();
            uint64_t* so = a.soff[f];
            uint8_t* chars = a.col[f];
            for (uint32_t k = tid; k <= nrec && R + k <= n; k += kBlock)
                if (k < nrec) so[R + k] = P + L.loff[k];
            const bool fits = ftot + 32 <= kImage;
            // copy each record's chars into the image (or straight to the output)
            for (uint32_t k = tid; k < nw; k += kBlock) {
                const uint32_t o = L.loff[k], len = L.loff[k + 1] - o;
                if (!len) continue;
                const uint64_t s = b0 + L.tbl[k];
                uint64_t pos = s + a.prefix_len;
                for (uint32_t g = 0; g < f; ++g) pos += a.size[g] ? a.size[g] : 8 + rd.u64(pos);
                pos += 8;
                if (fits) {
                    const uint32_t d = 16 + o;
                    if (rd.staged(pos, pos + len)) {
                        // LDS offsets from the start of L (the stage precedes the image)
                        uint8_t* l0 = reinterpret_cast<uint8_t*>(&L);
                        lds_copy_run(l0, static_cast<uint32_t>(L.img - l0) + d,
                                     static_cast<uint32_t>(L.st - l0) + static_cast<uint32_t>(pos - rd.base), len);
                    } else {
                        for (uint32_t x8 = 0; x8 < len; x8 += 8) {
                            const uint32_t kk = min<uint32_t>(8, len - x8);
                            uint64_t v = 0;
                            for (uint32_t bb = 0; bb < kk; ++bb) v |= static_cast<uint64_t>(w[pos + x8 + bb]) << (8 * bb);
                            lds_put_small(L.img, d + x8, v, kk);
                        }
                    }
                } else {
                    uint8_t* dst = chars + P + o;
                    for (uint32_t bb = 0; bb < len; ++bb) dst[bb] = rd.u8(pos + bb);
                }
            }
            __syncthreads();
            if (fits && ftot) {
                // chunk c of the output covers image bytes [16c - h, 16c + 16 - h)
                const uint32_t h = static_cast<uint32_t>(P & 15);
                const uint64_t gbase = P & ~15ull;
                const uint8_t* im = L.img + 16;
                const uint32_t span = h + static_cast<uint32_t>(ftot);
                const uint32_t nch = (span + 15) >> 4;
                const uint32_t sh = (16 - h) & 15;
                for (uint32_t c = tid; c < nch; c += kBlock) {
                    const uint32_t lo = max(h, 16 * c), hi2 = min(span, 16 * c + 16);
                    if (lo == 16 * c && hi2 == 16 * c + 16) {
                        const uint32_t* wd = reinterpret_cast<const uint32_t*>(im + 16 * c - h - sh);
                        const uint32_t w0 = wd[0], w1 = wd[1], w2 = wd[2], w3 = wd[3], w4 = wd[4], w5 = wd[5],
                                       w6 = wd[6], w7 = wd[7];
                        uint32_t o0, o1, o2, o3;
                        const uint32_t bsh = sh & 3;
                        switch (sh >> 2) {  // uniform
                        case 0:
                            o0 = __builtin_amdgcn_alignbyte(w1, w0, bsh); o1 = __builtin_amdgcn_alignbyte(w2, w1, bsh);
                            o2 = __builtin_amdgcn_alignbyte(w3, w2, bsh); o3 = __builtin_amdgcn_alignbyte(w4, w3, bsh);
                            break;
                        case 1:
                            o0 = __builtin_amdgcn_alignbyte(w2, w1, bsh); o1 = __builtin_amdgcn_alignbyte(w3, w2, bsh);
                            o2 = __builtin_amdgcn_alignbyte(w4, w3, bsh); o3 = __builtin_amdgcn_alignbyte(w5, w4, bsh);
                            break;
                        case 2:
                            o0 = __builtin_amdgcn_alignbyte(w3, w2, bsh); o1 = __builtin_amdgcn_alignbyte(w4, w3, bsh);
                            o2 = __builtin_amdgcn_alignbyte(w5, w4, bsh); o3 = __builtin_amdgcn_alignbyte(w6, w5, bsh);
                            break;
                        default:
                            o0 = __builtin_amdgcn_alignbyte(w4, w3, bsh); o1 = __builtin_amdgcn_alignbyte(w5, w4, bsh);
                            o2 = __builtin_amdgcn_alignbyte(w6, w5, bsh); o3 = __builtin_amdgcn_alignbyte(w7, w6, bsh);
                            break;
                        }
                        __builtin_nontemporal_store(u32x4{o0, o1, o2, o3}, reinterpret_cast<u32x4*>(chars + gbase + 16 * c));
                    } else {
                        for (uint32_t xx = lo; xx < hi2; ++xx) chars[gbase + xx] = im[xx - h];
                    }
                }
            }
            __syncthreads();
        }
    }
    SP(9);
}

// Records the stream holds, T, from the last block's state: rec_offs[T] =
// where the stream stopped (the failing record's start, or the end of the
// last record), rec_offs[T + 1 .. n] = W, str_offs[f][T .. n] = the chars
// total; with T < n the status names record T (PREFIX or BOUNDS, and BOUNDS
// for every record after it).  With T >= n every entry came from the blocks,
// except [n] when T == n.
template <int NC, bool kDecode>
__global__ __launch_bounds__(kBlock) void k_stream_finish(StreamArgs a, Scratch S, srpc_unpack_status* st,
                                                          const uint32_t* gate) {
    if (gate && !*gate) return;
    constexpr uint32_t IW = inc_words<NC>();
    uint64_t ex = 0, T = 0, ch[kMaxNC + 1] = {};
    uint32_t stp = 0;
    if (a.nb) {
        const uint64_t* iw = S.inc + static_cast<uint64_t>(a.nb - 1) * IW;
        ex = iw[0] & kValMask;
        T = iw[1] & kCnt40;
        stp = static_cast<uint32_t>((iw[1] >> 40) & 7);
#pragma unroll
        for (int k = 0; k < NC; ++k) ch[k] = iw[2 + k] & kValMask;
    }
    const uint64_t n = a.n;
    if (T > n) return;
    uint64_t tot[kMaxNC + 1];
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        tot[k] = ch[k];
        sum += ch[k];
    }
    tot[NC] = ex - T * a.fixed_bytes - sum;
    const uint64_t gs = static_cast<uint64_t>(gridDim.x) * kBlock;
    for (uint64_t r = T + static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; r <= n; r += gs) {
        a.rec_offs[r] = r == T ? ex : a.W;
        if (kDecode)
            for (uint32_t f = 0; f < a.nfields; ++f) {
                if (a.size[f]) continue;
                const uint32_t si = a.sord[f];
                uint64_t v = 0;
#pragma unroll
                for (int k = 0; k <= NC; ++k) v = si == static_cast<uint32_t>(k) ? tot[k] : v;
                a.soff[f][r] = v;
            }
    }
    if (kDecode && st && blockIdx.x == 0 && threadIdx.x == 0) {
        uint32_t fl = S.ctl[3] ? SRPC_STATUS_STALLED : 0;
        if (T < n) {
            const uint32_t kind = (stp & 1) ? (stp >> 1) & 3 : 0;
            fl |= (kind ? kind : SRPC_STATUS_BOUNDS) | (T + 1 < n ? SRPC_STATUS_BOUNDS : 0);
            st->first_bad_record = T;
        }
        st->flags |= fl;
    }
}

__global__ void k_stream_reset(Scratch S, srpc_unpack_status* st, const uint32_t* gate) {
    if (gate && !*gate) return;
    if (threadIdx.x == 0) {
        S.ctl[0] = 0xffffffffu;
        S.ctl[1] = 0;
        S.ctl[2] = 0;
        S.ctl[3] = 0;
        if (st) {
            st->flags = 0;
            st->reserved = 0;
            st->first_bad_record = ~0ull;
        }
    }
}

// Diagnostics (srpc_unpack_status.reserved): bit 1 = this decode ran, bit 2 =
// a block's chain left its speculation (explicit records, or an entry that was
// not the speculated start), bits 8-31 = blocks whose entry was in none of
// their candidates (each walked from it after its predecessor's state came;
// saturating).
__global__ void k_stream_note(Scratch S, srpc_unpack_status* st, const uint32_t* gate) {
    if (gate && !*gate) return;
    if (threadIdx.x == 0 && st)
        st->reserved |= 2u | ((S.ctl[1] & 1u) << 2) | (min<uint32_t>(S.ctl[2], 0xffffffu) << 8);
}

uint64_t r256(uint64_t b) { return (b + 255) & ~255ull; }

struct StreamLayout {
    uint64_t nb, flag, inc, agg, pri, ctl, total;
};

StreamLayout stream_layout(uint64_t wire_len, uint32_t nc) {
    StreamLayout L{};
    L.nb = (wire_len + kSB - 1) / kSB;
    uint64_t o = 0;
    L.flag = o;
    o += r256(8 * L.nb);
    L.inc = o;
    o += r256(8 * L.nb * (2 + nc));
    L.agg = o;
    o += r256(8 * L.nb * (2 + nc) * kWin);
    L.pri = o;
    o += r256(8 * L.nb * (5 + nc));
    L.ctl = o;
    o += 256;
    L.total = o;
    return L;
}

// This call's epoch: process-unique, starting at a random value so flag words
// left in recycled memory by another process do not match.
uint32_t next_epoch() {
    static std::atomic<uint32_t> ctr{static_cast<uint32_t>(
        std::chrono::steady_clock::now().time_since_epoch().count() * 2654435761u ^ static_cast<uint32_t>(getpid()))};
    uint32_t e;
    do e = ctr.fetch_add(1, std::memory_order_relaxed);
    while (e == 0);
    return e;
}

template <int NC, bool kDecode>
void launch_stream(const StreamArgs& a, const uint8_t* wire, const Scratch& S, srpc_unpack_status* st, hipStream_t s,
                   const uint32_t* gate) {
    launch(k_stream_reset, dim3(1), dim3(64), 0, s, S, kDecode ? st : nullptr, gate);
    if (a.nb) launch(k_stream_decode<NC, kDecode>, dim3(a.nb), dim3(kBlock), 0, s, a, wire, S, gate);
    const uint32_t g = static_cast<uint32_t>(std::min<uint64_t>(a.n / kBlock + 1, 4096));
    launch(k_stream_finish<NC, kDecode>, dim3(g), dim3(kBlock), 0, s, a, S, st, gate);
}

}  // namespace
}  // namespace srpc_impl

namespace srpc_impl {

bool stream1_decodes(const srpc_plan* p) { return p->nstrings <= kMaxNC + 1; }

uint64_t stream1_scratch_bytes(const srpc_plan* p, uint64_t wire_len) {
    return stream_layout(wire_len, stream1_decodes(p) ? p->nstrings - 1 : 0).total;
}

int stream1_launch(const srpc_plan* p, const uint8_t* wire, uint64_t wire_len, uint64_t n, uint64_t* rec_offs,
                   void* const* cols, uint64_t* const* str_offs, srpc_unpack_status* st, void* scratch,
                   const uint32_t* gate, hipStream_t s) {
    const bool decode = stream1_decodes(p);
    const uint32_t nc = decode ? p->nstrings - 1 : 0;
    const StreamLayout SL = stream_layout(wire_len, nc);
    // positions, counts and chars travel as 43-bit values in the look-back words
    if (SL.nb > 0x7fffffffull || p->fixed_bytes < 8 || wire_len >= (1ull << 40)) return SRPC_E_UNSUPPORTED;
    auto* base = static_cast<uint8_t*>(scratch);
    Scratch S{reinterpret_cast<uint64_t*>(base + SL.flag), reinterpret_cast<uint64_t*>(base + SL.inc),
              reinterpret_cast<uint64_t*>(base + SL.agg), reinterpret_cast<uint64_t*>(base + SL.pri),
              reinterpret_cast<uint32_t*>(base + SL.ctl)};
    StreamArgs a{};
    uint32_t si = 0;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        a.size[f] = p->size[f];
        a.sord[f] = p->size[f] ? 0 : si++;
        a.col[f] = static_cast<uint8_t*>(cols[f]);
        a.soff[f] = p->size[f] ? nullptr : str_offs[f];
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
    a.cap = 1 + kSC / p->fixed_bytes;
    a.nb = static_cast<uint32_t>(SL.nb);
    a.epoch = next_epoch();
    if (!decode) launch_stream<0, false>(a, wire, S, st, s, gate);
    else if (nc == 0) launch_stream<0, true>(a, wire, S, st, s, gate);
    else if (nc == 1) launch_stream<1, true>(a, wire, S, st, s, gate);
    else if (nc == 2) launch_stream<2, true>(a, wire, S, st, s, gate);
    else launch_stream<3, true>(a, wire, S, st, s, gate);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int stream1_note(const srpc_plan* p, uint64_t wire_len, void* scratch, srpc_unpack_status* st, const uint32_t* gate,
                 hipStream_t s) {
    const StreamLayout SL = stream_layout(wire_len, stream1_decodes(p) ? p->nstrings - 1 : 0);
    auto* base = static_cast<uint8_t*>(scratch);
    Scratch S{nullptr, nullptr, nullptr, nullptr, reinterpret_cast<uint32_t*>(base + SL.ctl)};
    if (st) hipLaunchKernelGGL(k_stream_note, dim3(1), dim3(64), 0, s, S, st, gate);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

}  // namespace srpc_impl

#ifdef SRPC_STREAM_PHASES
extern "C" {
// Diagnostics: per-block phase words go to d_buf (16 u64 per block, the
// caller zeroes it) for blocks below nblocks.
int srpc_debug_stream_phases(void* d_buf, uint64_t nblocks) {
    unsigned long long* p = static_cast<unsigned long long*>(d_buf);
    unsigned long long nb = nblocks;
    if (hipMemcpyToSymbol(HIP_SYMBOL(srpc_impl::g_sph), &p, sizeof(p)) != hipSuccess) return SRPC_E_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(srpc_impl::g_sph_blocks), &nb, sizeof(nb)) != hipSuccess) return SRPC_E_HIP;
    return SRPC_OK;
}
}
#endif
