// stream.hip -- decode a concatenated record stream with no index
// (srpc_gpu_unpack_var_stream).
//
// The reference decodes a batch with ONE shared cursor (buffer::_offset,
// core.hpp:39): each pipe_output advances it (packer.hpp:210-222, nested
// unpack sharing the buffer as in tests/packer_test.cpp:77-88), so where a
// record starts is only known once every record before it was read.  Here
// the record index is found on the device, then the indexed decode runs.
//
// 1. k_stream_chunks -- the wire is cut into chunks of kChunk bytes.  A
//    lane per chunk (its workgroup's chunks staged in LDS) finds the first
//    position p at which a.plaus records parse one after another (a
//    plausible record start: a string length read at a wrong offset is
//    almost always past the end of the wire; see k_stream_chunks for the one
//    exception), then walks records from there while they start inside the
//    chunk: their starts, count, the position after them ("exit": the first
//    record start at or past the chunk end, or where a record failed to
//    parse), and why the walk stopped.
// 2. the check (in k_stream_chunks; k_stream_check_edges for each
//    workgroup's leading chunks) -- chunk c is right when its start equals the exit of
//    chunk c - 1 (or chunk c holds no record start at all), chunk 0 when it
//    starts at 0.  By induction every chunk up to the first wrong one is
//    right.
// 3. repair rounds (k_stream_refix / k_stream_recheck, gated) walk the wrong
//    chunks again from entries that are final.  If chunks are still wrong
//    after them (data on which a wrong start parses too: zero-heavy strings,
//    records of zeros), k_stream_gate hands the stream to the single-pass
//    decode of stream1.hip, whose work is bounded for any input (per-block
//    candidate tables and a decoupled look-back, no serial walk over the
//    stream); its kernels are launched on the same stream and return at once
//    unless the gate is set.
// 4. the chunks' record counts are scanned to record numbers, and
//    k_stream_index copies each chunk's record starts into rec_offs[];
//    k_stream_tail fills what the stream does not hold.
// The walk is orc_unpack's cursor (oracle/packer_oracle.c): the prefix must
// match, every read must fit in the wire.  A record that fails stops the
// stream: its start becomes rec_offs[i], every later entry wire_len, so the
// indexed decode reports it (PREFIX or BOUNDS) as the first bad record, and
// every later record as BOUNDS.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>

#include "plan.h"
#include "scan.h"
#include "srpc_gpu.h"
#include "sdec.h"
#include "stream1.h"


namespace srpc_impl {
namespace {

#ifndef SRPC_STREAM_CHUNK
#define SRPC_STREAM_CHUNK 64
#endif
constexpr uint32_t kChunk = SRPC_STREAM_CHUNK;  // wire bytes per speculating lane (<= 64: the filter's mask)
static_assert(kChunk <= 64 && kChunk % 16 == 0, "a chunk's positions fit one 64-bit mask; 16-byte window reads");
// records that must parse from a candidate start: with an envelope prefix of
// 8 bytes or more a wrong start essentially never matches it, so one; else 2
// (a wrong start that hops onto a true one passes any count: see k_stream_scan)
constexpr uint32_t kPlausPrefixed = 1, kPlausBare = 2;
constexpr uint64_t kNone = ~0ull;   // chunk holds no plausible record start
constexpr uint32_t kStopEnd = 1;    // the walk reached the end of the wire exactly
constexpr uint32_t kStopBad = 2;    // a record failed to parse at the exit position
#ifndef SRPC_STREAM_ROUNDS
#define SRPC_STREAM_ROUNDS 3
#endif
constexpr int kRepairRounds = SRPC_STREAM_ROUNDS;  // parallel repair rounds before the hand-over

struct StreamArgs {
    uint32_t size[kMaxFields];  // fixed field bytes, 0 = string
    const uint8_t* prefix;      // device copy (16 zero bytes past the end)
    uint32_t nfields, prefix_len;
    uint32_t first_len_at;      // byte offset of the first string's u64 length in a record
    uint32_t plaus;             // records that must parse from a candidate start
    uint64_t pre8;              // the prefix's first 8 bytes (zero padded)
};

struct Chunks {      // per chunk (scratch, C entries each)
    uint64_t* start;  // first record start walked from (kNone: none in the chunk)
    uint64_t* cnt;    // records starting in [start, chunk end)
    uint64_t* exit;   // position after them
    uint32_t* stop;   // kStopEnd / kStopBad / 0
    uint32_t* bad;    // chunk disagrees with its predecessor
    uint32_t* blk;    // per 256 chunks: bit 0 some chunk is bad, bit 1 some chunk stops
    uint32_t* ctl;    // [0] any bad, [1] the stream's stop chunk, [2] the first bad chunk, [3..6] see below
    uint8_t* list;    // per chunk: its records' starts minus the chunk's first byte, cap entries each
    uint32_t cap;     // 1 + kChunk / the smallest record (fixed_bytes): a chunk's records at most
};

template <typename T>
__device__ __forceinline__ T ld(const uint8_t* p) {
    T v;
    __builtin_memcpy(&v, p, sizeof(T));
    return v;
}

typedef const uint8_t __attribute__((address_space(1))) global_u8;
typedef uint8_t __attribute__((address_space(3))) lds_u8;
typedef const uint8_t __attribute__((address_space(3))) lds_u8c;
typedef const uint32_t __attribute__((address_space(3))) lds_u32c;
typedef const uint64_t __attribute__((address_space(3))) lds_u64c;

// Wire readers: global memory, or a workgroup's LDS copy of wire bytes
// [lo, hi) with global memory past it (records that start near the end of the
// workgroup's span and run past its margin).  Typed address spaces, so the
// reads are ds_read / global_load, not flat.
struct GlobalRd {
    const uint8_t* w;
    const uint8_t* pre;  // the prefix (device copy)
    __device__ __forceinline__ uint64_t u64(uint64_t p) const { return ld<uint64_t>(w + p); }
    __device__ __forceinline__ uint8_t u8(uint64_t p) const { return w[p]; }
    __device__ __forceinline__ uint64_t pre64(uint32_t i) const { return ld<uint64_t>(pre + i); }
    __device__ __forceinline__ uint8_t pre8(uint32_t i) const { return pre[i]; }
};
struct StagedRd {
    global_u8* w;
    lds_u8c* lds;  // lds[x] = wire byte base + x, for wire offsets [lo, hi)
    uint64_t base, lo, hi;
    lds_u8c* pre;  // LDS copy of the prefix, 8-aligned
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
    __device__ __forceinline__ uint64_t pre64(uint32_t i) const { return *reinterpret_cast<lds_u64c*>(pre + i); }
    __device__ __forceinline__ uint8_t pre8(uint32_t i) const { return pre[i]; }
};
// The staged bytes only, for speculation: a read past them yields ~0 (no
// length fits, no prefix matches), so a candidate whose records run past the
// stage is not plausible -- a start one byte early whose length reads as
// len * 256 + a char would otherwise send every lane to global memory.  A true
// start of a record longer than the margin is missed the same way and left to
// the repair rounds.
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
// *err set (SRPC_STATUS_PREFIX / SRPC_STATUS_BOUNDS).
template <class Rd>
__device__ __forceinline__ uint64_t parse_rd(const StreamArgs& a, const Rd& r, uint64_t W, uint64_t p,
                                             uint32_t* err) {
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
    }
    return q;
}

__device__ uint64_t parse_at(const StreamArgs& a, const uint8_t* w, uint64_t W, uint64_t p, uint32_t* err) {
    return parse_rd(a, GlobalRd{w, a.prefix}, W, p, err);
}

// Walk from p while records start before hi: count, exit, stop reason.
template <class Rd>
__device__ __forceinline__ void walk_rd(const StreamArgs& a, const Rd& r, uint64_t W, uint64_t p, uint64_t hi,
                                        uint64_t* cnt, uint64_t* exit, uint32_t* stop, uint8_t* list, uint32_t cap) {
    uint64_t k = 0;
    *stop = 0;
    while (p < hi) {
        uint32_t err;
        const uint64_t q = parse_rd(a, r, W, p, &err);
        if (err) {
            *stop = kStopBad;
            break;
        }
        // always: records are >= fixed_bytes long; a start lies in [chunk, chunk + kChunk)
        if (k < cap) list[k] = static_cast<uint8_t>(p % kChunk);
        ++k;
        p = q;
    }
    if (!*stop && p >= W) *stop = kStopEnd;
    *cnt = k;
    *exit = p;
}
__device__ void walk(const StreamArgs& a, const uint8_t* w, uint64_t W, uint64_t p, uint64_t hi, uint64_t* cnt,
                     uint64_t* exit, uint32_t* stop, uint8_t* list, uint32_t cap) {
    walk_rd(a, GlobalRd{w, a.prefix}, W, p, hi, cnt, exit, stop, list, cap);
}

// Necessary for a record to parse at p: the prefix's first (up to 8) bytes
// match and the first string's length fits the wire.
template <class Rd>
__device__ __forceinline__ bool filter(const StreamArgs& a, const Rd& r, uint64_t W, uint64_t p) {
    if (a.first_len_at + 8 > W - p) return false;
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
__device__ __forceinline__ bool plausible(const StreamArgs& a, const Rd& r, uint64_t W, uint64_t p) {
    for (uint32_t k = 0; k < a.plaus; ++k) {
        if (p == W) return k > 0;  // the stream may end right after a record
        uint32_t err;
        const uint64_t q = parse_rd(a, r, W, p, &err);
        if (err) return false;
        p = q;
    }
    return true;
}

// The entry of chunk c (the first record start at or after its beginning):
// the exit of the nearest chunk before it with a record start, or a stop.
__device__ __forceinline__ uint64_t entry_of(const Chunks& ch, uint64_t c, bool* stopped) {
    *stopped = false;
    for (uint64_t j = c; j-- > 0;) {
        if (ch.start[j] == kNone) continue;  // passes its own entry through
        *stopped = ch.stop[j] != 0;
        return ch.exit[j];
    }
    return 0;  // unreachable: chunk 0 always starts at 0
}

// Chunk c agrees with its entry e when it starts exactly there, or -- e past
// the chunk's end -- when it found no record start.
__device__ __forceinline__ bool agrees(uint64_t e, uint64_t chunk_hi, uint64_t start) {
    return e >= chunk_hi ? start == kNone : start == e;
}

// A wave's bad chunks: one atomic per wave on the flags (every lane of the
// wave calls this: thousands of bad chunks on one control word serialised the
// check kernel), one per 256-chunk block word.
__device__ __forceinline__ void note_bad(const Chunks& ch, uint64_t c, bool bad, int any_at, int first_at) {
    const uint64_t m = __ballot(bad);
    if (!m) return;
    const uint32_t lane = threadIdx.x & 63, lead = __builtin_ctzll(m);
    if (lane == lead) {  // the wave's first bad chunk; a wave's 64 chunks share one block word
        atomicOr(&ch.ctl[any_at], 1u);
        atomicMin(&ch.ctl[first_at], static_cast<uint32_t>(min<uint64_t>(c, 0xfffffffeull)));
        atomicOr(&ch.blk[c >> 8], 1u);
    }
}

// The N dwords at LDS byte offset o & ~3 of the stage, in 16-byte reads (o
// mod 16 is the same for every lane of the workgroup: chunks are a multiple
// of 16 bytes apart, so the dword shift is a uniform switch).  Lanes' windows
// sit kChunk bytes apart on the same banks: dword reads made the 19-dword
// window 19 conflicted LDS ops (82 % of LDS cycles conflicted); 6 wide reads
// cut the stream decode 7-12 % (profiles/r02_stream_window_ab.log).
template <int N>
__device__ __forceinline__ void lds_window(const uint8_t* st, uint32_t o, uint32_t (&d)[N]) {
    constexpr int NQ = (N + 3 + 3) / 4;
    uint32_t w[4 * NQ];
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    typedef const u32x4v __attribute__((address_space(3))) lds_u32x4c;
    lds_u32x4c* q = reinterpret_cast<lds_u32x4c*>((lds_u8c*)st + (o & ~15u));
#pragma unroll
    for (int i = 0; i < NQ; ++i) {
        const u32x4v v = q[i];
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

// Chunk c's speculation and walk (k_stream_chunks, a lane per chunk of
// kChunk bytes): a workgroup stages its kBlock chunks plus a margin in LDS
// (LDS-DMA), and every lane, from LDS, finds its chunk's first plausible
// record start -- a cheap filter first (the prefix's first bytes, the first
// string's length fits the wire), then whole records parse from it (a
// plausible start) -- and walks the records from there that start inside the
// chunk: their starts, count, the position after them and why the walk
// stopped.  A start 1-3 bytes early is plausible too: its first string length
// reads the previous record's last chars as low bytes and the true length
// (little-endian, small) shifted up, and the jump it makes lands on a true
// record start about once per average record size -- after which every record
// parses.  So of the plausible starts within the 8 bytes of a length field the
// one with the smallest first string length is taken: the true start (random
// strings: ~0.05 % of chunks wrong).  A chunk with no plausible start (inside
// a long record) passes its entry through: start = exit = kNone, no records.
// Reads past the staged bytes (a record running past the margin) go to global
// memory.  (Round 2 before: a wave per 512-byte chunk speculating and a lane
// per chunk walking, both from global memory -- chains of dependent reads,
// 1.7 ms for a 4M-record stream of two strings; a wave per chunk from LDS with
// a lane-0 walk was compute-bound, profiles/r02_stream_lds_ab.log.)
constexpr uint32_t kStreamMargin = 2048;
constexpr uint32_t kStreamStage = kBlock * kChunk + kStreamMargin + 32;
__global__ __launch_bounds__(kBlock) void k_stream_chunks(StreamArgs a, const uint8_t* __restrict__ w, uint64_t W,
                                                          uint64_t C, Chunks ch) {
    __shared__ __attribute__((aligned(16))) uint8_t st[kStreamStage + 16];
    __shared__ __attribute__((aligned(16))) uint8_t pre[kMaxPrefix + 16];
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = threadIdx.x; i < a.prefix_len; i += kBlock) pre[i] = a.prefix[i];
    const uint64_t c0 = static_cast<uint64_t>(blockIdx.x) * kBlock;
    const uint64_t lo = c0 * kChunk;
    const uint64_t hi = min<uint64_t>(lo + kBlock * kChunk + kStreamMargin, W);
    const uint64_t A = (reinterpret_cast<uint64_t>(w) + lo) & ~15ull;
    const uint32_t ng = static_cast<uint32_t>((reinterpret_cast<uint64_t>(w) + hi - A + 15) >> 4);
    for (uint32_t w0 = threadIdx.x & ~63u; w0 < ng; w0 += kBlock) {
        const uint32_t gi = w0 + lane;
        if (gi < ng) {
            const uint32_t wb = __builtin_amdgcn_readfirstlane(w0);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<global_u8*>(A + 16ull * gi), (lds_u8*)(st + 16 * wb), 16,
                                             0, 0);
        }
    }
    __syncthreads();  // waits for the LDS-DMA and publishes the stage
    const StagedRd r{(global_u8*)w, (lds_u8c*)st, A - reinterpret_cast<uint64_t>(w), lo, hi, (lds_u8c*)pre};
    const StageOnlyRd so{r};
    const uint64_t c = c0 + threadIdx.x;
    const uint64_t clo = c * kChunk, chi = min(clo + kChunk, W);
    uint64_t b = kNone;
    if (c >= C) {
        // past the last chunk: nothing (the check below still needs the lane)
    } else if (c == 0) {
        b = 0;  // the stream starts at 0: no speculation
    } else {
        // the filter at the chunk's 64 positions, from two register windows of
        // the staged bytes (the first string's length at p + first_len_at, the
        // prefix's first 8 bytes at p), all lanes in step: a mask of the
        // positions that pass.  Then the passing positions are parsed in
        // order until one is plausible -- a lane parses only its few
        // candidates, instead of the wave running the parse at every position
        // some lane's filter passed (the divergent per-position loop issued
        // ~30K instructions per wave).
        const uint32_t at = static_cast<uint32_t>(clo - r.base);  // LDS offset of the chunk
        uint64_t mask = 0;
        {
            uint32_t d[kChunk / 4 + 3];
            const uint32_t o = at + a.first_len_at, sh = o & 3;
            lds_window(st, o, d);
#pragma unroll
            for (int k = 0; k < kChunk / 4 + 2; ++k) d[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
            // position j: bytes j .. j + 7 of the shifted window
            // position j passes when len + j <= lim0 = W - (clo + first_len_at + 8)
            // (a wrapped sum only adds a candidate: the filter stays necessary)
            const uint64_t need = clo + a.first_len_at + 8;
            const uint64_t lim0 = need <= W ? W - need : 0;
#pragma unroll
            for (int j = 0; j < static_cast<int>(kChunk); ++j) {
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
            uint32_t d[kChunk / 4 + 3];
            const uint32_t sh = at & 3;
            lds_window(st, at, d);
#pragma unroll
            for (int k = 0; k < kChunk / 4 + 2; ++k) d[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
            const uint32_t k8 = a.prefix_len < 8 ? a.prefix_len : 8;
            const uint64_t pm = k8 == 8 ? ~0ull : (1ull << (8 * k8)) - 1;
            uint64_t keep = 0;
#pragma unroll
            for (int j = 0; j < static_cast<int>(kChunk); ++j) {
                const int k = j >> 2, s8 = j & 3;
                const uint32_t lo32 = s8 ? __builtin_amdgcn_alignbyte(d[k + 1], d[k], s8) : d[k];
                const uint32_t hi32 = s8 ? __builtin_amdgcn_alignbyte(d[k + 2], d[k + 1], s8) : d[k + 1];
                const uint64_t v = (static_cast<uint64_t>(hi32) << 32) | lo32;
                keep |= static_cast<uint64_t>(((v ^ a.pre8) & pm) == 0) << j;
            }
            mask &= keep;
        }
        const uint64_t passing = mask;
        while (mask) {
            const uint32_t j = __builtin_ctzll(mask);
            if (plausible(a, so, W, clo + j)) {
                b = clo + j;
                break;
            }
            mask &= mask - 1;
        }
        if (b != kNone) {
            // candidates b .. b + 7 inside the chunk (filter-passing, plausible):
            // argmin of (first string length, position)
            const uint32_t jb = static_cast<uint32_t>(b - clo);
            uint64_t cand = (passing >> (jb + 1)) & 0x7f;
            uint64_t best = so.u64(b + a.first_len_at), pick = b;
            while (cand) {
                const uint64_t q = b + 1 + __builtin_ctzll(cand);
                cand &= cand - 1;
                const uint64_t l = so.u64(q + a.first_len_at);
                if (l < best && plausible(a, so, W, q)) {
                    best = l;
                    pick = q;
                }
            }
            b = pick;
        }
    }
    uint64_t cnt = 0, exit = kNone;
    uint32_t stop = 0;
    if (b != kNone) walk_rd(a, r, W, b, chi, &cnt, &exit, &stop, ch.list + c * ch.cap, ch.cap);
    __shared__ uint64_t s_start[kBlock], s_exit[kBlock];
    __shared__ uint32_t s_stop[kBlock];
    s_start[threadIdx.x] = b;
    s_exit[threadIdx.x] = exit;
    s_stop[threadIdx.x] = stop;
    if (c < C) {
        ch.start[c] = b;
        ch.cnt[c] = cnt;
        ch.exit[c] = exit;
        ch.stop[c] = stop;
        if (stop) atomicOr(&ch.blk[c >> 8], 2u);
    }
    __syncthreads();
    // the check (k_stream_check's rule) for chunks whose entry comes from a
    // chunk of this workgroup; the others -- the leading chunks up to the
    // first one with a record start -- are checked by k_stream_check_edges
    bool bad = false;
    if (c < C && c > 0) {
        int j = static_cast<int>(threadIdx.x) - 1;
        while (j >= 0 && s_start[j] == kNone) --j;  // chunks with no start pass their entry through
        if (j >= 0) bad = !(s_stop[j] != 0 || agrees(s_exit[j], chi, b));
    }
    if (c < C && (c == 0 || threadIdx.x > 0)) {
        bool edge = c > 0;
        for (int j = static_cast<int>(threadIdx.x) - 1; edge && j >= 0; --j) edge = s_start[j] == kNone;
        if (!edge) ch.bad[c] = bad ? 1u : 0u;
    }
    note_bad(ch, c, bad, 0, 2);
}

// The leading chunks of every workgroup of k_stream_chunks (those before and
// including its first chunk with a record start), whose entry is the exit of
// an earlier workgroup's chunk: a lane per workgroup, k_stream_check's rule.
__global__ __launch_bounds__(kBlock) void k_stream_check_edges(uint64_t W, uint64_t C, Chunks ch) {
    const uint64_t wg = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x + 1;  // workgroup 0 needs none
    if (wg * kBlock >= C) return;
    // every chunk visited before the first with a record start passes the
    // entry through: one look-back for the workgroup's leading chunks
    bool stopped;
    const uint64_t e = entry_of(ch, wg * kBlock, &stopped);
    for (uint64_t c = wg * kBlock; c < C && c < (wg + 1) * kBlock; ++c) {
        const uint64_t hi = min((c + 1) * kChunk, W);
        const bool ok = stopped || agrees(e, hi, ch.start[c]);
        ch.bad[c] = ok ? 0u : 1u;
        if (!ok) {
            atomicOr(&ch.ctl[0], 1u);
            atomicMin(&ch.ctl[2], static_cast<uint32_t>(min<uint64_t>(c, 0xfffffffeull)));
            atomicOr(&ch.blk[c >> 8], 1u);
        }
        if (ch.start[c] != kNone) break;  // later chunks of the workgroup were checked in k_stream_chunks
    }
}

// Parallel repair rounds (before the serial fixer): every bad chunk walks
// again from its entry as it stands, then the chunks whose entry may have
// changed are checked again.  The first bad chunk's entry is final, so each
// round repairs at least it, and isolated mis-speculations (the common case: a
// start one byte early whose u64 length reads as len * 256 + a char) all in
// one round.  Both kernels visit only 256-chunk blocks flagged in blk (bit 0:
// holds a bad chunk; bit 2: follows a chunk walked again), a workgroup per
// block on a grid-stride grid, so a round costs two launches of a few
// thousand workgroups at most.
constexpr uint32_t kBlkBad = 1, kBlkStop = 2, kBlkRecheck = 4;
constexpr uint32_t kChainMax = 64;  // chunks one repair lane walks behind its own
// Round r's recheck writes its any-bad / first-bad to ctl[kCtlRound + 2r] /
// [+ 1]; round r runs when the state before it (round r - 1's, or the first
// check's ctl[0] / ctl[2]) has a bad chunk -- no launch between rounds.
constexpr uint32_t kCtlRound = 8;
__device__ __forceinline__ uint32_t round_in(uint32_t r) { return r ? kCtlRound + 2 * (r - 1) : 0; }
// The state after the last round that ran: any bad chunk, *first = the first.
__device__ __forceinline__ bool final_bad(const Chunks& ch, uint32_t* first) {
    uint32_t any = ch.ctl[0];
    *first = ch.ctl[2];
    for (uint32_t r = 0; r < kRepairRounds && any; ++r) {
        any = ch.ctl[kCtlRound + 2 * r];
        *first = ch.ctl[kCtlRound + 2 * r + 1];
    }
    return any != 0;
}

__global__ __launch_bounds__(kBlock) void k_stream_refix(StreamArgs a, const uint8_t* __restrict__ w, uint64_t W,
                                                         uint64_t C, Chunks ch, uint32_t round) {
    if (ch.ctl[round_in(round)] == 0) return;
    const uint64_t nblk = (C + 255) / 256;
    for (uint64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        if (!(ch.blk[b] & kBlkBad)) continue;  // uniform
        const uint64_t c = b * 256 + threadIdx.x;
        if (c >= C || !ch.bad[c]) continue;
        // only a chunk whose entry is final: no bad chunk between it and the chunk
        // that provides its entry (a chunk marked bad only because its
        // predecessor was wrong keeps its own, probably right, speculation)
        bool final_entry = true;
        for (uint64_t j = c; j-- > 0;) {
            if (ch.bad[j]) {
                final_entry = false;
                break;
            }
            if (ch.start[j] != kNone) break;
        }
        if (!final_entry) continue;
        const uint64_t hi = min((c + 1) * kChunk, W);
        bool stopped;
        const uint64_t e = entry_of(ch, c, &stopped);
        if (stopped) continue;
        uint64_t cnt = 0, exit = kNone, start = kNone;
        uint32_t stop = 0;
        if (e < hi) {
            start = e;
            walk(a, w, W, e, hi, &cnt, &exit, &stop, ch.list + c * ch.cap, ch.cap);
        }
        ch.start[c] = start;
        ch.cnt[c] = cnt;
        ch.exit[c] = exit;
        ch.stop[c] = stop;
        if (stop) atomicOr(&ch.blk[c >> 8], kBlkStop);
        // the chain behind it: the following chunks that no longer agree with
        // their (new) entry are walked again here, in order, up to the first
        // that agrees -- runs of mis-speculated chunks (short records) are
        // repaired in one round instead of one chunk per round.  Every chunk
        // written and the chunks up to the next record start are rechecked.
        // The walk stops before the next bad chunk: that one is another lane's
        // (or a later round's), so no chunk is written by two lanes of a round
        // (bad flags change only in k_stream_recheck).
        uint64_t ent = start != kNone ? exit : e;
        bool stp = start != kNone && stop != 0;
        uint64_t mb = ~0ull;
        uint64_t j = c + 1;
        for (uint32_t steps = 0; j < C && steps < kChainMax && !stp; ++j, ++steps) {
            if ((j >> 8) != mb) {
                mb = j >> 8;
                atomicOr(&ch.blk[mb], kBlkRecheck);
            }
            const uint64_t hj = min((j + 1) * kChunk, W);
            if (ch.bad[j] || agrees(ent, hj, ch.start[j])) break;
            uint64_t cnt2 = 0, exit2 = kNone, start2 = kNone;
            uint32_t stop2 = 0;
            if (ent < hj) {
                start2 = ent;
                walk(a, w, W, ent, hj, &cnt2, &exit2, &stop2, ch.list + j * ch.cap, ch.cap);
            }
            ch.start[j] = start2;
            ch.cnt[j] = cnt2;
            ch.exit[j] = exit2;
            ch.stop[j] = stop2;
            if (stop2) atomicOr(&ch.blk[j >> 8], kBlkStop);
            if (start2 != kNone) {
                ent = exit2;
                stp = stop2 != 0;
            }
        }
        for (; j < C; ++j) {  // up to and including the next chunk with a record start
            if ((j >> 8) != mb) {
                mb = j >> 8;
                atomicOr(&ch.blk[mb], kBlkRecheck);
            }
            if (ch.start[j] != kNone) break;
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_stream_recheck(uint64_t W, uint64_t C, Chunks ch, uint32_t round) {
    if (ch.ctl[round_in(round)] == 0) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&ch.ctl[5], 1u);  // rounds that found something to repair
    const uint64_t nblk = (C + 255) / 256;
    for (uint64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
        const uint32_t f = ch.blk[b];
        if (!(f & (kBlkBad | kBlkRecheck))) continue;  // uniform: every chunk of the block agreed and kept its entry
        __syncthreads();  // every lane has read blk[b] before it changes
        if (threadIdx.x == 0 && (f & kBlkRecheck)) atomicAnd(&ch.blk[b], ~kBlkRecheck);
        const uint64_t c = b * 256 + threadIdx.x;
        bool ok = true;
        if (c < C && c > 0) {
            const uint64_t hi = min((c + 1) * kChunk, W);
            bool stopped;
            const uint64_t e = entry_of(ch, c, &stopped);
            ok = stopped || agrees(e, hi, ch.start[c]);
            ch.bad[c] = ok ? 0u : 1u;
        }
        note_bad(ch, c, !ok, kCtlRound + 2 * round, kCtlRound + 2 * round + 1);
    }
}


// The stream's stop among the chunks before the first bad one (all right).// The stream's stop among the chunks before the first bad one (all right).
__global__ __launch_bounds__(kBlock) void k_stream_stop(uint64_t C, Chunks ch) {
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    uint32_t first;
    (void)final_bad(ch, &first);
    if (c < C && c < first && ch.stop[c] && ch.start[c] != kNone)
        atomicMin(&ch.ctl[1], static_cast<uint32_t>(min<uint64_t>(c, 0xfffffffeull)));
}

// The hand-off: chunks still wrong before the stream's stop after the repair
// rounds -> ctl[6] = 1, the single-pass decode (stream1.hip) runs (it is
// bounded for any input; the round-2 one-thread in-order fixer here was not).
// `force` (a test hook, srpc_debug_stream_force_single) hands every stream over.
__global__ void k_stream_gate(Chunks ch, uint32_t force) {
    if (threadIdx.x != 0) return;
    uint32_t first;
    ch.ctl[6] = (force || (final_bad(ch, &first) && ch.ctl[1] >= first)) ? 1u : 0u;
}

std::atomic<uint32_t> g_force_single{0};

// Records of chunk c that enter the index: none past the stream's stop chunk.
__device__ __forceinline__ uint64_t chunk_count(const Chunks& ch, uint64_t c, uint64_t C, uint64_t stopc) {
    return c < C && c <= stopc ? ch.cnt[c] : 0;
}

// Exclusive scan over the workgroup's 256 lanes; *total = their sum.
__device__ __forceinline__ uint64_t wg_exclusive_scan(uint64_t x, uint64_t* total) {
    __shared__ uint64_t ws[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint64_t inc = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint64_t before = inc - x;
    for (int w = 0; w < wave; ++w) before += ws[w];
    *total = ws[0] + ws[1] + ws[2] + ws[3];
    return before;
}

// The index in three launches, with no per-chunk count or record-number
// arrays: per 256 chunks the number of records (k_stream_count), the scan of
// those block totals (k_xscan_partials), then per chunk its first record
// number (a workgroup scan plus its block's total) and its starts
// (k_stream_index) -- formerly a count array, a three-pass device scan into a
// record-number array and the index pass (mask 10 + scan 33 + index 19 us on
// 4M 0-64-byte strings).
__global__ __launch_bounds__(kBlock) void k_stream_count(uint64_t C, Chunks ch, uint64_t* __restrict__ parts) {
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    uint64_t tot;
    (void)wg_exclusive_scan(chunk_count(ch, c, C, ch.ctl[1]), &tot);
    if (threadIdx.x == 0) parts[blockIdx.x] = tot;
}

// rec_offs[first record of chunk c + k] = the chunk's k-th record start, up
// to index n (a lane per chunk, from the starts its walk kept).
// The workgroup's starts go through LDS when they fit (kIndexStage entries):
// a lane per chunk writes its few starts at scattered 8-byte slots, the
// staged copy leaves as contiguous 512-byte wave stores.
constexpr uint32_t kIndexStage = 2048;
__global__ __launch_bounds__(kBlock) void k_stream_index(uint64_t C, Chunks ch, const uint64_t* __restrict__ parts,
                                                         uint64_t n, uint64_t* __restrict__ rec_offs) {
    __shared__ uint64_t stage[kIndexStage];
    const uint64_t c = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const uint64_t cnt = chunk_count(ch, c, C, ch.ctl[1]);
    uint64_t tot;
    const uint64_t loc = wg_exclusive_scan(cnt, &tot);
    const uint64_t base = parts[blockIdx.x];
    if (base > n) return;  // uniform: every record of this workgroup is past n
    const uint64_t r0 = base + loc;
    const uint8_t* list = ch.list + c * ch.cap;
    if (tot > kIndexStage) {  // uniform
        if (cnt == 0 || r0 > n) return;
        const uint64_t k1 = min<uint64_t>(cnt, n - r0 + 1);  // [n]: the start of record n, if any
        for (uint64_t k = 0; k < k1; ++k) rec_offs[r0 + k] = c * kChunk + list[k];
        return;
    }
    for (uint64_t k = 0; k < cnt; ++k) stage[loc + k] = c * kChunk + list[k];
    __syncthreads();
    const uint64_t m = min<uint64_t>(tot, n - base + 1);  // entries up to index n
    for (uint32_t i = threadIdx.x; i < m; i += kBlock) rec_offs[base + i] = stage[i];
}

// Records the stream holds: T = sum of counts.  rec_offs[T] = where the stream
// stopped (the failing record's start, or the end of the last record);
// rec_offs[T + 1 .. n] = W.  With T >= n, rec_offs[n] = the start of record n
// (or the end of record n - 1).
__global__ __launch_bounds__(kBlock) void k_stream_tail(uint64_t W, uint64_t C, Chunks ch,
                                                        const uint64_t* __restrict__ total, uint64_t n,
                                                        uint64_t* __restrict__ rec_offs) {
    const uint64_t S = ch.ctl[1];
    const uint64_t T = *total;
    const uint64_t end = (C && S < C && ch.start[S] != kNone) ? ch.exit[S] : W;
    const uint64_t gs = static_cast<uint64_t>(gridDim.x) * kBlock;
    for (uint64_t r = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x; r <= n; r += gs) {
        if (r < T) continue;  // written by k_stream_index (r < n)
        rec_offs[r] = r == T ? end : W;
    }
}

// Diagnostic (srpc_unpack_status.reserved bit 0): some speculated chunk had
// to be walked again (the single pass adds its own bits, stream1.hip).
__global__ void k_stream_note(const Chunks ch, srpc_unpack_status* st) {
    if (threadIdx.x == 0 && (ch.ctl[5] || ch.ctl[6])) atomicOr(&st->reserved, 1u);
}

__global__ void k_stream_ctl_reset(Chunks ch, uint64_t nblk) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        ch.ctl[0] = 0;            // some chunk is bad
        ch.ctl[1] = 0xffffffffu;  // the chunk where the stream stops
        ch.ctl[2] = 0xffffffffu;  // the first bad chunk
        ch.ctl[5] = 0;            // repair rounds run
        ch.ctl[6] = 0;            // the single-pass decode takes over
        for (uint32_t r = 0; r < kRepairRounds; ++r) {
            ch.ctl[kCtlRound + 2 * r] = 0;                // round r: any bad
            ch.ctl[kCtlRound + 2 * r + 1] = 0xffffffffu;  // round r: first bad
        }
    }
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nblk;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
        ch.blk[i] = 0;
}

uint64_t r256(uint64_t b) { return (b + 255) & ~255ull; }

struct StreamLayout {
    uint64_t C, start, cnt, exit, stop, bad, blk, ctl, parts, list, cap, total;
};

StreamLayout stream_layout(uint64_t wire_len, uint32_t fixed_bytes) {
    StreamLayout L{};
    L.C = std::max<uint64_t>(1, (wire_len + kChunk - 1) / kChunk);
    uint64_t o = 0;
    L.start = o;
    o += r256(8 * L.C);
    L.cnt = o;
    o += r256(8 * L.C);
    L.exit = o;
    o += r256(8 * L.C);
    L.stop = o;
    o += r256(4 * L.C);
    L.bad = o;
    o += r256(4 * L.C);
    L.blk = o;
    o += r256(4 * ((L.C + 255) / 256));
    L.ctl = o;
    o += 256;
    L.parts = o;  // records per 256 chunks (then their exclusive scan), then the total
    o += r256(8 * ((L.C + kBlock - 1) / kBlock + 1));
    L.cap = 1 + kChunk / std::max<uint32_t>(fixed_bytes, 1);
    L.list = o;
    o += r256(L.C * L.cap);  // one byte per start
    L.total = o;
    return L;
}

}  // namespace
}  // namespace srpc_impl

using namespace srpc_impl;

extern "C" {

int srpc_legacy_var_stream_scratch_bytes(const srpc_plan* p, uint64_t n, uint64_t wire_len, uint64_t* out) {
    if (!p || !out || !p->has_string) return SRPC_E_INVALID;
    uint64_t var = 0;
    if (int rc = srpc_plan_var_scratch_bytes(p, n, wire_len, &var)) return rc;
    *out = r256(var) + r256(stream_layout(wire_len, p->fixed_bytes).total) + r256(stream1_scratch_bytes(p, wire_len)) +
           sdec_scratch_bytes(p, wire_len);
    return SRPC_OK;
}

int srpc_legacy_unpack_var_stream(const srpc_plan* p, const uint8_t* wire, uint64_t wire_len, uint64_t n,
                                  uint64_t* rec_offs, void* const* cols, uint64_t* const* str_offs,
                                  srpc_unpack_status* st, void* scratch, uint64_t scratch_bytes, void* stream) {
    if (!p || !p->has_string || !rec_offs || !scratch) return SRPC_E_INVALID;
    if (wire_len && !wire) return SRPC_E_INVALID;
    if (!aligned(rec_offs, 8) || !aligned(scratch, 256)) return SRPC_E_ALIGN;
    uint64_t need = 0, var = 0;
    if (int rc = srpc_legacy_var_stream_scratch_bytes(p, n, wire_len, &need)) return rc;
    if (scratch_bytes < need) return SRPC_E_CAPACITY;
    srpc_plan_var_scratch_bytes(p, n, wire_len, &var);
    auto s = static_cast<hipStream_t>(stream);
    auto* base = static_cast<uint8_t*>(scratch) + r256(var);
    const StreamLayout L = stream_layout(wire_len, p->fixed_bytes);
    Chunks ch{reinterpret_cast<uint64_t*>(base + L.start), reinterpret_cast<uint64_t*>(base + L.cnt),
              reinterpret_cast<uint64_t*>(base + L.exit),  reinterpret_cast<uint32_t*>(base + L.stop),
              reinterpret_cast<uint32_t*>(base + L.bad),   reinterpret_cast<uint32_t*>(base + L.blk),
              reinterpret_cast<uint32_t*>(base + L.ctl),   reinterpret_cast<uint8_t*>(base + L.list),
              static_cast<uint32_t>(L.cap)};
    StreamArgs a{};
    for (uint32_t f = 0; f < p->nfields; ++f) a.size[f] = p->size[f];
    a.prefix = p->d_prefix;
    a.nfields = p->nfields;
    a.prefix_len = p->prefix_len;
    a.first_len_at = p->prefix_len;
    for (uint32_t f = 0; f < p->nfields && p->size[f]; ++f) a.first_len_at += p->size[f];
    a.plaus = p->prefix_len >= 8 ? kPlausPrefixed : kPlausBare;
    for (uint32_t i = 0; i < 8 && i < p->prefix_len; ++i) a.pre8 |= static_cast<uint64_t>(p->h_prefix[i]) << (8 * i);
    const uint64_t C = L.C;
    const uint64_t g = (C + kBlock - 1) / kBlock;
    if (g > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
    const TimedCall timed;
    uint32_t mode = g_force_single.load(std::memory_order_relaxed);
    if (mode == 7) mode = 0;
    void* s1 = base + r256(L.total);
    if (mode == 2 && stream1_decodes(p)) {
        // the bounded single pass on its own
        if (int rc = stream1_launch(p, wire, wire_len, n, rec_offs, cols, str_offs, st, s1, nullptr, s)) return rc;
        return wire_len ? stream1_note(p, wire_len, s1, st, nullptr, s) : SRPC_OK;
    }
    void* sd = static_cast<uint8_t*>(s1) + r256(stream1_scratch_bytes(p, wire_len));
    const bool sdec = sdec_supports(p) && stream1_decodes(p);
    if ((mode == 1 || mode == 4 || mode == 5) && sdec) {
        // the speculative single pass (sdec.hip) alone; the bounded one when it gives up
        const uint32_t* abort_word = nullptr;
        if (int rc = sdec_launch(p, wire, wire_len, n, rec_offs, cols, str_offs, st, sd, mode == 4 ? ~0u : 0u,
                                 nullptr, &abort_word, s))
            return rc;
        const uint32_t* gate = mode == 1 ? nullptr : abort_word;  // mode 1: always (a test hook)
        if (int rc = stream1_launch(p, wire, wire_len, n, rec_offs, cols, str_offs, st, s1, gate, s)) return rc;
        return wire_len ? stream1_note(p, wire_len, s1, st, gate, s) : SRPC_OK;
    }
    // the chunk pipeline, its record index, the indexed decode; when its
    // chunks stay wrong after the repair rounds, the speculative single pass
    // (sdec.hip, per-block entry slots), and when that gives up the bounded
    // one (stream1.hip) -- each gated on the one before (mode 3: the bounded
    // pass right after the chunks; schemas beyond sdec: likewise)
    const uint64_t nblk = (C + 255) / 256;
    auto* parts = reinterpret_cast<uint64_t*>(base + L.parts);
    launch(k_stream_ctl_reset, dim3(static_cast<uint32_t>(std::min<uint64_t>((nblk + 255) / 256 + 1, 1024))),
           dim3(256), 0, s, ch, nblk);
    if (wire_len) {
        launch(k_stream_chunks, dim3(static_cast<uint32_t>(g)), dim3(kBlock), 0, s, a, wire, wire_len, C, ch);
        const uint64_t ge = (g + kBlock - 1) / kBlock;  // a lane per workgroup of k_stream_chunks
        launch(k_stream_check_edges, dim3(static_cast<uint32_t>(ge)), dim3(kBlock), 0, s, wire_len, C, ch);
        const uint32_t gr = static_cast<uint32_t>(std::min<uint64_t>(nblk, 2048));
        for (int r = 0; r < kRepairRounds; ++r) {  // gated: no-ops once every chunk agrees
            launch(k_stream_refix, dim3(gr), dim3(kBlock), 0, s, a, wire, wire_len, C, ch, static_cast<uint32_t>(r));
            launch(k_stream_recheck, dim3(gr), dim3(kBlock), 0, s, wire_len, C, ch, static_cast<uint32_t>(r));
        }
        launch(k_stream_stop, dim3(static_cast<uint32_t>(g)), dim3(kBlock), 0, s, C, ch);
        launch(k_stream_gate, dim3(1), dim3(64), 0, s, ch, mode == 6 ? 1u : 0u);
        launch(k_stream_count, dim3(static_cast<uint32_t>(g)), dim3(kBlock), 0, s, C, ch, parts);
    }
    const uint64_t nb = wire_len ? g : 0;
    launch(k_xscan_partials<1024>, dim3(1), dim3(1024), 0, s, parts, nb, parts + g);
    if (wire_len)
        launch(k_stream_index, dim3(static_cast<uint32_t>(g)), dim3(kBlock), 0, s, C, ch,
               static_cast<const uint64_t*>(parts), n, rec_offs);
    launch(k_stream_tail, dim3(static_cast<uint32_t>(std::min<uint64_t>(n / kBlock + 1, 4096))), dim3(kBlock), 0, s,
           wire_len, wire_len ? C : 0ull, ch, static_cast<const uint64_t*>(parts + g), n, rec_offs);
    if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
    // the single pass's gate (0 when the chunks settled or the wire is empty)
    const uint32_t* gate = wire_len ? ch.ctl + 6 : nullptr;
    const bool decodes = stream1_decodes(p);
    if (wire_len && !decodes)  // more string fields than it carries: its index replaces ours
        if (int rc = stream1_launch(p, wire, wire_len, n, rec_offs, cols, str_offs, st, s1, gate, s)) return rc;
    // the indexed decode over the index just built
    const int rc = srpc_gpu_unpack_var(p, wire, wire_len, n, rec_offs, cols, str_offs, st, scratch, var, stream);
    if (rc != SRPC_OK) return rc;
    if (wire_len && decodes && sdec && mode != 3) {  // rewrite every output when the gate is set
        if (int rc2 = sdec_launch(p, wire, wire_len, n, rec_offs, cols, str_offs, st, sd, 0u, gate, &gate, s))
            return rc2;
    }
    if (wire_len && decodes)  // rewrites every output when the gate is set
        if (int rc2 = stream1_launch(p, wire, wire_len, n, rec_offs, cols, str_offs, st, s1, gate, s)) return rc2;
    if (st) {
        hipLaunchKernelGGL(k_stream_note, dim3(1), dim3(64), 0, s, ch, st);
        if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
        if (wire_len) return stream1_note(p, wire_len, s1, st, gate, s);
    }
    return SRPC_OK;
}

}  // extern "C"

// Test hook (not part of the C ABI in include/): which decoders every later
// stream decode runs.  0 = the default (chunk pipeline; speculative single
// pass when its chunks stay wrong; bounded single pass when that gives up);
// 1 = speculative pass, then the bounded pass always; 2 = the bounded pass
// alone; 3 = chunk pipeline, the bounded pass when its chunks stay wrong;
// 4 = the speculative pass alone, never giving up; 5 = the speculative pass,
// the bounded one when it gives up; 6 = as 0 with the chunk pipeline's
// hand-over forced.  Returns the previous setting.
extern "C" __attribute__((visibility("default"))) int srpc_debug_stream_force_single(int on) {
    return static_cast<int>(srpc_impl::g_force_single.exchange(static_cast<uint32_t>(on < 0 ? 0 : on > 7 ? 7 : on)));
}
// Nonzero: srpc_gpu_unpack_var_stream runs these decoders (mode 7 = their
// default order, 1..6 as above); 0 = the table-scan decoder of sdx.hip.
extern "C" int srpc_legacy_stream_mode() { return static_cast<int>(srpc_impl::g_force_single.load()); }
