// sdec.hip -- decode a concatenated record stream with no index in ONE pass
// over the wire, speculatively: the first path of srpc_gpu_unpack_var_stream.
//
// The reference decodes a batch with ONE shared cursor (buffer::_offset,
// core.hpp:39): each pipe_output advances it (packer.hpp:210-222), so where a
// record starts is known only once every record before it was read.
//
// One launch, one workgroup per kSB-byte block of the wire.  Every block:
//  1. stages its bytes (+ kMargin) in LDS by LDS-DMA;
//  2. speculates, a lane per kSC-byte chunk: the chunk's first plausible
//     record start.  Candidates are the positions whose first string length
//     has four zero high bytes (a length read at a wrong offset almost never
//     has: a whole-chunk test from register windows of the stage); of the
//     candidates within 8 bytes the one with the smallest length (a start 1-3
//     bytes early reads the true length shifted up) whose records parse.  The
//     lane walks the records that start in its chunk: starts, count, chars per
//     string field, the position after them (exit);
//  3. links the chunks into the chain from the block's first speculated
//     start sF: when every chunk's start is its predecessor's exit (random
//     data: all of them), the chain is every chunk's records in order; else
//     one lane walks it (records one by one until a speculated start, then
//     whole segments);
//  4. publishes that chain's aggregate (AGG: sF, exit, records, chars) and
//     looks back (decoupled look-back, 64 blocks per round trip) for the
//     cursor's state at its start: from the nearest block whose inclusive
//     state is published (INC), the AGGs of the blocks between are summed --
//     each one only while the state's position is that block's sF (or passes
//     over a block with no start): an AGG speculated from a wrong start is
//     never used, the look-back waits for that block's own INC instead;
//  5. checks its own entry the same way.  A block entered at its sF uses its
//     chain; else (a miss) one lane walks the chain from the true entry.  It
//     publishes its INC and writes its records: rec_offs, fixed fields,
//     str_offs and chars (an LDS image per string field, aligned 16-byte
//     stores), each record read from the stage.
// Wire bytes are read from HBM once (the margin re-reads <= 25 % of a block
// from L2).  Misses make the look-back wait for walks, so on data where wrong
// starts parse too (zero-heavy strings, records of zeros) the decode gives
// up after miss_limit of them: every block then passes a stopped state on at
// once, and the caller runs the bounded decode of stream1.hip (per-block
// candidate tables), gated on the abort word.  A look-back that waits past
// kSpinMax polls gives up the same way (never a hang).
// Error semantics are the cursor's (oracle/packer_oracle.c orc_unpack): the
// first record that does not parse stops the stream; it is reported (PREFIX
// or BOUNDS) as the first bad record, every later record BOUNDS; rec_offs[T]
// = where the stream stopped, later entries wire_len.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <unistd.h>

#include "plan.h"
#include "sdec.h"
#include "srpc_gpu.h"

namespace srpc_impl {
namespace {

constexpr uint32_t kSB = 8192;                  // wire bytes per block (one workgroup)
constexpr uint32_t kSC = kSB / kBlock;          // 32: wire bytes per speculating lane
constexpr uint32_t kMargin = 1024;              // staged bytes past the block
constexpr uint32_t kStage = kSB + kMargin + 32; // + 16-byte alignment slack on both sides
constexpr uint32_t kImage = kSB + kMargin + 64; // chars image of one string field
constexpr uint32_t kMaxRec = kSB / 8;           // records starting in a block (each >= 8 bytes)
constexpr uint32_t kCap = 1 + kSC / 8;          // record starts a chunk can hold
constexpr int kMaxNS = 4;                       // string fields (chars of all but the last carried)
constexpr uint16_t kNoStart = 0xFFFF;
constexpr uint32_t kSlots = 8;                  // per block: chains from other plausible entries
constexpr uint32_t kSlotSpan = 128;             // ... in its first bytes (4 chunks)
constexpr uint32_t kSpinMax = 1u << 18;         // polls of one wait before giving up
constexpr uint32_t kAgg = 1, kInc = 2;          // flag states
constexpr uint64_t kValMask = (1ull << 43) - 1; // tagged words: 21-bit call tag over a 43-bit value
constexpr uint64_t kTagMax = (1ull << 21) - 1;
constexpr uint64_t kCnt40 = (1ull << 40) - 1;   // counts: 40 bits, stop bits above
enum : uint32_t { kCtlAbort = 0, kCtlMiss = 1, kCtlPastN = 2, kCtlStalled = 3, kCtlWords = 8 };

// Per-phase clock (A/B diagnostics, compiled only with -DSRPC_SDEC_PHASES):
// thread 0 of every block adds the clock64() cycles between its phase marks
// into 16 words of its own; srpc_debug_sdec_phases points them at a buffer.
#ifdef SRPC_SDEC_PHASES
__device__ unsigned long long* g_sdph = nullptr;
__device__ unsigned long long g_sdph_blocks = 0;
#define SD_BEGIN uint64_t sd_last_ = clock64();
#define SD_SLOT(i) g_sdph[static_cast<uint64_t>(blockIdx.x) * 16 + (i)]
#define SD(i)                                                                 \
    do {                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < g_sdph_blocks) {                 \
            const uint64_t now_ = clock64();                                  \
            SD_SLOT(i) += now_ - sd_last_;                                    \
            sd_last_ = now_;                                                  \
        }                                                                     \
    } while (0)
#define SD_ADD(i, v)                                                          \
    do {                                                                      \
        if (threadIdx.x == 0 && blockIdx.x < g_sdph_blocks) SD_SLOT(i) += (v); \
    } while (0)
#else
#define SD_BEGIN
#define SD(i)
#define SD_ADD(i, v)
#endif

typedef const uint8_t __attribute__((address_space(1))) global_u8;
typedef uint8_t __attribute__((address_space(3))) lds_u8;
typedef const uint8_t __attribute__((address_space(3))) lds_u8c;
typedef const uint32_t __attribute__((address_space(3))) lds_u32c;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef const u32x4 __attribute__((address_space(3))) lds_u32x4c;

struct SdArgs {
    uint32_t size[kMaxFields];   // fixed field bytes, 0 = string
    uint32_t sord[kMaxFields];   // string ordinal of a string field
    uint8_t* col[kMaxFields];    // fixed: column; string: chars
    uint64_t* soff[kMaxFields];  // string: n + 1 chars offsets
    const uint8_t* prefix;       // device copy (16 zero bytes past the end)
    uint64_t* rec_offs;
    uint64_t n, W;
    uint64_t pre8, pre8_mask;    // the prefix's first (up to) 8 bytes, and which of them count
    uint32_t nfields, P, fixed_bytes;
    uint32_t fla;                // byte offset of the first string's length in a record
    uint32_t run[kMaxNS + 1];    // fixed bytes before string s (after the prefix), after the last
    uint32_t plaus;              // records that must parse from a candidate
    uint32_t nb, epoch, miss_limit;
};

struct SdScratch {
    uint64_t* flag;  // per block: epoch << 32 | state << 8
    uint64_t* agg;   // per block: sF, exit, count | stop << 40, chars[NC]
    uint64_t* inc;   // per block: exit, count | stop << 40, chars[NC]
    uint64_t* slot;  // per block, kSlots of: entry (kValMask: none), exit, count | stop << 40, chars[NC]
    uint32_t* ctl;   // kCtl* words
};

template <int NC>
constexpr uint32_t agg_words() { return 3 + NC; }
template <int NC>
constexpr uint32_t inc_words() { return 2 + NC; }
template <int NC>
constexpr uint32_t slot_words() { return 3 + NC; }

__device__ __forceinline__ uint64_t ld_ac(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_ac(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_ctl(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t tg(uint64_t v, uint64_t t21) { return (v & kValMask) | (t21 << 43); }
__device__ __forceinline__ bool tag_ok(uint64_t w, uint64_t t21) { return (w >> 43) == t21; }
__device__ __forceinline__ uint32_t flag_state(uint64_t f, uint32_t epoch) {
    return (f >> 32) == epoch ? static_cast<uint32_t>((f >> 8) & 0xff) : 0;
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t l) {
    const uint32_t lo = __builtin_amdgcn_readlane(static_cast<uint32_t>(v), l);
    const uint32_t hi = __builtin_amdgcn_readlane(static_cast<uint32_t>(v >> 32), l);
    return (static_cast<uint64_t>(hi) << 32) | lo;
}

// ---- wire reader ---------------------------------------------------------------
// The workgroup's LDS copy of wire bytes [lo, hi) (lds[x] = byte base + x),
// global memory elsewhere; SO (stage only, for speculation): a read outside the
// stage yields bytes no record accepts.
struct Rd {
    global_u8* w;
    lds_u8c* lds;
    uint64_t base, lo, hi;
    lds_u8c* pre;  // LDS copy of the prefix, 16-aligned
    __device__ __forceinline__ uint64_t lds64(uint64_t p) const {
        const uint32_t off = static_cast<uint32_t>(p - base);
        lds_u32c* q = reinterpret_cast<lds_u32c*>(lds + (off & ~3u));
        const uint32_t sh = off & 3, w0 = q[0], w1 = q[1], w2 = q[2];
        return (static_cast<uint64_t>(__builtin_amdgcn_alignbyte(w2, w1, sh)) << 32) |
               __builtin_amdgcn_alignbyte(w1, w0, sh);
    }
    template <bool SO>
    __device__ __forceinline__ uint64_t u64(uint64_t p) const {
        if (p >= lo && p + 8 <= hi) return lds64(p);
        if (SO) return ~0ull;
        uint64_t v;
        __builtin_memcpy(&v, (const uint8_t*)(w + p), 8);
        return v;
    }
    template <bool SO>
    __device__ __forceinline__ uint8_t u8(uint64_t p, uint32_t i) const {
        if (p >= lo && p < hi) return lds[p - base];
        return SO ? static_cast<uint8_t>(~pre[i]) : w[p];
    }
    // the sz (1, 2, 4, 8) bytes of a fixed field at p, never a byte past them in global memory
    __device__ __forceinline__ uint64_t field(uint64_t p, uint32_t sz) const {
        if (p >= lo && p + sz <= hi) return lds64(p);  // the stage has slack past hi
        switch (sz) {
        case 1: return w[p];
        case 2: { uint16_t v; __builtin_memcpy(&v, (const uint8_t*)(w + p), 2); return v; }
        case 4: { uint32_t v; __builtin_memcpy(&v, (const uint8_t*)(w + p), 4); return v; }
        default: { uint64_t v; __builtin_memcpy(&v, (const uint8_t*)(w + p), 8); return v; }
        }
    }
    __device__ __forceinline__ uint64_t pre64(uint32_t i) const {
        lds_u32c* q = reinterpret_cast<lds_u32c*>(pre + i);
        return (static_cast<uint64_t>(q[1]) << 32) | q[0];
    }
    __device__ __forceinline__ bool staged(uint64_t p, uint64_t e) const { return p >= lo && e <= hi && p <= e; }
};

// orc_unpack's cursor over one record at p (p <= W): the position after it,
// or p with *err set (SRPC_STATUS_PREFIX / _BOUNDS); chars of string fields
// 0..NS-2 added to ch[].  Runs of fixed fields are checked as one (the
// cursor's first failing field is BOUNDS either way).
template <int NS, bool SO>
__device__ __forceinline__ uint64_t parse(const SdArgs& a, const Rd& r, uint64_t p, uint32_t* err,
                                          uint64_t (&ch)[kMaxNS]) {
    const uint64_t W = a.W;
    *err = 0;
    if (a.P) {
        if (a.P > W - p) {
            *err = SRPC_STATUS_BOUNDS;
            return p;
        }
        uint32_t i = 0;
        for (; i + 8 <= a.P; i += 8)
            if (r.u64<SO>(p + i) != r.pre64(i)) {
                *err = SRPC_STATUS_PREFIX;
                return p;
            }
        for (; i < a.P; ++i)
            if (r.u8<SO>(p + i, i) != r.pre[i]) {
                *err = SRPC_STATUS_PREFIX;
                return p;
            }
    }
    uint64_t q = p + a.P;
    uint64_t add[kMaxNS] = {};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const uint32_t F = a.run[s];
        if (F + 8ull > W - q) {
            *err = SRPC_STATUS_BOUNDS;
            return p;
        }
        q += F;
        const uint64_t len = r.u64<SO>(q);
        q += 8;
        if (len > W - q) {
            *err = SRPC_STATUS_BOUNDS;
            return p;
        }
        q += len;
        add[s] = len;
    }
    if (a.run[NS] > W - q) {
        *err = SRPC_STATUS_BOUNDS;
        return p;
    }
#pragma unroll
    for (int s = 0; s + 1 < NS; ++s) ch[s] += add[s];
    return q + a.run[NS];
}

template <int NS>
__device__ __forceinline__ bool plausible(const SdArgs& a, const Rd& r, uint64_t p) {
    uint64_t ch[kMaxNS];
    for (uint32_t k = 0; k < a.plaus; ++k) {
        if (p == a.W) return k > 0;  // the stream may end right after a record
        uint32_t err;
        const uint64_t q = parse<NS, true>(a, r, p, &err, ch);
        if (err) return false;
        p = q;
    }
    return true;
}

// Candidate starts of a chunk: bit j set when the four bytes at stage offset
// o + j (o = the chunk's first byte + fla + 4: the first string length's high
// half) are zero.  o mod 16 is the same for every lane of the block (chunks
// are 32 bytes apart), so the 16-byte LDS reads and the dword realignment
// are uniform; the test runs on all 32 positions at once from byte-zero
// indicators (0x80 per zero byte).
__device__ __forceinline__ uint32_t cand_mask(const uint8_t* st, uint32_t o) {
    lds_u32x4c* q = reinterpret_cast<lds_u32x4c*>((lds_u8c*)st + (o & ~15u));
    uint32_t w[16];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const u32x4 v = q[i];
        w[4 * i] = v.x;
        w[4 * i + 1] = v.y;
        w[4 * i + 2] = v.z;
        w[4 * i + 3] = v.w;
    }
    // d[k] = bytes o + 4k .. o + 4k + 3 (k < 9 covers positions 0..31 + 3)
    uint32_t d[10];
    const uint32_t sh = o & 3;
    switch (__builtin_amdgcn_readfirstlane((o >> 2) & 3)) {
    case 0:
#pragma unroll
        for (int k = 0; k < 10; ++k) d[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
        break;
    case 1:
#pragma unroll
        for (int k = 0; k < 10; ++k) d[k] = __builtin_amdgcn_alignbyte(w[k + 2], w[k + 1], sh);
        break;
    case 2:
#pragma unroll
        for (int k = 0; k < 10; ++k) d[k] = __builtin_amdgcn_alignbyte(w[k + 3], w[k + 2], sh);
        break;
    default:
#pragma unroll
        for (int k = 0; k < 10; ++k) d[k] = __builtin_amdgcn_alignbyte(w[k + 4], w[k + 3], sh);
        break;
    }
    uint32_t z[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) z[k] = ~(((d[k] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | d[k] | 0x7f7f7f7fu);
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t a4 = z[k] & __builtin_amdgcn_alignbyte(z[k + 1], z[k], 1) &
                            __builtin_amdgcn_alignbyte(z[k + 1], z[k], 2) &
                            __builtin_amdgcn_alignbyte(z[k + 1], z[k], 3);
        // bits 7, 15, 23, 31 -> a nibble
        m |= ((((a4 >> 7) * 0x00204081u) >> 21) & 15u) << (4 * k);
    }
    return m;
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

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

template <int NC>
struct Agg {
    uint64_t exit, cnt;
    uint64_t ch[kMaxNS];
    uint32_t stop;  // 0, or 1 | kind << 1
};

// The cursor's state at a block boundary.
template <int NC>
struct St {
    uint64_t ex, cn;
    uint64_t ch[kMaxNS];
    uint32_t stp;
};

template <int NC>
struct SdLds {
    alignas(16) uint8_t st[kStage + 16];   // wire bytes [base, base + kStage)
    alignas(16) uint8_t pre[kMaxPrefix + 16];
    union {
        alignas(16) uint8_t img[kImage + 32];  // chars image (once the record table is built)
        struct {                               // the chunks (until then)
            uint64_t exit[kBlock];                 // per chunk: position after its records
            uint64_t pch[NC ? NC : 1][kBlock + 1]; // per chunk, then exclusive scan: chars of fields 0..NC-1
            uint32_t pcnt[kBlock + 1];             // per chunk, then exclusive scan: records
            uint16_t start[kBlock];                // per chunk: first start (offset from the block), or none
            uint8_t list[kBlock * kCap];           // per chunk: its starts minus the chunk's first byte
            uint8_t stop[kBlock];                  // per chunk: 0, or 1 | kind << 1
        };
    };
    uint32_t loff[kMaxRec + 1];            // per local record: chars offset; the explicit start list while walking
    uint16_t tbl[kMaxRec + 1];             // the block's records in order: offset from the block
    uint64_t has[4], tail[4], jump[4];     // 256-bit masks over chunks
    uint64_t ws[kBlock / 64];
    uint32_t brk[kBlock / 64];             // per wave: some chunk breaks the plain chain
    uint32_t cm[kSlotSpan / kSC];          // candidate masks of the first chunks
    uint64_t slotpos[kSlots];              // this block's slot entries
    Agg<NC> g;                             // the chain from sF
    uint32_t g_nexp;                       // explicit starts of that walk (0: plain chain)
    uint64_t s_x, s_cnt, s_ch[kMaxNS];     // the entry and the state before the block
    uint32_t s_nexp, s_plain;
};

// The chain from x (x >= the block start): explicit records are parsed until
// the walk meets a speculated chunk start, whose segment is then taken whole
// from the scans, and so on.  REC: the explicit starts go to the list (LDS
// u16 offsets, ascending) and jumped chunks to the jump mask.
template <int NS, int NC, bool REC>
__device__ Agg<NC> walk_chain(const SdArgs& a, const Rd& rd, SdLds<NC>& L, uint64_t b0, uint64_t b1, uint64_t x,
                              uint16_t* xl, uint32_t* nx) {
    Agg<NC> g{};
    uint64_t q = x;
    uint32_t ne = 0;
    while (q < b1) {
        const uint32_t c = static_cast<uint32_t>((q - b0) / kSC);
        const uint16_t sc = L.start[c];
        if (sc != kNoStart && b0 + sc == q) {  // on a speculated segment: jump to its end
            const uint32_t e = next_bit(L.tail, c);
            g.cnt += L.pcnt[e + 1] - L.pcnt[c];
#pragma unroll
            for (int k = 0; k < NC; ++k) g.ch[k] += L.pch[k][e + 1] - L.pch[k][c];
            if (REC) {
                for (uint32_t j = c; j <= e;) {
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
        const uint64_t q2 = parse<NS, false>(a, rd, q, &err, g.ch);
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

// Wave-uniform sleep-and-count: false once the budget is spent or the
// decode was given up (then nothing this block waits for matters).
__device__ __forceinline__ bool spin(uint32_t* n, const uint32_t* ctl) {
    if (++*n >= kSpinMax || ld_ctl(ctl + kCtlAbort)) return false;
    __builtin_amdgcn_s_sleep(4);
    return true;
}

template <int NC>
__device__ __forceinline__ void publish_inc(const SdScratch& S, uint64_t b, const St<NC>& s, uint32_t epoch) {
    const uint64_t t21 = epoch & kTagMax;
    uint64_t* iw = S.inc + b * inc_words<NC>();
    st_ac(iw, tg(s.ex, t21));
    st_ac(iw + 1, tg((s.cn & kCnt40) | (static_cast<uint64_t>(s.stp) << 40), t21));
#pragma unroll
    for (int k = 0; k < NC; ++k) st_ac(iw + 2 + k, tg(s.ch[k], t21));
    st_ac(S.flag + b, (static_cast<uint64_t>(epoch) << 32) | (kInc << 8));
}

// Block j's INC (state after it) once published with every word's tag, else false.
template <int NC>
__device__ __forceinline__ bool load_inc(const SdScratch& S, uint64_t j, uint32_t epoch, St<NC>* s) {
    const uint64_t t21 = epoch & kTagMax;
    if (flag_state(ld_ac(S.flag + j), epoch) != kInc) return false;
    const uint64_t* iw = S.inc + j * inc_words<NC>();
    uint64_t w[2 + kMaxNS];
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 2 + NC; ++k) {
        w[k] = ld_ac(iw + k);
        ok = ok && tag_ok(w[k], t21);
    }
    if (!ok) return false;
    s->ex = w[0] & kValMask;
    s->cn = w[1] & kCnt40;
    s->stp = static_cast<uint32_t>((w[1] >> 40) & 7);
#pragma unroll
    for (int k = 0; k < NC; ++k) s->ch[k] = w[2 + k] & kValMask;
    return true;
}

// One lane per block of a look-back window: its INC (when published with
// every word's tag) and its AGG, loaded together -- one round trip.
template <int NC>
struct Win {
    bool inc_ok, agg_ok;
    uint64_t iw[2 + kMaxNS];  // exit, count | stop, chars
    uint64_t aw[3 + kMaxNS];  // sF, exit, count | stop, chars
    __device__ __forceinline__ void load(const SdScratch& S, int64_t j, uint64_t t21) {
        inc_ok = agg_ok = false;
        if (j < 0) return;
        const uint64_t* ip = S.inc + static_cast<uint64_t>(j) * inc_words<NC>();
        const uint64_t* ap = S.agg + static_cast<uint64_t>(j) * agg_words<NC>();
#pragma unroll
        for (int k = 0; k < 2 + NC; ++k) iw[k] = ld_ac(ip + k);
#pragma unroll
        for (int k = 0; k < 3 + NC; ++k) aw[k] = ld_ac(ap + k);
        bool io = true, ao = true;
#pragma unroll
        for (int k = 0; k < 2 + NC; ++k) io = io && tag_ok(iw[k], t21);
#pragma unroll
        for (int k = 0; k < 3 + NC; ++k) ao = ao && tag_ok(aw[k], t21);
        inc_ok = io;
        agg_ok = ao;
    }
};

// Fold lanes [first, cnt) of a window (lane l = block lo + l, AGGs) into s:
// each AGG applies while the state's position is that block's sF (or passes
// over a block without one); at a block whose AGG does not hold the state
// becomes that block's INC (waited for).  False when a wait gave up.
template <int NC>
__device__ bool fold(const SdArgs& a, const SdScratch& S, const Win<NC>& wv, uint64_t lo, uint32_t first, uint32_t cnt,
                     St<NC>& s, uint32_t* spins) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t W = a.W;
    const uint64_t j = lo + lane;
    const uint64_t sF = wv.aw[0] & kValMask, ex = wv.aw[1] & kValMask;
    const uint32_t gstop = static_cast<uint32_t>((wv.aw[2] >> 40) & 7);
    const uint64_t b1 = min<uint64_t>((j + 1) * kSB, W);
    while (first < cnt && !(s.stp & 1) && s.ex < W) {
        const bool act = lane >= first && lane < cnt;
        const bool hasS = act && sF != kValMask;
        // the position entering each lane's block: the exit of the nearest
        // earlier active block with a start (exits grow with the block), or s.ex
        uint64_t mx = hasS ? ex : 0;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(mx, d, 64);
            if (lane >= static_cast<uint32_t>(d)) mx = max<uint64_t>(mx, y);
        }
        uint64_t enter = __shfl_up(mx, 1, 64);
        if (lane == 0) enter = 0;
        enter = max<uint64_t>(enter, s.ex);
        const bool valid = !act || (hasS ? enter == sF : enter >= b1);
        const uint64_t inv = __ballot(!valid);
        const uint32_t f = inv ? __builtin_ctzll(inv) : 64;
        const uint64_t stm = __ballot(hasS && valid && (gstop & 1) && lane < f);
        const uint32_t g = stm ? __builtin_ctzll(stm) : 64;
        const uint32_t end = min(f, g + 1);  // lanes [first, end) apply
        const bool app = act && lane < end;
        s.cn += wave_sum(app ? (wv.aw[2] & kCnt40) : 0);
#pragma unroll
        for (int k = 0; k < NC; ++k) s.ch[k] += wave_sum(app ? (wv.aw[3 + k] & kValMask) : 0);
        if (end > first) {
            const uint64_t e = rl64(mx, end - 1);
            if (e) s.ex = max<uint64_t>(s.ex, e);
        }
        if (g < f) {  // the chain stops in block lo + g
            s.stp = __builtin_amdgcn_readlane(gstop, g);
            return true;
        }
        if (f >= cnt) return true;
        // block lo + f's AGG does not hold for the true entry (s.ex): one of
        // its slots (one round trip: a word per lane), else its INC
        {
            constexpr uint32_t SW = slot_words<NC>(), NW = kSlots * SW;
            const uint64_t t21 = a.epoch & kTagMax;
            const uint64_t* tb = S.slot + (lo + f) * NW;
            uint64_t v = 0;
            while (true) {
                v = lane < NW ? ld_ac(tb + lane) : 0;
                if (!__ballot(lane < NW && !tag_ok(v, t21))) break;
                if (!spin(spins, S.ctl)) return false;
            }
            int hit = -1;
#pragma unroll
            for (uint32_t k = 0; k < kSlots; ++k)
                if (hit < 0 && (rl64(v, k * SW) & kValMask) == s.ex) hit = static_cast<int>(k);
            if (hit >= 0) {
                const uint32_t o = static_cast<uint32_t>(hit) * SW;
                const uint64_t cw = rl64(v, o + 2);
                s.cn += cw & kCnt40;
#pragma unroll
                for (int k = 0; k < NC; ++k) s.ch[k] += rl64(v, o + 3 + k) & kValMask;
                s.ex = rl64(v, o + 1) & kValMask;
                s.stp = static_cast<uint32_t>((cw >> 40) & 7);
                first = f + 1;
                continue;
            }
        }
        SD_ADD(14, 1);
        while (!load_inc<NC>(S, lo + f, a.epoch, &s))
            if (!spin(spins, S.ctl)) return false;
        first = f + 1;
    }
    return true;
}

// The state before block b (wave 0, every lane the same result).  The window
// of the 64 blocks before b is loaded in one round trip (INC and AGG words of
// each); from its last INC the AGGs after it are folded.  With no INC in it,
// windows further back are searched for one (INC words only), then the
// windows between are loaded again and folded in order.
template <int NC>
__device__ St<NC> look_back(const SdArgs& a, const SdScratch& S, uint64_t b, bool* stalled) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t t21 = a.epoch & kTagMax;
    St<NC> s{};
    uint32_t spins = 0;
    const int64_t lo0 = static_cast<int64_t>(b) - 64;  // the first window: blocks lo0 .. b - 1 (lane l = lo0 + l)
    Win<NC> wv;
    while (true) {  // every block of the window with its INC or its AGG
        wv.load(S, lo0 + static_cast<int64_t>(lane), t21);
        if (!__ballot(lo0 + static_cast<int64_t>(lane) >= 0 && !wv.inc_ok && !wv.agg_ok)) break;
        if (!spin(&spins, S.ctl)) {
            *stalled = true;
            return s;
        }
    }
    uint64_t incm = __ballot(wv.inc_ok);
    int64_t base;  // the block whose INC starts the fold
    if (incm) {
        base = lo0 + 63 - __builtin_clzll(incm);
    } else {
        // further back, 64 INC flags per round trip (none yet down to block
        // 0, whose INC may still be coming: from the top again)
        int64_t top = lo0 - 1;
        while (true) {
            const int64_t jj = top - static_cast<int64_t>(lane);
            const uint32_t stt = jj >= 0 ? flag_state(ld_ac(S.flag + jj), a.epoch) : 0;
            const uint64_t m = __ballot(stt == kInc);
            if (m) {
                base = top - __builtin_ctzll(m);
                break;
            }
            top -= 64;
            if (top < 0) {
                if (!spin(&spins, S.ctl)) {
                    *stalled = true;
                    return s;
                }
                top = lo0 - 1;
            }
        }
    }
    while (!load_inc<NC>(S, static_cast<uint64_t>(base), a.epoch, &s))
        if (!spin(&spins, S.ctl)) {
            *stalled = true;
            return s;
        }
    // windows between base and the first window: loaded again, folded in order
    uint64_t lo = static_cast<uint64_t>(base) + 1;
    SD_ADD(13, b - 1 - static_cast<uint64_t>(base));
    SD_ADD(11, static_cast<uint64_t>(max<int64_t>(0, lo0 - static_cast<int64_t>(lo) + 63)) / 64);
    while (static_cast<int64_t>(lo) < lo0 && !(s.stp & 1) && s.ex < a.W) {
        const uint32_t cnt = static_cast<uint32_t>(min<uint64_t>(64, static_cast<uint64_t>(lo0) - lo));
        Win<NC> w2;
        while (true) {
            w2.load(S, lane < cnt ? static_cast<int64_t>(lo + lane) : -1, t21);
            if (!__ballot(lane < cnt && !w2.inc_ok && !w2.agg_ok)) break;
            if (!spin(&spins, S.ctl)) {
                *stalled = true;
                return s;
            }
        }
        // restart from its last INC
        const uint64_t m2 = __ballot(lane < cnt && w2.inc_ok);
        uint32_t first = 0;
        if (m2) {
            const uint32_t li = 63 - __builtin_clzll(m2);
            load_inc<NC>(S, lo + li, a.epoch, &s);
            first = li + 1;
        }
        if (!fold<NC>(a, S, w2, lo, first, cnt, s, &spins)) {
            *stalled = true;
            return s;
        }
        lo += cnt;
    }
    // the first window, from base (or its own last INC)
    if (!(s.stp & 1) && s.ex < a.W) {
        const int64_t from = max<int64_t>(static_cast<int64_t>(lo), static_cast<int64_t>(base) + 1);
        const uint32_t first = static_cast<uint32_t>(from - lo0);
        if (!fold<NC>(a, S, wv, static_cast<uint64_t>(lo0), first, 64, s, &spins)) *stalled = true;
    }
    return s;
}

// One launch decodes the whole stream; see the file comment.
template <int NS>
__global__ __launch_bounds__(kBlock) void k_sdec(SdArgs a, const uint8_t* __restrict__ w, SdScratch S,
                                                  const uint32_t* gate) {
    constexpr int NC = NS - 1;
    if (gate && !*gate) return;
    __shared__ SdLds<NC> L;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint64_t b = blockIdx.x;
    const uint64_t W = a.W;
    const uint64_t b0 = b * kSB, b1 = min<uint64_t>(b0 + kSB, W);

    // a given-up decode, or a block past the one that holds record n: pass a
    // stopped state on (nothing after it counts)
    if (ld_ctl(S.ctl + kCtlAbort) || (b > 0 && b > ld_ctl(S.ctl + kCtlPastN))) {
        if (tid == 0) {
            St<NC> st{};
            st.ex = W;
            st.cn = a.n + 1;
            st.stp = 1;
            publish_inc<NC>(S, b, st, a.epoch);
        }
        return;
    }

    SD_BEGIN
    SD_ADD(10, 1);
    // 1. prefix and stage (LDS-DMA)
    for (uint32_t i = tid; i < a.P + 16; i += kBlock) L.pre[i] = i < a.P ? a.prefix[i] : 0;
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
    if (tid < kSlotSpan / kSC) L.cm[tid] = 0;
    __syncthreads();
    const Rd rd{(global_u8*)w, (lds_u8c*)L.st, A - reinterpret_cast<uint64_t>(w), b0, hi, (lds_u8c*)L.pre};
    SD(0);

    // 2. speculation: chunk c = tid
    const uint64_t clo = b0 + static_cast<uint64_t>(tid) * kSC, chi = min<uint64_t>(clo + kSC, b1);
    uint64_t sp = ~0ull;
    if (clo < b1) {
        if (clo == 0) {
            sp = 0;  // the stream starts at 0
        } else {
            const uint64_t lim = chi - clo;  // positions in the chunk
            uint32_t m = cand_mask(L.st, static_cast<uint32_t>(clo - rd.base) + a.fla + 4);
            if (lim < 32) m &= (1u << lim) - 1;
            if (tid < kSlotSpan / kSC) L.cm[tid] = m;
            while (m && sp == ~0ull) {
                const uint32_t j0 = __builtin_ctz(m);
                uint32_t cl = (m >> j0) & 0xffu;  // candidates within 8 bytes of the first
                m &= ~(0xffu << j0);
                if (a.pre8_mask)  // an envelope: the prefix's first bytes, before any parse
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if (((cl >> k) & 1) && ((rd.u64<true>(clo + j0 + k) ^ a.pre8) & a.pre8_mask))
                            cl &= ~(1u << k);
                uint64_t len[8];
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    len[k] = (cl >> k) & 1 ? rd.u64<true>(clo + j0 + k + a.fla) : ~0ull;
                while (cl) {  // smallest first length first (ties: earliest)
                    uint32_t kb = 0;
                    uint64_t best = ~0ull;
#pragma unroll
                    for (int k = 7; k >= 0; --k)
                        if (((cl >> k) & 1) && len[k] <= best) {
                            best = len[k];
                            kb = k;
                        }
                    cl &= ~(1u << kb);
                    if (plausible<NS>(a, rd, clo + j0 + kb)) {
                        sp = clo + j0 + kb;
                        break;
                    }
                }
            }
        }
    }
    uint64_t cch[kMaxNS] = {};
    uint32_t ccnt = 0, cstop = 0;
    uint64_t cexit = ~0ull;
    if (sp != ~0ull) {  // the records that start in the chunk
        uint64_t p = sp;
        while (p < chi) {
            uint32_t err;
            const uint64_t q = parse<NS, false>(a, rd, p, &err, cch);
            if (err) {
                cstop = 1 | (err << 1);
                break;
            }
            if (ccnt < kCap) L.list[tid * kCap + ccnt] = static_cast<uint8_t>(p - clo);
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
    SD(1);

    // 3. segments: chunk c continues its predecessor's segment when that
    // chunk's exit is c's start; tails end segments.  The plain chain: every
    // chunk with a start continues (then the chain from sF is all of them).
    bool tail = false;
    const uint32_t F = next_bit(L.has, 0);
    if (sp != ~0ull) {
        const uint32_t nxt = next_bit(L.has, tid + 1);
        tail = cstop || nxt >= kBlock || cexit != b0 + L.start[nxt];
    }
    // a break: a tail that stops, is followed by another chunk with a start,
    // or (the last one) exits inside the block (a start no chunk found)
    const bool brk = sp != ~0ull && tail && (cstop || next_bit(L.has, tid + 1) < kBlock || cexit < b1);
    const uint64_t tm = __ballot(tail);
    const uint64_t bm = __ballot(brk);
    if (lane == 0) {
        L.tail[tid >> 6] = tm;
        L.brk[tid >> 6] = bm != 0;
    }
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
    const uint64_t sF = F < kBlock ? b0 + L.start[F] : ~0ull;
    const bool plain = !(L.brk[0] | L.brk[1] | L.brk[2] | L.brk[3]);
    SD(2);

    // 4. slots: the chains from the other plausible positions of the first
    // kSlotSpan bytes (where a predecessor's last record may end), published
    // (wave 0; two positions per lane, the first kSlots by position kept)
    if (tid < 64 && b > 0) {
        const uint64_t t21 = a.epoch & kTagMax;
        bool c[2];
        uint64_t p[2];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const uint32_t q = 2 * lane + e;
            p[e] = b0 + q;
            c[e] = ((L.cm[q / kSC] >> (q % kSC)) & 1) && p[e] < b1 && p[e] != sF && plausible<NS>(a, rd, p[e]);
        }
        const uint64_t m0 = __ballot(c[0]), m1 = __ballot(c[1]);
        const uint64_t below = (1ull << lane) - 1;
        const uint32_t r0 = __builtin_popcountll(m0 & below) + __builtin_popcountll(m1 & below);
        const uint32_t total = __builtin_popcountll(m0) + __builtin_popcountll(m1);
        uint64_t* tb = S.slot + b * kSlots * slot_words<NC>();
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const uint32_t r = r0 + (e ? c[0] : 0);
            if (c[e] && r < kSlots) {
                const Agg<NC> g = walk_chain<NS, NC, false>(a, rd, L, b0, b1, p[e], nullptr, nullptr);
                uint64_t* q = tb + r * slot_words<NC>();
                st_ac(q, tg(p[e], t21));
                st_ac(q + 1, tg(g.exit, t21));
                st_ac(q + 2, tg(g.cnt | (static_cast<uint64_t>(g.stop) << 40), t21));
#pragma unroll
                for (int k = 0; k < NC; ++k) st_ac(q + 3 + k, tg(g.ch[k], t21));
                L.slotpos[r] = p[e];
            }
        }
        if (lane >= total && lane < kSlots) {  // unused slots
            uint64_t* q = tb + lane * slot_words<NC>();
#pragma unroll
            for (int k = 0; k < 3 + NC; ++k) st_ac(q + k, tg(k == 0 ? kValMask : 0, t21));
            L.slotpos[lane] = ~0ull;
        }
    }
    // the chain from sF (AGG), published; then the look-back (wave 0)
    if (tid == 0) {
        Agg<NC> g{};
        uint32_t ne = 0;
        if (sF != ~0ull) {
            if (plain) {  // every chunk's records, in order
                const uint32_t e = next_bit(L.tail, F);  // the last chunk with a start
                g.cnt = L.pcnt[kBlock];
#pragma unroll
                for (int k = 0; k < NC; ++k) g.ch[k] = L.pch[k][kBlock];
                g.exit = L.exit[e];
                g.stop = 0;
            } else {
                g = walk_chain<NS, NC, true>(a, rd, L, b0, b1, sF, reinterpret_cast<uint16_t*>(L.loff), &ne);
            }
        }
        L.g = g;
        L.g_nexp = ne;
        if (b > 0) {
            const uint64_t t21 = a.epoch & kTagMax;
            uint64_t* q = S.agg + b * agg_words<NC>();
            st_ac(q, tg(sF == ~0ull ? kValMask : sF, t21));
            st_ac(q + 1, tg(g.exit, t21));
            st_ac(q + 2, tg(g.cnt | (static_cast<uint64_t>(g.stop) << 40), t21));
#pragma unroll
            for (int k = 0; k < NC; ++k) st_ac(q + 3 + k, tg(g.ch[k], t21));
            st_ac(S.flag + b, (static_cast<uint64_t>(a.epoch) << 32) | (kAgg << 8));
        }
    }
    __syncthreads();
    SD(3);
    if (tid < 64) {
        bool stalled = false;
        St<NC> s{};
        if (b > 0) s = look_back<NC>(a, S, b, &stalled);
        SD(4);
        if (!stalled && !(s.stp & 1) && s.ex < b0) stalled = true;  // never expected: a chain ended early
        if (stalled) s.stp = 1;  // reported; the result is not valid
        // 5. this block's own chain from its entry
        uint64_t x = ~0ull;
        uint32_t nexp = 0, isplain = 0;
        const St<NC> s0 = s;
        if (!(s.stp & 1) && s.ex < b1) {
            x = s.ex;
            Agg<NC> g;
            if (x == sF) {
                g = L.g;
                nexp = L.g_nexp;
                isplain = plain;
            } else {  // a miss: walk from the true entry (lane 0; the rest wait)
                g = Agg<NC>{};
                if (lane == 0) {
                    L.jump[0] = L.jump[1] = L.jump[2] = L.jump[3] = 0;
                    g = walk_chain<NS, NC, true>(a, rd, L, b0, b1, x, reinterpret_cast<uint16_t*>(L.loff), &nexp);
                    bool slot = false;
                    for (uint32_t k = 0; k < kSlots; ++k) slot = slot || L.slotpos[k] == x;
                    if (!slot) {  // every later look-back waited for this block's INC
                        SD_ADD(12, 1);
                        const uint32_t ms = atomicAdd(&S.ctl[kCtlMiss], 1u) + 1;
                        if (ms > a.miss_limit) atomicOr(&S.ctl[kCtlAbort], 1u);
                    }
                }
                g.exit = rl64(g.exit, 0);
                g.cnt = rl64(g.cnt, 0);
#pragma unroll
                for (int k = 0; k < NC; ++k) g.ch[k] = rl64(g.ch[k], 0);
                g.stop = __builtin_amdgcn_readfirstlane(g.stop);
                nexp = __builtin_amdgcn_readfirstlane(nexp);
            }
            s.ex = g.exit;
            s.cn += g.cnt;
#pragma unroll
            for (int k = 0; k < NC; ++k) s.ch[k] += g.ch[k];
            s.stp = g.stop;
        }
        if (lane == 0) {
            publish_inc<NC>(S, b, s, a.epoch);
            if (s.cn > a.n) atomicMin(&S.ctl[kCtlPastN], static_cast<uint32_t>(min<uint64_t>(b, 0xfffffffeull)));
            if (stalled) {
                atomicOr(&S.ctl[kCtlStalled], 1u);
                atomicOr(&S.ctl[kCtlAbort], 1u);
            }
            L.s_x = x;
            L.s_cnt = s0.cn;
#pragma unroll
            for (int k = 0; k < NC; ++k) L.s_ch[k] = s0.ch[k];
            L.s_nexp = nexp;
            L.s_plain = isplain;
        }
    }
    __syncthreads();
    SD(5);
    const uint64_t x = L.s_x;
    const uint64_t R = L.s_cnt;
    if (x == ~0ull || R > a.n) return;  // no record starts here (or all are past record n)

    // 6. the chain's records in order: chunk tid's explicit starts (binary
    // search in the ascending list), then its speculated starts if the chain
    // took them (every chunk of a plain chain from sF)
    const uint32_t ne = L.s_nexp;
    const uint16_t* xl = reinterpret_cast<const uint16_t*>(L.loff);
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
    const bool jumped = L.s_plain || ((L.jump[tid >> 6] >> (tid & 63)) & 1);
    const uint32_t ccount = L.pcnt[tid + 1] - L.pcnt[tid];
    const uint32_t fc = (e1 - e0) + (jumped ? ccount : 0);
    uint64_t tot;
    const uint32_t fb = static_cast<uint32_t>(block_xscan(fc, &tot, L.ws));
    for (uint32_t k = e0; k < e1; ++k) L.tbl[fb + (k - e0)] = xl[k];
    if (jumped)
        for (uint32_t k = 0; k < ccount; ++k)
            L.tbl[fb + (e1 - e0) + k] = static_cast<uint16_t>(tid * kSC + L.list[tid * kCap + k]);
    __syncthreads();
    const uint32_t nrec = static_cast<uint32_t>(min<uint64_t>(tot, kMaxRec));
    SD(6);

    // 7. outputs: record r = R + k of the batch (up to index n)
    const uint64_t n = a.n;
    for (uint32_t k = tid; k < nrec; k += kBlock) {
        const uint64_t r = R + k;
        if (r > n) break;
        const uint64_t s = b0 + L.tbl[k];
        a.rec_offs[r] = s;
        if (r == n) continue;
        uint64_t pos = s + a.P;
        for (uint32_t f = 0; f < a.nfields; ++f) {
            const uint32_t sz = a.size[f];
            if (sz) {
                const uint64_t v = rd.field(pos, sz);
                uint8_t* dst = a.col[f] + r * sz;
                switch (sz) {
                case 1: dst[0] = static_cast<uint8_t>(v); break;
                case 2: *reinterpret_cast<uint16_t*>(dst) = static_cast<uint16_t>(v); break;
                case 4: *reinterpret_cast<uint32_t*>(dst) = static_cast<uint32_t>(v); break;
                default: *reinterpret_cast<uint64_t*>(dst) = v; break;
                }
                pos += sz;
            } else {
                pos += 8 + rd.u64<false>(pos);
            }
        }
    }
    SD(7);
    // per string field: local offsets (a scan over the block's records),
    // str_offs, the chars image, aligned stores
    uint64_t Pbase[kMaxNS];
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
        for (uint32_t k = tid; k < nrec; k += kBlock) {
            uint64_t pos = b0 + L.tbl[k] + a.P, len = 0;
            for (uint32_t g = 0; g <= f; ++g) {
                const uint32_t sz = a.size[g];
                if (sz) {
                    pos += sz;
                    continue;
                }
                len = rd.u64<false>(pos);
                pos += 8 + (g < f ? len : 0);
            }
            L.loff[k] = k < nw ? static_cast<uint32_t>(len) : 0;
        }
        __syncthreads();
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
        for (uint32_t k = tid; k < nrec && R + k <= n; k += kBlock) so[R + k] = P + L.loff[k];
        const bool fits = ftot + 32 <= kImage;
        for (uint32_t k = tid; k < nw; k += kBlock) {
            const uint32_t o = L.loff[k], len = L.loff[k + 1] - o;
            if (!len) continue;
            uint64_t pos = b0 + L.tbl[k] + a.P;
            for (uint32_t g = 0; g < f; ++g) pos += a.size[g] ? a.size[g] : 8 + rd.u64<false>(pos);
            pos += 8;
            if (fits) {
                const uint32_t d = 16 + o;
                if (rd.staged(pos, pos + len)) {
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
                for (uint32_t bb = 0; bb < len; ++bb) dst[bb] = rd.u8<false>(pos + bb, 0);
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
    SD(8);
}

// Records the stream holds, T, from the last block's state: rec_offs[T] =
// where the stream stopped (the failing record's start, or the end of the
// last record), rec_offs[T + 1 .. n] = W, str_offs[f][T .. n] = the chars
// total; with T < n the status names record T (PREFIX or BOUNDS, and BOUNDS
// for every record after it).  Returns at once when the decode was given up.
template <int NS>
__global__ __launch_bounds__(kBlock) void k_sdec_finish(SdArgs a, SdScratch S, srpc_unpack_status* st,
                                                         const uint32_t* gate) {
    constexpr int NC = NS - 1;
    if (gate && !*gate) return;
    if (ld_ctl(S.ctl + kCtlAbort)) {
        if (st && blockIdx.x == 0 && threadIdx.x == 0) st->reserved |= 8u;
        return;
    }
    uint64_t ex = 0, T = 0, ch[kMaxNS] = {};
    uint32_t stp = 0;
    if (a.nb) {
        const uint64_t* iw = S.inc + static_cast<uint64_t>(a.nb - 1) * inc_words<NC>();
        ex = iw[0] & kValMask;
        T = iw[1] & kCnt40;
        stp = static_cast<uint32_t>((iw[1] >> 40) & 7);
#pragma unroll
        for (int k = 0; k < NC; ++k) ch[k] = iw[2 + k] & kValMask;
    }
    const uint64_t n = a.n;
    if (T <= n) {
        uint64_t tot[kMaxNS];
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
            for (uint32_t f = 0; f < a.nfields; ++f) {
                if (a.size[f]) continue;
                const uint32_t si = a.sord[f];
                uint64_t v = 0;
#pragma unroll
                for (int k = 0; k <= NC; ++k) v = si == static_cast<uint32_t>(k) ? tot[k] : v;
                a.soff[f][r] = v;
            }
        }
    }
    if (st && blockIdx.x == 0 && threadIdx.x == 0) {
        uint32_t fl = 0;
        if (T < n) {
            const uint32_t kind = (stp & 1) ? (stp >> 1) & 3 : 0;
            fl |= (kind ? kind : SRPC_STATUS_BOUNDS) | (T + 1 < n ? SRPC_STATUS_BOUNDS : 0);
            st->first_bad_record = T;
        }
        st->flags |= fl;
        st->reserved |= min<uint32_t>(ld_ctl(S.ctl + kCtlMiss), 0xffffffu) << 8;
    }
}

// The abort word always (the bounded decode after this one is gated on it);
// the rest only when this decode runs.
__global__ void k_sdec_reset(SdScratch S, srpc_unpack_status* st, const uint32_t* gate) {
    const uint32_t t = threadIdx.x;
    if (t == kCtlAbort) S.ctl[t] = 0;
    if (gate && !*gate) return;
    if (t < kCtlWords && t != kCtlAbort) S.ctl[t] = t == kCtlPastN ? 0xffffffffu : 0u;
    if (t == 0 && st) {
        st->flags = 0;
        st->reserved = 0;
        st->first_bad_record = ~0ull;
    }
}

uint64_t r256(uint64_t b) { return (b + 255) & ~255ull; }

struct SdLayout {
    uint64_t nb, flag, agg, inc, slot, ctl, total;
};

SdLayout sd_layout(uint64_t wire_len, uint32_t nc) {
    SdLayout L{};
    L.nb = (wire_len + kSB - 1) / kSB;
    uint64_t o = 0;
    L.flag = o;
    o += r256(8 * L.nb);
    L.agg = o;
    o += r256(8 * L.nb * (3 + nc));
    L.inc = o;
    o += r256(8 * L.nb * (2 + nc));
    L.slot = o;
    o += r256(8 * L.nb * kSlots * (3 + nc));
    L.ctl = o;
    o += 256;
    L.total = o;
    return L;
}

// This call's tag: process-unique, from a random start so flag words left in
// recycled memory by another process do not match.
uint32_t next_epoch() {
    static std::atomic<uint32_t> ctr{static_cast<uint32_t>(
        std::chrono::steady_clock::now().time_since_epoch().count() * 2246822519u ^
        (static_cast<uint32_t>(getpid()) << 7))};
    uint32_t e;
    do e = ctr.fetch_add(1, std::memory_order_relaxed);
    while ((e & kTagMax) == 0);
    return e;
}

template <int NS>
void launch_sdec(const SdArgs& a, const uint8_t* wire, const SdScratch& S, srpc_unpack_status* st, const uint32_t* gate,
                 hipStream_t s) {
    launch(k_sdec_reset, dim3(1), dim3(64), 0, s, S, st, gate);
    if (a.nb) launch(k_sdec<NS>, dim3(a.nb), dim3(kBlock), 0, s, a, wire, S, gate);
    const uint32_t g = static_cast<uint32_t>(std::min<uint64_t>(a.n / kBlock + 1, 4096));
    launch(k_sdec_finish<NS>, dim3(g), dim3(kBlock), 0, s, a, S, st, gate);
}

}  // namespace

bool sdec_supports(const srpc_plan* p) {
    return p && p->has_string && p->nstrings >= 1 && p->nstrings <= static_cast<uint32_t>(kMaxNS) &&
           p->fixed_bytes >= 8;
}

uint64_t sdec_scratch_bytes(const srpc_plan* p, uint64_t wire_len) {
    return sd_layout(wire_len, sdec_supports(p) ? p->nstrings - 1 : 0).total;
}

int sdec_launch(const srpc_plan* p, const uint8_t* wire, uint64_t wire_len, uint64_t n, uint64_t* rec_offs,
                void* const* cols, uint64_t* const* str_offs, srpc_unpack_status* st, void* scratch,
                uint32_t miss_limit, const uint32_t* gate, const uint32_t** abort_out, hipStream_t s) {
    if (!sdec_supports(p)) return SRPC_E_UNSUPPORTED;
    const uint32_t nc = p->nstrings - 1;
    const SdLayout SL = sd_layout(wire_len, nc);
    // positions, counts and chars travel as 43-bit values in the look-back words
    if (SL.nb > 0x7fffffffull || wire_len >= (1ull << 40)) return SRPC_E_UNSUPPORTED;
    auto* base = static_cast<uint8_t*>(scratch);
    SdScratch S{reinterpret_cast<uint64_t*>(base + SL.flag), reinterpret_cast<uint64_t*>(base + SL.agg),
                reinterpret_cast<uint64_t*>(base + SL.inc), reinterpret_cast<uint64_t*>(base + SL.slot),
                reinterpret_cast<uint32_t*>(base + SL.ctl)};
    SdArgs a{};
    uint32_t si = 0, run = 0;
    bool seen = false;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        a.size[f] = p->size[f];
        a.sord[f] = p->size[f] ? 0 : si;
        a.col[f] = static_cast<uint8_t*>(cols[f]);
        a.soff[f] = p->size[f] ? nullptr : str_offs[f];
        if (p->size[f]) {
            run += p->size[f];
        } else {
            a.run[si] = run;
            if (!seen) a.fla = p->prefix_len + run;
            seen = true;
            run = 0;
            ++si;
        }
    }
    a.run[si] = run;
    a.prefix = p->d_prefix;
    a.rec_offs = rec_offs;
    a.n = n;
    a.W = wire_len;
    a.nfields = p->nfields;
    a.P = p->prefix_len;
    a.fixed_bytes = p->fixed_bytes;
    a.plaus = p->prefix_len >= 8 ? 1 : 2;
    for (uint32_t i = 0; i < 8 && i < p->prefix_len; ++i) {
        a.pre8 |= static_cast<uint64_t>(p->h_prefix[i]) << (8 * i);
        a.pre8_mask |= 0xffull << (8 * i);
    }
    a.nb = static_cast<uint32_t>(SL.nb);
    a.epoch = next_epoch();
    // random data misses almost never (entry slots); data on which wrong
    // starts parse misses in most blocks, each miss a wait on the look-back
    // path: give up early
    a.miss_limit = miss_limit ? miss_limit : static_cast<uint32_t>(8 + SL.nb / 4096);
    *abort_out = S.ctl + kCtlAbort;
    switch (p->nstrings) {
    case 1: launch_sdec<1>(a, wire, S, st, gate, s); break;
    case 2: launch_sdec<2>(a, wire, S, st, gate, s); break;
    case 3: launch_sdec<3>(a, wire, S, st, gate, s); break;
    default: launch_sdec<4>(a, wire, S, st, gate, s); break;
    }
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

}  // namespace srpc_impl

#ifdef SRPC_SDEC_PHASES
extern "C" {
// Diagnostics: per-block phase words go to d_buf (16 u64 per block, the
// caller zeroes it) for blocks below nblocks.
int srpc_debug_sdec_phases(void* d_buf, uint64_t nblocks) {
    unsigned long long* p = static_cast<unsigned long long*>(d_buf);
    unsigned long long nb = nblocks;
    if (hipMemcpyToSymbol(HIP_SYMBOL(srpc_impl::g_sdph), &p, sizeof(p)) != hipSuccess) return SRPC_E_HIP;
    if (hipMemcpyToSymbol(HIP_SYMBOL(srpc_impl::g_sdph_blocks), &nb, sizeof(nb)) != hipSuccess) return SRPC_E_HIP;
    return SRPC_OK;
}
}
#endif
