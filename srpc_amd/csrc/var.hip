// var.hip -- records with string fields (SRPC_PATH_VAR).
//
// Wire format (reference include/srpc/packer.hpp): a string is a u64 LE length
// followed by its bytes (pack_arg<std::string> 193-198, pipe_output<std::string>
// 216-222); records are still back to back, so record i starts at the
// exclusive prefix sum of the record sizes before it.
//
// PACK  (srpc_gpu_pack_var)
//   1. k_scan_reduce / k_scan_partials / k_scan_apply: reduce-then-scan of the
//      record sizes  size(i) = fixed_bytes + sum_f len(i, f)  into
//      rec_offs[0..n] (u64).  Inside a workgroup: per-thread serial scan of 8
//      items, a 64-lane wavefront scan of the thread totals (__shfl_up), and
//      an LDS scan of the 4 wave totals.
//   2. k_pack_var: the wire is cut into 4 KiB tiles; a tile's first record
//      comes from the table the scan wrote (tile_first), the starts of the
//      records up to the next tile's first one are staged in LDS, and every
//      lane builds one 16-byte chunk of output: it walks the records/segments
//      (prefix, fixed fields, string length, string bytes) covering its 16
//      bytes, assembles them in an LDS staging slot and writes them with one
//      16-byte store.
// UNPACK (srpc_gpu_unpack_var) -- needs the record start index rec_offs
//   (produced by pack, or by frame lengths on a socket):
//   1. k_unpack_var_walk: one record per lane: prefix check, fixed fields to
//      their columns, string lengths and chars positions, record-size
//      consistency (status word on error).
//   2. scans of each string field's lengths -> str_offs[f][0..n].
//   3. k_unpack_var_chars: output-chunk-centric copy of string bytes.
// Byte movement uses unaligned 16-byte loads (one per record segment per
// 16-byte chunk), never one load per byte.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "plan.h"
#include "srpc_gpu.h"

namespace srpc_impl {
namespace {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kScanItems = 8;
constexpr uint64_t kScanBlock = static_cast<uint64_t>(kBlock) * kScanItems;  // 2048 items
constexpr uint32_t kTileBytes = kBlock * 16;                                  // 4 KiB output tile
constexpr uint32_t kWindow = 528;   // record starts staged in LDS per tile (>= 4096/8 + 2)
#ifndef SRPC_VAR_GRID
#define SRPC_VAR_GRID 2048  // 8192 / 32768 within +-5 % (profiles/r01_var_grid_ab.log)
#endif
constexpr int kVarGrid = SRPC_VAR_GRID;  // workgroups for grid-stride tiles
constexpr uint32_t kLongFlags = 256; // k_pack_short_records -> k_pack_var<true> flags, 64 bytes apart
constexpr uint32_t kShortRecord = 64; // records written one per lane are at most this long

struct VarArgs {
    const uint8_t* col[kMaxFields];   // fixed: column; string: chars
    const uint64_t* soff[kMaxFields]; // string: n+1 char offsets
    uint32_t size[kMaxFields];        // fixed size in bytes, 0 = string
    uint32_t sidx[kMaxFields];        // string ordinal of a string field
    uint32_t sfield[kMaxFields];      // field index of string ordinal si
    uint32_t ffield[kMaxFields];      // field index of fixed-field ordinal
    const uint8_t* prefix;            // device copy of the constant header
    uint32_t nfields, nstrings, prefix_len, fixed_bytes;
};

// ---- scans ------------------------------------------------------------------
struct PackSizes {
    VarArgs a;
    __device__ uint64_t operator()(uint64_t i) const {
        uint64_t s = a.fixed_bytes;
        for (uint32_t f = 0; f < a.nfields; ++f)
            if (a.size[f] == 0) s += a.soff[f][i + 1] - a.soff[f][i];
        return s;
    }
};

struct ArrayVals {
    const uint64_t* v;
    __device__ uint64_t operator()(uint64_t i) const { return v[i]; }
};

// Batched scan of every string field's lengths in one launch per phase:
// domain y = blockIdx.y = string ordinal, values v[y * n + i], output outs[y].
// The scan kernels offset partial and tile_first by y (a no-op for y = 0).
struct ArrayValsY {
    const uint64_t* v;
    uint64_t n;
    uint64_t* outs[kMaxFields];
    __device__ uint64_t operator()(uint64_t i) const { return v[blockIdx.y * n + i]; }
};
template <class F>
__device__ __forceinline__ uint64_t* scan_out(const F&, uint64_t* out) { return out; }
__device__ __forceinline__ uint64_t* scan_out(const ArrayValsY& f, uint64_t* /*out*/) { return f.outs[blockIdx.y]; }

// Tile metadata written by the scan for every tile whose first byte item i
// covers: item i itself (stride 1), which is all the chunk-walk kernels need.
struct FirstOnly {
    template <class F>
    __device__ void operator()(const F&, uint64_t i, uint64_t, uint64_t, uint64_t* out) const {
        out[0] = i;
    }
};

__device__ __forceinline__ uint64_t wave_inclusive_scan(uint64_t x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// Exclusive scan of one value per thread over the workgroup; returns the
// thread's exclusive prefix and writes the block total to *total.
__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t x, uint64_t* total) {
    __shared__ uint64_t wsum[kBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t inc = wave_inclusive_scan(x);
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint64_t before = 0, all = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
        before += (w < wave) ? wsum[w] : 0;
        all += wsum[w];
    }
    __syncthreads();
    *total = all;
    return before + inc - x;
}

// Every scan kernel takes `gate`: when non-null and *gate == 0 it does nothing
// (the single-string unpack's error path, see k_unpack_var_walk).  The reduce
// and apply kernels take scan block bx = blockIdx.x, blockIdx.x + gridDim.x,
// ... of nb: a gated scan is launched with a bounded grid, so on the (usual)
// exact batch its two no-op launches dispatch at most kGatedGrid workgroups
// instead of one per 2048 records (3.8 us each at 8M records,
// profiles/r04_short_string_unpack_kernels.csv).
constexpr uint32_t kGatedGrid = 512;
template <class F>
__global__ __launch_bounds__(kBlock) void k_scan_reduce(F f, uint64_t n, uint64_t* partial, const uint32_t* gate,
                                                        uint64_t nb) {
    if (gate && *gate == 0) return;
    for (uint64_t bx = blockIdx.x; bx < nb; bx += gridDim.x) {
        const uint64_t base = bx * kScanBlock;
        uint64_t s = 0;
#pragma unroll
        for (int j = 0; j < kScanItems; ++j) {
            const uint64_t i = base + static_cast<uint64_t>(j) * kBlock + threadIdx.x;
            if (i < n) s += f(i);
        }
        uint64_t tot;
        (void)block_exclusive_scan(s, &tot);
        if (threadIdx.x == 0) partial[blockIdx.y * (nb + 1) + bx] = tot;
    }
}

// One workgroup: exclusive scan of nb partials in place, partial[nb] = total.
__global__ __launch_bounds__(kBlock) void k_scan_partials(uint64_t* partial, uint64_t nb, const uint32_t* gate) {
    if (gate && *gate == 0) return;
    partial += blockIdx.y * (nb + 1);
    const uint64_t per = (nb + kBlock - 1) / kBlock;
    const uint64_t lo = threadIdx.x * per, hi = min(nb, lo + per);
    uint64_t s = 0;
    for (uint64_t i = lo; i < hi; ++i) s += partial[i];
    uint64_t tot;
    uint64_t run = block_exclusive_scan(s, &tot);
    for (uint64_t i = lo; i < hi; ++i) {
        const uint64_t v = partial[i];
        partial[i] = run;
        run += v;
    }
    if (threadIdx.x == 0) partial[nb] = tot;
}

// out[i] = exclusive prefix of f over [0, i); out[n] = total.  With
// tile_first, item i also writes the metadata M of every tile_bytes output
// tile whose first byte it covers (start_i <= t*tile_bytes < start_i + f(i)),
// at tile_first[t * meta_stride ...]: at least itself as the tile's first item,
// so a tile finds its first record with one load instead of a binary search.
template <class F, class M>
__global__ __launch_bounds__(kBlock) void k_scan_apply(F f, M meta, uint64_t n, const uint64_t* partial, uint64_t nb,
                                                       uint64_t* out, uint64_t* tile_first, uint64_t max_tiles,
                                                       uint64_t tile_bytes, uint32_t meta_stride,
                                                       const uint32_t* gate) {
    if (gate && *gate == 0) return;
    partial += blockIdx.y * (nb + 1);
    out = scan_out(f, out);
    if (tile_first) tile_first += blockIdx.y * max_tiles * meta_stride;
    __shared__ uint64_t v[kScanBlock];
    for (uint64_t bx = blockIdx.x; bx < nb; bx += gridDim.x) {
    const uint64_t base = bx * kScanBlock;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {  // coalesced reads, staged in LDS
        const uint32_t k = j * kBlock + threadIdx.x;
        v[k] = (base + k < n) ? f(base + k) : 0;
    }
    __syncthreads();
    uint64_t loc[kScanItems];
    uint64_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        loc[j] = s;
        s += v[threadIdx.x * kScanItems + j];
    }
    uint64_t tot;
    const uint64_t pre = block_exclusive_scan(s, &tot) + partial[bx];
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
        const uint32_t k = threadIdx.x * kScanItems + j;
        const uint64_t start = pre + loc[j], end = start + v[k];
        if (tile_first)
            for (uint64_t t = (start + tile_bytes - 1) / tile_bytes; t * tile_bytes < end && t < max_tiles; ++t)
                meta(f, base + k, start, t * tile_bytes, tile_first + t * meta_stride);
        v[k] = start;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {  // coalesced writes
        const uint32_t k = j * kBlock + threadIdx.x;
        if (base + k < n) out[base + k] = v[k];
    }
    if (bx == 0 && threadIdx.x == 0) out[n] = partial[nb];
    __syncthreads();  // (the next scan block overwrites v)
    }
}

// ---- record / chunk location -------------------------------------------------
// Largest r in [0, n] with offs[r] <= p (offs non-decreasing).  For a byte
// position p < offs[n] this is the record whose bytes cover p (records of
// zero length are skipped).
__device__ __forceinline__ uint64_t upper_index(const uint64_t* offs, uint64_t n, uint64_t p) {
    uint64_t lo = 0, hi = n;  // invariant: offs[lo] <= p, answer in [lo, hi]
    while (lo < hi) {
        const uint64_t mid = (lo + hi + 1) >> 1;
        if (offs[mid] <= p) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// Per-tile helper: a window of record starts from the tile's first covering
// record r0 (tile_first, written by the scan) on, staged in LDS.
struct Window {
    uint64_t r0;
    uint32_t len;  // entries valid in win[0..len)
};

// rz: the record covering the next tile's first byte (or n - 1): entries
// r0 .. rz + 1 cover every byte of this tile, so only those are staged.
__device__ __forceinline__ Window load_window(const uint64_t* offs, uint64_t n, uint64_t r0, uint64_t rz,
                                              uint64_t* win) {
    const uint32_t len = static_cast<uint32_t>(min<uint64_t>(min<uint64_t>(kWindow, n + 1 - r0), rz + 2 - r0));
    for (uint32_t k = threadIdx.x; k < len; k += kBlock) win[k] = offs[r0 + k];
    __syncthreads();
    return {r0, len};
}

// The window plus the same records' entries of a second offsets array.
__device__ __forceinline__ Window load_window2(const uint64_t* offs, const uint64_t* offs2, uint64_t n, uint64_t r0,
                                               uint64_t rz, uint64_t* win, uint64_t* win2) {
    const uint32_t len = static_cast<uint32_t>(min<uint64_t>(min<uint64_t>(kWindow, n + 1 - r0), rz + 2 - r0));
    for (uint32_t k = threadIdx.x; k < len; k += kBlock) {
        win[k] = offs[r0 + k];
        win2[k] = offs2[r0 + k];
    }
    __syncthreads();
    return {r0, len};
}

// Covering record of byte p using the window (global search when p lies past it).
__device__ __forceinline__ uint64_t find_record(const uint64_t* offs, uint64_t n, const Window& w,
                                                const uint64_t* win, uint64_t p) {
    if (win[w.len - 1] <= p) {
        if (w.r0 + w.len - 1 >= n) return n;
        return upper_index(offs, n, p);  // rare: window exhausted
    }
    uint32_t lo = 0, hi = w.len - 1;  // win[lo] <= p < win[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (win[mid] <= p) lo = mid;
        else hi = mid;
    }
    return w.r0 + lo;
}

// ---- byte movers ----------------------------------------------------------------
// Every output chunk (16 aligned bytes) is assembled in a 32-byte LDS slot of
// its lane -- one unaligned 16-byte global load and one 16-byte LDS write per
// record segment it touches -- and leaves with one 16-byte store.  (Merging
// in registers instead -- the load taken from src - b so the segment lands in
// place, then a byte mask -- measured 1.4-1.6x slower: profiles/r01_paths.log.)
// Sources are never read past their end (`end`): near it the copy falls back
// to bytes.
struct Slot {
    uint8_t* s;
};

__device__ __forceinline__ void put(Slot& c, const uint8_t* src, int b, int k, const uint8_t* end) {
    if (src + 16 <= end) {
        uint4 v;
        __builtin_memcpy(&v, src, 16);
        __builtin_memcpy(c.s + b, &v, 16);  // the slot has 16 bytes of room past any b < 16
    } else {
        for (int i = 0; i < k; ++i) c.s[b + i] = src[i];
    }
}

// Bytes [x, x + 8) of a u64 string length at slot byte b.
__device__ __forceinline__ void put_u64(Slot& c, uint64_t v, int x, int b) {
    v >>= 8 * x;
    __builtin_memcpy(c.s + b, &v, 8);
}

__device__ __forceinline__ void store_slot(uint8_t* dst, const Slot& c, uint32_t nb) {
    if (nb == 16) {
        const u64x2 v = *reinterpret_cast<const u64x2*>(c.s);
        __builtin_nontemporal_store(v, reinterpret_cast<u64x2*>(dst));
    } else {
        for (uint32_t i = 0; i < nb; ++i) dst[i] = c.s[i];
    }
}

template <typename T>
__device__ __forceinline__ T load_unaligned(const uint8_t* p) {
    T v;
    __builtin_memcpy(&v, p, sizeof(T));
    return v;
}

// ---- phase clock (A/B diagnostics, compiled only with -DSRPC_PHASES) -------------
#ifdef SRPC_PHASES
__device__ unsigned long long g_phase[8];
#define PHASE_BEGIN uint64_t ph_last_ = clock64(), ph_acc_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define PHASE(i)                                       \
    do {                                               \
        const uint64_t now_ = clock64();               \
        ph_acc_[i] += now_ - ph_last_;                 \
        ph_last_ = now_;                               \
    } while (0)
#define PHASE_COUNT(i) ph_acc_[i] += 1
#define PHASE_END                                                              \
    if (threadIdx.x == 0)                                                      \
        for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_phase[i_], ph_acc_[i_]);
#else
#define PHASE_BEGIN
#define PHASE(i)
#define PHASE_COUNT(i)
#define PHASE_END
#endif

// ---- pack ---------------------------------------------------------------------
// Merge `cnt` (<= 16) bytes of record r, from byte q of the record, into chunk
// bytes [b, b + cnt).  Segments in wire order: prefix, then every field
// (fixed value | u64 length, chars).  sw (may be null): LDS copy of
// soff[f0][r], soff[f0][r+1] for the first string field f0.
// pre: the prefix followed by 16 zero bytes (LDS copy in k_pack_var).
__device__ __forceinline__ void emit_record(const VarArgs& a, const uint8_t* pre, const uint64_t* climit, uint32_t f0,
                                            const uint64_t* sw, uint64_t n, uint64_t r, uint64_t q, uint32_t cnt,
                                            int b, Slot& c) {
    const uint64_t end = q + cnt;
    if (q < a.prefix_len) {
        const int k = static_cast<int>(min<uint64_t>(end, a.prefix_len) - q);
        put(c, pre + q, b, k, pre + a.prefix_len + 16);
        b += k;
        q += k;
    }
    uint64_t s = a.prefix_len;  // start of the current segment within the record
    for (uint32_t f = 0; f < a.nfields && q < end; ++f) {
        const uint32_t sz = a.size[f];
        if (sz) {
            if (q < s + sz) {
                const int k = static_cast<int>(min<uint64_t>(end, s + sz) - q);
                put(c, a.col[f] + r * sz + (q - s), b, k, a.col[f] + n * sz);
                b += k;
                q += k;
            }
            s += sz;
        } else {
            const bool staged = f == f0 && sw;
            const uint64_t b0 = staged ? sw[0] : a.soff[f][r];
            const uint64_t len = (staged ? sw[1] : a.soff[f][r + 1]) - b0;
            if (q < s + 8) {
                const int k = static_cast<int>(min<uint64_t>(end, s + 8) - q);
                put_u64(c, len, static_cast<int>(q - s), b);
                b += k;
                q += k;
            }
            s += 8;
            if (q < end && q < s + len) {
                const int k = static_cast<int>(min<uint64_t>(end, s + len) - q);
                put(c, a.col[f] + b0 + (q - s), b, k, a.col[f] + climit[f]);
                b += k;
                q += k;
            }
            s += len;
        }
    }
}

// kSkip: return at once when k_pack_short_records wrote every record.  All or nothing, and a separate instantiation: a
// per-tile skip test in this loop, in any form, made the kernel 40 % slower
// for every schema, even never taken (profiles/r01_var_short_copy_ab.log).
template <bool kSkip>
__global__ __launch_bounds__(kBlock) void k_pack_var(VarArgs a, const uint64_t* __restrict__ rec_offs, uint64_t n,
                                                     const uint64_t* __restrict__ tile_first,
                                                     uint8_t* __restrict__ wire, uint64_t wire_cap,
                                                     srpc_unpack_status* st, const uint32_t* __restrict__ some_long,
                                                     const uint64_t* __restrict__ soff0) {
    __shared__ uint64_t win[kWindow];
    __shared__ uint64_t swin[kWindow];       // char offsets of the first string field, same records
    __shared__ uint64_t climit[kMaxFields];  // end of each string field's chars
    __shared__ __attribute__((aligned(16))) uint8_t slots[kBlock * 32];
#ifndef SRPC_PACK_PREFIX_GLOBAL
    // the prefix segment is read from LDS: no L2 round trip per chunk that starts a record
    __shared__ __attribute__((aligned(16))) uint8_t pre[kMaxPrefix + 16];
    if (a.prefix_len)  // no device prefix (null) when the plan has none
        for (uint32_t i = threadIdx.x; i < a.prefix_len + 16; i += kBlock) pre[i] = a.prefix[i];
#else
    const uint8_t* pre = a.prefix;
#endif
    uint32_t f0 = 0;                         // the first string field
    while (a.size[f0]) ++f0;
    for (uint32_t f = threadIdx.x; f < a.nfields; f += kBlock) climit[f] = a.size[f] ? 0 : a.soff[f][n];
    const uint64_t total = rec_offs[n];
    const uint64_t limit = min(total, wire_cap);
    if (total > wire_cap && blockIdx.x == 0 && threadIdx.x == 0 && st)
        report_bad(st, SRPC_STATUS_BOUNDS, upper_index(rec_offs, n, wire_cap));
    const uint64_t ntiles = (limit + kTileBytes - 1) / kTileBytes;
    if constexpr (kSkip)  // k_pack_short_records wrote every record
        if (!__syncthreads_or(threadIdx.x < kLongFlags && some_long[threadIdx.x * 16])) return;
    PHASE_BEGIN
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t lo = t * kTileBytes;
        const uint64_t r0 = tile_first[t], rz = t + 1 < ntiles ? max(tile_first[t + 1], r0) : n - 1;
        PHASE(0);
        const Window w = load_window2(rec_offs, soff0, n, r0, rz, win, swin);
        PHASE(1);
        const uint64_t p0 = lo + 16ull * threadIdx.x;
        if (p0 < limit) {
            const uint32_t nb = static_cast<uint32_t>(min<uint64_t>(16, limit - p0));
            uint64_t r = find_record(rec_offs, n, w, win, p0);
            PHASE(2);
            uint64_t p = p0;
            uint32_t b = 0;
            Slot c{slots + 32 * threadIdx.x};
            while (b < nb && r < n) {
                const uint64_t k = r - w.r0;
                const uint64_t rs = k + 1 < w.len ? win[k] : rec_offs[r];
                const uint64_t re = k + 1 < w.len ? win[k + 1] : rec_offs[r + 1];
                const uint32_t cnt = static_cast<uint32_t>(min<uint64_t>(nb - b, re - p));
                emit_record(a, pre, climit, f0, k + 1 < w.len ? swin + k : nullptr, n, r, p - rs, cnt,
                            static_cast<int>(b), c);
                b += cnt;
                p += cnt;
                ++r;
            }
            PHASE(3);
            store_slot(wire + p0, c, nb);
            PHASE(4);
        }
        __syncthreads();  // the window is rewritten for the next tile
        PHASE(5);
        PHASE_COUNT(6);
    }
    PHASE_END
}

// ---- unpack -------------------------------------------------------------------
// One record per lane: prefix check, every string's length and chars position
// (lens/spos: [nstrings][n] scratch), and the fixed fields straight into their
// columns.  A string length past the record end (checked BEFORE it is used;
// the reference checks after the read, core.hpp:29-31) or a record whose size
// disagrees with the index is a BOUNDS error: that record's strings are
// decoded as empty.
//
// Single-string schemas (soff1 != null): the string's output offset needs no
// scan -- every record's string length is its size minus fixed_bytes, so
// str_offs[r] = rec_offs[r] - rec_offs[0] - r * fixed_bytes -- and its chars
// start len_at + 8 bytes into the record, so lens/spos are not written.  The
// walk writes str_offs and the chars tiles' first records itself; a record
// whose decoded length differs from that (any BOUNDS record, or a size
// mismatch under a PREFIX error) sets *bad, which runs the gated scan of
// SingleStrLen that rewrites both with the general path's semantics.
struct SingleFast {
    uint64_t* soff1;       // str_offs of the string field (n + 1)
    uint64_t* tiles;       // chars tiles' first records
    uint64_t max_tiles;
    uint32_t* bad;         // [0] some record is not exact, [16 k], k = 1 .. kLongFlags - 1: some chars tile is left to the chars kernel
    uint8_t* chars;        // the string field's output chars
    uint32_t* tile_long;   // per chars tile: 1 = it holds chars the walk did not copy
    uint32_t chars_at;     // chars start this many bytes into a record
    uint64_t first, last;  // rec_offs[0], rec_offs[n] (set by the walk)
};

// A wave whose 64 strings are all at most kShortCopy bytes copies them in the
// walk itself (one lane per string: an unaligned 16-byte load, stores of
// exactly len bytes); only chars tiles holding bytes of other waves' strings
// are left to k_unpack_var_chars (A/B: tools/ab_str.sh,
// profiles/r01_var_short_copy_ab.log -- per-lane copies of mixed lengths cost
// more than the chars kernel saves, hence the wave-uniform rule).
#ifndef SRPC_SHORT_COPY
#define SRPC_SHORT_COPY 32
#endif
constexpr uint32_t kShortCopy = SRPC_SHORT_COPY;

template <typename T>
__device__ __forceinline__ void store_unaligned(uint8_t* p, T v) {
    __builtin_memcpy(p, &v, sizeof(T));
}

// dst[0, len) := src[0, len); src bytes at or past src_end are never read.
__device__ __forceinline__ void copy_short(uint8_t* dst, const uint8_t* src, uint32_t len, const uint8_t* src_end) {
    while (len) {
        uint64_t lo = 0, hi = 0;
        if (src + 16 <= src_end) {
            lo = load_unaligned<uint64_t>(src);
            hi = load_unaligned<uint64_t>(src + 8);
        } else {
            for (uint32_t i = 0; i < 16 && src + i < src_end; ++i)
                (i < 8 ? lo : hi) |= static_cast<uint64_t>(src[i]) << (8 * (i & 7));
        }
        if (len >= 16) {
            store_unaligned(dst, lo);
            store_unaligned(dst + 8, hi);
            dst += 16;
            src += 16;
            len -= 16;
            continue;
        }
        uint32_t o = 0;
        if (len & 8) {
            store_unaligned(dst, lo);
            lo = hi;
            o = 8;
        }
        if (len & 4) {
            store_unaligned(dst + o, static_cast<uint32_t>(lo));
            lo >>= 32;
            o += 4;
        }
        if (len & 2) {
            store_unaligned(dst + o, static_cast<uint16_t>(lo));
            lo >>= 16;
            o += 2;
        }
        if (len & 1) dst[o] = static_cast<uint8_t>(lo);
        return;
    }
}

// k <= 8 low bytes of v at p (unaligned).
__device__ __forceinline__ void store_bytes(uint8_t* p, uint64_t v, uint32_t k) {
    if (k == 8) {
        store_unaligned(p, v);
        return;
    }
    uint32_t o = 0;
    if (k & 4) {
        store_unaligned(p, static_cast<uint32_t>(v));
        v >>= 32;
        o = 4;
    }
    if (k & 2) {
        store_unaligned(p + o, static_cast<uint16_t>(v));
        v >>= 16;
        o += 2;
    }
    if (k & 1) p[o] = static_cast<uint8_t>(v);
}

// Pack, before k_pack_var, one record per lane.  Single-string schemas
// (kSingle) need no scan for the record index: record r starts at
// (soff[r] - soff[0]) + r * fixed_bytes, and this kernel writes rec_offs[0..n]
// and the first record of every kTileBytes wire tile (what
// k_scan_apply<PackSizes> writes for other schemas, which run it first).  A
// wave whose strings are all <= kShortCopy bytes (when the batch fits
// wire_cap; the host passes wire_cap 0 for schemas whose records can exceed
// kShortRecord bytes) also writes its records' wire bytes -- prefix, fixed fields, u64
// lengths, chars -- with unaligned stores of exactly their bytes; any other
// wave sets *some_long, and then k_pack_var<true> writes the whole batch
// again (all or nothing, see k_pack_var).
template <bool kSingle>
__global__ __launch_bounds__(kBlock) void k_pack_short_records(VarArgs a, uint64_t n, uint64_t* __restrict__ rec_offs,
                                                               uint64_t* __restrict__ tile_first,
                                                               uint32_t* __restrict__ some_long, uint64_t max_tiles,
                                                               uint8_t* __restrict__ wire, uint64_t wire_cap) {
    const uint64_t r = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    uint64_t start, total;
    bool short_ok = true;
    if constexpr (kSingle) {
        const uint64_t* soff = a.soff[a.sfield[0]];
        const uint64_t s0 = soff[0], sr = soff[min(r, n)];
        start = sr - s0 + r * a.fixed_bytes;
        if (r <= n) rec_offs[r] = start;
        total = soff[n] - s0 + n * a.fixed_bytes;
        const uint64_t len = r < n ? soff[r + 1] - sr : 0;
        const uint64_t end = start + a.fixed_bytes + len;
        if (r < n)
            for (uint64_t t = (start + kTileBytes - 1) / kTileBytes; t * kTileBytes < end && t < max_tiles; ++t)
                tile_first[t] = r;
        short_ok = len <= kShortCopy;
    } else {
        start = rec_offs[min(r, n)];
        total = rec_offs[n];
        if (r < n)
            for (uint32_t si = 0; si < a.nstrings; ++si) {
                const uint64_t* so = a.soff[a.sfield[si]];
                short_ok &= so[r + 1] - so[r] <= kShortCopy;
            }
    }
    const bool all_short = __all(short_ok && total <= wire_cap);
    // some_long: kLongFlags flags 64 bytes apart, one store per long workgroup
    // (a single flag written by every long wave serialised them: 15 -> 63 us)
    if (__syncthreads_or(!all_short)) {
        if (threadIdx.x == 0) some_long[(blockIdx.x % kLongFlags) * 16] = 1;
        return;
    }
    if (r >= n) return;
    uint8_t* d = wire + start;
    for (uint32_t i = 0; i < a.prefix_len; i += 8)  // the device prefix has 16 zero bytes after it
        store_bytes(d + i, load_unaligned<uint64_t>(a.prefix + i), min(8u, a.prefix_len - i));
    d += a.prefix_len;
    for (uint32_t f = 0; f < a.nfields; ++f) {
        const uint32_t sz = a.size[f];
        if (sz) {
            const uint8_t* c = a.col[f] + r * sz;
            const uint64_t v = sz == 1   ? *c
                               : sz == 2 ? load_unaligned<uint16_t>(c)
                               : sz == 4 ? load_unaligned<uint32_t>(c)
                                         : load_unaligned<uint64_t>(c);
            store_bytes(d, v, sz);
            d += sz;
            continue;
        }
        const uint64_t* so = a.soff[f];
        const uint64_t s = so[r], len = so[r + 1] - s;
        store_unaligned(d, len);
        d += 8;
        copy_short(d, a.col[f] + s, static_cast<uint32_t>(len), a.col[f] + so[n]);
        d += len;
    }
}

// The walk's per-record parse.  src points at the record's first wire byte
// (in the LDS stage or in global memory), src_end bounds what may be read
// from it; positions are wire offsets (pos - start indexes src).
template <typename Pre>
__device__ __forceinline__ void walk_record(const VarArgs& a, const uint8_t* src, const uint8_t* src_end,
                                            const Pre* pre, uint64_t r, uint64_t start, uint64_t end,
                                            uint64_t wire_len, uint64_t n, uint64_t* lens, uint64_t* spos,
                                            srpc_unpack_status* st, const SingleFast& fast) {
    uint32_t flag = 0;
    if (start > end || end > wire_len || end - start < a.fixed_bytes) flag = SRPC_STATUS_BOUNDS;
    if (!flag) {
        uint32_t i = 0;
        for (; i + 8 <= a.prefix_len; i += 8)
            if (load_unaligned<uint64_t>(src + i) != load_unaligned<uint64_t>(pre + i)) flag = SRPC_STATUS_PREFIX;
        for (; i < a.prefix_len; ++i)
            if (src[i] != pre[i]) flag = SRPC_STATUS_PREFIX;
    }
    uint64_t pos = start + a.prefix_len;
    for (uint32_t f = 0; f < a.nfields; ++f) {
        const uint32_t sz = a.size[f];
        if (sz) {
            // a fixed field past the record end is never read (it could lie
            // past the wire buffer) and its column entry is left unwritten;
            // the record is then BOUNDS (or stays PREFIX) by the size check below
            if (flag != SRPC_STATUS_BOUNDS && pos + sz <= end) {
                uint8_t* dst = const_cast<uint8_t*>(a.col[f]) + r * sz;
                const uint8_t* q = src + (pos - start);
                switch (sz) {
                case 1: dst[0] = q[0]; break;
                case 2: *reinterpret_cast<uint16_t*>(dst) = load_unaligned<uint16_t>(q); break;
                case 4: *reinterpret_cast<uint32_t*>(dst) = load_unaligned<uint32_t>(q); break;
                default: *reinterpret_cast<uint64_t*>(dst) = load_unaligned<uint64_t>(q); break;
                }
            }
            pos += sz;
            continue;
        }
        const uint32_t si = a.sidx[f];
        uint64_t len = 0;
        if (flag != SRPC_STATUS_BOUNDS && pos + 8 <= end) {
            len = load_unaligned<uint64_t>(src + (pos - start));
            pos += 8;
            if (len > end - pos) {
                flag = SRPC_STATUS_BOUNDS;
                len = 0;
            }
        } else {
            flag = SRPC_STATUS_BOUNDS;
        }
        if (!fast.soff1) {
            spos[si * n + r] = pos;
            lens[si * n + r] = len;
        }
        pos += len;
    }
    if (!flag && pos != end) flag = SRPC_STATUS_BOUNDS;  // record size disagrees with the index
    if (fast.soff1) {
        const uint64_t first = fast.first;
        const uint64_t o = start - first - r * a.fixed_bytes;  // the output offset if every record is exact
        fast.soff1[r] = o;
        if (r == n - 1) fast.soff1[n] = fast.last - first - n * a.fixed_bytes;
        const uint64_t len = end - start - a.fixed_bytes;
        // exact: the decoded length (0 for BOUNDS) is the index's size - fixed_bytes,
        // and o is a real output offset.  o is only right when every earlier
        // record is exact too; when one is not (an empty frame, a non-monotonic
        // index), o can wrap or exceed the chars buffer (wire_len bytes), so a
        // record whose o + len does not fit is not exact either: *bad then
        // reruns the offsets through the scan and the chars kernel copies
        // every tile.  This keeps the walk's own copy inside the buffer.
        const bool exact = flag != SRPC_STATUS_BOUNDS && pos == end && start >= first &&
                           start - first >= r * a.fixed_bytes && o <= wire_len && len <= wire_len - o;
        // a wave whose strings are all short copies them here; otherwise its
        // strings' chars tiles are left to k_unpack_str1_tail (a flag below
        // says some tile is, else that launch has nothing to do)
        const bool all_short = __all(exact && len <= kShortCopy);
        if (exact) {
            for (uint64_t t = (o + kTileBytes - 1) / kTileBytes; t * kTileBytes < o + len && t < fast.max_tiles; ++t)
                fast.tiles[t] = r;
            if (all_short) {
                copy_short(fast.chars + o, src + fast.chars_at, static_cast<uint32_t>(len), src_end);
            } else {
                for (uint64_t t = o / kTileBytes; t * kTileBytes < o + len && t < fast.max_tiles; ++t)
                    fast.tile_long[t] = 1;
            }
        } else {
            atomicOr(fast.bad, 1u);
        }
        // some chars tile is left to the chars kernel: one store per wave, to
        // one of kLongFlags flags (a flag per lane of every long wave, all on
        // one address, cost 0-1024 B strings 108 us)
        const uint64_t act = __ballot(exact && !all_short);
        if (act && (threadIdx.x & 63) == static_cast<uint32_t>(__builtin_ctzll(__ballot(1))))
            fast.bad[16 * (1 + (blockIdx.x + (threadIdx.x >> 6)) % (kLongFlags - 1))] = 1;
    } else if (flag == SRPC_STATUS_BOUNDS) {  // positions are untrustworthy: decode nothing of this record's strings
        for (uint32_t si = 0; si < a.nstrings; ++si) lens[si * n + r] = 0;
    }
    if (flag && st) report_bad(st, flag, r);
}

// One record per lane.  The workgroup's 256 records are normally one
// contiguous wire span [rec_offs[r0], rec_offs[r0 + 256]); when it fits the
// LDS stage it is copied there first with coalesced 16-byte loads, so the
// per-record parse (prefix, fixed fields, a chain of dependent string
// lengths) reads LDS instead of paying an HBM round trip per length.  A
// record outside the staged span (a long span, or an index that is not
// monotonic) is parsed from global memory with the same code.
constexpr uint64_t kWalkStageMax = 49152;
#ifndef SRPC_STAGE_NUM
#define SRPC_STAGE_NUM 17
#endif
#ifndef SRPC_RTU_OFFLOAD
#define SRPC_RTU_OFFLOAD 1  // look-back waves' records built by the other waves (two strings 279 -> 270 us)
#endif
constexpr uint64_t kWalkTwoPerLane = 20;  // single-string walk: two records per lane at most this average
#ifndef SRPC_STAGE_DEN
#define SRPC_STAGE_DEN 16
#endif
#ifndef SRPC_STAGE_ROUND
#define SRPC_STAGE_ROUND 512
#endif
// the stage copy writes whole 16-byte chunks up to stage_bytes
static_assert((SRPC_STAGE_ROUND & (SRPC_STAGE_ROUND - 1)) == 0, "SRPC_STAGE_ROUND must be a power of two");
static_assert(SRPC_STAGE_ROUND % 16 == 0, "SRPC_STAGE_ROUND must be a multiple of 16");
static_assert(SRPC_STAGE_NUM >= SRPC_STAGE_DEN, "the stage must hold at least the average span");
// LDS stage of the unpack walk for an average record of avg bytes: the
// workgroup's 256 records with 6 % slack (a wider span parses from global;
// correct either way).  5/4 rounded to 4 KiB staged 32 KiB for ~100-byte
// records (4 workgroups per CU); 17/16 rounded to 512 B stages 27.5 KiB (5):
// two strings + envelope unpack 380 -> 361 us (r01_var_stage_slack_ab.log).
inline uint64_t stage_bytes_for(uint64_t avg, uint32_t rpl = 1) {
    return (avg * kBlock * rpl * SRPC_STAGE_NUM / SRPC_STAGE_DEN + 32 + SRPC_STAGE_ROUND - 1) &
           ~(SRPC_STAGE_ROUND - 1ull);
}

// STAGED (chosen by the host when 17/16 of the average span fits 48 KiB): the
// stage is dynamic LDS of exactly stage_bytes -- a fixed 32 KiB stage cost
// short-record schemas more in occupancy than it saved (0-16 B strings
// 105 -> 139 us), the sized one gains 4-8 % on them.
template <bool STAGED, int RPL>
__global__ __launch_bounds__(kBlock) void k_unpack_var_walk(VarArgs a, const uint8_t* __restrict__ wire,
                                                            uint64_t wire_len, const uint64_t* __restrict__ rec_offs,
                                                            uint64_t n, uint64_t* lens, uint64_t* spos,
                                                            srpc_unpack_status* st, SingleFast fast,
                                                            uint32_t stage_bytes) {
    __shared__ __attribute__((aligned(16))) uint8_t pre[kMaxPrefix + 16];
    extern __shared__ __attribute__((aligned(16))) uint8_t stage[];
    for (uint32_t i = threadIdx.x; i < a.prefix_len; i += kBlock) pre[i] = a.prefix[i];
    constexpr uint64_t kRecs = static_cast<uint64_t>(kBlock) * RPL;
    const uint64_t rA = static_cast<uint64_t>(blockIdx.x) * kRecs;
    const uint64_t rB = min<uint64_t>(rA + kRecs, n);
    // the lanes' own record bounds are loaded with the span's, before the
    // stage's barrier (one memory round trip less per workgroup: 0-16 B
    // strings 108.6 -> 99.2 us, profiles/r06_var_walk_ab.log)
    uint64_t start[RPL], end[RPL];
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
        const uint64_t r = rA + static_cast<uint64_t>(j) * kBlock + threadIdx.x;
        start[j] = r < n ? rec_offs[r] : 0;
        end[j] = r < n ? rec_offs[r + 1] : 0;
    }
    if (fast.soff1) {
        fast.first = rec_offs[0];
        fast.last = rec_offs[n];
    }
    const uint64_t lo = rec_offs[rA], hi = min(rec_offs[rB], wire_len);
    const uint64_t base = lo & ~15ull;
    // 16 bytes past the span: a fixed field after a string may be read up to
    // 7 bytes past its record's end (the record is then BOUNDS), as in global
    const uint64_t shi = min(hi + 16, wire_len);
    const bool staged = STAGED && lo < hi && shi - base <= stage_bytes;  // workgroup-uniform
    if (staged) {
        const uint32_t nch = static_cast<uint32_t>((shi - base + 15) >> 4);
        for (uint32_t c = threadIdx.x; c < nch; c += kBlock) {
            const uint64_t g = base + 16ull * c;
            if (g + 16 <= wire_len) {
                *reinterpret_cast<u64x2*>(stage + 16 * c) = *reinterpret_cast<const u64x2*>(wire + g);
            } else {
                for (uint32_t k = 0; k < 16 && g + k < wire_len; ++k) stage[16 * c + k] = wire[g + k];
            }
        }
    }
    __syncthreads();
    // (walk_record's all-short vote then runs per branch: it only chooses
    // between a lane copying its own string and flagging its chars tiles,
    // and either is correct per lane)
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
        const uint64_t r = rA + static_cast<uint64_t>(j) * kBlock + threadIdx.x;
        if (r >= n) continue;
        if (staged && start[j] >= lo && end[j] <= hi && start[j] <= end[j])
            walk_record(a, stage + (start[j] - base), stage + (shi - base), pre, r, start[j], end[j], wire_len, n,
                        lens, spos, st, fast);
        else
            walk_record(a, wire + start[j], wire + wire_len, pre, r, start[j], end[j], wire_len, n, lens, spos, st,
                        fast);
    }
}

// The single-string error path's lengths: exactly the length the walk
// decodes for record r (0 for a BOUNDS record).
struct SingleStrLen {
    const uint8_t* wire;
    uint64_t wire_len;
    const uint64_t* rec;
    const uint8_t* prefix;
    uint32_t prefix_len, len_at, fixed_bytes;
    __device__ uint64_t operator()(uint64_t r) const {
        const uint64_t start = rec[r], end = rec[r + 1];
        if (start > end || end > wire_len || end - start < fixed_bytes) return 0;
        const uint64_t len = load_unaligned<uint64_t>(wire + start + len_at);
        if (len > end - (start + len_at + 8)) return 0;
        if (len == end - start - fixed_bytes) return len;
        for (uint32_t i = 0; i < prefix_len; ++i)  // a PREFIX record keeps its length; otherwise it is BOUNDS
            if (wire[start + i] != prefix[i]) return len;
        return 0;
    }
};

// Chars of one string field, tile t: output chunk c = bytes [16c, 16c+16) of
// chars.  Record r's chars start at spos[r] in the wire, or (single-string
// schemas, spos == null) at rec_offs[r] + chars_at, staged with the window.
// r0/r1: tile_first[t], tile_first[t + 1].  Block-wide (syncs inside).
// Head: hoist the chunk's first two segments (multi-string schemas, whose
// strings are short next to the tile; with 0-1024 B single strings it costs 5 %).
template <bool Head>
__device__ __forceinline__ void chars_tile(const uint8_t* __restrict__ wire, uint64_t wire_len,
                                           const uint64_t* __restrict__ soff, const uint64_t* __restrict__ spos,
                                           uint64_t n, uint8_t* __restrict__ chars,
                                           const uint64_t* __restrict__ rec_offs, uint32_t chars_at, uint64_t t,
                                           uint64_t ntiles, uint64_t total, uint64_t r0, uint64_t r1, uint64_t* win,
                                           uint64_t* rwin, uint8_t* slots) {
    const uint64_t lo = t * kTileBytes;
    const uint64_t rz = t + 1 < ntiles ? max(r1, r0) : n - 1;
    const Window w = spos ? load_window(soff, n, r0, rz, win) : load_window2(soff, rec_offs, n, r0, rz, win, rwin);
    const uint64_t p0 = lo + 16ull * threadIdx.x;
    if (p0 < total) {
        const uint32_t nb = static_cast<uint32_t>(min<uint64_t>(16, total - p0));
        uint64_t r = find_record(soff, n, w, win, p0);
        uint64_t p = p0;
        uint32_t b = 0;
        Slot c{slots + 32 * threadIdx.x};
        // Head: the chunk's first two segments (records r and r + 1) with
        // their source offsets and 16-byte wire loads issued together, so
        // the two (offset -> chars) load chains overlap instead of running
        // back to back.  The loop below finishes chunks spanning more.
        if (Head && r < n) {
            const uint64_t k = r - w.r0;
            const uint64_t r1 = min(r + 1, n - 1);
            const uint64_t rs0 = k + 1 < w.len ? win[k] : soff[r];
            const uint64_t re0 = k + 1 < w.len ? win[k + 1] : soff[r + 1];
            const uint64_t re1 = k + 2 < w.len ? win[k + 2] : soff[r1 + 1];
            const uint64_t sp0 = spos ? spos[r] : (k + 1 < w.len ? rwin[k] : rec_offs[r]) + chars_at;
            const uint64_t sp1 = spos ? spos[r1] : (k + 2 < w.len ? rwin[k + 1] : rec_offs[r1]) + chars_at;
            const uint32_t cnt0 = static_cast<uint32_t>(min<uint64_t>(nb, re0 - p));
            const uint64_t p1 = p + cnt0;
            const uint32_t cnt1 = (cnt0 < nb && r + 1 < n)
                                      ? static_cast<uint32_t>(min<uint64_t>(nb - cnt0, re1 - p1))
                                      : 0u;
            const uint8_t* s0 = wire + sp0 + (p - rs0);
            const uint8_t* s1 = cnt1 ? wire + sp1 + (p1 - re0) : s0;
            const uint8_t* end = wire + wire_len;
            if (s0 + 16 <= end && s1 + 16 <= end) {
                uint4 v0, v1;
                __builtin_memcpy(&v0, s0, 16);
                __builtin_memcpy(&v1, s1, 16);
                __builtin_memcpy(c.s, &v0, 16);
                if (cnt1) __builtin_memcpy(c.s + cnt0, &v1, 16);
            } else {
                if (cnt0) put(c, s0, 0, static_cast<int>(cnt0), end);
                if (cnt1) put(c, s1, static_cast<int>(cnt0), static_cast<int>(cnt1), end);
            }
            b = cnt0 + cnt1;
            p = p1 + cnt1;
            r += cnt0 < nb ? 2 : 1;
        }
        while (b < nb && r < n) {
            const uint64_t k = r - w.r0;
            const uint64_t rs = k + 1 < w.len ? win[k] : soff[r];
            const uint64_t re = k + 1 < w.len ? win[k + 1] : soff[r + 1];
            const uint32_t cnt = static_cast<uint32_t>(min<uint64_t>(nb - b, re - p));
            if (cnt) {
                const uint64_t sp = spos ? spos[r] : (k + 1 < w.len ? rwin[k] : rec_offs[r]) + chars_at;
                put(c, wire + sp + (p - rs), static_cast<int>(b), static_cast<int>(cnt), wire + wire_len);
            }
            b += cnt;
            p += cnt;
            ++r;
        }
        store_slot(chars + p0, c, nb);
    }
}

__global__ __launch_bounds__(kBlock) void k_unpack_var_chars(const uint8_t* __restrict__ wire, uint64_t wire_len,
                                                             const uint64_t* __restrict__ soff,
                                                             const uint64_t* __restrict__ tile_first,
                                                             const uint64_t* __restrict__ spos, uint64_t n,
                                                             uint8_t* __restrict__ chars,
                                                             const uint64_t* __restrict__ rec_offs, uint32_t chars_at,
                                                             const uint32_t* __restrict__ tile_long,
                                                             const uint32_t* __restrict__ bad) {
    __shared__ uint64_t win[kWindow];
    __shared__ uint64_t rwin[kWindow];
    __shared__ __attribute__((aligned(16))) uint8_t slots[kBlock * 32];
    const uint64_t total = soff[n];
    const uint64_t ntiles = (total + kTileBytes - 1) / kTileBytes;
    // bad[0]: some record is not exact (then every tile is copied here)
    const bool skip_short = bad && bad[0] == 0;
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        // three independent scalar loads issued together (no branch between them)
        const uint32_t needed = tile_long[skip_short ? t : 0] | !skip_short;
        const uint64_t r0 = tile_first[t], r1 = tile_first[min(t + 1, ntiles - 1)];
        asm volatile("" ::"s"(r0), "s"(r1));  // keeps the tile_first loads above the branch
        if (!needed) continue;
        chars_tile<false>(wire, wire_len, soff, spos, n, chars, rec_offs, chars_at, t, ntiles, total, r0, r1, win, rwin,
                   slots);
        __syncthreads();
    }
}

// Every string field of a multi-string schema in ONE launch, the fields'
// tiles interleaved (work item u -> field u % nstr, tile u / nstr): tile t of
// every field covers about the same records, so the wire lines one field's
// tile pulls in are still in L2 / Infinity Cache when the other fields'
// tiles read them (separate launches stream the whole wire once per field).
struct CharsFields {
    const uint64_t* soff[kMaxFields];
    const uint64_t* tile_first[kMaxFields];
    const uint64_t* spos[kMaxFields];
    uint8_t* chars[kMaxFields];
    uint32_t nstr;
};

__global__ __launch_bounds__(kBlock) void k_unpack_var_chars_multi(const uint8_t* __restrict__ wire,
                                                                   uint64_t wire_len, CharsFields cf, uint64_t n,
                                                                   uint64_t max_tiles) {
    __shared__ uint64_t win[kWindow];
    __shared__ __attribute__((aligned(16))) uint8_t slots[kBlock * 32];
    uint64_t nt_max = 0;
    for (uint32_t j = 0; j < cf.nstr; ++j)
        nt_max = max(nt_max, min((cf.soff[j][n] + kTileBytes - 1) / kTileBytes, max_tiles));
    const uint64_t items = nt_max * cf.nstr;
    for (uint64_t u = blockIdx.x; u < items; u += gridDim.x) {
        const uint32_t j = static_cast<uint32_t>(u % cf.nstr);
        const uint64_t t = u / cf.nstr;
        const uint64_t* soff = cf.soff[j];
        const uint64_t total = soff[n];
        const uint64_t ntiles = (total + kTileBytes - 1) / kTileBytes;
        if (t >= ntiles) continue;
        const uint64_t r0 = cf.tile_first[j][t], r1 = cf.tile_first[j][min(t + 1, ntiles - 1)];
        chars_tile<true>(wire, wire_len, soff, cf.spos[j], n, cf.chars[j], nullptr, 0u, t, ntiles, total, r0, r1, win,
                   nullptr, slots);
        __syncthreads();
    }
}


// bad: nflags u32 flags, 64 bytes apart.
__global__ void k_reset_status(srpc_unpack_status* st, uint32_t* bad, uint32_t nflags) {
    if (threadIdx.x == 0 && st) {
        st->flags = 0;
        st->reserved = 0;
        st->first_bad_record = ~0ull;
    }
    if (bad)
        for (uint32_t i = threadIdx.x; i < nflags; i += blockDim.x) bad[16 * i] = 0;
}

// The single-string walk's per-call state in one launch (was three: the
// status, the exactness flag and a memset of the long-tile marks, ~4-5 us
// each on the call's critical path), and the error-path scan's look-back
// words (k_unpack_str1_tail).
__global__ void k_reset_walk1(srpc_unpack_status* st, uint32_t* bad, uint32_t* tile_long, uint64_t ntiles,
                              uint64_t* look, uint64_t nlook) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (st) {
            st->flags = 0;
            st->reserved = 0;
            st->first_bad_record = ~0ull;
        }
        bad[0] = 0;
    }
    if (blockIdx.x == 0)
        for (uint32_t i = 1 + threadIdx.x; i < kLongFlags; i += blockDim.x) bad[16 * i] = 0;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < ntiles;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
        tile_long[i] = 0;
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < nlook;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
        look[i] = 0;
}

// ---- record-tile pack: one pass over the inputs -------------------------------------
// k_pack_var_rt: a workgroup owns a tile of 256 consecutive records, one per
// lane, and moves every byte once:
//   1. wave 0 builds the tile's staging table: per string field its offsets
//      window soff[r0 .. r0+nr] and its chars [soff[r0], soff[r0+nr]), per
//      fixed field its column slice; every range is cut into 16-byte aligned
//      granules, numbered one after another;
//   2. the granules go to LDS by LDS-DMA, granule x at stage + 16 x (a granule
//      may hold up to 15 bytes outside its range, never outside the 16-byte
//      block of a valid byte: no fault, never used);
//   3. record r starts at r * fixed_bytes + sum_f (soff[f][r] - soff[f][0])
//      -- every record has fixed_bytes plus its strings' chars -- so the
//      wire offsets come from the staged windows with no scan -> rec_offs;
//   4. each lane writes its record -- prefix, fixed values, u64 lengths,
//      chars -- into an LDS image of the tile's wire span with exact-width
//      LDS stores (every image byte has one writer);
//   5. the image leaves with aligned 16-byte non-temporal stores; the two
//      16-byte blocks the tile shares with its neighbours are written byte
//      by byte (own bytes only).
// A tile whose chars or span do not fit the LDS budget writes its span with
// the chunk walk instead (emit_record, sources read from global memory).
// Reference semantics: pack_arg<std::string> (packer.hpp:193-198), records
// appended back to back (core.hpp:34).
constexpr uint32_t kRtRegions = 2 * kMaxFields;

struct RtRegion {
    uint64_t src;  // 16-aligned global address of the region's first granule
    uint32_t g0;   // its first granule number
    uint32_t dst;  // LDS offset of its first granule
};

struct RtArgs {
    uint32_t pre_at;     // prefix + 32 zero bytes
    uint32_t stage_at;   // staged granules (offsets windows, column slices, chars), stage_cap bytes
    uint32_t img_at;     // image, img_cap bytes
    uint32_t stage_cap, img_cap;
};
constexpr uint64_t kRtImageMin = kBlock * 32;  // the walk's lane slots live in the image
constexpr uint64_t kRtImageMax = 65536;
constexpr uint64_t kRtuMinAvg = 40;  // record-tile unpack: smallest average record (bytes)

typedef const uint8_t __attribute__((address_space(1))) global_u8;
typedef uint8_t __attribute__((address_space(3))) lds_u8;
typedef const uint8_t __attribute__((address_space(3))) lds_u8c;
typedef const u32x4 __attribute__((address_space(3))) lds_u32x4c;

// A workgroup is resident for the whole batch and takes tiles t, t + G, ...
// (G = the grid, sized by the host to what the chip holds at once), software
// pipelined so that its loads and stores overlap instead of following each
// other: the global values of tile t + G's staging table are loaded while tile
// t's stage is awaited, its granules are requested by LDS-DMA right after tile
// t's image stores are issued, and one wait covers both.  The barriers inside
// the loop wait on LDS only (lds_barrier): a __syncthreads() would also wait
// for every store in flight (vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void vm_wait_all() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Per-tile values of the staging table (double-buffered: tile t + G's are
// written while tile t's are read).
struct RtTile {
    uint64_t base;                // wire offset of the tile's first record
    uint32_t fits;                // every region incl. the chars is staged
    uint32_t fsw[kMaxFields];     // string ordinal -> LDS offset of its window entry 0
    uint32_t fch[kMaxFields];     // string ordinal -> LDS offset of char soff[f][r0]
    uint32_t ffx[kMaxFields];     // fixed ordinal -> LDS offset of its value of record r0
};

// Lane g of wave 0 describes region g of every tile: string ordinal g's
// offsets window (g < ns), fixed ordinal g - ns's column slice, string
// ordinal g - ns - nfx's chars.  Resolved once per workgroup: indexing the
// kernel arguments by lane is a chain of dependent vector loads.
struct RtLane {
    uint32_t kind = 0;  // 1 offsets window, 2 chars, 3 fixed column slice
    uint32_t ord = 0;
    uint32_t sz = 0;
    const uint64_t* so = nullptr;
    const uint8_t* col = nullptr;
};
__device__ __forceinline__ RtLane rt_lane(const VarArgs& a, uint32_t g) {
    RtLane r;
    const uint32_t ns = a.nstrings, nfx = a.nfields - a.nstrings;
    if (g < ns) {
        r.kind = 1;
        r.ord = g;
        r.so = a.soff[a.sfield[g]];
    } else if (g < ns + nfx) {
        r.kind = 3;
        r.ord = g - ns;
        const uint32_t f = a.ffield[r.ord];
        r.col = a.col[f];
        r.sz = a.size[f];
    } else if (g < 2 * ns + nfx) {
        r.kind = 2;
        r.ord = g - ns - nfx;
        const uint32_t f = a.sfield[r.ord];
        r.so = a.soff[f];
        r.col = a.col[f];
    }
    return r;
}

// The global values a lane needs for tile t's table: its string's soff[r0]
// and soff[0] (offsets window: the chars before the tile), or soff[r0] and
// soff[r0 + nr] (chars range).  Issued a tile ahead; used after a wait.
struct RtPend {
    uint64_t x0, x1;
};
__device__ __forceinline__ RtPend rt_issue(const RtLane& R, uint64_t n, uint64_t t) {
    RtPend v{0, 0};
    const uint64_t r0 = t * kBlock;
    const uint64_t nr = min<uint64_t>(kBlock, n - r0);
    if (R.kind == 1 || R.kind == 2) {
        v.x0 = R.so[r0];
        v.x1 = R.so[R.kind == 1 ? 0 : r0 + nr];
    }
    return v;
}

// Wave 0, one lane per region: region g's granules land in the stage in
// granule order, granule x at stage_at + 16 x.
__device__ __forceinline__ void rt_table(const RtLane& R, uint64_t fixed_bytes, const RtArgs& L, uint32_t stage_at,
                                         uint64_t n, uint64_t t, uint32_t g, RtPend v, RtTile& T, RtRegion* rt,
                                         uint32_t* s_ngran) {
    const uint64_t r0 = t * kBlock;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(kBlock, n - r0));
    uint64_t lo = 0, hi = 0;
    uint64_t before = 0;  // chars of this string field in the records before the tile
    if (R.kind == 1) {
        lo = reinterpret_cast<uint64_t>(R.so + r0);
        hi = reinterpret_cast<uint64_t>(R.so + r0 + nr + 1);
        before = v.x0 - v.x1;
    } else if (R.kind == 3) {
        lo = reinterpret_cast<uint64_t>(R.col + r0 * R.sz);
        hi = lo + static_cast<uint64_t>(nr) * R.sz;
    } else if (R.kind == 2) {
        lo = reinterpret_cast<uint64_t>(R.col + v.x0);
        hi = reinterpret_cast<uint64_t>(R.col + v.x1);
    }
    // record r starts at r * fixed_bytes + sum over string fields of
    // (soff[r] - soff[0]): the wire offsets need no scan
    const uint64_t chars_before = __shfl(wave_inclusive_scan(before), 63, 64);
    if (g == 0) T.base = r0 * fixed_bytes + chars_before;
    const uint64_t A = lo & ~15ull;
    uint64_t ng = hi > lo ? (hi - A + 15) >> 4 : 0;
    uint64_t inc = wave_inclusive_scan(ng);
    // the chars regions come last: when everything does not fit the stage,
    // the chars are not staged and the tile takes the global walk
    const bool fits = 16 * __shfl(inc, 63, 64) <= L.stage_cap;
    if (!fits) {
        if (R.kind == 2) ng = 0;
        inc = wave_inclusive_scan(ng);
    }
    if (R.kind) {
        const uint32_t g0 = static_cast<uint32_t>(inc - ng);
        rt[g] = {A, g0, 0};
        const uint32_t at = stage_at + 16 * g0 + static_cast<uint32_t>(lo - A);
        if (R.kind == 1) T.fsw[R.ord] = at;
        else if (R.kind == 2) T.fch[R.ord] = at;
        else T.ffx[R.ord] = at;
    }
    if (g == 63) {
        *s_ngran = static_cast<uint32_t>(inc);
        T.fits = fits;
    }
}

// Granules -> stage by LDS-DMA (global_load_lds_dwordx4: a wave instruction
// fills 1 KiB of LDS lane-linearly, no VGPRs hold the data, nothing waits
// here); a lane's granules increase, so its region index only moves forward.
__device__ __forceinline__ void rt_dma(uint32_t stage_at, uint32_t nreg, uint32_t ngran, const RtRegion* rt,
                                       uint8_t* lds) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t r = 0;
    for (uint32_t w0 = threadIdx.x & ~63u; w0 < ngran; w0 += kBlock) {
        const uint32_t gi = w0 + lane;
        if (gi < ngran) {
            while (r + 1 < nreg && rt[r + 1].g0 <= gi) ++r;
            const uint64_t src = rt[r].src + 16ull * (gi - rt[r].g0);
            const uint32_t wb = __builtin_amdgcn_readfirstlane(w0);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<global_u8*>(src),
                                             (lds_u8*)(lds + stage_at + 16 * wb), 16, 0, 0);
        }
    }
}

__global__ __launch_bounds__(kBlock) void k_pack_var_rt_loop(VarArgs a, RtArgs L, uint64_t n, uint8_t* __restrict__ wire,
                                                        uint64_t wire_cap, uint64_t* __restrict__ rec_offs,
                                                        srpc_unpack_status* st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ RtRegion rt[kRtRegions];
    __shared__ RtTile tl[2];
    __shared__ uint64_t lofs[kBlock + 1];     // local record starts (image positions minus h), [nr] = total
    __shared__ uint64_t climit[kMaxFields];   // string field: soff[f][n] (end of its chars)
    __shared__ uint32_t s_ngran;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ns = a.nstrings, nreg = 2 * ns + (a.nfields - a.nstrings);
    const uint64_t ntiles = (n + kBlock - 1) / kBlock;
    uint64_t t = blockIdx.x;
    // prefix + 32 zero bytes (emit_record reads 16 bytes at any prefix offset)
    for (uint32_t i = threadIdx.x; i < a.prefix_len + 32; i += kBlock)
        lds[L.pre_at + i] = i < a.prefix_len ? a.prefix[i] : 0;
    for (uint32_t f = threadIdx.x; f < a.nfields; f += kBlock) climit[f] = a.size[f] ? 0 : a.soff[f][n];
    RtLane R;
    if (threadIdx.x < 64) {
        R = rt_lane(a, lane);
        rt_table(R, a.fixed_bytes, L, L.stage_at, n, t, lane, rt_issue(R, n, t), tl[0], rt, &s_ngran);
    }
    __syncthreads();
    rt_dma(L.stage_at, nreg, s_ngran, rt, lds);
    for (uint32_t b = 0; t < ntiles; t += gridDim.x, b ^= 1) {
        const uint64_t tn = t + gridDim.x;
        const bool more = tn < ntiles;
        RtPend pend{0, 0};
        if (more && threadIdx.x < 64) pend = rt_issue(R, n, tn);
        vm_wait_all();  // this tile's granules (and the last tile's stores)
        lds_barrier();
        if (more && threadIdx.x < 64)
            rt_table(R, a.fixed_bytes, L, L.stage_at, n, tn, lane, pend, tl[b ^ 1], rt, &s_ngran);
        const RtTile& T = tl[b];
        const uint64_t r0 = t * kBlock;
        const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(kBlock, n - r0));
        // record starts from the staged offsets windows
        const uint32_t i = threadIdx.x;
        if (i < nr) {
            uint64_t e = static_cast<uint64_t>(i + 1) * a.fixed_bytes;
            for (uint32_t si = 0; si < ns; ++si) {
                const uint64_t* w = reinterpret_cast<const uint64_t*>(lds + T.fsw[si]);
                e += w[i + 1] - w[0];
            }
            lofs[i + 1] = e;
        }
        if (i == 0) lofs[0] = 0;
        lds_barrier();
        const uint64_t base = T.base, total = lofs[nr];
        if (i < nr) {
            const uint64_t start = base + lofs[i], end = base + lofs[i + 1];
            rec_offs[r0 + i] = start;
            if (st && start <= wire_cap && wire_cap < end) report_bad(st, SRPC_STATUS_BOUNDS, r0 + i);
        }
        if (i == 0 && r0 + nr == n) rec_offs[n] = base + total;
        const uint32_t h = static_cast<uint32_t>(base & 15);
        const uint64_t gbase = base & ~15ull;
        const uint64_t wend = min(base + total, wire_cap);  // wire bytes of this tile end here
        uint8_t* img = lds + L.img_at;
        if (T.fits && h + total <= L.img_cap) {
            // records -> LDS image
            if (i < nr) {
                uint32_t d = L.img_at + h + static_cast<uint32_t>(lofs[i]);
                if (a.prefix_len) {
                    lds_copy_run(lds, d, L.pre_at, a.prefix_len);
                    d += a.prefix_len;
                }
                uint32_t si = 0, fi = 0;
                for (uint32_t f = 0; f < a.nfields; ++f) {
                    const uint32_t sz = a.size[f];
                    if (sz) {
                        const uint8_t* v = lds + T.ffx[fi++] + i * sz;
                        const uint64_t x = sz == 1   ? *v
                                           : sz == 2 ? load_unaligned<uint16_t>(v)
                                           : sz == 4 ? load_unaligned<uint32_t>(v)
                                                     : load_unaligned<uint64_t>(v);
                        lds_put_small(lds, d, x, sz);
                        d += sz;
                        continue;
                    }
                    const uint64_t* w = reinterpret_cast<const uint64_t*>(lds + T.fsw[si]);
                    const uint64_t c0 = w[0], cb = w[i], len = w[i + 1] - cb;
                    lds_put_small(lds, d, len, 8);
                    d += 8;
                    lds_copy_run(lds, d, T.fch[si] + static_cast<uint32_t>(cb - c0), static_cast<uint32_t>(len));
                    d += static_cast<uint32_t>(len);
                    ++si;
                }
            }
            lds_barrier();  // image complete; the stage is free for the next tile
            // image -> wire
            const uint32_t span = h + static_cast<uint32_t>(total);
            const uint32_t nch = (span + 15) >> 4;
            for (uint32_t c = threadIdx.x; c < nch; c += kBlock) {
                const uint64_t g = gbase + 16ull * c;
                const uint32_t lo = max(h, 16 * c), hi = min(span, 16 * c + 16);
                if (lo == 16 * c && hi == 16 * c + 16 && g + 16 <= wire_cap) {
                    const u64x2 v = *reinterpret_cast<const u64x2*>(img + 16 * c);
                    __builtin_nontemporal_store(v, reinterpret_cast<u64x2*>(wire + g));
                } else {
                    for (uint32_t x = lo; x < hi && gbase + x < wend; ++x) wire[gbase + x] = img[x];
                }
            }
        } else {
            // span or chars too large for LDS: chunk walk over [base, base + total)
            // with global sources; the image region holds the lanes' 32-byte slots
            uint32_t f0 = 0;
            while (a.size[f0]) ++f0;
            Slot c{img + 32 * threadIdx.x};
            for (uint64_t p0 = gbase + 16ull * threadIdx.x; p0 < wend; p0 += 16ull * kBlock) {
                const uint64_t lo = max(p0, base), hi = min(p0 + 16, wend);
                if (lo >= hi) continue;
                // last record whose start <= lo (records may be empty)
                uint32_t k0 = 0, k1 = nr;  // lofs[k0] + base <= lo < lofs[k1] + base
                while (k1 - k0 > 1) {
                    const uint32_t mid = (k0 + k1) >> 1;
                    if (base + lofs[mid] <= lo) k0 = mid;
                    else k1 = mid;
                }
                uint64_t p = lo;
                uint32_t b2 = static_cast<uint32_t>(lo - p0);
                for (uint32_t k = k0; p < hi && k < nr; ++k) {
                    const uint64_t rs = base + lofs[k], re = base + lofs[k + 1];
                    if (re <= p) continue;
                    const uint32_t cnt = static_cast<uint32_t>(min(hi, re) - p);
                    emit_record(a, lds + L.pre_at, climit, f0, nullptr, n, r0 + k, p - rs, cnt, static_cast<int>(b2), c);
                    b2 += cnt;
                    p += cnt;
                }
                if (lo == p0 && hi == p0 + 16) {
                    store_slot(wire + p0, c, 16);
                } else {
                    for (uint64_t x = lo; x < hi; ++x) wire[x] = c.s[x - p0];
                }
            }
        }
        if (more) rt_dma(L.stage_at, nreg, s_ngran, rt, lds);
    }
}

// One tile of kBlock * RPL records per workgroup (records under kRtPersistMin
// bytes on average: the loop kernel's per-tile barriers and wider register
// state cost more than its overlap saves on 4-8 KiB tiles,
// profiles/r02_var_rt_persist_ab.log); lane i owns records i, i + kBlock, ...
// -- RPL > 1 makes a short-record tile as large as a long-record one.
template <int RPL>
__global__ __launch_bounds__(kBlock) void k_pack_var_rt(VarArgs a, RtArgs L, uint64_t n, uint8_t* __restrict__ wire,
                                                        uint64_t wire_cap, uint64_t* __restrict__ rec_offs,
                                                        srpc_unpack_status* st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ RtRegion rt[kRtRegions];
    constexpr uint32_t kTR = kBlock * RPL;   // records per tile
    __shared__ uint64_t lofs[kTR + 1];        // local record starts (image positions minus h), [nr] = total
    __shared__ uint64_t climit[kMaxFields];   // string field: soff[f][n] (end of its chars)
    __shared__ uint32_t fsw[kMaxFields];      // string ordinal -> LDS offset of its window entry 0
    __shared__ uint32_t fch[kMaxFields];      // string ordinal -> LDS offset of char soff[f][r0]
    __shared__ uint32_t ffx[kMaxFields];      // fixed ordinal -> LDS offset of its value of record r0
    __shared__ uint64_t s_base;
    __shared__ uint32_t s_ngran, s_fits;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t ns = a.nstrings, nfx = a.nfields - a.nstrings;
    // prefix + 32 zero bytes (emit_record reads 16 bytes at any prefix offset)
    for (uint32_t i = threadIdx.x; i < a.prefix_len + 32; i += kBlock)
        lds[L.pre_at + i] = i < a.prefix_len ? a.prefix[i] : 0;
    for (uint32_t f = threadIdx.x; f < a.nfields; f += kBlock) climit[f] = a.size[f] ? 0 : a.soff[f][n];
    const uint64_t r0 = static_cast<uint64_t>(blockIdx.x) * kTR;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(kTR, n - r0));
    // 1. staging table (wave 0, one lane per region): region g's granules
    // land in the stage in granule order, granule x at stage_at + 16 x
    if (threadIdx.x < 64) {
        const uint32_t g = lane;
        uint64_t lo = 0, hi = 0;
        uint32_t kind = 0;  // 1 offsets window, 2 chars, 3 fixed column slice
        uint32_t ord = 0;
        uint64_t before = 0;  // chars of this string field in the records before the tile
        if (g < ns) {
            kind = 1;
            ord = g;
            const uint64_t* so = a.soff[a.sfield[g]];
            lo = reinterpret_cast<uint64_t>(so + r0);
            hi = reinterpret_cast<uint64_t>(so + r0 + nr + 1);
            before = so[r0] - so[0];
        } else if (g < ns + nfx) {
            kind = 3;
            ord = g - ns;
            const uint32_t f = a.ffield[ord];
            lo = reinterpret_cast<uint64_t>(a.col[f] + r0 * a.size[f]);
            hi = lo + static_cast<uint64_t>(nr) * a.size[f];
        } else if (g < 2 * ns + nfx) {
            kind = 2;
            ord = g - ns - nfx;
            const uint32_t f = a.sfield[ord];
            const uint64_t* so = a.soff[f];
            lo = reinterpret_cast<uint64_t>(a.col[f] + so[r0]);
            hi = reinterpret_cast<uint64_t>(a.col[f] + so[r0 + nr]);
        }
        // record r starts at r * fixed_bytes + sum over string fields of
        // (soff[r] - soff[0]): the wire offsets need no scan
        const uint64_t chars_before = __shfl(wave_inclusive_scan(before), 63, 64);
        if (g == 0) s_base = r0 * a.fixed_bytes + chars_before;
        const uint64_t A = lo & ~15ull;
        uint64_t ng = hi > lo ? (hi - A + 15) >> 4 : 0;
        uint64_t inc = wave_inclusive_scan(ng);
        // the chars regions come last: when everything does not fit the stage,
        // the chars are not staged and the tile takes the global walk
        const bool fits = 16 * __shfl(inc, 63, 64) <= L.stage_cap;
        if (!fits) {
            if (kind == 2) ng = 0;
            inc = wave_inclusive_scan(ng);
        }
        if (kind) {
            const uint32_t g0 = static_cast<uint32_t>(inc - ng);
            rt[g] = {A, g0, 0};
            const uint32_t at = L.stage_at + 16 * g0 + static_cast<uint32_t>(lo - A);
            if (kind == 1) fsw[ord] = at;
            else if (kind == 2) fch[ord] = at;
            else ffx[ord] = at;
        }
        if (g == 63) {
            s_ngran = static_cast<uint32_t>(inc);
            s_fits = fits;
        }
    }
    __syncthreads();
    // 2. granules -> stage by LDS-DMA (global_load_lds_dwordx4: a wave
    // instruction fills 1 KiB of LDS lane-linearly, no VGPRs hold the data,
    // nothing waits until the barrier); a lane's granules increase, so its
    // region index only moves forward
    {
        const uint32_t ngran = s_ngran, nreg = 2 * ns + nfx;
        uint32_t r = 0;
        for (uint32_t w0 = threadIdx.x & ~63u; w0 < ngran; w0 += kBlock) {
            const uint32_t gi = w0 + lane;
            if (gi < ngran) {
                while (r + 1 < nreg && rt[r + 1].g0 <= gi) ++r;
                const uint64_t src = rt[r].src + 16ull * (gi - rt[r].g0);
                const uint32_t wb = __builtin_amdgcn_readfirstlane(w0);
                __builtin_amdgcn_global_load_lds(reinterpret_cast<global_u8*>(src),
                                                 (lds_u8*)(lds + L.stage_at + 16 * wb), 16, 0, 0);
            }
        }
    }
    __syncthreads();  // waits for the LDS-DMA (vmcnt(0)) and publishes the stage
    // 3. record starts from the staged offsets windows
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const uint32_t i = threadIdx.x + q * kBlock;
        if (i < nr) {
            uint64_t e = static_cast<uint64_t>(i + 1) * a.fixed_bytes;
            for (uint32_t si = 0; si < ns; ++si) {
                const uint64_t* w = reinterpret_cast<const uint64_t*>(lds + fsw[si]);
                e += w[i + 1] - w[0];
            }
            lofs[i + 1] = e;
        }
    }
    if (threadIdx.x == 0) lofs[0] = 0;
    __syncthreads();
    const uint64_t base = s_base, total = lofs[nr];
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const uint32_t i = threadIdx.x + q * kBlock;
        if (i < nr) {
            const uint64_t start = base + lofs[i], end = base + lofs[i + 1];
            rec_offs[r0 + i] = start;
            if (st && start <= wire_cap && wire_cap < end) report_bad(st, SRPC_STATUS_BOUNDS, r0 + i);
        }
    }
    if (threadIdx.x == 0 && r0 + nr == n) rec_offs[n] = base + total;
    const uint32_t h = static_cast<uint32_t>(base & 15);
    const uint64_t gbase = base & ~15ull;
    const uint64_t wend = min(base + total, wire_cap);  // wire bytes of this tile end here
    uint8_t* img = lds + L.img_at;
    if (s_fits && h + total <= L.img_cap) {
        // 4. records -> LDS image
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const uint32_t i = threadIdx.x + q * kBlock;
            if (i >= nr) break;
            uint32_t d = L.img_at + h + static_cast<uint32_t>(lofs[i]);
            if (a.prefix_len) {
                lds_copy_run(lds, d, L.pre_at, a.prefix_len);
                d += a.prefix_len;
            }
            uint32_t si = 0, fi = 0;
            for (uint32_t f = 0; f < a.nfields; ++f) {
                const uint32_t sz = a.size[f];
                if (sz) {
                    const uint8_t* v = lds + ffx[fi++] + i * sz;
                    const uint64_t x = sz == 1   ? *v
                                       : sz == 2 ? load_unaligned<uint16_t>(v)
                                       : sz == 4 ? load_unaligned<uint32_t>(v)
                                                 : load_unaligned<uint64_t>(v);
                    lds_put_small(lds, d, x, sz);
                    d += sz;
                    continue;
                }
                const uint64_t* w = reinterpret_cast<const uint64_t*>(lds + fsw[si]);
                const uint64_t c0 = w[0], cb = w[i], len = w[i + 1] - cb;
                lds_put_small(lds, d, len, 8);
                d += 8;
                lds_copy_run(lds, d, fch[si] + static_cast<uint32_t>(cb - c0), static_cast<uint32_t>(len));
                d += static_cast<uint32_t>(len);
                ++si;
            }
        }
        __syncthreads();
        // 5. image -> wire
        const uint32_t span = h + static_cast<uint32_t>(total);
        const uint32_t nch = (span + 15) >> 4;
        for (uint32_t c = threadIdx.x; c < nch; c += kBlock) {
            const uint64_t g = gbase + 16ull * c;
            const uint32_t lo = max(h, 16 * c), hi = min(span, 16 * c + 16);
            if (lo == 16 * c && hi == 16 * c + 16 && g + 16 <= wire_cap) {
                const u64x2 v = *reinterpret_cast<const u64x2*>(img + 16 * c);
                __builtin_nontemporal_store(v, reinterpret_cast<u64x2*>(wire + g));
            } else {
                for (uint32_t x = lo; x < hi && gbase + x < wend; ++x) wire[gbase + x] = img[x];
            }
        }
        return;
    }
    // 4'. span or chars too large for LDS: chunk walk over [base, base + total)
    // with global sources; the image region holds the lanes' 32-byte slots
    uint32_t f0 = 0;
    while (a.size[f0]) ++f0;
    Slot c{img + 32 * threadIdx.x};
    for (uint64_t p0 = gbase + 16ull * threadIdx.x; p0 < wend; p0 += 16ull * kBlock) {
        const uint64_t lo = max(p0, base), hi = min(p0 + 16, wend);
        if (lo >= hi) continue;
        // last record whose start <= lo (records may be empty)
        uint32_t k0 = 0, k1 = nr;  // lofs[k0] + base <= lo < lofs[k1] + base
        while (k1 - k0 > 1) {
            const uint32_t mid = (k0 + k1) >> 1;
            if (base + lofs[mid] <= lo) k0 = mid;
            else k1 = mid;
        }
        uint64_t p = lo;
        uint32_t b = static_cast<uint32_t>(lo - p0);
        for (uint32_t k = k0; p < hi && k < nr; ++k) {
            const uint64_t rs = base + lofs[k], re = base + lofs[k + 1];
            if (re <= p) continue;
            const uint32_t cnt = static_cast<uint32_t>(min(hi, re) - p);
            emit_record(a, lds + L.pre_at, climit, f0, nullptr, n, r0 + k, p - rs, cnt, static_cast<int>(b), c);
            b += cnt;
            p += cnt;
        }
        if (lo == p0 && hi == p0 + 16) {
            store_slot(wire + p0, c, 16);
        } else {
            for (uint64_t x = lo; x < hi; ++x) wire[x] = c.s[x - p0];
        }
    }
}

// ---- record-tile unpack: one pass over the wire --------------------------------------
// k_unpack_var_rt: a workgroup owns 256 consecutive records of the index, one
// per lane:
//   1. the tile's index window rec_offs[r0 .. r0+nr] and its wire span
//      [rec_offs[r0], rec_offs[r0+nr]) go to LDS by LDS-DMA (16-byte
//      granules, as in k_pack_var_rt);
//   2. each lane parses its record from the stage (or from global memory when
//      the record lies outside the staged span: a non-monotonic index, or a
//      span too large to stage) with the general error semantics of
//      walk_record: prefix check, fixed fields straight to their columns
//      (coalesced: lane i writes element r0 + i), every string's length
//      checked against the record end BEFORE it is used (the reference reads
//      first: core.hpp:29-31), a BOUNDS record's strings decoded as empty;
//   3. per string field, a workgroup scan of the lengths gives the chars'
//      offsets inside the tile, and a decoupled look-back over the tiles'
//      published chars totals (tile ids from an atomic ticket: every earlier
//      tile is running and publishes before it looks back) gives the tile's
//      base -> str_offs;
//   4. per string field, the lanes copy their chars into an LDS image of the
//      field's output range, which leaves with aligned 16-byte stores (the
//      two blocks shared with the neighbouring tiles byte by byte).
// Reference semantics: pipe_output<T> / pipe_output<std::string>
// (packer.hpp:210-222) over records appended back to back (core.hpp:34).
constexpr uint64_t kLookAgg = 1ull << 62, kLookIncl = 2ull << 62, kLookVal = (1ull << 62) - 1;
#ifndef SRPC_RTU_TICKET
#define SRPC_RTU_TICKET 0
#endif
#ifndef SRPC_RTU_NOLOOK
#define SRPC_RTU_NOLOOK 0
#endif
#ifndef SRPC_RTU_NOCHARS
#define SRPC_RTU_NOCHARS 0
#endif
// Spin budget of one look-back wait (s_sleep 1 per round, ~0.1 s in all):
// past it the tile gives up, sets SRPC_STATUS_STALLED and uses what it has --
// a wrong result that is reported, never a hung GPU.
constexpr uint32_t kLookSpinMax = 1u << 21;
// the budget in force (a test hook lowers it to force the STALLED report)
__device__ uint32_t g_look_spin_max = kLookSpinMax;

__device__ __forceinline__ uint64_t look_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void look_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Two-level decoupled look-back (wave 0).  look1[t] holds tile t's value
// (AGG: its own total; INCL: the inclusive prefix); look2[b] the same for
// blocks of 64 tiles (AGG: the block's total, published by the block's last
// tile once every tile of the block published its AGG; INCL: the inclusive
// prefix at the block's end).  Tile t sums its own block's earlier tiles
// (one round of loads), then whole blocks, 64 per round.  A flat look-back
// walked back 64 tiles per round until it met an INCL and took 25 us per
// tile at 2,048 tiles in flight (agent-scope loads pay the Infinity-Cache
// latency on MI355X, profiles/r02_var_rtu_ab.log); blocks cut that to about
// two rounds.  Values of one string field, `stride` words apart per tile.
__device__ __forceinline__ uint64_t look_back2(uint64_t* look1, uint64_t* look2, uint64_t t, uint32_t stride,
                                               uint64_t total, bool* stalled) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t q = static_cast<uint32_t>(t & 63);
    const uint64_t blk = t >> 6;
    uint64_t pre = 0;
    bool done = false;
    uint32_t spins = 0;
    const uint32_t spin_max = g_look_spin_max;
    // 1. earlier tiles of the own block, nearest INCL first
    if (q) {
        while (true) {
            const uint64_t v = lane < q ? look_load(look1 + ((blk << 6) + lane) * stride) : kLookAgg;
            const uint64_t incl = __ballot(lane < q && v >= kLookIncl);
            const uint32_t from = incl ? 63 - __builtin_clzll(incl) : 0;  // highest INCL lane, or 0
            const uint64_t wait = __ballot(lane < q && lane >= from && v < kLookAgg);
            if (wait && ++spins < spin_max) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            if (wait) *stalled = true;
            const uint64_t part = (lane < q && lane >= from) ? (v & kLookVal) : 0;
            pre = __shfl(wave_inclusive_scan(part), 63, 64);
            done = incl != 0;
            break;
        }
    } else {
        done = blk == 0;
    }
    if (q == 63 && lane == 0)  // the block's total (or already its inclusive prefix)
        look_store(look2 + blk * stride, (done ? kLookIncl : kLookAgg) | ((pre + total) & kLookVal));
    // 2. whole blocks before the own block, 64 per round
    int64_t j = static_cast<int64_t>(blk) - 1;
    while (!done && j >= 0) {
        const int64_t idx = j - static_cast<int64_t>(lane);
        const uint64_t v = idx >= 0 ? look_load(look2 + static_cast<uint64_t>(idx) * stride) : kLookIncl;
        const uint64_t incl = __ballot(v >= kLookIncl);
        const uint64_t wait = __ballot(v < kLookAgg);
        const uint32_t first = incl ? __builtin_ctzll(incl) : 64;
        const uint64_t upto = first >= 63 ? ~0ull : (2ull << first) - 1;
        if ((wait & upto) && ++spins < spin_max) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        if (wait & upto) *stalled = true;
        const uint64_t part = lane <= first ? (v & kLookVal) : 0;
        pre += __shfl(wave_inclusive_scan(part), 63, 64);
        if (first < 64) break;
        j -= 64;
    }
    if (lane == 0) {
        look_store(look1 + t * stride, kLookIncl | ((pre + total) & kLookVal));
        if (q == 63 && !done) look_store(look2 + blk * stride, kLookIncl | ((pre + total) & kLookVal));
    }
    return pre;
}

// The gated error-path scan in ONE launch (was reduce + partials + apply,
// three launches of ~3.7 us each even as no-ops on an exact batch): out[i] =
// exclusive prefix of f over [0, i), out[n] = total, tile metadata as
// k_scan_apply's.  Scan block b = ticket order (look[0]), its base by the
// decoupled look-back over the blocks' totals (look + 1, look2); a bounded
// grid takes tickets until the blocks run out (a block waits only on lower
// tickets, taken by running workgroups that wait on nothing later).
template <class F>
__global__ __launch_bounds__(kBlock) void k_scan1(F f, uint64_t n, uint64_t* out, uint64_t* tile_first,
                                                  uint64_t max_tiles, const uint32_t* gate, uint64_t* look,
                                                  uint64_t* look2, srpc_unpack_status* st) {
    if (*gate == 0) return;
    __shared__ uint64_t v[kScanBlock];
    __shared__ uint64_t s_bx, s_pre;
    const uint64_t nb = (n + kScanBlock - 1) / kScanBlock;
    for (;;) {
        if (threadIdx.x == 0) s_bx = atomicAdd(reinterpret_cast<unsigned long long*>(look), 1ull);
        __syncthreads();
        const uint64_t bx = s_bx;
        if (bx >= nb) break;
        const uint64_t base = bx * kScanBlock;
#pragma unroll
        for (int j = 0; j < kScanItems; ++j) {
            const uint32_t k = j * kBlock + threadIdx.x;
            v[k] = (base + k < n) ? f(base + k) : 0;
        }
        __syncthreads();
        uint64_t loc[kScanItems];
        uint64_t sum = 0;
#pragma unroll
        for (int j = 0; j < kScanItems; ++j) {
            loc[j] = sum;
            sum += v[threadIdx.x * kScanItems + j];
        }
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(sum, &tot);
        if (threadIdx.x < 64) {
            bool stalled = false;
            const uint64_t pre = look_back2(look + 1, look2, bx, 1, tot, &stalled);
            if (threadIdx.x == 0) {
                s_pre = pre;
                if (stalled && st) report_bad(st, SRPC_STATUS_STALLED, base);
            }
        }
        __syncthreads();
        const uint64_t pre = s_pre + ex;
#pragma unroll
        for (int j = 0; j < kScanItems; ++j) {
            const uint32_t k = threadIdx.x * kScanItems + j;
            const uint64_t start = pre + loc[j], end = start + v[k];
            for (uint64_t t = (start + kTileBytes - 1) / kTileBytes; t * kTileBytes < end && t < max_tiles; ++t)
                tile_first[t] = base + k;
            v[k] = start;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kScanItems; ++j) {
            const uint32_t k = j * kBlock + threadIdx.x;
            if (base + k < n) out[base + k] = v[k];
        }
        if (bx == nb - 1 && threadIdx.x == 0) out[n] = s_pre + tot;
        __syncthreads();  // (v and s_bx are rewritten by the next block)
    }
}

// The single-string walk's tail in ONE gated launch (was the error path's
// reduce + partials + apply and the chars kernel: four launches of ~3.7 us
// each, no-ops on an exact batch of short strings):
// - bad[0] (some record is not exact): str_offs[i] = exclusive prefix of the
//   decoded lengths (SingleStrLen), str_offs[n] = total, and every record's
//   chars copied by its lane.  Scan block b = ticket order (look[0]), its
//   base by the decoupled look-back over the blocks' totals (look + 1,
//   look2); the grid takes tickets until the blocks run out (a block waits
//   only on lower tickets, taken by running workgroups that wait on nothing
//   later);
// - else one of the long flags bad[16 k] (a wave left long strings): the
//   chars tiles it marked (tile_long), as k_unpack_var_chars;
// - else nothing.
__global__ __launch_bounds__(kBlock) void k_unpack_str1_tail(SingleStrLen f, uint64_t n, uint64_t* soff,
                                                             uint8_t* __restrict__ chars, uint32_t chars_at,
                                                             const uint64_t* __restrict__ tiles,
                                                             const uint32_t* __restrict__ tile_long,
                                                             const uint32_t* bad, uint64_t* look, uint64_t* look2,
                                                             srpc_unpack_status* st) {
    const bool dirty = bad[0] != 0;
    const bool lng = threadIdx.x >= 1 && threadIdx.x < kLongFlags && bad[16 * threadIdx.x] != 0;
    if (!__syncthreads_or(dirty || lng)) return;
    // one LDS region: the chars tiles' windows and slots, or the scan block
    // (members of one __shared__ object, so every access stays an LDS one)
    __shared__ union {
        struct {
            uint64_t win[kWindow];
            uint64_t rwin[kWindow];
            __attribute__((aligned(16))) uint8_t slots[kBlock * 32];
        } c;
        uint64_t v[kScanBlock];
    } U;
    if (!dirty) {
        const uint64_t total = soff[n];
        const uint64_t ntiles = (total + kTileBytes - 1) / kTileBytes;
        for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
            const uint32_t needed = tile_long[t];
            const uint64_t r0 = tiles[t], r1 = tiles[min(t + 1, ntiles - 1)];
            asm volatile("" ::"s"(r0), "s"(r1));  // keeps the tile_first loads above the branch
            if (!needed) continue;
            chars_tile<false>(f.wire, f.wire_len, soff, nullptr, n, chars, f.rec, chars_at, t, ntiles, total, r0, r1,
                              U.c.win, U.c.rwin, U.c.slots);
            __syncthreads();
        }
        return;
    }
    uint64_t* v = U.v;  // the scan block's values
    __shared__ uint64_t s_bx, s_pre;
    const uint64_t nb = (n + kScanBlock - 1) / kScanBlock;
    for (;;) {
        if (threadIdx.x == 0) s_bx = atomicAdd(reinterpret_cast<unsigned long long*>(look), 1ull);
        __syncthreads();
        const uint64_t bx = s_bx;
        if (bx >= nb) break;
        const uint64_t base = bx * kScanBlock;
#pragma unroll 2
        for (int j = 0; j < kScanItems; ++j) {
            const uint32_t k = j * kBlock + threadIdx.x;
            v[k] = (base + k < n) ? f(base + k) : 0;
        }
        __syncthreads();
        uint64_t sum = 0;
#pragma unroll
        for (int j = 0; j < kScanItems; ++j) sum += v[threadIdx.x * kScanItems + j];
        uint64_t tot;
        const uint64_t ex = block_exclusive_scan(sum, &tot);
        if (threadIdx.x < 64) {
            bool stalled = false;
            const uint64_t pre = look_back2(look + 1, look2, bx, 1, tot, &stalled);
            if (threadIdx.x == 0) {
                s_pre = pre;
                if (stalled && st) report_bad(st, SRPC_STATUS_STALLED, base);
            }
        }
        __syncthreads();
        uint64_t run = s_pre + ex;  // this thread's items' offsets, from the lengths still in v
        const uint8_t* wend = f.wire + f.wire_len;
#pragma unroll 1
        for (int j = 0; j < kScanItems; ++j) {
            const uint32_t k = threadIdx.x * kScanItems + j;
            const uint64_t len = v[k];
            if (len) copy_short(chars + run, f.wire + f.rec[base + k] + chars_at, static_cast<uint32_t>(len), wend);
            v[k] = run;
            run += len;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kScanItems; ++j) {
            const uint32_t k = j * kBlock + threadIdx.x;
            if (base + k < n) soff[base + k] = v[k];
        }
        if (bx == nb - 1 && threadIdx.x == 0) soff[n] = s_pre + tot;
        __syncthreads();  // (v and s_bx are rewritten by the next block)
    }
}

struct RtuArgs {
    uint32_t pre_at;     // prefix + 16 bytes
    uint32_t stage_at;   // the wire span's granules (stage_cap bytes)
    uint32_t len_at;     // per string ordinal: 256 u64 lengths, then offsets inside the tile's chars
    uint32_t img_at;     // chars image, img_cap bytes
    uint32_t stage_cap, img_cap;
};

// len bytes from the LDS stage at byte offset so to global memory at d: byte
// stores up to a 4-byte boundary of d, dwords up to a 16-byte one, 16-byte
// stores, then dwords and bytes (the stage reads are aligned dwords funnel-
// shifted; the stage has a dword of slack past any run).
__device__ __forceinline__ void copy_stage_run(uint8_t* d, const uint8_t* lds, uint32_t so, uint32_t len) {
    const lds_u8c* l8 = (const lds_u8c*)lds;
    const uint32_t head = min<uint32_t>(len, (4 - (reinterpret_cast<uintptr_t>(d) & 3)) & 3);
    uint32_t i = 0;
#pragma nounroll
    for (; i < head; ++i) d[i] = l8[so + i];
    typedef const uint32_t __attribute__((address_space(3))) lds_u32c;
    const uint32_t sa = (so + i) & 3;
    lds_u32c* sw = reinterpret_cast<lds_u32c*>(l8 + ((so + i) & ~3u));
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
    for (i += 4 * nd; i < len; ++i) d[i] = l8[so + i];
}

// General decode of record r (walk_record's multi-string semantics); string
// ordinal si's length goes to len_l[si * 256 + lane] (its chars position is
// found again by string_pos when the chars are copied).
template <typename Pre>
__device__ __forceinline__ uint32_t parse_record(const VarArgs& a, const uint8_t* src, const Pre* pre, uint64_t r,
                                                 uint64_t start, uint64_t end, uint64_t wire_len, uint64_t* len_l,
                                                 uint32_t i) {
    uint32_t flag = 0;
    if (start > end || end > wire_len || end - start < a.fixed_bytes) flag = SRPC_STATUS_BOUNDS;
    if (!flag) {
        uint32_t k = 0;
        for (; k + 8 <= a.prefix_len; k += 8)
            if (load_unaligned<uint64_t>(src + k) != load_unaligned<uint64_t>(pre + k)) flag = SRPC_STATUS_PREFIX;
        for (; k < a.prefix_len; ++k)
            if (src[k] != pre[k]) flag = SRPC_STATUS_PREFIX;
    }
    uint64_t pos = start + a.prefix_len;
    uint32_t si = 0;
    for (uint32_t f = 0; f < a.nfields; ++f) {
        const uint32_t sz = a.size[f];
        if (sz) {
            if (flag != SRPC_STATUS_BOUNDS && pos + sz <= end) {
                uint8_t* dst = const_cast<uint8_t*>(a.col[f]) + r * sz;
                const uint8_t* q = src + (pos - start);
                switch (sz) {
                case 1: dst[0] = q[0]; break;
                case 2: *reinterpret_cast<uint16_t*>(dst) = load_unaligned<uint16_t>(q); break;
                case 4: *reinterpret_cast<uint32_t*>(dst) = load_unaligned<uint32_t>(q); break;
                default: *reinterpret_cast<uint64_t*>(dst) = load_unaligned<uint64_t>(q); break;
                }
            }
            pos += sz;
            continue;
        }
        uint64_t len = 0;
        if (flag != SRPC_STATUS_BOUNDS && pos + 8 <= end) {
            len = load_unaligned<uint64_t>(src + (pos - start));
            pos += 8;
            if (len > end - pos) {
                flag = SRPC_STATUS_BOUNDS;
                len = 0;
            }
        } else {
            flag = SRPC_STATUS_BOUNDS;
        }
        len_l[si * kBlock + i] = len;
        ++si;
        pos += len;
    }
    if (!flag && pos != end) flag = SRPC_STATUS_BOUNDS;  // record size disagrees with the index
    if (flag == SRPC_STATUS_BOUNDS)
        for (uint32_t k = 0; k < a.nstrings; ++k) len_l[k * kBlock + i] = 0;
    return flag;
}

// Wire offset of string ordinal si's chars in a record that decoded without a
// BOUNDS error (every length fits the record), walking its fields again;
// rd(p) reads the u64 at wire offset p (the LDS stage or global memory).
template <class Rd>
__device__ __forceinline__ uint64_t string_pos(const VarArgs& a, uint64_t start, uint32_t si, Rd rd) {
    uint64_t pos = start + a.prefix_len;
    uint32_t k = 0;
    for (uint32_t f = 0; f < a.nfields; ++f) {
        const uint32_t sz = a.size[f];
        if (sz) {
            pos += sz;
            continue;
        }
        const uint64_t len = rd(pos);
        pos += 8;
        if (k++ == si) break;
        pos += len;
    }
    return pos;
}

// parse_record for a record staged in LDS at byte offset `so` (wire offset
// `start`), the prefix at LDS offset `po` (16-aligned): every read is aligned.
__device__ __forceinline__ uint32_t parse_record_lds(const VarArgs& a, const uint8_t* lds, uint32_t so, uint32_t po,
                                                     uint64_t r, uint64_t start, uint64_t end, uint64_t wire_len,
                                                     uint64_t* len_l, uint32_t i) {
    uint32_t flag = 0;
    if (start > end || end > wire_len || end - start < a.fixed_bytes) flag = SRPC_STATUS_BOUNDS;
    if (!flag && a.prefix_len) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (so & ~3u));
        const uint32_t* p = reinterpret_cast<const uint32_t*>(lds + po);
        const uint32_t s = so & 3;
        uint32_t w0 = w[0], diff = 0;
        const uint32_t nd = (a.prefix_len + 3) >> 2;
        for (uint32_t k = 0; k < nd; ++k) {
            const uint32_t w1 = w[k + 1];
            const uint32_t x = __builtin_amdgcn_alignbyte(w1, w0, s) ^ p[k];
            const uint32_t left = a.prefix_len - 4 * k;
            diff |= left >= 4 ? x : (x & ((1u << (8 * left)) - 1));
            w0 = w1;
        }
        if (diff) flag = SRPC_STATUS_PREFIX;
    }
    uint64_t pos = start + a.prefix_len;
    uint32_t si = 0;
    for (uint32_t f = 0; f < a.nfields; ++f) {
        const uint32_t sz = a.size[f];
        if (sz) {
            if (flag != SRPC_STATUS_BOUNDS && pos + sz <= end) {
                const uint64_t v = lds_u64(lds, so + static_cast<uint32_t>(pos - start));
                uint8_t* dst = const_cast<uint8_t*>(a.col[f]) + r * sz;
                switch (sz) {
                case 1: dst[0] = static_cast<uint8_t>(v); break;
                case 2: *reinterpret_cast<uint16_t*>(dst) = static_cast<uint16_t>(v); break;
                case 4: *reinterpret_cast<uint32_t*>(dst) = static_cast<uint32_t>(v); break;
                default: *reinterpret_cast<uint64_t*>(dst) = v; break;
                }
            }
            pos += sz;
            continue;
        }
        uint64_t len = 0;
        if (flag != SRPC_STATUS_BOUNDS && pos + 8 <= end) {
            len = lds_u64(lds, so + static_cast<uint32_t>(pos - start));
            pos += 8;
            if (len > end - pos) {
                flag = SRPC_STATUS_BOUNDS;
                len = 0;
            }
        } else {
            flag = SRPC_STATUS_BOUNDS;
        }
        len_l[si * kBlock + i] = len;
        ++si;
        pos += len;
    }
    if (!flag && pos != end) flag = SRPC_STATUS_BOUNDS;  // record size disagrees with the index
    if (flag == SRPC_STATUS_BOUNDS)
        for (uint32_t k = 0; k < a.nstrings; ++k) len_l[k * kBlock + i] = 0;
    return flag;
}

// kOpt (single-string schemas): no look-back -- when every record is exact
// (its decoded string length is its index size minus fixed_bytes), string
// chars of record r start at rec_offs[r] - rec_offs[0] - r * fixed_bytes, so
// the tile's base comes from its index window alone.  A tile holding a record
// that is not exact (or whose base would leave the chars buffer) sets *bad;
// then the general kernel (kOpt = false, gated on *bad) decodes the whole
// batch again with the look-back and rewrites every output.
// table (kOpt = false, several string fields): the caller's tile table
// (srpc_gpu_var_tile_table: chars of each string field before every 256-record
// tile) gives each tile its output bases instead of the look-back; each tile
// checks its own totals against the table's differences (and table[0] = 0,
// bases inside the chars buffers), so a wrong table is caught: *bad is set and
// the look-back pass (gated on *bad) decodes the batch again.
template <bool kOpt>
__global__ __launch_bounds__(kBlock) void k_unpack_var_rt(VarArgs a, RtuArgs L, const uint8_t* __restrict__ wire,
                                                          uint64_t wire_len, const uint64_t* __restrict__ rec_offs,
                                                          uint64_t n, uint64_t* __restrict__ look,
                                                          uint64_t* __restrict__ look2, uint32_t* __restrict__ ticket,
                                                          srpc_unpack_status* st, uint32_t* __restrict__ bad,
                                                          const uint64_t* __restrict__ table) {
    if constexpr (!kOpt)
        if (!table && bad && *bad == 0) return;  // the optimistic pass was exact everywhere
    PHASE_BEGIN
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    __shared__ uint64_t s_tile, s_lo, s_hi, s_src, s_first;
    __shared__ uint32_t s_inexact;
    __shared__ uint64_t s_tot[kMaxFields], s_pre[kMaxFields];
    __shared__ uint32_t s_ioff[kMaxFields];
    __shared__ uint32_t s_ngran, s_fits;
#if SRPC_RTU_OFFLOAD
    __shared__ uint32_t s_bnd[kBlock / 32];  // records whose strings are not copied (BOUNDS, or past the tile)
#endif
    const uint32_t lane = threadIdx.x & 63, i = threadIdx.x;
    const uint32_t ns = a.nstrings;
#if SRPC_RTU_OFFLOAD
    if (i < kBlock / 32) s_bnd[i] = 0;
#endif
#if SRPC_RTU_TICKET
    if (i == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint64_t t = s_tile;
#else
    // tile = blockIdx.x: every XCD dispatches its workgroups in increasing
    // order, so the smallest unfinished tile is always resident and every
    // look-back ends (one ticket atomic per tile, all on one address, cost
    // ~10 ns each at the memory side: 32K tiles -> 300 us, r02_var_rtu_ab.log);
    // the spin limit in the look-back guarantees termination regardless
    const uint64_t t = blockIdx.x;
#endif
    const uint64_t r0 = t * kBlock;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(kBlock, n - r0));
    // the lane's record bounds stay in registers (coalesced loads, issued
    // with the prefix bytes and before the table's wait)
    const uint64_t start = i < nr ? rec_offs[r0 + i] : 0, end = i < nr ? rec_offs[r0 + i + 1] : 0;
    // the caller's tile table: this tile's bases, loaded with the index (its
    // round trip overlaps the index's and the stage's instead of following
    // the scan)
    uint64_t tab_lo = 0, tab_hi = 0;
    if (!kOpt && table && i < ns) {
        tab_lo = table[t * ns + i];
        tab_hi = table[(t + 1) * ns + i];
    }
    // the prefix's first kBlock bytes are loaded here and written to LDS after
    // the table, so their round trip overlaps the index loads (one barrier
    // less before the stage can be requested)
    const uint8_t pb = i < a.prefix_len ? a.prefix[i] : 0;
    // 1. the tile's wire span [rec_offs[r0], rec_offs[r0 + nr]) in 16-byte granules
    if (i == 0) {
        const uint64_t w0 = rec_offs[r0], w1 = rec_offs[r0 + nr];
        s_lo = w0;
        s_hi = w1;
        if (kOpt) {
            s_first = rec_offs[0];
            s_inexact = 0;
        }
        uint64_t A = 0, ng = 0;
        if (w0 < w1 && w1 <= wire_len) {
            A = reinterpret_cast<uint64_t>(wire + w0) & ~15ull;
            ng = (reinterpret_cast<uint64_t>(wire + w1) - A + 15) >> 4;
            if (16 * ng > L.stage_cap) ng = 0;  // span too large: parse from global memory
        }
        s_src = A;
        s_ngran = static_cast<uint32_t>(ng);
    }
    if (i < a.prefix_len + 16) lds[L.pre_at + i] = pb;
    for (uint32_t k = i + kBlock; k < a.prefix_len + 16; k += kBlock)
        lds[L.pre_at + k] = k < a.prefix_len ? a.prefix[k] : 0;
    __syncthreads();
    PHASE(0);
    // 2. span -> stage by LDS-DMA (global_load_lds_dwordx4: a wave
    // instruction fills 1 KiB of LDS, no VGPRs hold the data)
    const uint32_t ngran = s_ngran;
    const uint64_t src0 = s_src;
    for (uint32_t w0 = i & ~63u; w0 < ngran; w0 += kBlock) {
        const uint32_t gi = w0 + lane;
        if (gi < ngran) {
            const uint32_t wb = __builtin_amdgcn_readfirstlane(w0);
            __builtin_amdgcn_global_load_lds(reinterpret_cast<global_u8*>(src0 + 16ull * gi),
                                             (lds_u8*)(lds + L.stage_at + 16 * wb), 16, 0, 0);
        }
    }
    __syncthreads();  // waits for the LDS-DMA (vmcnt(0)) and publishes the stage
    PHASE(1);
    const bool staged = ngran != 0;
    const uint64_t slo = s_lo, shi = s_hi;
    const uint32_t sb = L.stage_at;                       // LDS offset of the stage's first granule
    const uint64_t sw = src0 - reinterpret_cast<uint64_t>(wire);  // its wire offset
    uint64_t* len_l = reinterpret_cast<uint64_t*>(lds + L.len_at);
    // 3. parse (the record's chars positions are walked again when copied)
    uint32_t flag = SRPC_STATUS_BOUNDS;  // lanes past the tile: nothing to copy
    const bool in_stage = staged && start >= slo && end <= shi && start <= end;
    if (i < nr) {
        if (in_stage)
            flag = parse_record_lds(a, lds, sb + static_cast<uint32_t>(start - sw), L.pre_at, r0 + i, start, end,
                                    wire_len, len_l, i);
        else
            flag = parse_record(a, wire + start, lds + L.pre_at, r0 + i, start, end, wire_len, len_l, i);
        if (flag && st) report_bad(st, flag, r0 + i);
        if (kOpt && (start > end || end - start < a.fixed_bytes || len_l[i] != end - start - a.fixed_bytes))
            s_inexact = 1;
    } else {
        for (uint32_t k = 0; k < ns; ++k) len_l[k * kBlock + i] = 0;
    }
#if SRPC_RTU_OFFLOAD
    if (flag == SRPC_STATUS_BOUNDS) atomicOr(&s_bnd[i >> 5], 1u << (i & 31));
#endif
    __syncthreads();
    PHASE(2);
    // per string field: offsets inside the tile, tile totals
    for (uint32_t si = 0; si < ns; ++si) {
        uint64_t tot;
        // lengths become exclusive offsets in place (len = next offset - offset)
        const uint64_t x = block_exclusive_scan(len_l[si * kBlock + i], &tot);
        len_l[si * kBlock + i] = x;
        if (i == 0) {
            s_tot[si] = tot;
            if (!kOpt && !table) look_store(look + t * ns + si, (t == 0 ? kLookIncl : kLookAgg) | (tot & kLookVal));
        }
    }
    if (!kOpt && table) {  // the tile's bases from the caller's table, checked
        if (i == 0) s_inexact = 0;
        __syncthreads();
        if (i < ns) {
            const uint64_t lo = tab_lo, hi = tab_hi;
            const bool ok = (t > 0 || lo == 0) && hi >= lo && hi - lo == s_tot[i] && hi <= wire_len;
            s_pre[i] = lo;
            if (!ok) s_inexact = 1;
        }
        __syncthreads();
        if (s_inexact) {
            if (i == 0) atomicOr(bad, 1u);
            return;  // the look-back pass rewrites the batch
        }
    }
    if (kOpt) {  // the tile's chars base, valid when every record before it is exact
        if (i == 0) {
            const uint64_t first = s_first, w0 = start;
            const uint64_t fixed_before = r0 * a.fixed_bytes;
            const bool ok = !s_inexact && w0 >= first && w0 - first >= fixed_before &&
                            w0 - first - fixed_before <= wire_len && s_tot[0] <= wire_len - (w0 - first - fixed_before);
            s_pre[0] = ok ? w0 - first - fixed_before : 0;
            if (!ok) {
                atomicOr(bad, 1u);
                s_inexact = 1;
            }
        }
        __syncthreads();
        if (s_inexact) return;  // the general pass rewrites this tile
    }
    // every field's chars image at local offsets (16 bytes of slack on each
    // side), independent of the tile's output base: waves 1-3 build theirs
    // while wave 0 looks back, then wave 0 builds its own
    if (i == 0) {
        uint64_t at = 16;
        for (uint32_t k = 0; k < ns; ++k) {
            s_ioff[k] = static_cast<uint32_t>(min<uint64_t>(at, 0xffffffffull));
            at += ((s_tot[k] + 15) & ~15ull) + 16;
        }
        s_fits = at + 16 <= L.img_cap;
    }
    __syncthreads();
    PHASE(3);
    const bool fits = s_fits;
    // string chars positions: from the stage for a staged record, else from global memory
    auto rd = [&](uint64_t p) -> uint64_t {
        return in_stage ? lds_u64(lds, sb + static_cast<uint32_t>(p - sw)) : load_unaligned<uint64_t>(wire + p);
    };
    // record j's chars into the image (its wire start, whether it is staged)
    auto build_at = [&](uint32_t j, uint64_t start, bool in_stage) {
        uint64_t pos = start + a.prefix_len;
        uint32_t k = 0;
        for (uint32_t f = 0; f < a.nfields; ++f) {
            const uint32_t sz = a.size[f];
            if (sz) {
                pos += sz;
                continue;
            }
            pos += 8;  // the length (the scan's offsets give it back)
            const uint64_t o = len_l[k * kBlock + j];
            const uint64_t len = (j + 1 < kBlock ? len_l[k * kBlock + j + 1] : s_tot[k]) - o;
            if (len) {
                const uint32_t d = L.img_at + s_ioff[k] + static_cast<uint32_t>(o);
                if (in_stage) {
                    lds_copy_run(lds, d, sb + static_cast<uint32_t>(pos - sw), static_cast<uint32_t>(len));
                } else {
                    for (uint64_t x = 0; x < len; x += 8) {
                        const uint32_t kk = static_cast<uint32_t>(min<uint64_t>(8, len - x));
                        uint64_t v = 0;
                        for (uint32_t b = 0; b < kk; ++b) v |= static_cast<uint64_t>(wire[pos + x + b]) << (8 * b);
                        lds_put_small(lds, d + static_cast<uint32_t>(x), v, kk);
                    }
                }
            }
            pos += len;
            ++k;
        }
    };
    auto build = [&]() {
        if (fits && flag != SRPC_STATUS_BOUNDS) build_at(i, start, in_stage);
    };
    // string field si's look-back runs on wave si mod 4: the fields' round
    // trips overlap instead of adding up (two strings: one wave each)
    if (!kOpt && !table && (i >> 6) < ns) {
        bool stalled = false;
        for (uint32_t si = i >> 6; si < ns; si += kBlock / 64) {
#if SRPC_RTU_NOLOOK  // A/B timing only: wrong offsets
            const uint64_t pre = 0;
#else
            const uint64_t pre = t ? look_back2(look + si, look2 + si, t, ns, s_tot[si], &stalled) : 0;
#endif
            if (lane == 0) s_pre[si] = pre;
        }
        if (stalled && lane == 0 && st) report_bad(st, SRPC_STATUS_STALLED, r0);
    }
#if SRPC_RTU_OFFLOAD
    // the waves that do not look back build every record's chars (the
    // look-back waves' records too), so the look-back is off the build's path
    if (!kOpt && !table && ns < kBlock / 64) {
        const uint32_t w = i >> 6, nb = kBlock - 64 * ns;
        if (w >= ns && fits) {
            for (uint32_t j = i - 64 * ns; j < nr; j += nb) {
                if ((s_bnd[j >> 5] >> (j & 31)) & 1) continue;
                const uint64_t sj = rec_offs[r0 + j], ej = rec_offs[r0 + j + 1];
                build_at(j, sj, staged && sj >= slo && ej <= shi && sj <= ej);
            }
        }
    } else {
        build();
    }
#else
    build();
#endif
    __syncthreads();
    PHASE(4);
    // 4. str_offs and chars, per string field; chunk c of the output covers
    // image bytes [16c - h, 16c + 16 - h), h = the base's offset in its 16-byte
    // block, the same for every chunk: a uniform byte shift of two aligned
    // 16-byte image reads
    uint8_t* img = lds + L.img_at;
    uint32_t si = 0;
    for (uint32_t f = 0; f < a.nfields; ++f) {
        if (a.size[f]) continue;
        const uint64_t P = s_pre[si], tot = s_tot[si];
        uint64_t* so = const_cast<uint64_t*>(a.soff[f]);
        uint8_t* chars = const_cast<uint8_t*>(a.col[f]);
        const uint64_t o = len_l[si * kBlock + i];
        if (i < nr) so[r0 + i] = P + o;
        if (i == 0 && r0 + nr == n) so[n] = P + tot;
        const uint32_t h = static_cast<uint32_t>(P & 15);
        const uint64_t gbase = P & ~15ull;
        if (fits && !SRPC_RTU_NOCHARS) {
            const uint8_t* im = img + s_ioff[si];  // local chars x at im[x]; 16 bytes of slack either side
            const uint32_t span = h + static_cast<uint32_t>(tot);
            const uint32_t nch = (span + 15) >> 4;
            const uint32_t sh = (16 - h) & 15;  // (16c - h) mod 16
            for (uint32_t c = i; c < nch; c += kBlock) {
                const uint32_t lo = max(h, 16 * c), hi = min(span, 16 * c + 16);
                if (lo == 16 * c && hi == 16 * c + 16) {
                    // image bytes [16c - h, 16c - h + 16) = bytes sh.. of the aligned pair at 16c - h - sh,
                    // read as two 16-byte LDS quads (ds_read_b128: lanes 16 bytes apart are conflict-free;
                    // the dword pairs the compiler made of plain reads hit every 16th lane's bank)
                    const lds_u32x4c* q = reinterpret_cast<const lds_u32x4c*>(
                        (const lds_u8c*)lds + (L.img_at + s_ioff[si] + 16 * c - h - sh));
                    const u32x4 qa = q[0], qb = sh ? q[1] : u32x4{0, 0, 0, 0};
                    const uint32_t w0 = qa.x, w1 = qa.y, w2 = qa.z, w3 = qa.w, w4 = qb.x, w5 = qb.y, w6 = qb.z,
                                   w7 = qb.w;
                    uint32_t o0, o1, o2, o3;
                    const uint32_t b = sh & 3;
                    switch (sh >> 2) {  // uniform
                    case 0:
                        o0 = __builtin_amdgcn_alignbyte(w1, w0, b); o1 = __builtin_amdgcn_alignbyte(w2, w1, b);
                        o2 = __builtin_amdgcn_alignbyte(w3, w2, b); o3 = __builtin_amdgcn_alignbyte(w4, w3, b);
                        break;
                    case 1:
                        o0 = __builtin_amdgcn_alignbyte(w2, w1, b); o1 = __builtin_amdgcn_alignbyte(w3, w2, b);
                        o2 = __builtin_amdgcn_alignbyte(w4, w3, b); o3 = __builtin_amdgcn_alignbyte(w5, w4, b);
                        break;
                    case 2:
                        o0 = __builtin_amdgcn_alignbyte(w3, w2, b); o1 = __builtin_amdgcn_alignbyte(w4, w3, b);
                        o2 = __builtin_amdgcn_alignbyte(w5, w4, b); o3 = __builtin_amdgcn_alignbyte(w6, w5, b);
                        break;
                    default:
                        o0 = __builtin_amdgcn_alignbyte(w4, w3, b); o1 = __builtin_amdgcn_alignbyte(w5, w4, b);
                        o2 = __builtin_amdgcn_alignbyte(w6, w5, b); o3 = __builtin_amdgcn_alignbyte(w7, w6, b);
                        break;
                    }
                    __builtin_nontemporal_store(u32x4{o0, o1, o2, o3}, reinterpret_cast<u32x4*>(chars + gbase + 16 * c));
                } else {
                    for (uint32_t x = lo; x < hi; ++x) chars[gbase + x] = im[x - h];
                }
            }
        } else if (!SRPC_RTU_NOCHARS && i < nr && flag != SRPC_STATUS_BOUNDS) {
            // the tile's chars exceed the image: copied lane by lane
            const uint64_t len = (i + 1 < kBlock ? len_l[si * kBlock + i + 1] : tot) - o;
            if (len) {
                const uint64_t pos = string_pos(a, start, si, rd);
                uint8_t* dst = chars + P + o;
                if (in_stage) {
                    copy_stage_run(dst, lds, sb + static_cast<uint32_t>(pos - sw), static_cast<uint32_t>(len));
                } else {
                    const uint8_t* src = wire + pos;
                    for (uint64_t k = 0; k < len; ++k) dst[k] = src[k];
                }
            }
        }
        ++si;
    }
    PHASE(5);
    PHASE_COUNT(6);
    PHASE_END
}

// The tile table of a batch from its string offsets: entry t * ns + s = chars
// of string ordinal s before record min(256 t, n).
struct TileTableArgs {
    const uint64_t* soff[kMaxFields];
    uint32_t ns;
};
__global__ void k_tile_table(TileTableArgs t, uint64_t n, uint64_t* __restrict__ table, uint64_t entries) {
    for (uint64_t e = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; e < entries;
         e += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
        const uint64_t tile = e / t.ns;
        const uint32_t si = static_cast<uint32_t>(e % t.ns);
        const uint64_t* so = t.soff[si];
        table[e] = so[min<uint64_t>(tile * kBlock, n)] - so[0];
    }
}

__global__ void k_str_offs_zero(VarArgs a) {  // n == 0: str_offs[f][0] = 0
    const uint32_t f = threadIdx.x;
    if (f < a.nfields && !a.size[f]) const_cast<uint64_t*>(a.soff[f])[0] = 0;
}

__global__ void k_zero_u64(uint64_t* p, uint64_t count) {
    for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < count;
         i += static_cast<uint64_t>(gridDim.x) * blockDim.x)
        p[i] = 0;
}

// ---- host helpers -------------------------------------------------------------
uint64_t scan_blocks(uint64_t n) { return (n + kScanBlock - 1) / kScanBlock; }

template <class F, class M = FirstOnly>
int launch_scan(F f, uint64_t n, uint64_t* partial, uint64_t* out, uint64_t* tile_first, uint64_t max_tiles,
                hipStream_t s, uint64_t tile_bytes = kTileBytes, uint32_t meta_stride = 1,
                const uint32_t* gate = nullptr, uint32_t domains = 1) {
    const uint64_t nb = std::max<uint64_t>(1, scan_blocks(n));
    if (nb > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
    const uint32_t gx = static_cast<uint32_t>(gate ? std::min<uint64_t>(nb, kGatedGrid) : nb);
    launch(k_scan_reduce<F>, dim3(gx, domains), dim3(kBlock), 0, s, f, n, partial, gate, nb);
    launch(k_scan_partials, dim3(1, domains), dim3(kBlock), 0, s, partial, nb, gate);
    launch(k_scan_apply<F, M>, dim3(gx, domains), dim3(kBlock), 0, s, f, M{}, n, partial, nb, out,
           tile_first, max_tiles, tile_bytes, meta_stride, gate);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

VarArgs make_var_args(const srpc_plan* p, const void* const* cols, const uint64_t* const* str_offs) {
    VarArgs a{};
    uint32_t si = 0, fi = 0;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        a.col[f] = static_cast<const uint8_t*>(cols[f]);
        a.size[f] = p->size[f];
        if (p->size[f] == 0) {
            a.soff[f] = str_offs ? str_offs[f] : nullptr;
            a.sfield[si] = f;
            a.sidx[f] = si++;
        } else {
            a.ffield[fi++] = f;
        }
    }
    a.prefix = p->d_prefix;
    a.nfields = p->nfields;
    a.nstrings = p->nstrings;
    a.prefix_len = p->prefix_len;
    a.fixed_bytes = p->fixed_bytes;
    return a;
}

// Scratch layout (each region 256-byte aligned):
//   [partials: nb+1 u64] [tile_first: per tile domain, max_tiles u64]
//   unpack only: [lens: ns*n u64] [spos: ns*n u64]
// Pack has one tile domain (the wire); unpack one per string field (its chars).
struct ScratchLayout {
    uint64_t partial_off, tiles_off, lens_off, spos_off, bad_off, long_off, look_off, total;
    uint64_t max_tiles;
};

uint64_t round256(uint64_t b) { return (b + 255) & ~255ull; }

// max_tiles covers tile index wire_bytes / kTileBytes + 1.
ScratchLayout scratch_layout(const srpc_plan* p, uint64_t n, uint64_t wire_bytes, bool unpack) {
    ScratchLayout L{};
    L.max_tiles = wire_bytes / kTileBytes + 2;
    L.partial_off = 0;
    const uint64_t domains = unpack ? p->nstrings : 1;
    // one partials array per string field: multi-string unpack scans them all in one launch
    L.tiles_off = round256(8 * (std::max<uint64_t>(1, scan_blocks(n)) + 1) * std::max<uint64_t>(1, domains));
    L.lens_off = L.tiles_off + round256(8 * L.max_tiles * domains);
    L.spos_off = L.lens_off + (unpack ? round256(8 * static_cast<uint64_t>(p->nstrings) * n) : 0);
    L.bad_off = L.spos_off + (unpack ? round256(8 * static_cast<uint64_t>(p->nstrings) * n) : 0);
    L.long_off = L.bad_off + 64 * kLongFlags;
    // record-tile unpack: ticket + a look-back word per 256-record tile and string field
    L.look_off = L.long_off + round256(4 * L.max_tiles);
    const uint64_t nt = (n + kBlock - 1) / kBlock;
    L.total = L.look_off + round256(8 * (1 + (nt + (nt + 63) / 64) * p->nstrings));
    return L;
}

uint32_t round16(uint32_t b) { return (b + 15) & ~15u; }

// Workgroups of `kernel` (kBlock threads, `lds` dynamic LDS bytes) the device
// holds at once, times SRPC_RT_GRID_MULT (A/B builds; default 1).
#ifndef SRPC_RT_GRID_MULT
#define SRPC_RT_GRID_MULT 1
#endif
#ifndef SRPC_RT_PERSIST_MIN
#define SRPC_RT_PERSIST_MIN 40
#endif
constexpr uint64_t kRtPersistMin = SRPC_RT_PERSIST_MIN;
constexpr uint64_t kRtTwoPerLane = 20;
template <typename K>
uint64_t resident_grid(K kernel, uint32_t lds, int device) {
    int per_cu = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, lds) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || per_cu < 1 ||
        cus < 1) {
        per_cu = 2;
        cus = 256;
    }
    return static_cast<uint64_t>(per_cu) * cus * SRPC_RT_GRID_MULT;
}

// LDS carve of k_pack_var_rt (see RtArgs).  The image holds a tile's wire
// span: 256 records of `avg` bytes (the caller's wire_cap / n, exact when the
// caller sizes the wire buffer to the batch) with 1/16 slack, unless the plan
// fixes it (SRPC_TUNE_VAR_IMAGE_BYTES); the stage holds the tile's offsets
// windows and column slices plus the chars that such a span can hold.  Tiles
// that do not fit take the chunk walk.
RtArgs rt_layout(const srpc_plan* p, uint64_t avg, uint32_t* total, uint32_t rpl = 1) {
    RtArgs L{};
    const uint32_t tr = kBlock * rpl;  // records per tile
    uint32_t off = 0;
    L.pre_at = off;
    off += round16(p->prefix_len + 32);
    uint64_t img = p->rt_img_cap;
    if (!img) {
        img = std::min<uint64_t>(avg, kRtImageMax) * tr;
        img = std::min<uint64_t>(std::max<uint64_t>(img + img / 16 + 64, kRtImageMin), kRtImageMax);
    }
    L.img_cap = round16(static_cast<uint32_t>(img));
    uint64_t chars = p->rt_ch_cap;
    if (p->rt_ch_cap_auto) {
        const uint64_t fixed_span = static_cast<uint64_t>(tr) * p->fixed_bytes;
        chars = L.img_cap > fixed_span ? L.img_cap - fixed_span : 0;
    }
    uint32_t fixed = p->nstrings * (((tr + 1) * 8 + 16 + 15) & ~15u);  // offsets windows
    for (uint32_t f = 0; f < p->nfields; ++f)
        if (p->size[f]) fixed += round16(tr * p->size[f] + 16);
    L.stage_cap = fixed + round16(static_cast<uint32_t>(chars)) + 16 * p->nstrings;
    L.stage_at = off;
    off += L.stage_cap + 16;  // lds_copy_run may read a dword past a chars run
    L.img_at = off;
    off += L.img_cap + 16;
    *total = off;
    return L;
}

// LDS carve of k_unpack_var_rt: the stage holds the index window and a
// tile's wire span (256 records of wire_len / n bytes with 1/16 slack); the
// chars image one string field's chars of a tile.  Returns false when the
// span would not fit (long records keep the walk + scans + chars kernels).
bool rtu_layout(const srpc_plan* p, uint64_t avg, RtuArgs* out, uint32_t* total) {
    RtuArgs L{};
    const uint64_t span = std::min<uint64_t>(avg, kRtImageMax) * kBlock;
    const uint64_t cap = span + span / 16 + 64;
    if (cap > kRtImageMax * 3 / 4) return false;
    uint32_t off = 0;
    L.pre_at = off;
    off += round16(p->prefix_len + 16);
    L.stage_cap = round16(static_cast<uint32_t>(cap));
    L.stage_at = off;
    off += L.stage_cap + 16;  // lds_copy_run may read a dword past a run
    L.len_at = off;
    off += 8 * kBlock * p->nstrings;
    const uint64_t fixed_span = static_cast<uint64_t>(kBlock) * p->fixed_bytes;
    // every string field's chars of a tile, 16 bytes of slack around each
    // (without the image -- each record's lane copying its own chars -- the
    // tiles ran 0.44 -> 0.32 on 0-64 B strings: fewer, wider stores won)
    L.img_cap = round16(static_cast<uint32_t>(std::max<uint64_t>(1024, cap > fixed_span ? cap - fixed_span : 0) +
                                              32 * (p->nstrings + 1)));
    L.img_at = off;
    off += L.img_cap + 32;
    *out = L;
    *total = off;
    return true;
}

}  // namespace

}  // namespace srpc_impl

using namespace srpc_impl;

extern "C" {

// Test hook (not part of the C ABI in include/): the multi-string unpack's
// look-back spin budget (0 = the default, 2^21 polls); a tiny budget makes
// tiles give up and report SRPC_STATUS_STALLED.  Returns SRPC_OK.
__attribute__((visibility("default"))) int srpc_debug_var_spin_limit(uint32_t spins) {
    const uint32_t v = spins ? spins : kLookSpinMax;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_look_spin_max), &v, sizeof(v)) == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

#ifdef SRPC_PHASES
int srpc_debug_phases(uint64_t* host8, int reset) {
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_phase), sizeof(h)) != hipSuccess) return SRPC_E_HIP;
    for (int i = 0; i < 8; ++i) host8[i] = h[i];
    if (reset) {
        const unsigned long long z[8] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof(z)) != hipSuccess) return SRPC_E_HIP;
    }
    return SRPC_OK;
}
#endif

int srpc_plan_var_scratch_bytes(const srpc_plan* p, uint64_t n, uint64_t wire_bytes, uint64_t* out) {
    if (!p || !out) return SRPC_E_INVALID;
    if (!p->has_string) {
        *out = 0;
        return SRPC_OK;
    }
    *out = std::max(scratch_layout(p, n, wire_bytes, false).total, scratch_layout(p, n, wire_bytes, true).total);
    return SRPC_OK;
}

int srpc_gpu_pack_var(const srpc_plan* p, const void* const* cols, const uint64_t* const* str_offs, uint64_t n,
                      uint8_t* wire, uint64_t wire_cap, uint64_t* rec_offs, srpc_unpack_status* st,
                      void* scratch, uint64_t scratch_bytes, void* stream) {
    const TimedCall timed;
    if (!p || !p->has_string) return SRPC_E_INVALID;
    auto s = static_cast<hipStream_t>(stream);
    if (st) {
        hipLaunchKernelGGL(k_reset_status, dim3(1), dim3(64), 0, s, st, nullptr, 0u);
        if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
    }
    if (!rec_offs || !cols || !str_offs || !scratch) return SRPC_E_INVALID;
    const ScratchLayout L = scratch_layout(p, n, wire_cap, false);
    if (scratch_bytes < L.total) return SRPC_E_CAPACITY;
    if (!aligned(wire, 16) || !aligned(rec_offs, 8) || !aligned(scratch, 8)) return SRPC_E_ALIGN;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        if (!cols[f]) return SRPC_E_INVALID;
        if (p->size[f] == 0 && (!str_offs[f] || !aligned(str_offs[f], 8))) return SRPC_E_INVALID;
    }
    const VarArgs a = make_var_args(p, cols, str_offs);
    auto* base = static_cast<uint8_t*>(scratch);
    // record tiles, one pass (default) -- unless a tile's span would not fit
    // the LDS image (records averaging more than ~240 bytes: the scan +
    // chunk walk below moves long strings at 0.38 of HBM peak, the record
    // tiles' per-tile walk fallback at 0.10, profiles/r02_var_rt_ab.log)
    const uint64_t avg = n ? wire_cap / n : 0;
    if (p->var_kernel == 1 && (p->rt_img_cap || avg * kBlock * 17 / 16 + 64 <= kRtImageMax * 15 / 16)) {
        if (n == 0) {  // rec_offs[0] = 0
            launch(k_zero_u64, dim3(1), dim3(64), 0, s, rec_offs, 1ull);
            return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
        }
        const uint64_t ntiles = (n + kBlock - 1) / kBlock;
        if (ntiles > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
        if (!wire) return SRPC_E_INVALID;
        uint32_t lds = 0;
        const bool loop = wire_cap / n >= kRtPersistMin;
        // records under kRtTwoPerLane bytes on average: two per lane (a tile of
        // 512 records; 0-16 B strings 114 -> 98 us, but 0-32 B 67 -> 79 us and
        // four per lane slower on both, profiles/r02_var_rt_rpl_ab.log)
        const uint32_t rpl = !loop && wire_cap / n < kRtTwoPerLane ? 2 : 1;
        const RtArgs R = rt_layout(p, wire_cap / n, &lds, rpl);
        // records of >= SRPC_RT_PERSIST_MIN bytes on average: resident workgroups
        // only, each looping over its tiles with the next tile's loads in flight
        // (two strings + request envelope 228 -> 193 us, 0-64 B 134 -> 127 us);
        // shorter records: a workgroup per tile, as the loop's per-tile barriers
        // cost more than the overlap saves on 4-8 KiB tiles (0-16 B strings
        // 112 -> 134 us persistent, profiles/r02_var_rt_persist_ab.log)
        if (loop) {
            const uint64_t grid = std::min<uint64_t>(ntiles, resident_grid(k_pack_var_rt_loop, lds, p->device));
            launch(k_pack_var_rt_loop, dim3(static_cast<uint32_t>(grid)), dim3(kBlock), lds, s, a, R, n, wire,
                   wire_cap, rec_offs, st);
        } else {
            const uint64_t tiles = (n + kBlock * rpl - 1) / (kBlock * rpl);
            if (rpl == 2)
                launch(k_pack_var_rt<2>, dim3(static_cast<uint32_t>(tiles)), dim3(kBlock), lds, s, a, R, n, wire,
                       wire_cap, rec_offs, st);
            else
                launch(k_pack_var_rt<1>, dim3(static_cast<uint32_t>(tiles)), dim3(kBlock), lds, s, a, R, n, wire,
                       wire_cap, rec_offs, st);
        }
        return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    }
    auto* tiles = reinterpret_cast<uint64_t*>(base + L.tiles_off);
    auto* partial = reinterpret_cast<uint64_t*>(base + L.partial_off);
    const uint64_t g1 = n / kBlock + 1;
    if (g1 > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
    if (n && !wire) return SRPC_E_INVALID;
    uint32_t* some_long = reinterpret_cast<uint32_t*>(base + L.bad_off);
    // records that may be written one per lane: small ones only (wide per-lane
    // records write partial cache lines: 94-byte records took 723 us against
    // the walk's 313, profiles/r01_var_pack_short_ab.log)
    const bool small = p->fixed_bytes + p->nstrings * kShortCopy <= kShortRecord;
    // skip_test: k_pack_short_records ran and its flags say whether the walk
    // has work; otherwise the walk runs unconditionally (k_pack_var<false>,
    // no flag reset / set launches: 2 tiny kernels, ~7 us)
    bool skip_test = true;
    if (p->nstrings == 1) {
        hipLaunchKernelGGL(k_reset_status, dim3(1), dim3(64), 0, s, nullptr, some_long, kLongFlags);
        launch(k_pack_short_records<true>, dim3(static_cast<uint32_t>(g1)), dim3(kBlock), 0, s, a, n, rec_offs,
               tiles, some_long, L.max_tiles, wire, small ? wire_cap : 0);
    } else {
        int rc = launch_scan(PackSizes{a}, n, partial, rec_offs, tiles, L.max_tiles, s);
        if (rc) return rc;
        if (n && small) {
            hipLaunchKernelGGL(k_reset_status, dim3(1), dim3(64), 0, s, nullptr, some_long, kLongFlags);
            launch(k_pack_short_records<false>, dim3(static_cast<uint32_t>(g1)), dim3(kBlock), 0, s, a, n, rec_offs,
                   tiles, some_long, L.max_tiles, wire, wire_cap);
        } else {
            skip_test = false;
        }
    }
    if (n == 0) return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    if (!wire) return SRPC_E_INVALID;
    // soff0 = a.soff[first string field] as its own argument: indexed out of
    // VarArgs, the compiler re-loads it from the kernarg segment inside the
    // tile loop (a dependent scalar load per tile, +40 % kernel time,
    // profiles/r01_var_short_copy_ab.log)
    uint32_t f0 = 0;
    while (p->size[f0]) ++f0;
    launch(skip_test ? k_pack_var<true> : k_pack_var<false>, dim3(kVarGrid), dim3(kBlock), 0, s, a, rec_offs, n,
           tiles, wire, wire_cap, st, static_cast<const uint32_t*>(some_long), a.soff[f0]);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int srpc_gpu_unpack_var_tiled(const srpc_plan* p, const uint8_t* wire, uint64_t wire_len, uint64_t n,
                              const uint64_t* rec_offs, const uint64_t* table, void* const* cols,
                              uint64_t* const* str_offs, srpc_unpack_status* st, void* scratch, uint64_t scratch_bytes,
                              void* stream) {
    const TimedCall timed;
    if (!p || !p->has_string) return SRPC_E_INVALID;
    auto s = static_cast<hipStream_t>(stream);
    // the status is reset on every path before its first reporting kernel --
    // fused into the paths' own reset launches where they have one
    bool st_done = !st;
    auto reset_st = [&]() -> bool {
        if (!st_done) {
            hipLaunchKernelGGL(k_reset_status, dim3(1), dim3(64), 0, s, st, nullptr, 0u);
            st_done = true;
        }
        return hipGetLastError() == hipSuccess;
    };
    auto fail = [&](int rc) { return reset_st() ? rc : SRPC_E_HIP; };
    if (!rec_offs || !cols || !str_offs || !scratch) return fail(SRPC_E_INVALID);
    const ScratchLayout L = scratch_layout(p, n, wire_len, true);
    if (scratch_bytes < L.total) return fail(SRPC_E_CAPACITY);
    if (!aligned(scratch, 8) || !aligned(rec_offs, 8)) return fail(SRPC_E_ALIGN);
    for (uint32_t f = 0; f < p->nfields; ++f) {
        if (!cols[f]) return fail(SRPC_E_INVALID);
        if (p->size[f] && !aligned(cols[f], p->size[f])) return fail(SRPC_E_ALIGN);
        if (p->size[f] == 0 && (!str_offs[f] || !aligned(str_offs[f], 8) || !aligned(cols[f], 16)))
            return fail(SRPC_E_ALIGN);
    }
    const VarArgs a = make_var_args(p, reinterpret_cast<const void* const*>(cols),
                                    reinterpret_cast<const uint64_t* const*>(str_offs));
    auto* base = static_cast<uint8_t*>(scratch);
    auto* partial = reinterpret_cast<uint64_t*>(base + L.partial_off);
    auto* tiles = reinterpret_cast<uint64_t*>(base + L.tiles_off);
    auto* lens = reinterpret_cast<uint64_t*>(base + L.lens_off);
    auto* spos = reinterpret_cast<uint64_t*>(base + L.spos_off);
    const uint64_t grid = (n + kBlock - 1) / kBlock;
    if (grid > 0x7fffffffull) return fail(SRPC_E_UNSUPPORTED);
    auto* bad = reinterpret_cast<uint32_t*>(base + L.bad_off);
    // record tiles, one pass (default), for batches whose tiles' wire spans fit LDS
    RtuArgs R{};
    uint32_t rlds = 0;
    // (multi-string schemas look back on the tiles' chars totals, one wave per
    // string field: two strings + request envelope 358 us with the walk + scans
    // + chars kernels -> 305 us, profiles/r02_var_rtu_parlook_ab.log)
    // Very short records (under ~40 bytes on average) keep the staged walk +
    // chars kernels as well: their 256-record tiles are too small to pay for a
    // tile's fixed cost (0-16 B strings 104 vs 142 us, 0-32 B 71 vs 88 us;
    // 50-byte records 206 -> 146 us with the tiles, profiles/r02_var_rtu_ab.log).
    if (p->var_kernel == 1 &&
        (n == 0 || ((wire_len / n >= kRtuMinAvg || p->var_rt_general) && rtu_layout(p, wire_len / n, &R, &rlds)))) {
        if (n == 0) {
            if (!reset_st()) return SRPC_E_HIP;
            launch(k_str_offs_zero, dim3(1), dim3(64), 0, s, a);
            return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
        }
        if (!wire) return fail(SRPC_E_INVALID);
        auto* look = reinterpret_cast<uint64_t*>(base + L.look_off);
        // ticket + look-back words per tile and per 64-tile block, per string field
        const uint64_t w1 = grid * p->nstrings, w2 = ((grid + 63) / 64) * p->nstrings;
        const uint64_t words = 1 + w1 + w2;
        const uint32_t zgrid = static_cast<uint32_t>(std::min<uint64_t>((words + 255) / 256, 1024));
        const uint64_t* no_table = nullptr;
        // (the optimistic passes below never touch the look-back words: the
        // status, the flag and the words of the gated look-back pass are
        // reset in one launch before them, not by a gated launch between)
        if (p->nstrings == 1) {
            hipLaunchKernelGGL(k_reset_walk1, dim3(zgrid), dim3(256), 0, s, st_done ? nullptr : st, bad,
                               static_cast<uint32_t*>(nullptr), 0ull, look, words);
            st_done = true;
            launch(k_unpack_var_rt<true>, dim3(static_cast<uint32_t>(grid)), dim3(kBlock), rlds, s, a, R, wire,
                   wire_len, rec_offs, n, look + 1, look + 1 + w1, reinterpret_cast<uint32_t*>(look), st, bad,
                   no_table);
        } else if (table) {
            // the tiles' bases from the caller's table; the look-back pass only
            // when a tile's totals disagree with it
            hipLaunchKernelGGL(k_reset_walk1, dim3(zgrid), dim3(256), 0, s, st_done ? nullptr : st, bad,
                               static_cast<uint32_t*>(nullptr), 0ull, look, words);
            st_done = true;
            launch(k_unpack_var_rt<false>, dim3(static_cast<uint32_t>(grid)), dim3(kBlock), rlds, s, a, R, wire,
                   wire_len, rec_offs, n, look + 1, look + 1 + w1, reinterpret_cast<uint32_t*>(look), st, bad, table);
        } else {
            if (!reset_st()) return SRPC_E_HIP;
            launch(k_zero_u64, dim3(zgrid), dim3(256), 0, s, look, words);
        }
        launch(k_unpack_var_rt<false>, dim3(static_cast<uint32_t>(grid)), dim3(kBlock), rlds, s, a, R, wire, wire_len,
               rec_offs, n, look + 1, look + 1 + w1, reinterpret_cast<uint32_t*>(look), st,
               p->nstrings == 1 || table ? bad : nullptr, no_table);
        return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    }
    if (p->nstrings == 1 && n) {  // single-string fast path: no scan unless a record is not exact
        if (!wire) return fail(SRPC_E_INVALID);
        const uint32_t f = a.sfield[0];
        uint32_t len_at = p->prefix_len;  // the u64 length follows the prefix and the fixed fields before it
        for (uint32_t g = 0; g < f; ++g) len_at += p->size[g];
        auto* tile_long = reinterpret_cast<uint32_t*>(base + L.long_off);
        const uint32_t rgrid = static_cast<uint32_t>(std::min<uint64_t>((L.max_tiles + 255) / 256 + 1, 1024));
        auto* look = reinterpret_cast<uint64_t*>(base + L.look_off);
        const uint64_t snb = std::max<uint64_t>(1, scan_blocks(n));
        const uint64_t nlook = 1 + snb + (snb + 63) / 64;  // ticket, per scan block, per 64 blocks
        hipLaunchKernelGGL(k_reset_walk1, dim3(rgrid), dim3(256), 0, s, st_done ? nullptr : st, bad, tile_long,
                           static_cast<uint64_t>(L.max_tiles), look, nlook);
        st_done = true;
        if (hipGetLastError() != hipSuccess) return SRPC_E_HIP;
        const SingleFast fast{str_offs[f], tiles, L.max_tiles, bad, static_cast<uint8_t*>(cols[f]), tile_long,
                              len_at + 8};
        // the walk stages its span as in the multi-string path when it fits
        // (0-32 B strings 77 -> 71 us, r01_var_staged_walk_ab.log)
        const uint64_t avg1 = wire_len / n;
        // records under kWalkTwoPerLane bytes on average: two per lane (512-record
        // workgroups; 0-16 B strings' walk 89 -> 76 us, 0-32 B unchanged,
        // four per lane slower on both: profiles/r06_var_walk_ab.log)
        const uint32_t kR = avg1 <= kWalkTwoPerLane ? 2 : 1;
        const uint64_t want1 = avg1 > kWalkStageMax ? ~0ull : stage_bytes_for(avg1, kR);
        const uint64_t want1s = avg1 > kWalkStageMax ? ~0ull : stage_bytes_for(avg1);
        if (kR > 1 && want1 <= kWalkStageMax) {
            const uint64_t g = (n + kBlock * kR - 1) / (kBlock * kR);
            launch(k_unpack_var_walk<true, 2>, dim3(static_cast<uint32_t>(g)), dim3(kBlock),
                   static_cast<uint32_t>(want1), s, a, wire, wire_len, rec_offs, n, lens, spos, st, fast,
                   static_cast<uint32_t>(want1));
        } else if (want1s <= kWalkStageMax) {
            launch(k_unpack_var_walk<true, 1>, dim3(static_cast<uint32_t>(grid)), dim3(kBlock),
                   static_cast<uint32_t>(want1s), s, a, wire, wire_len, rec_offs, n, lens, spos, st, fast,
                   static_cast<uint32_t>(want1s));
        } else {
            launch(k_unpack_var_walk<false, 1>, dim3(static_cast<uint32_t>(grid)), dim3(kBlock), 0, s, a, wire,
                   wire_len, rec_offs, n, lens, spos, st, fast, 0u);
        }
        if (snb > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
        const SingleStrLen lens1{wire, wire_len, rec_offs, p->d_prefix, p->prefix_len, len_at, p->fixed_bytes};
        if (avg1 <= p->fixed_bytes + kShortCopy) {
            // short strings: the tail in one gated launch
            launch(k_unpack_str1_tail, dim3(kVarGrid), dim3(kBlock), 0, s, lens1, n, str_offs[f],
                   static_cast<uint8_t*>(cols[f]), len_at + 8, static_cast<const uint64_t*>(tiles),
                   static_cast<const uint32_t*>(tile_long), static_cast<const uint32_t*>(bad), look, look + 1 + snb,
                   st);
        } else {
            // long strings (the chars kernel copies most tiles): the gated scan,
            // then the chars kernel on its own (in the tail kernel its tiles ran
            // 0-1024 B strings 311 -> 420 us, profiles/r06_var_walk_ab.log)
            launch(k_scan1<SingleStrLen>, dim3(static_cast<uint32_t>(std::min<uint64_t>(snb, kGatedGrid))),
                   dim3(kBlock), 0, s, lens1, n, str_offs[f], tiles, static_cast<uint64_t>(L.max_tiles),
                   static_cast<const uint32_t*>(bad), look, look + 1 + snb, st);
            launch(k_unpack_var_chars, dim3(kVarGrid), dim3(kBlock), 0, s, wire, wire_len, str_offs[f], tiles,
                   static_cast<const uint64_t*>(nullptr), n, static_cast<uint8_t*>(cols[f]), rec_offs, len_at + 8,
                   static_cast<const uint32_t*>(tile_long), static_cast<const uint32_t*>(bad));
        }
        return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    }
    if (!reset_st()) return SRPC_E_HIP;
    if (n) {
        if (!wire) return SRPC_E_INVALID;
        // stage a workgroup's span when 17/16 of the average span fits 48 KiB
        const uint64_t avg = wire_len / n;
        const uint64_t want = avg > kWalkStageMax ? ~0ull : stage_bytes_for(avg);
        if (want <= kWalkStageMax)
            launch(k_unpack_var_walk<true, 1>, dim3(static_cast<uint32_t>(grid)), dim3(kBlock),
                   static_cast<uint32_t>(want), s, a, wire, wire_len, rec_offs, n, lens, spos, st, SingleFast{},
                   static_cast<uint32_t>(want));
        else
            launch(k_unpack_var_walk<false, 1>, dim3(static_cast<uint32_t>(grid)), dim3(kBlock), 0, s, a, wire,
                   wire_len, rec_offs, n, lens, spos, st, SingleFast{}, 0u);
    }
#ifndef SRPC_SCAN_PERFIELD
    if (p->nstrings > 1) {  // all string fields' offsets in one scan launch per phase
        ArrayValsY fy{lens, n, {}};
        for (uint32_t f = 0; f < p->nfields; ++f)
            if (!p->size[f]) fy.outs[a.sidx[f]] = str_offs[f];
        int rc = launch_scan(fy, n, partial, nullptr, tiles, L.max_tiles, s, kTileBytes, 1, nullptr, p->nstrings);
        if (rc) return rc;
    } else
#endif
    for (uint32_t f = 0; f < p->nfields; ++f) {
        if (p->size[f]) continue;
        int rc = launch_scan(ArrayVals{lens + a.sidx[f] * n}, n, partial, str_offs[f],
                             tiles + a.sidx[f] * L.max_tiles, L.max_tiles, s);
        if (rc) return rc;
    }
    if (n == 0) return SRPC_OK;
#ifndef SRPC_CHARS_PERFIELD
    if (p->nstrings > 1) {  // one interleaved launch: the wire is streamed once, not once per field
        CharsFields cf{};
        for (uint32_t f = 0; f < p->nfields; ++f) {
            if (p->size[f]) continue;
            const uint32_t j = cf.nstr++;
            cf.soff[j] = str_offs[f];
            cf.tile_first[j] = tiles + a.sidx[f] * L.max_tiles;
            cf.spos[j] = spos + a.sidx[f] * n;
            cf.chars[j] = static_cast<uint8_t*>(cols[f]);
        }
        launch(k_unpack_var_chars_multi, dim3(kVarGrid), dim3(kBlock), 0, s, wire, wire_len, cf, n, L.max_tiles);
        return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    }
#endif
    for (uint32_t f = 0; f < p->nfields; ++f) {
        if (p->size[f]) continue;
        launch(k_unpack_var_chars, dim3(kVarGrid), dim3(kBlock), 0, s, wire, wire_len, str_offs[f],
               tiles + a.sidx[f] * L.max_tiles, spos + a.sidx[f] * n, n, static_cast<uint8_t*>(cols[f]),
               static_cast<const uint64_t*>(nullptr), 0u, reinterpret_cast<const uint32_t*>(tiles),
               static_cast<const uint32_t*>(nullptr));
    }
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int srpc_gpu_unpack_var(const srpc_plan* p, const uint8_t* wire, uint64_t wire_len, uint64_t n,
                        const uint64_t* rec_offs, void* const* cols, uint64_t* const* str_offs,
                        srpc_unpack_status* st, void* scratch, uint64_t scratch_bytes, void* stream) {
    return srpc_gpu_unpack_var_tiled(p, wire, wire_len, n, rec_offs, nullptr, cols, str_offs, st, scratch,
                                     scratch_bytes, stream);
}

int srpc_var_tile_table_words(const srpc_plan* p, uint64_t n, uint64_t* out) {
    if (!p || !out || !p->has_string) return SRPC_E_INVALID;
    *out = ((n + kBlock - 1) / kBlock + 1) * p->nstrings;
    return SRPC_OK;
}

int srpc_gpu_var_tile_table(const srpc_plan* p, const uint64_t* const* str_offs, uint64_t n, uint64_t* table,
                            void* stream) {
    const TimedCall timed;
    if (!p || !p->has_string || !str_offs || !table) return SRPC_E_INVALID;
    if (!aligned(table, 8)) return SRPC_E_ALIGN;
    TileTableArgs t{};
    uint32_t si = 0;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        if (p->size[f]) continue;
        if (!str_offs[f] || !aligned(str_offs[f], 8)) return SRPC_E_INVALID;
        t.soff[si++] = str_offs[f];
    }
    t.ns = p->nstrings;
    const uint64_t entries = ((n + kBlock - 1) / kBlock + 1) * t.ns;
    launch(k_tile_table, dim3(static_cast<uint32_t>(std::min<uint64_t>((entries + 255) / 256, 4096))), dim3(256), 0,
           static_cast<hipStream_t>(stream), t, n, table, entries);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

}  // extern "C"
