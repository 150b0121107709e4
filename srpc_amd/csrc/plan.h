// plan.h -- internal: the srpc_plan object and helpers shared by the kernel
// translation units of libsrpc_gpu.so (srpc_gpu.hip: fixed-size records,
// var.hip: records with string fields).  Not part of the public ABI.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>

#include "srpc_gpu.h"

namespace srpc_impl {

constexpr int kBlock = 256;          // 4 waves of 64
constexpr int kMaxFields = SRPC_MAX_FIELDS;
constexpr int kMaxDwords = 8;        // DWORD path: records of up to 32 bytes
constexpr uint32_t kTileTarget = 8192;   // TILE path: ~8 KiB LDS image per tile
constexpr uint32_t kMaxTileStride = 2048;
constexpr uint32_t kMaxPrefix = SRPC_MAX_PREFIX;
// every schema within the limits has a TILE kernel (records of <= 1280 bytes)
static_assert(kMaxPrefix + 8u * kMaxFields <= kMaxTileStride, "fixed records within the limits fit a tile");

// Variant bits (srpc_plan_tune SRPC_TUNE_NT): non-temporal stores / loads.
constexpr int kNtStore = 1;
constexpr int kNtLoad = 2;

// DWORD-path variant: records per lane (1 or 4), iterations per lane, NT bits.
// Default = the fastest in the steady-state bench loop on MI355X (16M Quad,
// profiles/r01_tune.log): one record per lane, one iteration, non-temporal
// loads and stores (streamed bytes are touched once per kernel).
struct DwordVariant {
    int rpl = 1;
    int iter = 1;
    int nt = kNtStore | kNtLoad;
    int grid = 0;  // 0: one workgroup per 256*iter records; >0: at most this many (grid-stride)
};

__device__ __forceinline__ void report_bad(srpc_unpack_status* st, uint32_t flag, uint64_t rec) {
    atomicOr(&st->flags, flag);
    atomicMin(reinterpret_cast<unsigned long long*>(&st->first_bad_record),
              static_cast<unsigned long long>(rec));
}

inline int kind_size(int32_t k) {
    switch (k) {
    case SRPC_KIND_BOOL:
    case SRPC_KIND_INT8:
    case SRPC_KIND_CHAR: return 1;
    case SRPC_KIND_INT16: return 2;
    case SRPC_KIND_INT32: return 4;
    case SRPC_KIND_INT64: return 8;
    case SRPC_KIND_STRING: return 0;
    default: return -1;
    }
}

inline uint32_t gcd_u32(uint32_t a, uint32_t b) {
    while (b) {
        uint32_t t = a % b;
        a = b;
        b = t;
    }
    return a;
}

inline uint32_t ilog2(uint32_t s) { return s == 1 ? 0 : s == 2 ? 1 : s == 4 ? 2 : 3; }

inline bool aligned(const void* p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) & (a - 1)) == 0; }

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// Kernel timing armed by srpc_time_next_call: the data-path kernels of the
// next C-ABI call on this host thread are launched with hipExtLaunchKernel,
// which writes the dispatch packet's own begin/end timestamps into the
// events -- kernel-only time, the same interval rocprofv3 --kernel-trace
// reports, with no event packets between the launches being timed.
struct LaunchTimer {
    hipEvent_t start = nullptr;
    hipEvent_t stop = nullptr;
    bool armed = false;
    bool started = false;
    int depth = 0;  // C-ABI calls in progress (one calls another: srpc_gpu_unpack_var_stream)
};

inline LaunchTimer& launch_timer() {
    static thread_local LaunchTimer t;
    return t;
}

// Disarms the timer when the outermost C-ABI call returns (whatever it and
// the calls it made launched).
struct TimedCall {
    TimedCall() { ++launch_timer().depth; }
    ~TimedCall() {
        LaunchTimer& t = launch_timer();
        if (--t.depth <= 0) t = LaunchTimer{};
    }
};

// Launch a data-path kernel: the first launch of an armed call stamps
// `start`, every launch stamps `stop` (the last one wins).
template <typename K, typename... Args>
inline void launch(K kernel, dim3 grid, dim3 block, uint32_t lds, hipStream_t s, Args... args) {
    LaunchTimer& t = launch_timer();
    if (t.armed) {
        hipExtLaunchKernelGGL(kernel, grid, block, lds, s, t.started ? nullptr : t.start, t.stop, 0u, args...);
        t.started = true;
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
    }
}

// ---- LDS byte access with aligned instructions (every file's kernels) ----
// The k <= 8 low bytes of v at LDS byte d, each byte written once, with the
// widest naturally aligned stores that fit.
__device__ __forceinline__ void lds_put_small(uint8_t* lds, uint32_t d, uint64_t v, uint32_t k) {
    if (k && (d & 1)) {
        lds[d] = static_cast<uint8_t>(v);
        v >>= 8;
        ++d;
        --k;
    }
    if (k >= 2 && (d & 2)) {
        *reinterpret_cast<uint16_t*>(lds + d) = static_cast<uint16_t>(v);
        v >>= 16;
        d += 2;
        k -= 2;
    }
    while (k >= 4) {
        *reinterpret_cast<uint32_t*>(lds + d) = static_cast<uint32_t>(v);
        v >>= 32;
        d += 4;
        k -= 4;
    }
    if (k >= 2) {
        *reinterpret_cast<uint16_t*>(lds + d) = static_cast<uint16_t>(v);
        v >>= 16;
        d += 2;
        k -= 2;
    }
    if (k) lds[d] = static_cast<uint8_t>(v);
}

// 8 bytes at any LDS byte offset from three aligned dword reads and two byte
// funnel shifts: a misaligned ds_read_b64 costs ~6x an aligned one on gfx950
// (profiles/r01_lds_unaligned.log).  Reads up to 4 bytes past the value,
// inside the LDS allocation.
__device__ __forceinline__ uint64_t lds_u64(const uint8_t* lds, uint32_t off) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(lds + (off & ~3u));
    const uint32_t s = off & 3;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
    return (static_cast<uint64_t>(__builtin_amdgcn_alignbyte(w2, w1, s)) << 32) | __builtin_amdgcn_alignbyte(w1, w0, s);
}

// LDS bytes [s, s + len) -> LDS bytes [d, d + len): aligned dword stores in
// the body, each built from two aligned dword loads of the source and a byte
// funnel shift (the load may read up to 3 bytes past the run, inside the LDS
// allocation, never used).
__device__ __forceinline__ void lds_copy_run(uint8_t* lds, uint32_t d, uint32_t s, uint32_t len) {
    while (len && (d & 3)) {
        lds[d++] = lds[s++];
        --len;
    }
    if (len >= 4) {
        const uint32_t sa = s & 3;
        const uint32_t* sw = reinterpret_cast<const uint32_t*>(lds + (s - sa));
        uint32_t* dw = reinterpret_cast<uint32_t*>(lds + d);
        const uint32_t nd = len >> 2;
        uint32_t w0 = sw[0];
        for (uint32_t k = 0; k < nd; ++k) {
            const uint32_t w1 = sw[k + 1];
            dw[k] = sa ? __builtin_amdgcn_alignbyte(w1, w0, sa) : w0;
            w0 = w1;
        }
        d += 4 * nd;
        s += 4 * nd;
        len &= 3;
    }
    while (len--) lds[d++] = lds[s++];
}

}  // namespace srpc_impl

// The object behind the opaque srpc_plan* of include/srpc_gpu.h.
struct srpc_plan {
    int device = 0;
    uint32_t nfields = 0;
    int32_t kinds[srpc_impl::kMaxFields] = {};
    uint32_t size[srpc_impl::kMaxFields] = {};
    uint32_t off[srpc_impl::kMaxFields] = {};   // offset within record, prefix included
    uint32_t prefix_len = 0;
    uint8_t h_prefix[srpc_impl::kMaxPrefix] = {};
    uint8_t* d_prefix = nullptr;       // device copy (d_prefix_alloc + 16, zero-padded 16 B each side)
    uint8_t* d_prefix_alloc = nullptr;
    uint8_t* d_period = nullptr;     // TILE: template | mask of one period lcm(stride, 16) (prefixed schemas)
    uint64_t stride = 0;             // fixed record bytes (0 for string schemas)
    bool has_string = false;
    bool dword_ok = false;
    int path = 0;
    uint32_t tile_R = 0, tile_L = 0;
    int tile_grid = 0;               // resident workgroups for grid-stride tiles
    bool tile_full_grid = true;      // image kernels: one workgroup per tile
    int tile_lb = 8;                 // pack image kernel: 16-byte column loads in flight per lane
    int tile_flat_k = 0;             // pack: flat kernel's loads per lane (0 = per-field kernel)
    uint32_t ptile_R = 0;            // pack image kernel: records per tile
    size_t ptile_lds = 0;
    size_t tile_lds = 0;
    // TILE wave tiles (one wave per tile), per direction; R = 0: workgroup tiles
    struct WaveTile {
        uint32_t R = 0;              // records per tile
        size_t lds = 0;
        int k = 0, kw = 0;           // column chunks / wire chunks per lane
    } wtp, wtu;                      // pack, unpack
    bool all4 = false;              // every field 4 bytes (DWORD x4 variant eligible)
    int rec_id = -1;                 // TILE: schema-specialised kernels (rec.hip), -1 none
    bool rec_pack = false, rec_unpack = false;  // ... used for pack / unpack
    srpc_impl::DwordVariant dv;      // DWORD-path variant (srpc_plan_tune)
    // string schemas (SRPC_PATH_VAR)
    uint32_t nstrings = 0;
    uint32_t fixed_bytes = 0;        // prefix + fixed fields + 8 per string field
    int var_kernel = 1;              // SRPC_TUNE_VAR_KERNEL: 1 record tiles (one pass), 0 scan + chunk walk
    bool var_rt_general = false;     // unpack: record tiles for short records too (A/B)
    uint32_t rt_img_cap = 0;         // record tiles: LDS image bytes, 0 = from wire_cap / n (SRPC_TUNE_VAR_IMAGE_BYTES)
    uint32_t rt_ch_cap = 0;          // record tiles: LDS chars stage bytes (SRPC_TUNE_VAR_CHARS_BYTES)
    bool rt_ch_cap_auto = true;      //   ... or what the image's span can hold
};
