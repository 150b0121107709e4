// aos.hip -- fixed-size records packed from / unpacked into an array of the
// caller's own structs (AoS) in device memory.
//
// A C++ caller of the reference holds std::vector<T> and packs with
// `packer p; for (r : recs) p << r;` (packer.hpp:73 -> pack_struct 172-178).
// Going through SoA columns costs a host-side transpose (host_columns in
// include/srpc/gpu.hpp: 14 ns per Quad record, 87 ns per multiple_primitives
// record, profiles/r02_host_columns.log) that dwarfs the GPU pack.  Here the
// struct array itself is the input: the caller copies the raw bytes of its
// vector to the device (one DMA) and the kernel reads each leaf field at its
// byte offset inside T; unpack writes only the leaf fields' bytes into a
// device copy of the array (everything else -- vtable pointer, padding --
// stays as the copy brought it), which the caller copies back.
//
// Kernels (struct array 16-byte aligned, the usual case): a workgroup owns a
// tile of R records (R a multiple of 16, so the tile's struct bytes are whole
// 16-byte pieces).  Both the tile's struct bytes and its wire bytes move
// between HBM and LDS in coalesced 16-byte pieces; the fields move between
// the two LDS images, one struct per lane.  Pack: structs -> LDS, fields ->
// wire image, wire image (+ the envelope prefix from the plan's periodic
// template) -> HBM.  Unpack: wire -> LDS (prefix checked), fields -> struct
// image, struct image -> HBM; when the leaf fields do not cover every byte of
// the struct (padding, a vtable pointer) the struct tile is read first so
// those bytes are written back unchanged.  When the struct's layout is the
// wire body's (same offsets and stride, no prefix -- e.g. Quad) the two images
// are one and the kernels are tile copies.  When the fields are one run of the
// struct (Quad behind a vtable pointer), one lane moves each record's run
// straight between HBM arrays (k_pack_aos_run).  A struct array that is only
// naturally aligned takes the per-field kernels (one struct per lane, fields
// straight between HBM and the wire image).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "plan.h"
#include "srpc_gpu.h"

namespace srpc_impl {
namespace {

constexpr uint32_t kAosFillMax = 256;  // struct bytes srpc_gpu_unpack_aos_fill takes as its fill record

struct AosArgs {
    uint32_t roff[kMaxFields];  // leaf field offset inside the caller's struct
    uint32_t size[kMaxFields];  // 1, 2, 4 or 8
    uint32_t woff[kMaxFields];  // offset inside the wire record (prefix included)
    const uint8_t* period;      // template | mask of one period (prefix_len > 0)
    uint32_t nfields, wstride, rstride, prefix_len, R, L;
    uint32_t simg;              // staged kernels: LDS offset of the struct image (0: the wire image's, ident)
    bool ident;                 // struct layout == wire layout
    bool cover;                 // the leaf fields cover every byte of the struct
    int32_t boff;               // >= 0: the wire body is struct bytes [boff, boff + wstride) (no prefix)
    bool fill;                  // unpack into fresh objects: bytes no field covers come from fillw
    uint32_t fill_at;           // staged kernels: LDS offset of the fill bytes
    uint32_t fillw[kAosFillMax / 4];  // the fill record (rstride bytes, zero padded)
};

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t load_field(const uint8_t* p, uint32_t sz) {
    switch (sz) {  // naturally aligned (checked on the host)
    case 1: return *p;
    case 2: return *reinterpret_cast<const uint16_t*>(p);
    case 4: return *reinterpret_cast<const uint32_t*>(p);
    default: return *reinterpret_cast<const uint64_t*>(p);
    }
}

__device__ __forceinline__ void store_field(uint8_t* p, uint64_t v, uint32_t sz) {
    switch (sz) {
    case 1: *p = static_cast<uint8_t>(v); break;
    case 2: *reinterpret_cast<uint16_t*>(p) = static_cast<uint16_t>(v); break;
    case 4: *reinterpret_cast<uint32_t*>(p) = static_cast<uint32_t>(v); break;
    default: *reinterpret_cast<uint64_t*>(p) = v; break;
    }
}

__device__ __forceinline__ void load_period(const AosArgs& a, uint8_t* tmpl) {
    for (uint32_t i = threadIdx.x; i < (2 * a.L) >> 4; i += kBlock)
        reinterpret_cast<uint4*>(tmpl)[i] = reinterpret_cast<const uint4*>(a.period)[i];
}

__global__ __launch_bounds__(kBlock) void k_pack_aos(AosArgs a, const uint8_t* __restrict__ recs,
                                                     uint8_t* __restrict__ wire, uint64_t n) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* tmpl = lds + a.R * a.wstride;
    uint8_t* mask = tmpl + a.L;
    if (a.prefix_len) load_period(a, tmpl);
    const uint64_t rbase = static_cast<uint64_t>(blockIdx.x) * a.R;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
    // structs -> image, one struct per lane (consecutive lanes, consecutive structs)
    for (uint32_t e = threadIdx.x; e < nr; e += kBlock) {
        const uint8_t* src = recs + (rbase + e) * a.rstride;
        const uint32_t d = e * a.wstride;
        for (uint32_t f = 0; f < a.nfields; ++f)
            lds_put_small(lds, d + a.woff[f], load_field(src + a.roff[f], a.size[f]), a.size[f]);
    }
    __syncthreads();
    // image (+ prefix template) -> wire, aligned 16-byte stores
    uint8_t* dst = wire + rbase * a.wstride;
    const uint32_t tbytes = nr * a.wstride, full = tbytes >> 4;
    for (uint32_t c = threadIdx.x; c < full; c += kBlock) {
        uint4 v = reinterpret_cast<const uint4*>(lds)[c];
        if (a.prefix_len) {
            const uint32_t ph = (16 * c) % a.L;
            const uint4 m = *reinterpret_cast<const uint4*>(mask + ph), t = *reinterpret_cast<const uint4*>(tmpl + ph);
            v = make_uint4((v.x & ~m.x) | t.x, (v.y & ~m.y) | t.y, (v.z & ~m.z) | t.z, (v.w & ~m.w) | t.w);
        }
        __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u*>(dst + 16 * c));
    }
    if (threadIdx.x == 0)
        for (uint32_t i = full * 16; i < tbytes; ++i) {
            const uint32_t ph = i % a.L;
            dst[i] = a.prefix_len && mask[ph] ? tmpl[ph] : lds[i];
        }
}

__global__ __launch_bounds__(kBlock) void k_unpack_aos(AosArgs a, const uint8_t* __restrict__ wire,
                                                       uint8_t* __restrict__ recs, uint64_t n,
                                                       srpc_unpack_status* st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* tmpl = lds + a.R * a.wstride;
    uint8_t* mask = tmpl + a.L;
    if (a.prefix_len) load_period(a, tmpl);
    __syncthreads();
    const uint64_t rbase = static_cast<uint64_t>(blockIdx.x) * a.R;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
    const uint8_t* src = wire + rbase * a.wstride;
    const uint32_t tbytes = nr * a.wstride, full = tbytes >> 4;
    // wire -> image, every prefix byte checked against the template
    for (uint32_t c = threadIdx.x; c < full; c += kBlock) {
        const uint4 v = reinterpret_cast<const uint4*>(src)[c];
        if (a.prefix_len && st) {
            const uint32_t ph = (16 * c) % a.L;
            const uint4 m = *reinterpret_cast<const uint4*>(mask + ph), t = *reinterpret_cast<const uint4*>(tmpl + ph);
            const uint32_t d[4] = {(v.x & m.x) ^ t.x, (v.y & m.y) ^ t.y, (v.z & m.z) ^ t.z, (v.w & m.w) ^ t.w};
            for (uint32_t w = 0; w < 4; ++w)
                if (d[w]) {
                    const uint32_t i = 16 * c + 4 * w + (__builtin_ctz(d[w]) >> 3);
                    report_bad(st, SRPC_STATUS_PREFIX, rbase + i / a.wstride);
                    break;
                }
        }
        reinterpret_cast<uint4*>(lds)[c] = v;
    }
    if (threadIdx.x == 0)
        for (uint32_t i = full * 16; i < tbytes; ++i) {
            const uint8_t b = src[i];
            const uint32_t ph = i % a.L;
            if (a.prefix_len && st && (b & mask[ph]) != tmpl[ph]) report_bad(st, SRPC_STATUS_PREFIX, rbase + i / a.wstride);
            lds[i] = b;
        }
    __syncthreads();
    // image -> the leaf fields of the structs (nothing else in them is written)
    for (uint32_t e = threadIdx.x; e < nr; e += kBlock) {
        uint8_t* dst = recs + (rbase + e) * a.rstride;
        const uint32_t s = e * a.wstride;
        for (uint32_t f = 0; f < a.nfields; ++f) store_field(dst + a.roff[f], lds_u64(lds, s + a.woff[f]), a.size[f]);
    }
}

// A struct whose leaf fields sit back to back in wire order (Quad behind a
// vtable pointer: bytes 8..23 of 24) and no prefix: each record is one run of
// W bytes, moved between the struct array and the wire in 8-byte pieces
// straight from HBM to HBM, one record per lane (no LDS: the wire side is
// contiguous, the struct side is strided runs the L2 merges into lines).
template <uint32_t W>
__global__ __launch_bounds__(kBlock) void k_pack_aos_run(const uint8_t* __restrict__ recs, uint32_t rstride,
                                                         uint32_t boff, uint8_t* __restrict__ wire, uint64_t n) {
    const uint64_t e = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (e >= n) return;
    const uint64_t* s = reinterpret_cast<const uint64_t*>(recs + e * rstride + boff);
    uint64_t* d = reinterpret_cast<uint64_t*>(wire + e * W);
    uint64_t v[W / 8];
#pragma unroll
    for (uint32_t k = 0; k < W / 8; ++k) v[k] = __builtin_nontemporal_load(s + k);
#pragma unroll
    for (uint32_t k = 0; k < W / 8; ++k) __builtin_nontemporal_store(v[k], d + k);
}

template <uint32_t W>
__global__ __launch_bounds__(kBlock) void k_unpack_aos_run(const uint8_t* __restrict__ wire, uint8_t* __restrict__ recs,
                                                           uint32_t rstride, uint32_t boff, uint64_t n) {
    const uint64_t e = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (e >= n) return;
    const uint64_t* s = reinterpret_cast<const uint64_t*>(wire + e * W);
    uint64_t* d = reinterpret_cast<uint64_t*>(recs + e * rstride + boff);
    uint64_t v[W / 8];
#pragma unroll
    for (uint32_t k = 0; k < W / 8; ++k) v[k] = __builtin_nontemporal_load(s + k);
#pragma unroll
    for (uint32_t k = 0; k < W / 8; ++k) __builtin_nontemporal_store(v[k], d + k);
}

// k_unpack_aos_run into fresh objects: a lane writes its WHOLE struct (the
// run from the wire, every other 8-byte word from the fill record), so the
// lanes' stores cover whole lines and nothing of the old array is read (the
// partial-struct writes of k_unpack_aos_run make the memory system read every
// line they touch: ~64 bytes moved per 40 algorithmic for Quad + vptr).
template <uint32_t W>
__global__ __launch_bounds__(kBlock) void k_unpack_aos_run_fill(const uint8_t* __restrict__ wire,
                                                                uint8_t* __restrict__ recs, AosArgs a, uint64_t n) {
    const uint64_t e = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (e >= n) return;
    const uint64_t* s = reinterpret_cast<const uint64_t*>(wire + e * W);
    uint64_t* d = reinterpret_cast<uint64_t*>(recs + e * a.rstride);
    uint64_t v[W / 8];
#pragma unroll
    for (uint32_t k = 0; k < W / 8; ++k) v[k] = __builtin_nontemporal_load(s + k);
    // plain stores: the L2 merges a wave's strided 8-byte pieces into whole
    // lines (non-temporal ones stream out partial lines: 0.27 of peak)
    const uint32_t b0 = static_cast<uint32_t>(a.boff) >> 3, nw = a.rstride >> 3;  // uniform
    for (uint32_t k = 0; k < b0; ++k)
        d[k] = static_cast<uint64_t>(a.fillw[2 * k]) | (static_cast<uint64_t>(a.fillw[2 * k + 1]) << 32);
#pragma unroll
    for (uint32_t k = 0; k < W / 8; ++k) d[b0 + k] = v[k];
    for (uint32_t k = b0 + W / 8; k < nw; ++k)
        d[k] = static_cast<uint64_t>(a.fillw[2 * k]) | (static_cast<uint64_t>(a.fillw[2 * k + 1]) << 32);
}

// k_unpack_aos_run(_fill) with whole-line stores: a wave per 256 structs,
// the wire tile in LDS; lane c writes bytes [16c, 16c + 16) of the tile's
// structs (every store instruction covers 1 KiB of the array contiguously),
// each dword from the run (the LDS tile) or, outside it, from the fill record
// (fresh objects) or the array itself (in place: a coalesced load of the
// piece when it has such a dword).  Struct stride and run offset multiples of
// 8, the array 16-byte aligned.
template <uint32_t W, bool kFill>
__global__ __launch_bounds__(64, 8) void k_unpack_aos_run_piece(const uint8_t* __restrict__ wire,
                                                                uint8_t* __restrict__ recs, AosArgs a, uint64_t n) {
    constexpr uint32_t TR = 256;
    __shared__ __attribute__((aligned(16))) uint32_t img[TR * W / 4];
    const uint32_t lane = threadIdx.x;
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * TR;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(TR, n - t0));
    const uint32_t wbytes = nr * W;  // a multiple of 8
    const v4u* src = reinterpret_cast<const v4u*>(wire + t0 * W);
    for (uint32_t c = lane; c < wbytes / 16; c += 64) reinterpret_cast<v4u*>(img)[c] = __builtin_nontemporal_load(src + c);
    if (wbytes & 8 && lane == 0)
        reinterpret_cast<uint64_t*>(img)[wbytes / 8 - 1] = reinterpret_cast<const uint64_t*>(wire + t0 * W)[wbytes / 8 - 1];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes before its reads
    const uint32_t rs = a.rstride, boff = static_cast<uint32_t>(a.boff);
    const uint32_t obytes = nr * rs;  // a multiple of 8
    v4u* out = reinterpret_cast<v4u*>(recs + t0 * rs);
    for (uint32_t c = lane; 16 * c < obytes; c += 64) {
        const uint32_t gb = 16 * c;
        uint32_t sidx = gb / rs, ob = gb - sidx * rs;
        uint32_t o[4];
        bool need_old = false;
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const bool in_run = ob >= boff && ob < boff + W;
            o[d] = in_run ? img[(sidx * W + ob - boff) >> 2] : a.fillw[ob >> 2];
            need_old |= !in_run;
            ob += 4;
            if (ob == rs) {
                ob = 0;
                ++sidx;
            }
        }
        const bool whole = gb + 16 <= obytes;
        if constexpr (!kFill) {
            if (need_old) {  // the dwords outside the run as they are
                uint32_t od[4];
                if (whole) {
                    const v4u v = out[c];
                    od[0] = v.x, od[1] = v.y, od[2] = v.z, od[3] = v.w;
                } else {
                    od[0] = reinterpret_cast<const uint32_t*>(out + c)[0];
                    od[1] = reinterpret_cast<const uint32_t*>(out + c)[1];
                    od[2] = od[3] = 0;
                }
                uint32_t ob2 = gb - (gb / rs) * rs;
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    if (!(ob2 >= boff && ob2 < boff + W)) o[d] = od[d];
                    ob2 += 4;
                    if (ob2 == rs) ob2 = 0;
                }
            }
        }
        if (whole) {
            out[c] = v4u{o[0], o[1], o[2], o[3]};
        } else {  // the array's last 8 bytes
            reinterpret_cast<uint32_t*>(out + c)[0] = o[0];
            reinterpret_cast<uint32_t*>(out + c)[1] = o[1];
        }
    }
}

// The fill record into every struct of [0, n) (the per-field fallback's first
// pass when unpacking into fresh objects): a lane per 4 bytes, or per byte.
__global__ __launch_bounds__(kBlock) void k_aos_fill(uint8_t* __restrict__ recs, AosArgs a, uint64_t n) {
    __shared__ uint32_t f[kAosFillMax / 4];
    if (threadIdx.x < kAosFillMax / 4) f[threadIdx.x] = a.fillw[threadIdx.x];
    __syncthreads();
    const uint64_t bytes = n * a.rstride, gs = static_cast<uint64_t>(gridDim.x) * kBlock;
    const uint64_t i0 = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (a.rstride % 4 == 0 && (reinterpret_cast<uintptr_t>(recs) & 3) == 0) {
        const uint32_t rw = a.rstride / 4;
        for (uint64_t i = i0; i < bytes / 4; i += gs) reinterpret_cast<uint32_t*>(recs)[i] = f[i % rw];
    } else {
        const uint8_t* fb = reinterpret_cast<const uint8_t*>(f);
        for (uint64_t i = i0; i < bytes; i += gs) recs[i] = fb[i % a.rstride];
    }
}

// A/B switch (SRPC_AOS_RUN_PIECE=0 at load): the run kernels' unpack without
// the piece kernel.
const bool g_aos_run_piece = [] {
    const char* e = std::getenv("SRPC_AOS_RUN_PIECE");
    return !(e && e[0] == '0');
}();

// The run kernels for wire bodies of 8, 16, 24 or 32 bytes (8-byte aligned
// struct array, stride and body offset), else false.
bool launch_aos_run(const AosArgs& a, bool pack, const uint8_t* src, uint8_t* dst, uint64_t n, hipStream_t s) {
    if (a.boff < 0 || (a.wstride != 8 && a.wstride != 16 && a.wstride != 24 && a.wstride != 32) || a.rstride % 8 ||
        a.boff % 8 || !aligned(src, 8) || !aligned(dst, 8))
        return false;
    const uint64_t g = (n + kBlock - 1) / kBlock;
    if (g > 0x7fffffffull) return false;
    const uint32_t boff = static_cast<uint32_t>(a.boff);
    // unpack: whole-line piece stores when the array is 16-byte aligned and
    // the struct fits the fill record (the run kernels' strided stores: 0.65
    // into fresh objects, profiles/r04z_aos_piece_ab.log)
    const uint64_t gpn = (n + 255) / 256;
    // (16-byte wire loads: the wire 16-byte aligned too, else the lane-per-struct kernels)
    const bool pieces = !pack && g_aos_run_piece && aligned(dst, 16) && aligned(src, 16) && a.rstride <= kAosFillMax &&
                        gpn <= 0x7fffffffull;
    const dim3 gp(static_cast<uint32_t>(gpn));
#define SRPC_AOS_RUN(Wb)                                                                                         \
    if (a.wstride == Wb) {                                                                                       \
        if (pack) launch(k_pack_aos_run<Wb>, dim3(static_cast<uint32_t>(g)), dim3(kBlock), 0, s, src, a.rstride, \
                         boff, dst, n);                                                                          \
        else if (pieces && a.fill) launch(k_unpack_aos_run_piece<Wb, true>, gp, dim3(64), 0, s, src, dst, a, n);  \
        else if (pieces) launch(k_unpack_aos_run_piece<Wb, false>, gp, dim3(64), 0, s, src, dst, a, n);           \
        else if (a.fill) launch(k_unpack_aos_run_fill<Wb>, dim3(static_cast<uint32_t>(g)), dim3(kBlock), 0, s,  \
                                src, dst, a, n);                                                         \
        else launch(k_unpack_aos_run<Wb>, dim3(static_cast<uint32_t>(g)), dim3(kBlock), 0, s, src, dst,         \
                    a.rstride, boff, n);                                                                         \
        return true;                                                                                             \
    }
    SRPC_AOS_RUN(8)
    SRPC_AOS_RUN(16)
    SRPC_AOS_RUN(24)
    SRPC_AOS_RUN(32)
#undef SRPC_AOS_RUN
    return false;
}

// ---- layouts known at compile time -------------------------------------------
// The staged kernels below move each field between the two LDS images at
// offsets known only at run time (byte-wide LDS traffic, ~55% bank conflicts
// on the all-kinds struct: profiles/r04_pmc_aos.txt).  For the struct layouts
// the benchmarks and the reference's examples use, the layout is a template
// instead (as rec.hip does for columns): a lane holds G structs in registers
// (16-byte PLAIN loads straight from HBM: the wave's loads cover whole lines,
// which stay in the caches between its instructions -- non-temporal loads
// refetched them, 0.35 of peak; staging the struct side through LDS instead
// measured 0.70 pack / 0.41 fresh-object unpack: profiles/r04_aos_lay_ab.log), builds
// its G wire records as dwords with byte permutes fixed at compile time, and
// the wave streams its wire tile through LDS in coalesced 16-byte pieces (an
// odd dword stride per lane: no bank conflicts).  Unpack is the mirror; bytes
// of a struct no field covers come from the fill record (fresh objects) or
// from the struct itself (in place: the lane reads it first).  That mirror's
// strided whole-struct stores ran 0.78 on some boxes and 0.41 on others, so
// the default unpack is k_unpack_aos_piece below (a lane per 16-byte piece of
// the array: whole-line stores, 0.69 on a 0.41 box).
struct AosLayAllKindsV {  // {vtable*, bool, int8, char, int16, int32, int64}: 32 bytes
    static constexpr int RS = 32, NF = 6;
    static constexpr int ROFF[NF] = {8, 9, 10, 12, 16, 24}, SZ[NF] = {1, 1, 1, 2, 4, 8};
};
struct AosLayAllKinds {  // the same without the vtable slot: 24 bytes
    static constexpr int RS = 24, NF = 6;
    static constexpr int ROFF[NF] = {0, 1, 2, 4, 8, 16}, SZ[NF] = {1, 1, 1, 2, 4, 8};
};

template <class L>
struct AosT {
    static constexpr int WS = [] {
        int w = 0;
        for (int f = 0; f < L::NF; ++f) w += L::SZ[f];
        return w;
    }();
    static constexpr int woff(int f) {
        int o = 0;
        for (int i = 0; i < f; ++i) o += L::SZ[i];
        return o;
    }
    static constexpr int wfield(int b) {  // field of wire byte b
        int o = 0;
        for (int i = 0; i < L::NF; ++i) {
            if (b < o + L::SZ[i]) return i;
            o += L::SZ[i];
        }
        return L::NF - 1;
    }
    static constexpr int rfield(int b) {  // field of struct byte b, or -1
        for (int i = 0; i < L::NF; ++i)
            if (b >= L::ROFF[i] && b < L::ROFF[i] + L::SZ[i]) return i;
        return -1;
    }
    static constexpr bool dword_used(int d) {  // dword d of a lane's structs holds a field byte
        for (int b = 4 * d; b < 4 * d + 4; ++b)
            if (rfield(b % L::RS) >= 0) return true;
        return false;
    }
    static constexpr bool piece_used(int q) {  // 16-byte piece q of a lane's structs holds a field byte
        return dword_used(4 * q) || dword_used(4 * q + 1) || dword_used(4 * q + 2) || dword_used(4 * q + 3);
    }
};

__device__ __forceinline__ uint32_t aos_byte(const uint32_t* w, int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xffu; }

constexpr int kAosLayG = 4;  // structs per lane
constexpr int kAosWave = 64;

template <class L>
__global__ __launch_bounds__(kAosWave, 8) void k_pack_aos_lay(const uint8_t* __restrict__ recs, uint8_t* __restrict__ wire,
                                                          uint64_t n) {
    using T = AosT<L>;
    constexpr int G = kAosLayG, SD = G * L::RS / 4, WD = G * T::WS / 4, TR = kAosWave * G;
    static_assert((G * L::RS) % 16 == 0 && L::RS % 4 == 0 && (G * T::WS) % 4 == 0,
                  "16-byte pieces of a lane's structs, whole wire dwords per lane");
    __shared__ __attribute__((aligned(16))) uint32_t img[kAosWave * WD + 4];
    const uint32_t lane = threadIdx.x;
    const uint64_t r0 = static_cast<uint64_t>(blockIdx.x) * TR + lane * G;  // the lane's first struct
    uint32_t sd[SD] = {};
    if (r0 + G <= n) {  // the lane's structs in 16-byte pieces (those holding a field byte)
        const v4u* src = reinterpret_cast<const v4u*>(recs + r0 * L::RS);
#pragma unroll
        for (int q = 0; q < SD / 4; ++q) {
            if (!T::piece_used(q)) continue;
            const v4u v = src[q];  // plain: the wave's strided pieces share lines (non-temporal ones refetch them)
            sd[4 * q] = v.x;
            sd[4 * q + 1] = v.y;
            sd[4 * q + 2] = v.z;
            sd[4 * q + 3] = v.w;
        }
    } else {  // the array's last lane: its structs below n, a dword at a time
        const uint32_t* src = reinterpret_cast<const uint32_t*>(recs + r0 * L::RS);
#pragma unroll
        for (int d = 0; d < SD; ++d)
            if (T::dword_used(d) && r0 + (4 * d) / L::RS < n) sd[d] = src[d];
    }
#pragma unroll
    for (int d = 0; d < WD; ++d) {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = 4 * d + i, r = j / T::WS, b = j % T::WS, f = T::wfield(b);
            v |= aos_byte(sd, r * L::RS + L::ROFF[f] + (b - T::woff(f))) << (8 * i);
        }
        img[lane * WD + d] = v;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes before its reads
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * TR;
    const uint64_t nr = min<uint64_t>(TR, n - t0);
    const uint32_t bytes = static_cast<uint32_t>(nr) * T::WS, full = bytes >> 4;
    uint8_t* dst = wire + t0 * T::WS;
    for (uint32_t c = lane; c < full; c += kAosWave) {
        const v4u v = reinterpret_cast<const v4u*>(img)[c];
        __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(dst) + c);
    }
    for (uint32_t i = 16 * full + lane; i < bytes; i += kAosWave) dst[i] = reinterpret_cast<const uint8_t*>(img)[i];
}

template <class L, bool kFill>
__global__ __launch_bounds__(kAosWave) void k_unpack_aos_lay(const uint8_t* __restrict__ wire, uint8_t* __restrict__ recs,
                                                            uint64_t n, AosArgs a) {
    using T = AosT<L>;
    constexpr int G = kAosLayG, SD = G * L::RS / 4, WD = G * T::WS / 4, TR = kAosWave * G;
    __shared__ __attribute__((aligned(16))) uint32_t img[kAosWave * WD + 4];
    const uint32_t lane = threadIdx.x;
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * TR;
    const uint64_t nr = min<uint64_t>(TR, n - t0);
    const uint32_t bytes = static_cast<uint32_t>(nr) * T::WS, full = bytes >> 4;
    const uint8_t* src = wire + t0 * T::WS;
    for (uint32_t c = lane; c < full; c += kAosWave)
        reinterpret_cast<v4u*>(img)[c] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + c);
    for (uint32_t i = 16 * full + lane; i < bytes; i += kAosWave) reinterpret_cast<uint8_t*>(img)[i] = src[i];
    const uint64_t r0 = t0 + lane * G;
    v4u* out = reinterpret_cast<v4u*>(recs + r0 * L::RS);
    // in place: the lane's structs as they are (the bytes no field covers stay)
    const bool whole = r0 + G <= n;
    uint32_t old[SD] = {};
    if constexpr (!kFill) {
        if (whole) {
#pragma unroll
            for (int q = 0; q < SD / 4; ++q) {
                const v4u v = out[q];
                old[4 * q] = v.x;
                old[4 * q + 1] = v.y;
                old[4 * q + 2] = v.z;
                old[4 * q + 3] = v.w;
            }
        } else {
            const uint32_t* o32 = reinterpret_cast<const uint32_t*>(out);
#pragma unroll
            for (int d = 0; d < SD; ++d)
                if (r0 + (4 * d) / L::RS < n) old[d] = o32[d];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);
    uint32_t w[WD];
#pragma unroll
    for (int d = 0; d < WD; ++d) w[d] = img[lane * WD + d];
    uint32_t o[SD];
#pragma unroll
    for (int d = 0; d < SD; ++d) {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int sb = 4 * d + i, r = sb / L::RS, ob = sb % L::RS, f = T::rfield(ob);
            uint32_t byte;
            if (f >= 0) byte = aos_byte(w, r * T::WS + T::woff(f) + (ob - L::ROFF[f]));
            else if (kFill) byte = (a.fillw[ob >> 2] >> (8 * (ob & 3))) & 0xffu;
            else byte = aos_byte(old, sb);
            v |= byte << (8 * i);
        }
        o[d] = v;
    }
    if (whole) {
        // plain stores: the L2 merges the wave's strided pieces into whole lines
#pragma unroll
        for (int q = 0; q < SD / 4; ++q) out[q] = v4u{o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]};
    } else {
        uint32_t* o32 = reinterpret_cast<uint32_t*>(out);
#pragma unroll
        for (int d = 0; d < SD; ++d)
            if (r0 + (4 * d) / L::RS < n) o32[d] = o[d];
    }
}

template <class L>
bool aos_lay_match(const AosArgs& a) {
    if (a.prefix_len || a.rstride != static_cast<uint32_t>(L::RS) || a.nfields != static_cast<uint32_t>(L::NF)) return false;
    for (int f = 0; f < L::NF; ++f)
        if (a.roff[f] != static_cast<uint32_t>(L::ROFF[f]) || a.size[f] != static_cast<uint32_t>(L::SZ[f])) return false;
    return true;
}

// Unpack with whole-line stores (struct sizes a multiple of 16 bytes, P =
// RS / 16 pieces per struct): lane c of the wave writes bytes [16c, 16c + 16)
// of the tile's structs, so every store instruction covers 1 KiB of the array
// contiguously and no line is written in parts by several instructions.  The
// lane assembles its piece (half H of struct c / P) from the wire tile in LDS:
// the record bytes [lo, hi) the piece's fields come from, funnel-shifted from
// dwords; struct bytes no field covers come from the fill record (fresh
// objects) or from the struct as it is (in place: a coalesced load of the
// same piece).
template <class L, int H>
struct AosPiece {
    using T = AosT<L>;
    static constexpr int lo = [] {
        int m = T::WS;
        for (int ob = 16 * H; ob < 16 * H + 16; ++ob) {
            const int f = T::rfield(ob);
            if (f >= 0 && T::woff(f) + (ob - L::ROFF[f]) < m) m = T::woff(f) + (ob - L::ROFF[f]);
        }
        return m == T::WS ? 0 : m;
    }();
    static constexpr int hi = [] {
        int m = 0;
        for (int ob = 16 * H; ob < 16 * H + 16; ++ob) {
            const int f = T::rfield(ob);
            if (f >= 0 && T::woff(f) + (ob - L::ROFF[f]) + 1 > m) m = T::woff(f) + (ob - L::ROFF[f]) + 1;
        }
        return m;
    }();
    static constexpr int ND = hi > lo ? (hi - lo + 3) / 4 : 1;  // record dwords the piece reads
};

template <class L, int H, bool kFill>
__device__ __forceinline__ v4u aos_piece(const uint32_t* img, uint32_t srec, const v4u& old, const AosArgs& a) {
    using T = AosT<L>;
    using PC = AosPiece<L, H>;
    const uint32_t at = srec * T::WS + PC::lo, base = at >> 2, sh = at & 3;
    uint32_t raw[PC::ND + 1];
#pragma unroll
    for (int j = 0; j <= PC::ND; ++j) raw[j] = img[base + j];
    uint32_t w[PC::ND];
#pragma unroll
    for (int j = 0; j < PC::ND; ++j) w[j] = __builtin_amdgcn_alignbyte(raw[j + 1], raw[j], sh);
    const uint32_t od[4] = {old.x, old.y, old.z, old.w};
    uint32_t o[4];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ob = 16 * H + 4 * d + i, f = T::rfield(ob);
            uint32_t byte;
            if (f >= 0) byte = aos_byte(w, T::woff(f) + (ob - L::ROFF[f]) - PC::lo);
            else if (kFill) byte = (a.fillw[ob >> 2] >> (8 * (ob & 3))) & 0xffu;
            else byte = (od[d] >> (8 * i)) & 0xffu;
            v |= byte << (8 * i);
        }
        o[d] = v;
    }
    return v4u{o[0], o[1], o[2], o[3]};
}

template <class L, bool kFill>
__global__ __launch_bounds__(kAosWave, 8) void k_unpack_aos_piece(const uint8_t* __restrict__ wire,
                                                                  uint8_t* __restrict__ recs, uint64_t n, AosArgs a) {
    using T = AosT<L>;
    constexpr int G = kAosLayG, WD = G * T::WS / 4, TR = kAosWave * G, P = L::RS / 16;
    static_assert(L::RS % 16 == 0 && (P == 1 || P == 2), "structs of 16 or 32 bytes");
    __shared__ __attribute__((aligned(16))) uint32_t img[kAosWave * WD + 8];
    const uint32_t lane = threadIdx.x;
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * TR;
    const uint64_t nr = min<uint64_t>(TR, n - t0);
    const uint32_t bytes = static_cast<uint32_t>(nr) * T::WS, full = bytes >> 4;
    const uint8_t* src = wire + t0 * T::WS;
    for (uint32_t c = lane; c < full; c += kAosWave)
        reinterpret_cast<v4u*>(img)[c] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + c);
    for (uint32_t i = 16 * full + lane; i < bytes; i += kAosWave) reinterpret_cast<uint8_t*>(img)[i] = src[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes before its reads
    v4u* out = reinterpret_cast<v4u*>(recs + t0 * L::RS);
    const uint32_t npieces = static_cast<uint32_t>(nr) * P;
#pragma unroll
    for (int k = 0; k < TR * P / kAosWave; ++k) {
        const uint32_t c = lane + kAosWave * k;
        if (c >= npieces) break;
        v4u old{0, 0, 0, 0};
        if constexpr (!kFill) old = out[c];
        v4u v;
        if constexpr (P == 1) v = aos_piece<L, 0, kFill>(img, c, old, a);
        else v = (lane & 1) ? aos_piece<L, 1, kFill>(img, c >> 1, old, a) : aos_piece<L, 0, kFill>(img, c >> 1, old, a);
        out[c] = v;
    }
}

// The layout kernels for a struct array that matches one (16-byte aligned
// array and wire), else false.  Unpack: umode 1 takes the per-lane struct
// kernel, umode 2 the whole-line piece kernel where the struct size allows it
// (else false: the staged kernels).
template <class L>
bool launch_aos_lay1(const AosArgs& a, bool pack, const uint8_t* src, uint8_t* dst, uint64_t n, hipStream_t s,
                     int umode) {
    if (!aos_lay_match<L>(a)) return false;
    const uint64_t g = (n + kAosWave * kAosLayG - 1) / (kAosWave * kAosLayG);
    if (g > 0x7fffffffull) return false;
    const dim3 grid(static_cast<uint32_t>(g));
    constexpr bool kPieces = L::RS == 16 || L::RS == 32;
    if constexpr (!kPieces) {
        if (!pack && umode == 2) return false;  // the staged kernels (coalesced stores)
    } else {
        if (!pack && umode == 2) {
            if (a.fill) launch(k_unpack_aos_piece<L, true>, grid, dim3(kAosWave), 0, s, src, dst, n, a);
            else launch(k_unpack_aos_piece<L, false>, grid, dim3(kAosWave), 0, s, src, dst, n, a);
            return true;
        }
    }
    if (pack) launch(k_pack_aos_lay<L>, grid, dim3(kAosWave), 0, s, src, dst, n);
    else if (a.fill) launch(k_unpack_aos_lay<L, true>, grid, dim3(kAosWave), 0, s, src, dst, n, a);
    else launch(k_unpack_aos_lay<L, false>, grid, dim3(kAosWave), 0, s, src, dst, n, a);
    return true;
}

bool launch_aos_lay(const AosArgs& a, bool pack, const uint8_t* src, uint8_t* dst, uint64_t n, hipStream_t s,
                    int umode = 0) {
    if (!aligned(src, 16) || !aligned(dst, 16)) return false;
    return launch_aos_lay1<AosLayAllKindsV>(a, pack, src, dst, n, s, umode) ||
           launch_aos_lay1<AosLayAllKinds>(a, pack, src, dst, n, s, umode);
}

// HBM bytes [0, bytes) of a tile -> LDS (16-byte pieces, then single bytes).
__device__ __forceinline__ void tile_in(uint8_t* lds, const uint8_t* __restrict__ g, uint32_t bytes) {
    const uint32_t full = bytes >> 4;
    for (uint32_t c = threadIdx.x; c < full; c += kBlock)
        reinterpret_cast<v4u*>(lds)[c] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(g) + c);
    for (uint32_t i = full * 16 + threadIdx.x; i < bytes; i += kBlock) lds[i] = g[i];
}

// LDS -> HBM bytes [0, bytes) of a tile.
__device__ __forceinline__ void tile_out(uint8_t* __restrict__ g, const uint8_t* lds, uint32_t bytes) {
    const uint32_t full = bytes >> 4;
    for (uint32_t c = threadIdx.x; c < full; c += kBlock) {
        const uint4 v = reinterpret_cast<const uint4*>(lds)[c];
        __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u*>(g + 16 * c));
    }
    for (uint32_t i = full * 16 + threadIdx.x; i < bytes; i += kBlock) g[i] = lds[i];
}

// Wire image (+ prefix template) -> wire, aligned 16-byte stores.
__device__ __forceinline__ void wire_out(const AosArgs& a, const uint8_t* img, const uint8_t* tmpl, const uint8_t* mask,
                                         uint8_t* __restrict__ dst, uint32_t tbytes) {
    const uint32_t full = tbytes >> 4;
    for (uint32_t c = threadIdx.x; c < full; c += kBlock) {
        uint4 v = reinterpret_cast<const uint4*>(img)[c];
        if (a.prefix_len) {
            const uint32_t ph = (16 * c) % a.L;
            const uint4 m = *reinterpret_cast<const uint4*>(mask + ph), t = *reinterpret_cast<const uint4*>(tmpl + ph);
            v = make_uint4((v.x & ~m.x) | t.x, (v.y & ~m.y) | t.y, (v.z & ~m.z) | t.z, (v.w & ~m.w) | t.w);
        }
        __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u*>(dst + 16 * c));
    }
    for (uint32_t i = full * 16 + threadIdx.x; i < tbytes; i += kBlock) {
        const uint32_t ph = i % a.L;
        dst[i] = a.prefix_len && mask[ph] ? tmpl[ph] : img[i];
    }
}

// Wire -> wire image, every prefix byte checked against the template.
__device__ __forceinline__ void wire_in(const AosArgs& a, uint8_t* img, const uint8_t* tmpl, const uint8_t* mask,
                                        const uint8_t* __restrict__ src, uint32_t tbytes, uint64_t rbase,
                                        srpc_unpack_status* st) {
    const uint32_t full = tbytes >> 4;
    for (uint32_t c = threadIdx.x; c < full; c += kBlock) {
        const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + c);
        const uint4 v = make_uint4(w.x, w.y, w.z, w.w);
        if (a.prefix_len && st) {
            const uint32_t ph = (16 * c) % a.L;
            const uint4 m = *reinterpret_cast<const uint4*>(mask + ph), t = *reinterpret_cast<const uint4*>(tmpl + ph);
            const uint32_t d[4] = {(v.x & m.x) ^ t.x, (v.y & m.y) ^ t.y, (v.z & m.z) ^ t.z, (v.w & m.w) ^ t.w};
            for (uint32_t w = 0; w < 4; ++w)
                if (d[w]) {
                    const uint32_t i = 16 * c + 4 * w + (__builtin_ctz(d[w]) >> 3);
                    report_bad(st, SRPC_STATUS_PREFIX, rbase + i / a.wstride);
                    break;
                }
        }
        reinterpret_cast<uint4*>(img)[c] = v;
    }
    for (uint32_t i = full * 16 + threadIdx.x; i < tbytes; i += kBlock) {
        const uint8_t b = src[i];
        const uint32_t ph = i % a.L;
        if (a.prefix_len && st && (b & mask[ph]) != tmpl[ph]) report_bad(st, SRPC_STATUS_PREFIX, rbase + i / a.wstride);
        img[i] = b;
    }
}

// LDS: wire image (R * wstride, 16-byte rounded) | struct image at a.simg
// (unless ident) | template | mask.
__global__ __launch_bounds__(kBlock) void k_pack_aos_staged(AosArgs a, const uint8_t* __restrict__ recs,
                                                            uint8_t* __restrict__ wire, uint64_t n, uint32_t tmpl_at) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* tmpl = lds + tmpl_at;
    uint8_t* mask = tmpl + a.L;
    if (a.prefix_len) load_period(a, tmpl);
    const uint64_t rbase = static_cast<uint64_t>(blockIdx.x) * a.R;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
    uint8_t* simg = lds + a.simg;
    tile_in(simg, recs + rbase * a.rstride, nr * a.rstride);
    __syncthreads();
    if (!a.ident) {
        for (uint32_t e = threadIdx.x; e < nr; e += kBlock) {
            const uint8_t* src = simg + e * a.rstride;
            const uint32_t d = e * a.wstride;
            for (uint32_t f = 0; f < a.nfields; ++f)
                lds_put_small(lds, d + a.woff[f], load_field(src + a.roff[f], a.size[f]), a.size[f]);
        }
        __syncthreads();
    }
    wire_out(a, lds, tmpl, mask, wire + rbase * a.wstride, nr * a.wstride);
}

__global__ __launch_bounds__(kBlock) void k_unpack_aos_staged(AosArgs a, const uint8_t* __restrict__ wire,
                                                              uint8_t* __restrict__ recs, uint64_t n,
                                                              srpc_unpack_status* st, uint32_t tmpl_at) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    uint8_t* tmpl = lds + tmpl_at;
    uint8_t* mask = tmpl + a.L;
    if (a.prefix_len) load_period(a, tmpl);
    const uint64_t rbase = static_cast<uint64_t>(blockIdx.x) * a.R;
    const uint32_t nr = static_cast<uint32_t>(min<uint64_t>(a.R, n - rbase));
    uint8_t* simg = lds + a.simg;
    uint8_t* g = recs + rbase * a.rstride;
    if (!a.ident && !a.cover) {
        if (a.fill) {  // fresh objects: the fill record, repeated (no read of the old structs)
            uint32_t* fl = reinterpret_cast<uint32_t*>(lds + a.fill_at);
            if (threadIdx.x < kAosFillMax / 4) fl[threadIdx.x] = a.fillw[threadIdx.x];
            __syncthreads();
            const uint32_t tb = nr * a.rstride;
            if (a.rstride % 4 == 0) {
                const uint32_t rw = a.rstride / 4;
                for (uint32_t i = threadIdx.x; i < tb / 4; i += kBlock) reinterpret_cast<uint32_t*>(simg)[i] = fl[i % rw];
            } else {
                const uint8_t* fb = lds + a.fill_at;
                for (uint32_t i = threadIdx.x; i < tb; i += kBlock) simg[i] = fb[i % a.rstride];
            }
        } else {
            tile_in(simg, g, nr * a.rstride);  // bytes no field covers are written back as they were
        }
    }
    __syncthreads();  // the template, before wire_in reads it
    wire_in(a, lds, tmpl, mask, wire + rbase * a.wstride, nr * a.wstride, rbase, st);
    __syncthreads();
    if (!a.ident) {
        for (uint32_t e = threadIdx.x; e < nr; e += kBlock) {
            uint8_t* dst = simg + e * a.rstride;
            const uint32_t s = e * a.wstride;
            for (uint32_t f = 0; f < a.nfields; ++f) store_field(dst + a.roff[f], lds_u64(lds, s + a.woff[f]), a.size[f]);
        }
        __syncthreads();
    }
    tile_out(g, simg, nr * a.rstride);
}

// Staged-kernel tiling: R (a multiple of 16) records whose two images fill
// about kAosTileBytes of LDS; returns the LDS bytes, sets a->R / a->simg.
constexpr uint32_t kAosTileBytes = 24 * 1024;  // (12 / 16 KiB measured slower: profiles/r04_aos_lay_ab.log)
uint32_t staged_tiling(AosArgs* a) {
    const uint32_t per = a->ident ? a->wstride : a->wstride + a->rstride;
    uint32_t R = std::max<uint32_t>(16, (kAosTileBytes / per) & ~15u);
    a->R = R;
    const uint32_t wimg = (R * a->wstride + 15) & ~15u;
    a->simg = a->ident ? 0 : wimg;
    const uint32_t end = a->ident ? wimg : wimg + ((R * a->rstride + 15) & ~15u);
    a->fill_at = end + (a->prefix_len ? 2 * a->L : 0);
    return a->fill_at + (a->fill ? kAosFillMax : 0);
}

__global__ void k_aos_status(srpc_unpack_status* st, uint32_t flags, uint64_t first_bad) {
    if (threadIdx.x == 0) {
        st->flags = flags;
        st->reserved = 0;
        st->first_bad_record = first_bad;
    }
}

// Validates the layout and fills the kernel arguments.
int aos_args(const srpc_plan* p, const void* recs, uint64_t stride, const uint32_t* offs, AosArgs* a) {
    if (!p || p->has_string || !offs || stride == 0 || stride > 0xffffffffull) return SRPC_E_INVALID;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        const uint32_t sz = p->size[f];
        if (offs[f] + static_cast<uint64_t>(sz) > stride) return SRPC_E_INVALID;
        if (offs[f] % sz || stride % sz || !aligned(recs, sz)) return SRPC_E_ALIGN;  // natural alignment, as in C++ structs
        a->roff[f] = offs[f];
        a->size[f] = sz;
        a->woff[f] = p->off[f];
    }
    a->period = p->d_period;
    a->nfields = p->nfields;
    a->wstride = static_cast<uint32_t>(p->stride);
    a->rstride = static_cast<uint32_t>(stride);
    a->prefix_len = p->prefix_len;
    a->L = p->tile_L;
    a->ident = p->prefix_len == 0 && stride == p->stride;
    uint64_t covered = 0;
    for (uint32_t f = 0; f < p->nfields; ++f) {
        a->ident = a->ident && offs[f] == p->off[f];
        covered += p->size[f];
    }
    // fields do not overlap (each has its own bytes in a C++ struct), so they
    // cover the struct when their sizes add up to its stride
    a->cover = covered == stride;
    // the body as one run of the struct: every field at the same shift from its wire offset
    a->boff = -1;
    if (p->prefix_len == 0 && p->nfields && offs[0] >= p->off[0]) {
        const uint32_t sh = offs[0] - p->off[0];
        bool run = sh + p->stride <= stride;
        for (uint32_t f = 0; f < p->nfields; ++f) run = run && offs[f] == p->off[f] + sh;
        if (run) a->boff = static_cast<int32_t>(sh);
    }
    return SRPC_OK;
}

// A/B switch (SRPC_AOS_FILL_STAGED=1 at load): fresh-object unpacks of run
// layouts take the staged kernels instead of k_unpack_aos_run_fill.
const bool g_aos_fill_staged = [] {
    const char* e = std::getenv("SRPC_AOS_FILL_STAGED");
    return e && e[0] == '1';
}();

// A/B switch (SRPC_AOS_UNSTAGED=1 in the environment at load): the per-field kernels only.
const bool g_aos_unstaged = [] {
    const char* e = std::getenv("SRPC_AOS_UNSTAGED");
    return e && e[0] == '1';
}();

// Which kernels unpack takes for the layouts above (SRPC_AOS_LAY_UNPACK=N at
// load, or the srpc_debug_aos_lay_unpack test hook): 0 the staged ones, 1 the
// per-lane struct kernel, 2 (default) the whole-line piece kernel.
std::atomic<int> g_aos_lay_unpack{[] {
    const char* e = std::getenv("SRPC_AOS_LAY_UNPACK");
    return e && e[0] >= '0' && e[0] <= '2' ? e[0] - '0' : 2;
}()};

// A/B switch (SRPC_AOS_NOLAY=1 at load): the staged kernels for the layouts above too.
const bool g_aos_nolay = [] {
    const char* e = std::getenv("SRPC_AOS_NOLAY");
    return e && e[0] == '1';
}();

}  // namespace
}  // namespace srpc_impl

using namespace srpc_impl;

extern "C" {

int srpc_gpu_pack_aos(const srpc_plan* p, const void* d_records, uint64_t record_stride,
                      const uint32_t* field_offsets, uint64_t n, uint8_t* d_wire, uint64_t wire_cap, void* stream) {
    const TimedCall timed;
    AosArgs a{};
    if (int rc = aos_args(p, d_records, record_stride, field_offsets, &a)) return rc;
    if (n == 0) return SRPC_OK;
    if (!d_records || !d_wire) return SRPC_E_INVALID;
    if (n > UINT64_MAX / p->stride || n * p->stride > wire_cap) return SRPC_E_CAPACITY;
    if (!aligned(d_wire, 16)) return SRPC_E_ALIGN;
    if (!a.ident && !g_aos_unstaged &&
        launch_aos_run(a, true, static_cast<const uint8_t*>(d_records), d_wire, n, static_cast<hipStream_t>(stream)))
        return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    if (!g_aos_unstaged && !g_aos_nolay &&
        launch_aos_lay(a, true, static_cast<const uint8_t*>(d_records), d_wire, n, static_cast<hipStream_t>(stream)))
        return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    if (aligned(d_records, 16) && !g_aos_unstaged) {
        const uint32_t lds = staged_tiling(&a);
        const uint64_t tiles = (n + a.R - 1) / a.R;
        if (tiles > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
        launch(k_pack_aos_staged, dim3(static_cast<uint32_t>(tiles)), dim3(kBlock), lds, static_cast<hipStream_t>(stream),
               a, static_cast<const uint8_t*>(d_records), d_wire, n, lds - (a.prefix_len ? 2 * a.L : 0));
        return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    }
    a.R = p->ptile_R;
    const uint64_t tiles = (n + a.R - 1) / a.R;
    if (tiles > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
    launch(k_pack_aos, dim3(static_cast<uint32_t>(tiles)), dim3(kBlock), static_cast<uint32_t>(p->ptile_lds),
           static_cast<hipStream_t>(stream), a, static_cast<const uint8_t*>(d_records), d_wire, n);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

static int unpack_aos(const srpc_plan* p, const uint8_t* d_wire, uint64_t wire_len, uint64_t n, void* d_records,
                      uint64_t record_stride, const uint32_t* field_offsets, const void* h_fill,
                      srpc_unpack_status* d_status, void* stream) {
    const TimedCall timed;
    AosArgs a{};
    if (int rc = aos_args(p, d_records, record_stride, field_offsets, &a)) return rc;
    if (h_fill && !a.ident && !a.cover) {  // a struct the fields cover needs no fill
        if (record_stride > kAosFillMax) return SRPC_E_UNSUPPORTED;
        std::memcpy(a.fillw, h_fill, record_stride);
        a.fill = true;
    }
    auto s = static_cast<hipStream_t>(stream);
    if (d_status) hipLaunchKernelGGL(k_aos_status, dim3(1), dim3(64), 0, s, d_status, 0u, ~0ull);
    if (n == 0) return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    if (!d_records || !d_wire) return SRPC_E_INVALID;
    if (!aligned(d_wire, 16)) return SRPC_E_ALIGN;
    uint64_t n_fit = wire_len / p->stride;
    int ret = SRPC_OK;
    if (n_fit < n) {  // the records that fit are decoded; the status names the first that does not
        if (d_status) hipLaunchKernelGGL(k_aos_status, dim3(1), dim3(64), 0, s, d_status, SRPC_STATUS_BOUNDS, n_fit);
        ret = SRPC_ERR_BOUNDS;
    } else {
        n_fit = n;
    }
    if (n_fit && !a.ident && !g_aos_unstaged && !(a.fill && g_aos_fill_staged) &&
        launch_aos_run(a, false, d_wire, static_cast<uint8_t*>(d_records), n_fit, s))
        return hipGetLastError() == hipSuccess ? ret : SRPC_E_HIP;
    // the layout kernels: the 32-byte struct a lane per 16-byte piece
    // (whole-line stores: 0.69 into fresh objects where the lane-per-struct
    // kernel's strided stores run 0.41 and the staged kernels 0.55,
    // profiles/r04z_aos_piece_ab.log); the 24-byte one takes the staged kernels
    const int umode = g_aos_lay_unpack.load(std::memory_order_relaxed);
    if (n_fit && !g_aos_unstaged && !g_aos_nolay && umode &&
        launch_aos_lay(a, false, d_wire, static_cast<uint8_t*>(d_records), n_fit, s, umode))
        return hipGetLastError() == hipSuccess ? ret : SRPC_E_HIP;
    if (n_fit && aligned(d_records, 16) && !g_aos_unstaged) {
        const uint32_t lds = staged_tiling(&a);
        const uint64_t tiles = (n_fit + a.R - 1) / a.R;
        if (tiles > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
        launch(k_unpack_aos_staged, dim3(static_cast<uint32_t>(tiles)), dim3(kBlock), lds, s, a, d_wire,
               static_cast<uint8_t*>(d_records), n_fit, d_status, a.fill_at - (a.prefix_len ? 2 * a.L : 0));
    } else if (n_fit) {
        a.R = p->tile_R;
        const uint64_t tiles = (n_fit + a.R - 1) / a.R;
        if (tiles > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
        if (a.fill)  // the per-field kernel writes only the fields: fill every struct first
            launch(k_aos_fill, dim3(static_cast<uint32_t>(std::min<uint64_t>(tiles, 8192))), dim3(kBlock), 0, s,
                   static_cast<uint8_t*>(d_records), a, n_fit);
        launch(k_unpack_aos, dim3(static_cast<uint32_t>(tiles)), dim3(kBlock), static_cast<uint32_t>(p->tile_lds), s, a,
               d_wire, static_cast<uint8_t*>(d_records), n_fit, d_status);
    }
    return hipGetLastError() == hipSuccess ? ret : SRPC_E_HIP;
}

int srpc_gpu_unpack_aos(const srpc_plan* p, const uint8_t* d_wire, uint64_t wire_len, uint64_t n,
                        void* d_records, uint64_t record_stride, const uint32_t* field_offsets,
                        srpc_unpack_status* d_status, void* stream) {
    return unpack_aos(p, d_wire, wire_len, n, d_records, record_stride, field_offsets, nullptr, d_status, stream);
}

int srpc_gpu_unpack_aos_fill(const srpc_plan* p, const uint8_t* d_wire, uint64_t wire_len, uint64_t n,
                             void* d_records, uint64_t record_stride, const uint32_t* field_offsets,
                             const void* h_fill, srpc_unpack_status* d_status, void* stream) {
    if (!h_fill) return SRPC_E_INVALID;
    return unpack_aos(p, d_wire, wire_len, n, d_records, record_stride, field_offsets, h_fill, d_status, stream);
}

// Test hook (not part of the C ABI in include/): which kernels unpack takes
// for the layout-kernel structs (0 staged, 1 per-lane structs, 2 whole-line
// pieces); returns the previous setting.
__attribute__((visibility("default"))) int srpc_debug_aos_lay_unpack(int mode) {
    return g_aos_lay_unpack.exchange(mode < 0 ? 0 : mode > 2 ? 2 : mode);
}

}  // extern "C"
