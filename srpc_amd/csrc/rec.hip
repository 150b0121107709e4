// rec.hip -- schema-specialised TILE kernels for common fixed record layouts
// (pack_struct of a record's fields behind the
// request / response envelope, reference packer.hpp:77-91,172-191).
//
// The generic TILE kernels (srpc_gpu.hip) move a field's 16-byte column
// chunks into an LDS image of the tile's records element by element, at
// unaligned LDS offsets decided at run time: for a record of mixed widths
// (the 17-byte all-kinds record) that is byte-wide LDS traffic and a chain of
// runtime switches per chunk, and the kernel stalls on it with HBM idle
// (profiles/r02_pmc_all_kinds_flat.txt).  Here the record layout is a
// template -- envelope prefix length P and the field sizes S... -- so every
// byte's place is known at compile time:
//
//   pack:   lane l of a wave loads the G records' worth of every column
//           (coalesced: consecutive lanes, consecutive column bytes), builds
//           the G wire records as G*stride/4 dwords in registers (byte
//           permutes the compiler folds into v_perm / v_alignbyte; prefix
//           bytes are wave-uniform kernel arguments), writes them to LDS at
//           l*G*stride with dword stores (an odd dword stride for the 17- and
//           53-byte records: no bank conflicts), and the wave streams the
//           image out with 16-byte non-temporal stores.
//   unpack: the mirror: 16-byte wire loads -> LDS -> each lane's G records as
//           dwords -> every column's G values -> coalesced column stores; the
//           prefix bytes are compared in registers and the first mismatching
//           record is reported.
//
// A tile is one wave (a workgroup of 64 lanes: no barriers, the image needs
// only the wave's own LDS ordering) and K groups of G records per lane.  The
// kernels cover whole tiles only; the host runs the generic kernels on the
// remainder (tail records).  Which layouts get an instance: the ones the
// benchmarks and the reference's examples use (rec_kernel_for below).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>
#include <utility>

#include "plan.h"
#include "rec.h"
#include "srpc_gpu.h"

namespace srpc_impl {
namespace {

constexpr int kRecMaxPrefix = 64;

// fn(std::integral_constant<int, i>) for i in [0, N): a loop whose index is a
// compile-time constant (template arguments inside the body).
template <int... I, class Fn>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, I...>, Fn&& fn) {
    (fn(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
    static_for_impl(std::make_integer_sequence<int, N>{}, fn);
}

struct RecArgs {
    const uint8_t* col[8];
    uint8_t pre[kRecMaxPrefix];  // the envelope prefix (P bytes used)
};

template <int P, int... S>
struct Lay {
    static constexpr int NF = sizeof...(S);
    static constexpr int SZ[NF] = {S...};
    static constexpr int STRIDE = P + (S + ...);
    static constexpr int off(int f) {
        int o = P;
        for (int i = 0; i < f; ++i) o += SZ[i];
        return o;
    }
    static constexpr int field_of(int b) {
        int o = P;
        for (int i = 0; i < NF; ++i) {
            if (b < o + SZ[i]) return i;
            o += SZ[i];
        }
        return NF - 1;
    }
};

typedef uint32_t v2u __attribute__((ext_vector_type(2)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

// N bytes (a multiple of 4) at p -> d[0 .. N/4)
template <int N>
__device__ __forceinline__ void load_bytes(const uint8_t* p, uint32_t* d) {
    if constexpr (N == 4) {
        d[0] = *reinterpret_cast<const uint32_t*>(p);
    } else if constexpr (N == 8) {
        const v2u v = *reinterpret_cast<const v2u*>(p);
        d[0] = v.x;
        d[1] = v.y;
    } else {
        static_assert(N % 16 == 0, "column slice of 4, 8 or 16k bytes");
#pragma unroll
        for (int i = 0; i < N / 16; ++i) {
            const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p) + i);
            d[4 * i] = v.x;
            d[4 * i + 1] = v.y;
            d[4 * i + 2] = v.z;
            d[4 * i + 3] = v.w;
        }
    }
}

template <int N>
__device__ __forceinline__ void store_bytes(uint8_t* p, const uint32_t* d) {
    if constexpr (N == 4) {
        *reinterpret_cast<uint32_t*>(p) = d[0];
    } else if constexpr (N == 8) {
        *reinterpret_cast<v2u*>(p) = v2u{d[0], d[1]};
    } else {
        static_assert(N % 16 == 0, "column slice of 4, 8 or 16k bytes");
#pragma unroll
        for (int i = 0; i < N / 16; ++i)
            __builtin_nontemporal_store(v4u{d[4 * i], d[4 * i + 1], d[4 * i + 2], d[4 * i + 3]},
                                        reinterpret_cast<v4u*>(p) + i);
    }
}

__device__ __forceinline__ uint32_t byte_of(const uint32_t* w, int i) { return (w[i >> 2] >> (8 * (i & 3))) & 0xffu; }

// Dword offset of field f's G values in a lane's column buffer.
template <class L, int G>
constexpr int col_base(int f) {
    int b = 0;
    for (int i = 0; i < f; ++i) b += G * L::SZ[i] / 4;
    return b;
}
template <class L, int G>
constexpr int col_dwords() {
    return col_base<L, G>(L::NF);
}

// Lane columns (G values of each field) -> G wire records as dwords.
template <class L, int G>
__device__ __forceinline__ void build_records(const RecArgs& a, const uint32_t* in, uint32_t* w) {
#pragma unroll
    for (int d = 0; d < G * L::STRIDE / 4; ++d) {
        uint32_t v = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int j = 4 * d + i, r = j / L::STRIDE, b = j % L::STRIDE;
            uint32_t byte;
            if (b < L::off(0)) {
                byte = a.pre[b];
            } else {
                const int f = L::field_of(b), k = b - L::off(f);
                byte = byte_of(in + col_base<L, G>(f), r * L::SZ[f] + k);
            }
            v |= byte << (8 * i);
        }
        w[d] = v;
    }
}

// G wire records (dwords) -> lane columns; returns a mask of the records
// whose prefix differs from the plan's.
template <class L, int G>
__device__ __forceinline__ uint32_t split_records(const RecArgs& a, const uint32_t* w, uint32_t* out) {
#pragma unroll
    for (int f = 0; f < L::NF; ++f) {
#pragma unroll
        for (int d = 0; d < G * L::SZ[f] / 4; ++d) {
            uint32_t v = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int j = 4 * d + i, r = j / L::SZ[f], k = j % L::SZ[f];
                v |= byte_of(w, r * L::STRIDE + L::off(f) + k) << (8 * i);
            }
            out[col_base<L, G>(f) + d] = v;
        }
    }
    uint32_t bad = 0;
    if constexpr (L::off(0) > 0) {
#pragma unroll
        for (int r = 0; r < G; ++r) {
            uint32_t x = 0;
#pragma unroll
            for (int b = 0; b < L::off(0); ++b) x |= byte_of(w, r * L::STRIDE + b) ^ a.pre[b];
            bad |= (x ? 1u : 0u) << r;
        }
    }
    return bad;
}

constexpr int kRecWave = 64;

__device__ __forceinline__ void rec_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <class L, int G, int K>
__global__ __launch_bounds__(kRecWave) void k_pack_rec(RecArgs a, uint8_t* __restrict__ wire) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int TR = kRecWave * G * K;  // records per tile
    constexpr int W = G * L::STRIDE / 4;  // dwords of a lane's G records
    const uint32_t lane = threadIdx.x;
    const uint64_t tile = blockIdx.x;
    uint32_t in[K][col_dwords<L, G>()];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t q = (tile * K + k) * kRecWave + lane;  // the lane's group of G records
        static_for<L::NF>([&](auto fc) {
            constexpr int f = decltype(fc)::value;
            load_bytes<G * L::SZ[f]>(a.col[f] + q * (G * L::SZ[f]), in[k] + col_base<L, G>(f));
        });
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint32_t w[W];
        build_records<L, G>(a, in[k], w);
        uint32_t* dst = reinterpret_cast<uint32_t*>(lds + (k * kRecWave + lane) * (G * L::STRIDE));
#pragma unroll
        for (int d = 0; d < W; ++d) dst[d] = w[d];
    }
    rec_wave_sync();
    constexpr int CH = TR * L::STRIDE / 16;
    uint8_t* out = wire + tile * (static_cast<uint64_t>(TR) * L::STRIDE);
#pragma unroll
    for (int c0 = 0; c0 < CH; c0 += kRecWave) {
        const int c = c0 + static_cast<int>(lane);
        if (c0 + kRecWave <= CH || c < CH) {
            const v4u v = reinterpret_cast<const v4u*>(lds)[c];
            __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(out) + c);
        }
    }
}

template <class L, int G, int K>
__global__ __launch_bounds__(kRecWave) void k_unpack_rec(RecArgs a, const uint8_t* __restrict__ wire,
                                                         srpc_unpack_status* st) {
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    constexpr int TR = kRecWave * G * K;
    constexpr int W = G * L::STRIDE / 4;
    constexpr int CH = TR * L::STRIDE / 16;
    constexpr int PER = (CH + kRecWave - 1) / kRecWave;
    const uint32_t lane = threadIdx.x;
    const uint64_t tile = blockIdx.x;
    const uint8_t* src = wire + tile * (static_cast<uint64_t>(TR) * L::STRIDE);
    v4u v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int c = u * kRecWave + static_cast<int>(lane);
        if (c < CH) v[u] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(src) + c);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int c = u * kRecWave + static_cast<int>(lane);
        if (c < CH) reinterpret_cast<v4u*>(lds)[c] = v[u];
    }
    rec_wave_sync();
    uint32_t first_bad = ~0u;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint32_t w[W];
        const uint32_t* s = reinterpret_cast<const uint32_t*>(lds + (k * kRecWave + lane) * (G * L::STRIDE));
#pragma unroll
        for (int d = 0; d < W; ++d) w[d] = s[d];
        uint32_t out[col_dwords<L, G>()];
        const uint32_t bad = split_records<L, G>(a, w, out);
        const uint64_t q = (tile * K + k) * kRecWave + lane;
        if (bad && first_bad == ~0u) first_bad = static_cast<uint32_t>(k * kRecWave * G) + __builtin_ctz(bad);
        static_for<L::NF>([&](auto fc) {
            constexpr int f = decltype(fc)::value;
            store_bytes<G * L::SZ[f]>(const_cast<uint8_t*>(a.col[f]) + q * (G * L::SZ[f]), out + col_base<L, G>(f));
        });
    }
    if (st && first_bad != ~0u) {
        // first_bad encodes (round k, record r of the lane's group): record index
        const uint32_t k = first_bad / (kRecWave * G), r = first_bad % (kRecWave * G);
        report_bad(st, SRPC_STATUS_PREFIX, tile * TR + (static_cast<uint64_t>(k) * kRecWave + lane) * G + r);
    }
}

// ---- enveloped records: pack straight into 16-byte wire chunks --------------
// A request record is mostly its envelope (49-55 of 53-63 bytes are the same
// in every record), so the wire is a periodic template -- 16 records = S
// chunks of 16 bytes -- with each record's field bytes (one run of V <= 16
// bytes after the P >= 16 prefix bytes: at most one run meets a chunk) merged
// in.  A lane per chunk: the period's template chunk from LDS, the run's
// record and offset from the chunk index (32-bit math on constants), its
// field values loaded from the columns, a masked 128-bit merge, one
// non-temporal 16-byte store.  No LDS image, no barrier after the template:
// the generic TILE pack scatters 4-byte values into its image at odd offsets
// (misaligned LDS stores) and is at 0.71-0.75 of peak on these layouts.
template <class L, int U>
__global__ __launch_bounds__(kBlock) void k_pack_env(RecArgs a, uint8_t* __restrict__ wire, uint64_t nch) {
    constexpr int S = L::STRIDE, P = L::off(0), V = S - P;
    static_assert(P >= 16 && V <= 16 && V % 4 == 0, "one value run of whole dwords per 16-byte chunk");
    typedef unsigned __int128 u128;
    __shared__ uint32_t tmpl[4 * S];  // one period: S chunks = 16 records
    for (int t = threadIdx.x; t < 4 * S; t += kBlock) {
        uint32_t v = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int b = (4 * t + j) % S;
            v |= (b < P ? static_cast<uint32_t>(a.pre[b]) : 0u) << (8 * j);
        }
        tmpl[t] = v;
    }
    __syncthreads();
    const uint64_t c0 = static_cast<uint64_t>(blockIdx.x) * (U * kBlock) + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t c = c0 + static_cast<uint64_t>(u) * kBlock;
        if (c >= nch) break;
        const uint64_t T = c / S;                                  // period: records 16 T ..
        const uint32_t tc = static_cast<uint32_t>(c - T * S);     // chunk in the period
        const uint32_t lb = 16 * tc;                               // its first byte in the period
        const v4u tv = reinterpret_cast<const v4u*>(tmpl)[tc];
        u128 out = (static_cast<u128>((static_cast<uint64_t>(tv.w) << 32) | tv.z) << 64) |
                   ((static_cast<uint64_t>(tv.y) << 32) | tv.x);
        const int32_t e = static_cast<int32_t>(lb) + 15 - P;      // >= 0: some run starts by the chunk's end
        if (e >= 0) {
            const uint32_t lr = static_cast<uint32_t>(e) / S;      // that record, in the period
            const int32_t o = static_cast<int32_t>(S * lr + P) - static_cast<int32_t>(lb);  // (-V, 16)
            if (o + V > 0) {
                const uint64_t r = 16 * T + lr;
                u128 val = 0;
                static_for<L::NF>([&](auto fc) {
                    constexpr int f = decltype(fc)::value;
                    constexpr int at = L::off(f) - P;
                    static_assert(L::SZ[f] == 4 || L::SZ[f] == 8, "dword fields");
                    if constexpr (L::SZ[f] == 4) {
                        const uint32_t x = reinterpret_cast<const uint32_t*>(a.col[f])[r];
                        val |= static_cast<u128>(x) << (8 * at);
                    } else {
                        const uint64_t x = reinterpret_cast<const uint64_t*>(a.col[f])[r];
                        val |= static_cast<u128>(x) << (8 * at);
                    }
                });
                u128 m = V == 16 ? ~static_cast<u128>(0) : ((static_cast<u128>(1) << (8 * V)) - 1);
                if (o >= 0) {
                    val <<= 8 * o;
                    m <<= 8 * o;
                } else {
                    val >>= -8 * o;
                    m >>= -8 * o;
                }
                out = (out & ~m) | (val & m);
            }
        }
        const uint64_t lo = static_cast<uint64_t>(out), hi = static_cast<uint64_t>(out >> 64);
        __builtin_nontemporal_store(v4u{static_cast<uint32_t>(lo), static_cast<uint32_t>(lo >> 32),
                                        static_cast<uint32_t>(hi), static_cast<uint32_t>(hi >> 32)},
                                    reinterpret_cast<v4u*>(wire) + c);
    }
}

constexpr int kEnvU = 4;  // chunks per lane

// ---- instances ---------------------------------------------------------------
struct RecKernel {
    bool use_pack, use_unpack;  // measured faster than the generic kernels (rec_default)
    int prefix_len;
    int nf;
    int size[8];
    int tile_records;
    size_t lds;
    void (*pack)(RecArgs, uint8_t*);
    void (*unpack)(RecArgs, const uint8_t*, srpc_unpack_status*);
    void (*env_pack)(RecArgs, uint8_t*, uint64_t);  // enveloped layouts: the chunk pack (16-record periods)
    int stride;
};

template <class L, int G, int K>
constexpr RecKernel make_rec(bool use_pack, bool use_unpack) {
    RecKernel r{use_pack, use_unpack, L::off(0), L::NF, {}, kRecWave * G * K, static_cast<size_t>(kRecWave) * G * K * L::STRIDE,
                k_pack_rec<L, G, K>, k_unpack_rec<L, G, K>, nullptr, L::STRIDE};
    for (int f = 0; f < L::NF; ++f) r.size[f] = L::SZ[f];
    return r;
}
template <class L, int G, int K>
constexpr RecKernel make_rec_env(bool use_pack, bool use_unpack) {
    RecKernel r = make_rec<L, G, K>(use_pack, use_unpack);
    r.env_pack = k_pack_env<L, kEnvU>;
    return r;
}

// all_kinds {bool, int8, char, int16, int32, int64} (17 B); Number behind the
// square request (49-byte prefix, 53 B) and a response (15-byte prefix, 19
// B); TwoNumbers behind the add request (50-byte prefix), the subtract /
// multiply requests (55) and a response (19).  A layout matches by prefix
// length and field sizes, whatever the prefix bytes.
const RecKernel kRec[] = {
    // (pack, unpack): where each measured faster than the generic TILE kernels
    // (profiles/r03_paths_rec_ab.log, profiles/r04_rec_unpack_ab.log;
    // differences under ~0.02 of peak are noise).  Tile depth K: the records
    // behind an envelope unpack best one round per wave (K = 1: a 53-63 byte
    // record's tile is ~14 KiB of LDS, ~11 waves per CU instead of ~5 at K =
    // 2), the short responses at K = 2.
    make_rec<Lay<0, 1, 1, 1, 2, 4, 8>, 4, 4>(true, true),  // 0.64 / 0.68 -> 0.80 / 0.72
    make_rec_env<Lay<49, 4>, 4, 1>(true, true),             // unpack 0.76 -> 0.77; pack 0.715 -> 0.755 (chunk kernel)
    make_rec<Lay<15, 4>, 4, 2>(false, true),                // 0.74 -> 0.77
    make_rec_env<Lay<50, 4, 4>, 4, 1>(true, true),          // 0.72 (K = 2) -> 0.76; pack 0.75 -> 0.765 (chunk)
    make_rec<Lay<55, 4, 4>, 4, 1>(false, true),             // 0.69 -> 0.78; pack: the generic TILE kernel
                                                            // (0.77-0.79; the chunk kernel 0.74, r05)
    make_rec<Lay<19, 4, 4>, 4, 2>(false, true),             // 0.76 (K = 4) -> 0.78
};
constexpr int kNumRec = sizeof(kRec) / sizeof(kRec[0]);

}  // namespace

int rec_kernel_for(const srpc_plan* p) {
    if (!p || p->has_string || p->prefix_len > static_cast<uint32_t>(kRecMaxPrefix) || p->nfields > 8) return -1;
    for (int i = 0; i < kNumRec; ++i) {
        const RecKernel& r = kRec[i];
        if (r.prefix_len != static_cast<int>(p->prefix_len) || r.nf != static_cast<int>(p->nfields)) continue;
        bool same = true;
        for (uint32_t f = 0; f < p->nfields; ++f) same = same && r.size[f] == static_cast<int>(p->size[f]);
        if (same) return i;
    }
    return -1;
}

bool rec_default(int id, bool pack) {
    return id >= 0 && id < kNumRec && (pack ? kRec[id].use_pack : kRec[id].use_unpack);
}

uint64_t rec_tile_records(int id, bool pack) {
    if (id < 0 || id >= kNumRec) return 0;
    return pack && kRec[id].env_pack ? 16 : static_cast<uint64_t>(kRec[id].tile_records);
}

static RecArgs rec_args(const srpc_plan* p, const void* const* cols) {
    RecArgs a{};
    for (uint32_t f = 0; f < p->nfields; ++f) a.col[f] = static_cast<const uint8_t*>(cols[f]);
    for (uint32_t i = 0; i < p->prefix_len; ++i) a.pre[i] = p->h_prefix[i];
    return a;
}

int rec_pack(int id, const srpc_plan* p, const void* const* cols, uint64_t tiles, uint8_t* wire, hipStream_t s) {
    if (id < 0 || id >= kNumRec || !tiles) return SRPC_OK;
    if (tiles > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
    const RecKernel& r = kRec[id];
    if (r.env_pack) {  // tiles of 16 records = `stride` 16-byte chunks
        const uint64_t nch = tiles * static_cast<uint64_t>(r.stride);
        const uint64_t g = (nch + kEnvU * kBlock - 1) / (kEnvU * kBlock);
        if (g > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
        launch(r.env_pack, dim3(static_cast<uint32_t>(g)), dim3(kBlock), 0, s, rec_args(p, cols), wire, nch);
        return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
    }
    launch(r.pack, dim3(static_cast<uint32_t>(tiles)), dim3(kRecWave), static_cast<uint32_t>(r.lds), s, rec_args(p, cols),
           wire);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

int rec_unpack(int id, const srpc_plan* p, const uint8_t* wire, uint64_t tiles, void* const* cols,
               srpc_unpack_status* st, hipStream_t s) {
    if (id < 0 || id >= kNumRec || !tiles) return SRPC_OK;
    if (tiles > 0x7fffffffull) return SRPC_E_UNSUPPORTED;
    const RecKernel& r = kRec[id];
    launch(r.unpack, dim3(static_cast<uint32_t>(tiles)), dim3(kRecWave), static_cast<uint32_t>(r.lds), s,
           rec_args(p, reinterpret_cast<const void* const*>(cols)), wire, st);
    return hipGetLastError() == hipSuccess ? SRPC_OK : SRPC_E_HIP;
}

}  // namespace srpc_impl
