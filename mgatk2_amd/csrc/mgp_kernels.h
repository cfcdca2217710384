// mgp_kernels.h — device-side helpers shared by the engine kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mgp {

constexpr int kWave = 64;        // CDNA wavefront width (never 32)
constexpr int kBlock = 256;      // 4 waves per workgroup

// error bits accumulated in DevStats::err during a run
constexpr uint32_t ERR_UNSORTED = 1u;   // start[i] < start[i-1]
constexpr uint32_t ERR_BADREAD = 2u;    // kept read without SEQ/QUAL
constexpr uint32_t ERR_SPAN = 4u;       // CIGAR reach larger than declared span
constexpr uint32_t ERR_BADBC = 8u;      // bc >= n_cells
constexpr uint32_t ERR_OVERFLOW = 16u;  // scatter destination outside its cell segment
constexpr uint32_t ERR_PACKED = 32u;    // MGP_FLAG_PACKED record outside the packed layout's limits
constexpr uint32_t ERR_RESPEC = 64u;    // a read does not fit the speculative compact grouping (mgp_sync reruns)
constexpr uint32_t ERR_BOUNDS = 128u;   // start-bin read ranges not monotone (unsorted input): grouping and
                                        // pileup kernels exit at entry, so no slot leaves its buffer
constexpr uint32_t ERR_BADOFF = 256u;   // a pushed record (offset, header, CIGAR) lies outside its batch's payload
                                        // (k_check_records at push; set with ERR_BOUNDS: no kernel reads records)

// Counters written by the kernels of one run (zeroed at run start).
struct DevStats {
    unsigned long long dup_len;        // duplicate_reads_with_length
    unsigned long long dup_pos;        // duplicate_reads_position_only
    unsigned long long filtered;       // kept reads (after dedup)
    unsigned long long n_barcodes;     // cells with >= 1 kept read
    unsigned long long cells_passed;   // cells producing a result
    unsigned long long valid;          // reads passing flag + barcode filters
    unsigned int max_span;             // max declared span over valid reads
    unsigned int err;                  // ERR_* bits
};

// Geometry of the cell-major grouping and the position windows.
struct Geom {
    int L;        // mito_len
    int G;        // start-bin width (positions per bin)
    int nb_reg;   // ceil(L / G) regular bins; bin nb_reg holds starts >= L
    int nbins;    // nb_reg + 1
    int W;        // window width (positions), multiple of G
    int Wp;       // LDS plane pitch (odd => conflict-free plane offsets)
    int nwin;     // ceil(L / W)
    int nc;       // cells
    int cpb;      // cells per pileup workgroup
    int nchunks;  // ceil(nc / cpb)
};

__device__ __forceinline__ int bin_of(int s, const Geom& g) {
    if (s < 0) return 0;
    if (s >= g.L) return g.nb_reg;
    return s / g.G;
}

// start-bin window edges of pileup window k, given the reach R (multiple of G)
__device__ __forceinline__ int win_lo_bin(int k, int R, const Geom& g) {
    long long lo = (long long)k * g.W - R;
    return lo <= 0 ? 0 : (int)(lo / g.G);
}
__device__ __forceinline__ int win_hi_bin(int k, const Geom& g) {
    long long hi = (long long)(k + 1) * g.W / g.G;
    return hi > g.nb_reg ? g.nb_reg : (int)hi;
}

__device__ __forceinline__ unsigned long long lanemask_lt() {
    const unsigned lane = threadIdx.x & (kWave - 1);
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// The lanes of the wave holding the same key as this lane, among the `act` lanes:
// the AND over the key's bits of the ballot of the lanes that agree on the bit. One
// v_cmp per bit makes the ballot (the plain __ballot of a compound predicate costs a
// select and a second compare), and the bit itself gives the agree mask (0: set, take
// the ballot; ~0: clear, take its complement). Inactive lanes take key 0 and are
// outside the initial mask. Callers ranking several keys per lane run the bit steps
// of all their keys together (independent dependency chains).
struct PeerAcc {
    uint32_t kv, lo, hi;
};
__device__ __forceinline__ PeerAcc peer_begin(bool act, uint32_t key) {
    const unsigned long long vb = __ballot(act);
    return PeerAcc{act ? key : 0u, (uint32_t)vb, (uint32_t)(vb >> 32)};
}
__device__ __forceinline__ void peer_bit(PeerAcc& p, int bit) {
    const uint32_t x = (p.kv >> bit) & 1u;
    const unsigned long long m = __builtin_amdgcn_uicmp(x, 0u, 33);  // ballot(x != 0)
    const uint32_t agree = x - 1u;
    p.lo &= (uint32_t)m ^ agree;
    p.hi &= (uint32_t)(m >> 32) ^ agree;
}
__device__ __forceinline__ unsigned long long peer_end(const PeerAcc& p) {
    return (unsigned long long)p.hi << 32 | p.lo;
}
// one key: kBits bits unrolled, then bits [kBits, nbits) in a wave-uniform loop
template <int kBits>
__device__ __forceinline__ unsigned long long peer_mask(bool act, uint32_t key, int nbits = kBits) {
    PeerAcc p = peer_begin(act, key);
#pragma unroll
    for (int bit = 0; bit < kBits; ++bit) peer_bit(p, bit);
    for (int bit = kBits; bit < nbits; ++bit) peer_bit(p, bit);
    return peer_end(p);
}

// Wave reductions over all 64 lanes (every caller enters with the whole wave
// active), result in every lane. They are the device library's DPP reductions
// (row shifts + row broadcasts, then a lane read): ALU work only. A butterfly of
// __shfl_xor is six ds_bpermute round trips through the LDS pipe.
extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);
extern "C" __device__ uint32_t __ockl_wfred_min_u32(uint32_t);
extern "C" __device__ uint32_t __ockl_wfred_max_u32(uint32_t);
extern "C" __device__ uint32_t __ockl_wfred_or_u32(uint32_t);
extern "C" __device__ int __ockl_wfred_min_i32(int);
extern "C" __device__ int __ockl_wfred_max_i32(int);
extern "C" __device__ unsigned long long __ockl_wfred_add_u64(unsigned long long);
extern "C" __device__ unsigned long long __ockl_wfred_max_u64(unsigned long long);
extern "C" __device__ unsigned long long __ockl_wfred_or_u64(unsigned long long);

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "wave_sum: 32- or 64-bit integers");
    if constexpr (sizeof(T) == 4) return (T)__ockl_wfred_add_u32((uint32_t)v);  // two's complement: signed too
    else return (T)__ockl_wfred_add_u64((unsigned long long)v);
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
    if constexpr (sizeof(T) == 4 && T(-1) < T(0)) return (T)__ockl_wfred_max_i32((int)v);
    else if constexpr (sizeof(T) == 4) return (T)__ockl_wfred_max_u32((uint32_t)v);
    else {
        static_assert(sizeof(T) == 8 && !(T(-1) < T(0)), "wave_max: 32-bit or unsigned 64-bit");
        return (T)__ockl_wfred_max_u64((unsigned long long)v);
    }
}
template <typename T>
__device__ __forceinline__ T wave_or(T v) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "wave_or: 32- or 64-bit integers");
    if constexpr (sizeof(T) == 4) return (T)__ockl_wfred_or_u32((uint32_t)v);
    else return (T)__ockl_wfred_or_u64((unsigned long long)v);
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
    static_assert(sizeof(T) == 4, "wave_min: 32-bit integers");
    if constexpr (T(-1) < T(0)) return (T)__ockl_wfred_min_i32((int)v);
    else return (T)__ockl_wfred_min_u32((uint32_t)v);
}

// splitmix64 finaliser + counter-based stream hash (synthetic generator; the
// host mirror in mgatk2_amd/synth.py computes the same values with numpy uint64).
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t shash(uint64_t seed, uint64_t i, uint64_t k) {
    return mix64(seed * 0x9E3779B97F4A7C15ull + i * 0xD1B54A32D192ED03ull + k * 0x8CB92BA72F3D8DD7ull);
}

}  // namespace mgp
