// mgp_synth.hip — device-side synthetic chrM workload, used by
// bench.py so that 200M-read inputs are created directly in HBM. The generator is
// counter-based (every field is a pure function of (seed, read index, field id)),
// so mgatk2_amd/synth.py reproduces it bit for bit on the host with numpy; the
// tests check that equality. Nothing here is on the timed path.
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/mgpileup.h"
#include "mgp_kernels.h"

using namespace mgp;

namespace {

// Integer thresholds on a 24-bit uniform (x * 2^24, floored). Mirrored in synth.py.
constexpr uint32_t DUP_FULL = 2516582;   // 0.15 : copy (bc, start, strand, |tlen|) of previous read
constexpr uint32_t DUP_PART = 3019898;   // 0.18 : copy (bc, start, strand), fresh tlen
// CAT_NONWL = 503316 (0.03, non-whitelisted barcode) and CAT_NOCB both map to bc = -1
constexpr uint32_t CAT_NOCB = 671088;    // 0.04  (+0.01) no CB tag
constexpr uint32_t CAT_SEC = 754974;     // 0.045 (+0.005) secondary
constexpr uint32_t CAT_SUPP = 838860;    // 0.05  (+0.005) supplementary
constexpr uint32_t CAT_UNMAP = 872415;   // 0.052 (+0.002) unmapped (placed)
constexpr uint32_t MAPQ0 = 838860;       // 0.05  MAPQ 0, else 60
constexpr uint32_t CIG_M = 15099494;     // 0.90  50M
constexpr uint32_t CIG_S = 15938355;     // 0.95  kS(L-k)M
constexpr uint32_t CIG_I = 16441671;     // 0.98  aM bI cM ; else aM bD cM
constexpr uint32_t QUAL37 = 13421772;    // 0.80
constexpr uint32_t BASE_N = 16777;       // 0.001
constexpr uint32_t BASE_SUB = 184549;    // 0.011 (+0.01)

enum { T_ORIG = 0, T_FULL = 1, T_PART = 2 };
enum { C_M = 0, C_S = 1, C_I = 2, C_D = 3 };

__device__ __forceinline__ uint32_t u24(uint64_t h) { return (uint32_t)(h >> 40); }

__device__ __forceinline__ int read_type(uint64_t seed, int64_t i) {
    if (i == 0) return T_ORIG;
    const uint32_t t = u24(shash(seed, i, 1));
    return t < DUP_FULL ? T_FULL : (t < DUP_PART ? T_PART : T_ORIG);
}

struct Cig {
    int cls, a, b, n;
};

__device__ __forceinline__ Cig cig_of(uint64_t seed, int64_t i) {
    const uint32_t x = u24(shash(seed, i, 8));
    const uint64_t p = shash(seed, i, 9);
    Cig c;
    c.a = 0;
    c.b = 0;
    if (x < CIG_M) {
        c.cls = C_M;
        c.n = 1;
    } else if (x < CIG_S) {
        c.cls = C_S;
        c.a = 1 + (int)(p % 10);
        c.n = 2;
    } else if (x < CIG_I) {
        c.cls = C_I;
        c.a = 10 + (int)(p % 31);
        c.b = 1 + (int)((p >> 16) % 3);
        c.n = 3;
    } else {
        c.cls = C_D;
        c.a = 10 + (int)(p % 31);
        c.b = 1 + (int)((p >> 16) % 3);
        c.n = 3;
    }
    return c;
}

__device__ __forceinline__ int cigar_offset(int rl) { return (int)mgp_cigar_offset((uint32_t)rl); }

__device__ __forceinline__ uint64_t rec_size(int ncig, int rl, int align) {
    return (uint64_t)((cigar_offset(rl) + 4 * ncig + align - 1) & ~(align - 1));
}

// every synthetic read fits the packed layouts when rl <= MGP_PACK_MAX_LEN: quals
// are <= 37, at most 3 CIGAR operations with 2 aligned blocks, lengths < 64, starts
// in [0, 16569) (pack 1: 64-byte records, pack 2: 32-byte ones)
__device__ __forceinline__ bool packs(int rl, int pack) { return pack && rl <= MGP_PACK_MAX_LEN; }
__device__ __forceinline__ uint64_t packed_size(int pack, int align) {
    const int b = pack == 2 ? MGP_PACK32_BYTES : MGP_PACK_BYTES;
    const int a = pack == 2 && align > MGP_PACK32_BYTES ? MGP_PACK32_BYTES : align;
    return (uint64_t)((b + a - 1) & ~(a - 1));
}

// Cell-range filter (mgp_synth_params.cell_lo/hi, shard_rank/world): a shard of the
// global read set keeps the reads of its cells (barcode rebased to cell_lo) and, of the
// reads without a whitelisted barcode, those with index % shard_world == shard_rank.
struct Filt {
    int lo, hi, rank, world;  // hi > lo: active
    const uint64_t* map;      // read index -> index in the shard (exclusive scan of keep)
};

__device__ __forceinline__ bool keeps(const Filt& f, int64_t i, int b) {
    if (f.hi <= f.lo) return true;
    if (b >= 0) return b >= f.lo && b < f.hi;
    return f.world > 0 && (int)(i % f.world) == f.rank;
}

__device__ int cell_of(uint64_t h, const uint32_t* cdf, int nc);
__device__ int read_bc(uint64_t seed, int64_t i, int nc, const uint32_t* cdf);

__global__ void k_synth_sizes(uint64_t seed, int64_t n, int rl, int align, int pack, int nc,
                              const uint32_t* __restrict__ cdf, Filt f, uint64_t* __restrict__ sz) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int64_t j = i;
    if (f.hi > f.lo) {
        if (!keeps(f, i, read_bc(seed, i, nc, cdf))) return;
        j = (int64_t)f.map[i];
    }
    sz[j] = packs(rl, pack) ? packed_size(pack, align) : rec_size(cig_of(seed, i).n, rl, align);
}

__global__ void k_synth_keep(uint64_t seed, int64_t n, int nc, const uint32_t* __restrict__ cdf, Filt f,
                             uint64_t* __restrict__ keep) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keep[i] = keeps(f, i, read_bc(seed, i, nc, cdf)) ? 1u : 0u;
}

// ---- generic exclusive scan of u64 (3-phase, 4096 items per block) ----------
constexpr int kItems = 16;

__global__ void __launch_bounds__(kBlock) k_scan_block_sums(const uint64_t* __restrict__ a, int64_t n,
                                                            uint64_t* __restrict__ bsum) {
    const int64_t b0 = (int64_t)blockIdx.x * kBlock * kItems;
    uint64_t acc = 0;
    for (int k = 0; k < kItems; ++k) {
        const int64_t i = b0 + (int64_t)k * kBlock + threadIdx.x;
        if (i < n) acc += a[i];
    }
    acc = wave_sum(acc);
    __shared__ uint64_t ws[kBlock / kWave];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t t = 0;
        for (int w = 0; w < kBlock / kWave; ++w) t += ws[w];
        bsum[blockIdx.x] = t;
    }
}

// exclusive scan of one block's items in place, adding offs[blockIdx.x]
__global__ void __launch_bounds__(kBlock) k_scan_block_apply(uint64_t* __restrict__ a, int64_t n,
                                                             const uint64_t* __restrict__ offs) {
    const int64_t b0 = (int64_t)blockIdx.x * kBlock * kItems;
    // thread t owns items b0 + t*kItems .. +kItems (contiguous)
    uint64_t v[kItems];
    uint64_t sum = 0;
    const int64_t i0 = b0 + (int64_t)threadIdx.x * kItems;
    for (int k = 0; k < kItems; ++k) {
        const int64_t i = i0 + k;
        v[k] = i < n ? a[i] : 0;
        sum += v[k];
    }
    // block exclusive scan of per-thread sums
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint64_t x = sum;
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    __shared__ uint64_t ws[kBlock / kWave];
    if (lane == 63) ws[wid] = x;
    __syncthreads();
    uint64_t woff = 0;
    for (int w = 0; w < wid; ++w) woff += ws[w];
    uint64_t run = offs[blockIdx.x] + woff + x - sum;
    for (int k = 0; k < kItems; ++k) {
        const int64_t i = i0 + k;
        if (i < n) a[i] = run;
        run += v[k];
    }
}

int scan_exclusive_u64(uint64_t* a, int64_t n, hipStream_t s, uint64_t* total) {
    if (n <= 0) {
        *total = 0;
        return MGP_OK;
    }
    const int64_t per = (int64_t)kBlock * kItems;
    const int64_t nb = (n + per - 1) / per;
    uint64_t* bs = nullptr;
    if (hipMalloc(&bs, (size_t)(nb + 1) * 8) != hipSuccess) return MGP_E_OOM;
    k_scan_block_sums<<<(unsigned)nb, kBlock, 0, s>>>(a, n, bs);
    uint64_t btot = 0;
    int r = MGP_OK;
    if (nb > 1) {
        r = scan_exclusive_u64(bs, nb, s, &btot);
    } else {
        uint64_t t = 0;
        (void)hipMemcpyAsync(&t, bs, 8, hipMemcpyDeviceToHost, s);
        (void)hipStreamSynchronize(s);
        btot = t;
        (void)hipMemsetAsync(bs, 0, 8, s);
    }
    if (r == MGP_OK) {
        k_scan_block_apply<<<(unsigned)nb, kBlock, 0, s>>>(a, n, bs);
        if (hipStreamSynchronize(s) != hipSuccess) r = MGP_E_HIP;
    }
    (void)hipFree(bs);
    *total = btot;
    return r;
}

__device__ int cell_of(uint64_t h, const uint32_t* cdf, int nc) {
    const uint32_t u = (uint32_t)(h & 0xFFFFFFFFull);
    int lo = 0, hi = nc;  // first c with u < cdf[c]
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid;
        else lo = mid + 1;
    }
    return lo < nc ? lo : nc - 1;
}

// the barcode column of read i: its origin read's cell, or -1 (no CB / not whitelisted)
__device__ int read_bc(uint64_t seed, int64_t i, int nc, const uint32_t* cdf) {
    int64_t A = i;
    while (read_type(seed, A) != T_ORIG) --A;
    const int cell = nc > 0 ? cell_of(shash(seed, A, 3), cdf, nc) : -1;
    return u24(shash(seed, i, 6)) < CAT_NOCB ? -1 : cell;
}

__device__ __forceinline__ uint32_t code_idx(uint32_t c) { return c == 1 ? 0 : c == 2 ? 1 : c == 4 ? 2 : 3; }

__global__ void k_synth_fill(uint64_t seed, int64_t n, int rl, int nc, int L, const uint32_t* __restrict__ cdf,
                             const uint8_t* __restrict__ ref, int32_t* __restrict__ start, int32_t* __restrict__ bc,
                             int32_t* __restrict__ tlen, uint16_t* __restrict__ flag, uint8_t* __restrict__ mapq,
                             uint32_t* __restrict__ span, const uint64_t* __restrict__ roff,
                             uint8_t* __restrict__ payload, int pack, int p32_minq, int p32_dist, Filt flt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t spanpos = (uint64_t)(L - rl + 1);
    int64_t A = i;
    while (read_type(seed, A) != T_ORIG) --A;
    int64_t B = i;
    while (read_type(seed, B) == T_FULL) --B;
    const int s0 = (int)(((uint64_t)A * spanpos + (((uint64_t)u24(shash(seed, A, 2)) * spanpos) >> 24)) / (uint64_t)n);
    const int cell = nc > 0 ? cell_of(shash(seed, A, 3), cdf, nc) : -1;
    const int strand = (int)(shash(seed, A, 4) >> 63);
    const int tabs = 60 + (int)(shash(seed, B, 5) % 541);

    const uint32_t cat = u24(shash(seed, i, 6));
    int b = cell;
    uint16_t f = MGP_FLAG_PAIRED | (strand ? MGP_FLAG_REVERSE : 0);
    if (cat < CAT_NOCB) b = -1;
    else if (cat < CAT_SEC) f |= MGP_FLAG_SECONDARY;
    else if (cat < CAT_SUPP) f |= MGP_FLAG_SUPPLEMENTARY;
    else if (cat < CAT_UNMAP) f |= MGP_FLAG_UNMAPPED;
    const uint8_t mq = u24(shash(seed, i, 7)) < MAPQ0 ? 0 : 60;
    const Cig cg = cig_of(seed, i);

    const bool pk = packs(rl, pack);
    const bool p32 = pk && pack == 2;
    if (pk) f |= p32 ? MGP_FLAG_PACK32 : MGP_FLAG_PACKED;
    int64_t j = i;  // the read's index in the (shard's) read set
    if (flt.hi > flt.lo) {
        if (!keeps(flt, i, b)) return;
        j = (int64_t)flt.map[i];
        if (b >= 0) b -= flt.lo;
    }
    start[j] = s0;
    bc[j] = b;
    tlen[j] = strand ? -tabs : tabs;
    flag[j] = f;
    mapq[j] = mq;
    span[j] = (uint32_t)(cg.cls == C_D ? rl + cg.b : rl);

    uint32_t cw[3] = {0, 0, 0};
    if (cg.cls == C_M) {
        cw[0] = ((uint32_t)rl << 4) | 0;
    } else if (cg.cls == C_S) {
        cw[0] = ((uint32_t)cg.a << 4) | 4;
        cw[1] = ((uint32_t)(rl - cg.a) << 4) | 0;
    } else if (cg.cls == C_I) {
        cw[0] = ((uint32_t)cg.a << 4) | 0;
        cw[1] = ((uint32_t)cg.b << 4) | 1;
        cw[2] = ((uint32_t)(rl - cg.a - cg.b) << 4) | 0;
    } else {
        cw[0] = ((uint32_t)cg.a << 4) | 0;
        cw[1] = ((uint32_t)cg.b << 4) | 2;
        cw[2] = ((uint32_t)(rl - cg.a) << 4) | 0;
    }
    uint8_t* rec = payload + roff[j];
    uint8_t* qual = rec + 16;
    uint8_t* seq = rec + mgp_seq_offset((uint32_t)rl);
    uint32_t w32[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};  // a 32-byte record, written at the end
    if (p32) {  // 32-byte layout (include/mgpileup.h): header here, 3-bit codes per base below
        const int md = p32_dist > 0 ? p32_dist : 0;
        w32[0] = (uint32_t)s0 | ((uint32_t)rl << 16) | ((uint32_t)(cg.n | (md << 3) | (strand ? 0x80 : 0)) << 24);
        w32[1] = (cw[0] & 0xFFFFu) | ((cw[1] & 0xFFFFu) << 16);
        w32[2] = (cw[2] & 0xFFFFu);
        w32[7] = (uint32_t)(uint8_t)(int8_t)p32_minq << 24;
    } else if (pk) {  // packed layout (include/mgpileup.h); base bytes are written per base below
        *reinterpret_cast<int32_t*>(rec) = s0;
        rec[4] = (uint8_t)rl;
        rec[5] = (uint8_t)(cg.n | (strand ? 0x80 : 0));
        for (int k = 0; k < 4; ++k) {
            const uint32_t c = k < 3 ? cw[k] : 0u;
            rec[6 + 2 * k] = (uint8_t)c;
            rec[7 + 2 * k] = (uint8_t)(c >> 8);
        }
        for (int k = rl; k < MGP_PACK_MAX_LEN; ++k) rec[14 + k] = 0xFF;
    } else {
        *reinterpret_cast<int32_t*>(rec) = s0;
        *reinterpret_cast<uint32_t*>(rec + 4) = (uint32_t)rl;
        *reinterpret_cast<uint16_t*>(rec + 8) = (uint16_t)cg.n;
        *reinterpret_cast<uint16_t*>(rec + 10) = f;
        *reinterpret_cast<uint32_t*>(rec + 12) = (uint32_t)cigar_offset(rl);
        uint32_t* cig = reinterpret_cast<uint32_t*>(rec + cigar_offset(rl));
        for (int k = 0; k < cg.n; ++k) cig[k] = cw[k];
    }
    const uint8_t kCodes[4] = {1, 2, 4, 8};
    uint8_t hi_nib = 0;
    for (int q = 0; q < rl; ++q) {
        const uint64_t hq = shash(seed, i, 1000 + (uint64_t)q);
        const uint8_t qv = u24(hq) < QUAL37 ? 37 : (uint8_t)(2 + hq % 35);
        int d;
        bool rnd = false;
        if (cg.cls == C_M) d = q;
        else if (cg.cls == C_S) { rnd = q < cg.a; d = q - cg.a; }
        else if (cg.cls == C_I) {
            if (q < cg.a) d = q;
            else if (q < cg.a + cg.b) { rnd = true; d = 0; }
            else d = q - cg.b;
        } else d = q < cg.a ? q : q + cg.b;
        const uint64_t hs = shash(seed, i, 100000 + (uint64_t)q);
        uint8_t code;
        if (rnd) {
            code = kCodes[hs & 3];
        } else {
            const uint8_t rc = ref[(uint32_t)(s0 + d) % (uint32_t)L];
            const uint32_t m = u24(hs);
            if (m < BASE_N) code = 15;
            else if (m < BASE_SUB) code = kCodes[(code_idx(rc) + 1 + (uint32_t)((hs & 255) % 3)) & 3];
            else code = rc;
        }
        if (p32) {
            // counted (include/mgpileup.h): inside an aligned operation's query range (an
            // insertion does not advance q: the last b positions of aM bI cM are outside),
            // min_dist <= q < rl - min_dist, int8(qual) >= min_baseq, A/C/G/T
            const int md = p32_dist > 0 ? p32_dist : 0;
            const bool inblk = cg.cls == C_S ? q >= cg.a : cg.cls == C_I ? q < rl - cg.b : true;
            const bool cnt = inblk && q >= md && q < rl - md && (int)(int8_t)qv >= p32_minq && code != 15;
            const uint32_t v = cnt ? code_idx(code) : 4u;
            const int bit = 96 + 3 * q;
            w32[bit >> 5] |= v << (bit & 31);
            if ((bit & 31) > 29) w32[(bit >> 5) + 1] |= v >> (32 - (bit & 31));
            continue;
        }
        if (pk) {
            rec[14 + q] = code == 15 ? (uint8_t)0xFF : (uint8_t)((qv << 2) | code_idx(code));
            continue;
        }
        qual[q] = qv;
        if ((q & 1) == 0) hi_nib = code;
        else seq[q >> 1] = (uint8_t)((hi_nib << 4) | code);
    }
    if ((rl & 1) && !pk) seq[rl >> 1] = (uint8_t)(hi_nib << 4);
    if (p32) {
        for (int q = rl; q < MGP_PACK_MAX_LEN; ++q) {  // never counted
            const int bit = 96 + 3 * q;
            w32[bit >> 5] |= 4u << (bit & 31);
            if ((bit & 31) > 29) w32[(bit >> 5) + 1] |= 4u >> (32 - (bit & 31));
        }
        uint4* r4 = reinterpret_cast<uint4*>(rec);
        r4[0] = make_uint4(w32[0], w32[1], w32[2], w32[3]);
        r4[1] = make_uint4(w32[4], w32[5], w32[6], w32[7]);
    }
}

}  // namespace

// n: reads of the global set; with an active filter (cell_hi > cell_lo) only the
// shard's reads are written, *n_out of them, barcodes rebased to cell_lo.
extern "C" int mgp_synth_fill(void* stream, uint64_t seed, int64_t n, int read_len, int n_cells, int mito_len,
                              const uint32_t* d_cdf, const uint8_t* d_ref, int32_t* start, int32_t* bc,
                              int32_t* tlen, uint16_t* flag, uint8_t* mapq, uint32_t* span, uint64_t* roff,
                              uint8_t* payload, int64_t* payload_bytes, int rec_align, int pack, int placed,
                              int cell_lo, int cell_hi, int shard_rank, int shard_world, uint64_t* d_map,
                              int64_t* n_out, int p32_minq, int p32_dist) {
    hipStream_t s = (hipStream_t)stream;
    if (read_len < 48) return MGP_E_INVALID;
    *n_out = n;
    if (n == 0) {
        *payload_bytes = 0;
        return MGP_OK;
    }
    const unsigned nb = (unsigned)((n + kBlock - 1) / kBlock);
    Filt flt{cell_lo, cell_hi, shard_rank, shard_world, d_map};
    int64_t nk = n;
    if (cell_hi > cell_lo) {  // the shard's read indices: exclusive scan of the keep flags
        k_synth_keep<<<nb, kBlock, 0, s>>>(seed, n, n_cells, d_cdf, flt, d_map);
        if (hipGetLastError() != hipSuccess) return MGP_E_HIP;
        uint64_t tot = 0;
        int r = scan_exclusive_u64(d_map, n, s, &tot);
        if (r != MGP_OK) return r;
        nk = (int64_t)tot;
    }
    *n_out = nk;
    if (placed < 0) return MGP_OK;  // the shard's read count only (its placement comes next)
    uint64_t total = (uint64_t)*payload_bytes;
    if (!placed) {  // dense: offsets = exclusive scan of the record sizes; else roff holds the placement
        k_synth_sizes<<<nb, kBlock, 0, s>>>(seed, n, read_len, rec_align, pack, n_cells, d_cdf, flt, roff);
        if (hipGetLastError() != hipSuccess) return MGP_E_HIP;
        int r = scan_exclusive_u64(roff, nk, s, &total);
        if (r != MGP_OK) return r;
    }
    if (total && hipMemsetAsync(payload, 0, (size_t)total, s) != hipSuccess) return MGP_E_HIP;
    k_synth_fill<<<nb, kBlock, 0, s>>>(seed, n, read_len, n_cells, mito_len, d_cdf, d_ref, start, bc, tlen, flag,
                                       mapq, span, roff, payload, pack, p32_minq, p32_dist, flt);
    if (hipGetLastError() != hipSuccess) return MGP_E_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return MGP_E_HIP;
    *payload_bytes = (int64_t)total;
    return MGP_OK;
}
