// mgp_txtgz.hip — mgatk's txt count files formatted and gzip-deflated on the device
// (gfx950, wave64). See mgp_txtgz.h for what is written; the layout of one member:
//
//   gzip header (10 B) | one deflate block (BFINAL) | CRC-32 | ISIZE
//
// One 256-thread workgroup per (file, cell) member. Thread t owns positions
// [t P, (t + 1) P) of chrM (P = ceil(L / 256)) and with them a contiguous run of the
// member's lines (a "segment"):
//   1. format: each thread counts its lines' bytes, a block scan places the segments,
//      each thread writes its text and a line table (start and field offsets);
//   2. parse (twice: default prices, then the member's own Huffman lengths): each
//      thread runs a backward optimal-parse DP over its segment's bytes. The match
//      candidates are line-aligned: for each of the 16 previous lines, the byte at the
//      same offset from the start of the current field and the byte at the same offset
//      from the line's end. Along a line those distances are constant, so a
//      candidate's match length follows L(i) = T[i] == T[i - d] ? L(i + 1) + 1 : 0
//      and only a field change costs a forward compare. Tokens never cross a segment
//      (the cost: one token per ~65 positions). On C4-like text this parse gives
//      85-94 % of zlib level 9's bytes (tests/test_gpu_txtgz.py measures it);
//   3. Huffman: length-limited codes from the parse's symbol counts (rank sort over the
//      workgroup, two-queue merge on one lane), the dynamic header, and the fixed-code
//      and stored alternatives; the smallest is written;
//   4. encode: a block scan of the segments' bit counts, each thread writes its bits
//      (atomic OR only on the words it shares with a neighbour);
//   5. CRC-32 of the text: per segment (table in LDS), combined up a tree with
//      GF(2) shift matrices.
// No shared state between members: the grid is members, nothing is global but the
// scratch each member owns.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mgp_kernels.h"
#include "mgp_txtgz.h"

namespace mgp {
namespace txtgz {

constexpr int kT = 256;        // threads per member (one segment each)
static_assert(kT == 256, "h5_seg_bytes / h5_tok_words (mgp_txtgz.h) assume 256 threads per chunk");
constexpr int kJ = 16;         // previous lines searched for matches
constexpr int kLMax = 31;      // longest match tried (longer ones gain nothing on C4-like text)
constexpr int kMaxDist = 32768;
constexpr int kLit = 286, kDist = 30;
constexpr int kWinBytes = 24 * 1024;  // LDS text window of the match finder

__constant__ uint16_t c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint16_t c_dist_base[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,   65,    97,    129,
                                         193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};

__constant__ uint8_t c_cl_ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ int len_code(int l) {  // 3..258 -> 0..28
    if (l <= 10) return l - 3;
    if (l == 258) return 28;
    const int x = l - 3, n = 31 - __clz(x);
    return 4 * (n - 1) + ((x >> (n - 2)) & 3);
}
__device__ __forceinline__ int len_xb(int c) { return (c < 8 || c == 28) ? 0 : (c >> 2) - 1; }
__device__ __forceinline__ int dist_code(int d) {  // 1..32768 -> 0..29
    if (d <= 4) return d - 1;
    const int x = d - 1, n = 31 - __clz(x);
    return 2 * n + ((x >> (n - 1)) & 1);
}
__device__ __forceinline__ int dist_xb(int c) { return c < 4 ? 0 : (c >> 1) - 1; }

__device__ __forceinline__ uint32_t ndig(uint32_t v) {
    uint32_t n = 1;
    while (v >= 10) {
        v /= 10;
        ++n;
    }
    return n;
}
__device__ __forceinline__ uint8_t* put_num(uint8_t* p, uint32_t v, uint32_t nd) {
    for (uint32_t k = nd; k-- > 0;) {
        p[k] = (uint8_t)('0' + v % 10);
        v /= 10;
    }
    return p + nd;
}

// ---- the count rows ----
// the line of position p in file f (0 coverage, 1..4 A..T): its length (0: none) and values.
// u16: the position's window has exact 16-bit rows (rows16, decided by the caller from the
// cell's wide flags staged in LDS); the depth and the counts are loaded together
__device__ __forceinline__ uint32_t line_of(const Rows& r, int c, int p, int f, uint32_t bclen, uint32_t& v1,
                                            uint32_t& v2, bool u16) {
    const size_t P = (size_t)c * r.L + p;
    uint32_t d, a = 0, b = 0;
    if (u16) {
        d = r.d16[P];
        if (f) {
            const uint4 q = r.c16[P];
            const uint32_t w = f == 1 ? q.x : f == 2 ? q.y : f == 3 ? q.z : q.w;
            a = w & 0xFFFFu;
            b = w >> 16;
        }
    } else {
        d = r.d32[P];
        if (f) {
            a = r.c32[P * 8 + 2 * (f - 1)];
            b = r.c32[P * 8 + 2 * (f - 1) + 1];
        }
    }
    if (!d) return 0;
    if (f == 0) {
        v1 = d;
        v2 = 0;
        return ndig((uint32_t)p + 1) + bclen + ndig(d) + 3;
    }
    v1 = a;
    v2 = b;
    if (!(v1 | v2)) return 0;
    return ndig((uint32_t)p + 1) + bclen + ndig(v1) + ndig(v2) + 4;
}
constexpr int kMaxWin = 256;  // wide flags of a cell staged in LDS (the first kMaxWin windows)
__device__ __forceinline__ bool wide_at(const Rows& r, int c, int win) {
    return r.c16 == nullptr || (r.wide && r.wide[(size_t)c * r.nwin + win]);
}
// the cell's wide flags into LDS (all threads; 1: the u32 rows)
__device__ __forceinline__ void stage_wide(const Rows& r, int c, uint8_t* wf) {
    for (int q = threadIdx.x; q < min(r.nwin, kMaxWin); q += blockDim.x) wf[q] = wide_at(r, c, q) ? 1 : 0;
}
// window win of cell c has exact 16-bit rows
__device__ __forceinline__ bool u16_at(const Rows& r, int c, int win, const uint8_t* wf) {
    return win < kMaxWin ? !wf[win] : !wide_at(r, c, win);
}

// ---- block-wide helpers (256 threads = 4 waves) ----
__device__ uint64_t block_excl_scan(uint64_t x, uint64_t* wsum, uint64_t& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t v = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    if (lane == 63) wsum[w] = v;
    __syncthreads();
    uint64_t base = 0;
    for (int k = 0; k < w; ++k) base += wsum[k];
    total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
    return base + v - x;
}

// ---- Huffman code lengths (length-limited), all threads call ----
struct HuffLds {
    uint32_t f[kLit];
    uint16_t order[kLit];
    uint32_t w[2 * kLit];
    uint16_t par[2 * kLit];
    uint8_t dep[2 * kLit];
    int m;
};
// len[s] for s < n from freq[s] (LDS), lengths <= mb; every used symbol gets a code and
// the code is complete (Kraft sum 1, as inflate requires). One Huffman tree; leaves deeper
// than mb are clipped to mb, then the per-length counts are repaired (the deepest shorter
// leaf moved one level down until the Kraft sum fits, then leaves moved up until it is
// exactly 1) and the lengths dealt out by frequency, the longest to the rarest (zlib's
// gen_bitlen does the same repair; halving the counts and rebuilding, as before, took
// ~7 rebuilds on count planes: 0.5 ms per chunk).
__device__ void huff_lengths(const uint32_t* freq, int n, int mb, uint8_t* len, HuffLds& h) {
    const int t = threadIdx.x;
    for (int s = t; s < n; s += kT) h.f[s] = freq[s];
    if (t == 0) h.m = 0;
    __syncthreads();
    // rank sort of the used symbols by (count, symbol)
    for (int s = t; s < n; s += kT) {
        const uint32_t fs = h.f[s];
        if (!fs) continue;
        int r = 0;
        for (int q = 0; q < n; ++q) {
            const uint32_t fq = h.f[q];
            r += (fq != 0) & ((fq < fs) | ((fq == fs) & (q < s)));
        }
        h.order[r] = (uint16_t)s;
        atomicAdd(&h.m, 1);
    }
    __syncthreads();
    if (t == 0) {
        const int m = h.m;
        for (int s = 0; s < n; ++s) len[s] = 0;
        if (m == 1) {
            len[h.order[0]] = 1;
        } else if (m > 1) {
            // two queues: the sorted leaves 0..m-1 and the internal nodes m.. in creation order
            for (int i = 0; i < m; ++i) h.w[i] = h.f[h.order[i]];
            int li = 0, ni = m, nn = m;
            auto take = [&]() -> int {
                if (li < m && (ni >= nn || h.w[li] <= h.w[ni])) return li++;
                return ni++;
            };
            for (int k = 0; k < m - 1; ++k) {
                const int a = take(), b = take();
                h.w[nn] = h.w[a] + h.w[b];
                h.par[a] = (uint16_t)nn;
                h.par[b] = (uint16_t)nn;
                ++nn;
            }
            h.dep[nn - 1] = 0;
            uint32_t cnt[16] = {0};  // leaves per length (clipped to mb)
            for (int x = nn - 2; x >= 0; --x) {
                const int d = h.dep[h.par[x]] + 1;
                h.dep[x] = (uint8_t)(d < 255 ? d : 255);
                if (x < m) cnt[d < mb ? d : mb]++;
            }
            // Kraft sum in units of 2^-mb
            int64_t K = 0;
            for (int l = 1; l <= mb; ++l) K += (int64_t)cnt[l] << (mb - l);
            const int64_t full = (int64_t)1 << mb;
            while (K > full) {  // the deepest leaf above mb one level down
                int b = mb - 1;
                while (cnt[b] == 0) --b;
                cnt[b]--;
                cnt[b + 1]++;
                K -= (int64_t)1 << (mb - b - 1);
            }
            while (K < full) {  // a leaf whose move up fits, the deepest first
                int b = mb;
                while (cnt[b] == 0 || ((int64_t)1 << (mb - b)) > full - K) --b;
                cnt[b]--;
                cnt[b - 1]++;
                K += (int64_t)1 << (mb - b);
            }
            // the rarest symbols (order ascending) get the longest codes
            int i = 0;
            for (int l = mb; l >= 1; --l)
                for (uint32_t c = 0; c < cnt[l]; ++c) len[h.order[i++]] = (uint8_t)l;
        }
    }
    __syncthreads();
}

// canonical codes (bit-reversed for LSB-first output), one thread
__device__ void canon(const uint8_t* len, int n, uint16_t* code) {
    uint16_t cnt[16] = {0}, next[16];
    for (int s = 0; s < n; ++s) cnt[len[s]]++;
    cnt[0] = 0;
    uint32_t c = 0;
    for (int b = 1; b < 16; ++b) {
        c = (c + cnt[b - 1]) << 1;
        next[b] = (uint16_t)c;
    }
    for (int s = 0; s < n; ++s) {
        const int l = len[s];
        code[s] = l ? (uint16_t)(__brev((uint32_t)next[l]++) >> (32 - l)) : 0;
    }
}

// ---- the LDS of the coding kernel (k_txt_code) ----
struct CodeLds {
    uint64_t wsum[4];
    uint32_t lit_f[kLit], dist_f[kDist];
    uint8_t lit_len[kLit], dist_len[kDist];
    uint16_t lit_code[kLit], dist_code[kDist];
    uint8_t litcost[256], lencost[kLMax + 1], dcost[kDist];
    HuffLds h;
    uint32_t cl_f[19];
    uint8_t cl_len[19];
    uint16_t cl_code[19];
    uint16_t rle[kLit + kDist];  // code-length symbols: sym | extra << 8
    int n_rle, hlit, hdist, hclen;
    uint64_t hdr_bits;
};

__device__ __forceinline__ void lds_prices_default(CodeLds& S) {
    for (int s = threadIdx.x; s < 256; s += kT)
        S.litcost[s] = (uint8_t)((s >= '0' && s <= '9') || s == ',' ? 4 : s == '\n' ? 5 : 6);
    for (int l = threadIdx.x; l <= kLMax; l += kT) S.lencost[l] = l < 3 ? 0 : (uint8_t)(7 + len_xb(len_code(l)));
    for (int c = threadIdx.x; c < kDist; c += kT) S.dcost[c] = (uint8_t)(5 + dist_xb(c));
}
__device__ __forceinline__ void lds_prices_from_lengths(CodeLds& S) {
    for (int s = threadIdx.x; s < 256; s += kT) S.litcost[s] = S.lit_len[s] ? S.lit_len[s] : 16;
    for (int l = threadIdx.x; l <= kLMax; l += kT) {
        if (l < 3) {
            S.lencost[l] = 0;
            continue;
        }
        const int c = len_code(l);
        S.lencost[l] = (uint8_t)((S.lit_len[257 + c] ? S.lit_len[257 + c] : 16) + len_xb(c));
    }
    for (int c = threadIdx.x; c < kDist; c += kT) S.dcost[c] = (uint8_t)((S.dist_len[c] ? S.dist_len[c] : 16) + dist_xb(c));
}

#ifndef MGP_TXT_FWD_CAP
#define MGP_TXT_FWD_CAP 8  // (8 and 12 gave the same members on C4 text, 31: 0.04 % smaller, match 12 % slower)
#endif
// forward match length at distance d from i (at most cap and MGP_TXT_FWD_CAP), text staged in LDS
__device__ __forceinline__ int fwd_match(const uint8_t* W, int i, int d, int cap) {
    cap = min(cap, MGP_TXT_FWD_CAP);
    int L = 0;
    while (L < cap && W[i + L] == W[i - d + L]) ++L;
    return L;
}

// The match finder over one window of lines [k0, k1), the text staged in LDS (W[x] =
// T[x + base], lines k0 - kJ .. k1 and 64 bytes beyond): each thread takes whole lines
// and walks them backward. Candidates per previous line m = k - 1 - j (j < kJ): the same
// offset from the start of the current field (distance constant along the field) and
// from the line's end (constant along the line); along a run of one distance the
// length follows L(i) = T[i] == T[i - d] ? L(i + 1) + 1 : 0, so only the first byte
// visited (the line end, a field's last byte) costs a forward compare. Every position
// keeps its longest candidate (the nearest on ties): cand[i] = d | L << 16, 0 if L < 3.
__device__ void match_window(const uint8_t* W, int64_t base, int64_t wend, const uint32_t* ln, int k0, int k1,
                             int kb, int nf, uint32_t* cand) {
    // ln: the window's line table in LDS, lines kb .. k1 - 1
    auto line = [&](int k) -> const uint32_t* { return ln + 3 * (size_t)(k - kb); };
    for (int k = k0 + (int)threadIdx.x; k < k1; k += kT) {
        const uint32_t* le = line(k);
        const int s = (int)((int64_t)le[0] - base);
        const int A1 = s + (int)(le[1] & 0xFFFFu), A2 = s + (int)(le[1] >> 16), A3 = s + (int)(le[2] & 0xFFFFu);
        const int e = s + (int)(le[2] >> 16) - 1;  // the '\n'
        // per previous line j: distances dd = dE | dF << 16 and lengths ll = LE | LF << 8
        // (packed: 32 registers for the 32 candidates)
        uint32_t dd[kJ], ll[kJ];
#pragma unroll
        for (int j = 0; j < kJ; ++j) {
            dd[j] = 0;
            ll[j] = 0;
            if (k - j - 1 < kb) continue;  // (lines before the window: no candidate)
            const uint32_t* lp = line(k - j - 1);
            const int d = e - ((int)((int64_t)lp[0] - base) + (int)(lp[2] >> 16) - 1);
            if (d > 0 && d <= kMaxDist) dd[j] = (uint32_t)d;
        }
        const int cap_e = (int)min((int64_t)kLMax, wend - base - e);
        int field = -1;
        for (int i = e; i >= s; --i) {
            const int f = (nf > 3 && i >= A3) ? 3 : i >= A2 ? 2 : i >= A1 ? 1 : 0;
            const uint8_t ti = W[i];
            const int cap = min(kLMax, cap_e + (e - i));
            if (f != field) {
                const int Af = f == 0 ? s : f == 1 ? A1 : f == 2 ? A2 : A3;
#pragma unroll
                for (int j = 0; j < kJ; ++j) {
                    const int dE = (int)(dd[j] & 0xFFFFu);
                    int LE = (int)(ll[j] & 0xFFu);
                    if (dE) {
                        if (field < 0) LE = i - dE >= 0 ? fwd_match(W, i, dE, cap) : 0;
                        else LE = (i - dE >= 0 && W[i - dE] == ti) ? min(LE + 1, cap) : 0;
                    }
                    int dF = 0, LF = 0;
                    if (k - j - 1 >= kb) {
                        const uint32_t* lp = line(k - j - 1);
                        const int sp = (int)((int64_t)lp[0] - base);
                        const int Bf = f == 0 ? sp
                                     : f == 1 ? sp + (int)(lp[1] & 0xFFFFu)
                                     : f == 2 ? sp + (int)(lp[1] >> 16)
                                              : sp + (int)(lp[2] & 0xFFFFu);
                        const int d = Af - Bf;
                        if (d > 0 && d <= kMaxDist && d != dE) {
                            dF = d;
                            LF = fwd_match(W, i, d, cap);
                        }
                    }
                    dd[j] = (uint32_t)dE | (uint32_t)dF << 16;
                    ll[j] = (uint32_t)LE | (uint32_t)LF << 8;
                }
                field = f;
            } else {
                // (a field-anchored source stays inside the earlier line's field; an
                // end-anchored one can run off the window's start when that line is short)
#pragma unroll
                for (int j = 0; j < kJ; ++j) {
                    const int dE = (int)(dd[j] & 0xFFFFu), dF = (int)(dd[j] >> 16);
                    int LE = (int)(ll[j] & 0xFFu), LF = (int)(ll[j] >> 8);
                    if (dF) LF = (W[i - dF] == ti) ? min(LF + 1, cap) : 0;
                    if (dE) LE = (i - dE >= 0 && W[i - dE] == ti) ? min(LE + 1, cap) : 0;
                    ll[j] = (uint32_t)LE | (uint32_t)LF << 8;
                }
            }
            int bl = 0, bd = 0;
#pragma unroll
            for (int j = 0; j < kJ; ++j) {  // nearest first: a later candidate must be longer
                const int dE = (int)(dd[j] & 0xFFFFu), dF = (int)(dd[j] >> 16);
                const int LE = (int)(ll[j] & 0xFFu), LF = (int)(ll[j] >> 8);
                if (LF > bl || (LF == bl && dF && dF < bd)) {
                    bl = LF;
                    bd = dF;
                }
                if (LE > bl || (LE == bl && dE && dE < bd)) {
                    bl = LE;
                    bd = dE;
                }
            }
            cand[i + base] = bl >= 3 ? ((uint32_t)bd | (uint32_t)bl << 16) : 0u;
        }
    }
}

// The default prices of the parse (bits): a literal by class, a length symbol 7 bits and
// a distance symbol 5, plus their extra bits (a second pass at the member's own code
// lengths gained 0.4-1 % on C4-like text for twice the parse time).
__host__ __device__ constexpr int lit_price(int b) {
    return ((b >= '0' && b <= '9') || b == ',') ? 4 : b == '\n' ? 5 : 6;
}
__device__ __forceinline__ constexpr int len_price(int l) {
    return 7 + ((l <= 10) ? 0 : (l < 258 ? ((4 * (31 - __builtin_clz(l - 3) - 1) + (((l - 3) >> (31 - __builtin_clz(l - 3) - 2)) & 3)) >> 2) - 1 : 0));
}

// One segment's backward optimal parse over its candidates (tok[i] = d | L << 16 from
// match_window): the chosen length (0: a literal, else 3..L at distance d) goes into
// bits 22-27 of tok[i]. Positions go in blocks of 32 aligned to the member's text, the
// costs of the 31 positions after the current one in a register ring whose indices are
// static inside the block (the position loop and the length loop unrolled): no LDS and
// no dynamic register indexing on the relaxation's path.
__device__ void dp_segment(const uint8_t* T, uint32_t* tok, int t0, int t1, const CodeLds& S) {
    if (t1 <= t0) return;
    uint32_t ring[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) ring[k] = 0;  // cost[t1] = 0; the others are never read
    for (int b0 = (t1 - 1) & ~31; b0 + 31 >= t0; b0 -= 32) {
        // the block's 32 candidates and bytes in 10 aligned 16-byte loads, all in flight
        // together (member texts start 16-byte aligned; positions outside [t0, t1) are read
        // but never used, and the buffers have slack past the last member)
        uint32_t w[32];
        uint32_t tb[32];
        const uint4* const w4 = reinterpret_cast<const uint4*>(tok + b0);
        const uint4* const t4 = reinterpret_cast<const uint4*>(T + b0);
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint4 v = w4[q];
            w[4 * q] = v.x;
            w[4 * q + 1] = v.y;
            w[4 * q + 2] = v.z;
            w[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint4 v = t4[q];
            const uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int u = 0; u < 16; ++u) tb[16 * q + u] = (ws[u >> 2] >> (8 * (u & 3))) & 0xFFu;
        }
#pragma unroll
        for (int u = 31; u >= 0; --u) {
            const int p = b0 + u;
            if (p < t0 || p >= t1) continue;
            uint32_t best = S.litcost[tb[u]] + ring[(u + 1) & 31];
            uint32_t bl = 0;
            const int L = min((int)((w[u] >> 16) & 63u), t1 - p);
            if (L >= 3) {
                const int d = (int)(w[u] & 0xFFFFu);
                const int dc = dist_code(d);
                const uint32_t dp = 5u + (uint32_t)dist_xb(dc);
#pragma unroll
                for (int l = 3; l <= kLMax; ++l) {
                    const uint32_t v = (uint32_t)len_price(l) + dp + ring[(u + l) & 31];
                    const bool take = l <= L && v < best;
                    best = take ? v : best;
                    bl = take ? (uint32_t)l : bl;
                }
            }
            ring[u] = best;
            tok[p] = (w[u] & 0x3FFFFFu) | (bl << 22);
        }
    }
}

// zero-byte CRC operator applied n times (GF(2) matrices M[b] = one-byte operator ^ 2^b)
__device__ uint32_t crc_shift(uint32_t c, uint64_t n, const uint32_t* M) {
    for (int b = 0; n && b < kShiftPow; ++b, n >>= 1) {
        if (!(n & 1)) continue;
        const uint32_t* m = M + 32 * b;
        uint32_t r = 0;
        for (int k = 0; k < 32; ++k)
            if ((c >> k) & 1u) r ^= m[k];
        c = r;
    }
    return c;
}

// bit writer over the member's u32 words: atomics on the words shared with neighbours
struct BitW {
    uint32_t* w;
    uint64_t word;
    uint64_t acc;
    int n;
    bool first;
    __device__ BitW(uint32_t* out, uint64_t bit) : w(out), word(bit >> 5), acc(0), n((int)(bit & 31)), first(true) {}
    __device__ void put(uint32_t v, int nb) {
        acc |= (uint64_t)v << n;
        n += nb;
        while (n >= 32) {
            if (first) atomicOr(&w[word], (uint32_t)acc);
            else w[word] = (uint32_t)acc;
            first = false;
            ++word;
            acc >>= 32;
            n -= 32;
        }
    }
    __device__ void done() {
        if (n > 0) atomicOr(&w[word], (uint32_t)acc);
    }
};

__device__ __forceinline__ void put_token(BitW& bw, uint32_t tk, const uint16_t* lc, const uint8_t* ll, const uint16_t* dcd,
                                          const uint8_t* dl) {
    const uint32_t l = tk >> 16;
    if (!l) {
        bw.put(lc[tk], ll[tk]);
        return;
    }
    const int d = (int)(tk & 0xFFFFu);
    const int c = len_code((int)l), xb = len_xb(c);
    bw.put(lc[257 + c], ll[257 + c]);
    if (xb) bw.put(l - c_len_base[c], xb);
    const int e = dist_code(d), yb = dist_xb(e);
    bw.put(dcd[e], dl[e]);
    if (yb) bw.put((uint32_t)(d - c_dist_base[e]), yb);
}
__device__ __forceinline__ uint32_t token_bits(uint32_t tk, const uint8_t* ll, const uint8_t* dl) {
    const uint32_t l = tk >> 16;
    if (!l) return ll[tk];
    const int c = len_code((int)l), e = dist_code((int)(tk & 0xFFFFu));
    return ll[257 + c] + len_xb(c) + dl[e] + dist_xb(e);
}
__device__ __forceinline__ uint8_t fixed_len(int s) { return s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8; }

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kT) k_txt_sizes(Job job, uint64_t* __restrict__ sizes, uint64_t* __restrict__ nlines) {
    __shared__ unsigned long long acc[2 * kFiles];
    __shared__ uint8_t wf[kMaxWin];
    const int k = blockIdx.x, t = threadIdx.x;
    if (t < 2 * kFiles) acc[t] = 0;
    const int c = job.cells[k];
    stage_wide(job.rows, c, wf);
    __syncthreads();
    const uint32_t bclen = (uint32_t)(job.name_off[k + 1] - job.name_off[k]);
    uint64_t b[kFiles] = {0, 0, 0, 0, 0};
    uint32_t n[kFiles] = {0, 0, 0, 0, 0};
    for (int p = t; p < job.rows.L; p += kT) {
        const bool u16 = u16_at(job.rows, c, p / job.rows.W, wf);
        for (int f = 0; f < kFiles; ++f) {
            uint32_t v1, v2;
            const uint32_t len = line_of(job.rows, c, p, f, bclen, v1, v2, u16);
            if (!len) {
                if (f == 0) break;  // depth 0: no line in any file
                continue;
            }
            b[f] += len;
            ++n[f];
        }
    }
    for (int f = 0; f < kFiles; ++f) {
        atomicAdd(&acc[f], (unsigned long long)b[f]);
        atomicAdd(&acc[kFiles + f], (unsigned long long)n[f]);
    }
    __syncthreads();
    if (t < kFiles) {
        sizes[(size_t)t * job.n + k] = acc[t];
        nlines[(size_t)t * job.n + k] = acc[kFiles + t];
    }
}

// MGP_TXT_PROF: thread 0 stamps the 100 MHz wall clock when a kernel's member is done
#define PROF_STAMP(k)                                                            \
    do {                                                                         \
        if (sc.prof) {                                                           \
            __syncthreads();                                                     \
            if (threadIdx.x == 0) sc.prof[m * 8 + (k)] = wall_clock64();         \
        }                                                                        \
    } while (0)

// A thread's text written through a 16-byte staging block: byte stores until the address
// is 16-byte aligned, then whole aligned 16-byte stores, byte stores for the last partial
// block (its other bytes are the next thread's): one store instruction per 16 bytes instead
// of one per byte, each lane's to its own line.
struct TextOut {
    uint8_t* T;
    uint64_t pos;  // index in T of the next byte
    uint64_t lo = 0, hi = 0;
    int nb = 0;    // staged bytes: [pos - nb, pos), the block starting 16-aligned
    bool stg = false;
    __device__ TextOut(uint8_t* t, uint64_t p) : T(t), pos(p) {
        stg = (reinterpret_cast<uintptr_t>(T + pos) & 15u) == 0;
    }
    // n <= 8 bytes, little-endian in x (zero above them)
    __device__ __forceinline__ void put(uint64_t x, int n) {
        if (!stg) {  // (the head, up to the first 16-byte boundary)
            int k = 0;
            for (; k < n && !stg; ++k) {
                T[pos++] = (uint8_t)(x >> (8 * k));
                stg = (reinterpret_cast<uintptr_t>(T + pos) & 15u) == 0;
            }
            if (k == n) return;
            x >>= 8 * k;
            n -= k;
        }
        uint64_t carry = 0;
        if (nb < 8) {
            lo |= x << (8 * nb);
            if (nb + n > 8) hi |= x >> (8 * (8 - nb));
        } else {
            hi |= x << (8 * (nb - 8));
            if (nb + n > 16) carry = x >> (8 * (16 - nb));
        }
        nb += n;
        pos += (uint64_t)n;
        if (nb >= 16) {
            *reinterpret_cast<uint4*>(T + pos - nb) =
                make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
            nb -= 16;
            lo = carry;
            hi = 0;
        }
    }
    __device__ void flush() {
        uint8_t* const b = T + pos - nb;
        for (int k = 0; k < nb; ++k) b[k] = (uint8_t)((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8))) & 0xFFu);
        nb = 0;
    }
    // exactly nd <= 8 digits of v, most significant first
    __device__ __forceinline__ void digits(uint32_t v, uint32_t nd) {
        uint64_t x = 0;
        for (uint32_t k = 0; k < nd; ++k) {
            x = (x << 8) | (uint64_t)('0' + v % 10u);
            v /= 10u;
        }
        put(x, (int)nd);
    }
    // the decimal digits of v (no leading zeros; "0" for 0)
    __device__ __forceinline__ void num(uint32_t v) {
        if (v >= 100000000u) {
            digits(v / 100000000u, ndig(v / 100000000u));
            digits(v % 100000000u, 8);
        } else {
            digits(v, ndig(v));
        }
    }
};

struct FormatLds {
    uint8_t bc[4096 + 8];  // the member's barcode (the same on every line)
    uint64_t wsum[4];
    uint8_t wf[kMaxWin];
    uint32_t crc_tab[4][256];  // slicing-by-4 tables (crc_tab[0]: the byte table)
    uint32_t shift[kShiftPow * 32];  // the zero-byte operator's powers (Scratch::crc_shift)
    uint32_t crc_x[kT / 64];   // the waves' XORs
};

// Kernel 1 (per member): the text, the line table, the segments' starts and the CRC-32.
__global__ void __launch_bounds__(kT) k_txt_format(Job job, Scratch sc) {
    __shared__ FormatLds S;
    const int t = threadIdx.x;
    const int64_t m = blockIdx.x;
    const int f = (int)(m / job.n);
    const int64_t kc = m - (int64_t)f * job.n;
    const int c = job.cells[kc];
    const char* bc = job.names + job.name_off[kc];
    const uint32_t bclen = (uint32_t)(job.name_off[kc + 1] - job.name_off[kc]);
    const int L = job.rows.L;
    uint8_t* const T = sc.text + sc.text_off[m];
    uint32_t* const lines = sc.lines + 3 * sc.line_off[m];
    const uint64_t n_text = sc.text_n[m];
    if (n_text == 0) return;
    PROF_STAMP(0);
    for (int s = t; s < 256; s += kT) {
        uint32_t r = (uint32_t)s;
        for (int b = 0; b < 8; ++b) r = (r >> 1) ^ (0xEDB88320u & (0u - (r & 1u)));
        S.crc_tab[0][s] = r;
    }
    for (int q = t; q < kShiftPow * 32; q += kT) S.shift[q] = sc.crc_shift[q];
    stage_wide(job.rows, c, S.wf);
    for (uint32_t q = t; q < bclen; q += kT) S.bc[q] = (uint8_t)bc[q];
    __syncthreads();
    for (int s = t; s < 256; s += kT) {
        uint32_t r = S.crc_tab[0][s];
        for (int k = 1; k < 4; ++k) {
            r = (r >> 8) ^ S.crc_tab[0][r & 0xFFu];
            S.crc_tab[k][s] = r;
        }
    }
    // ---- 1. format ----
    const int P = (L + kT - 1) / kT;
    const int p0 = min(L, t * P), p1 = min(L, p0 + P);
    uint32_t my_b = 0, my_n = 0;
    const int W = job.rows.W;
    {
        int win = p0 / W, wnext = (win + 1) * W;
        for (int p = p0; p < p1; ++p) {
            if (p >= wnext) {
                ++win;
                wnext += W;
            }
            uint32_t v1, v2;
            const uint32_t len = line_of(job.rows, c, p, f, bclen, v1, v2, u16_at(job.rows, c, win, S.wf));
            my_b += len;
            my_n += len != 0;
        }
    }
    uint64_t tot;
    const uint64_t pre = block_excl_scan(((uint64_t)my_b << 24) | my_n, S.wsum, tot);
    PROF_STAMP(5);
    const int t0 = (int)(pre >> 24), t1 = t0 + (int)my_b;
    const int l0 = (int)(pre & 0xFFFFFFu);
    {
        TextOut o(T, (uint64_t)t0);
        int k = l0;
        int win = p0 / W, wnext = (win + 1) * W;
        for (int p = p0; p < p1; ++p) {
            if (p >= wnext) {
                ++win;
                wnext += W;
            }
            uint32_t v1 = 0, v2 = 0;
            const uint32_t len = line_of(job.rows, c, p, f, bclen, v1, v2, u16_at(job.rows, c, win, S.wf));
            if (!len) continue;
            const uint64_t s = o.pos;
            o.num((uint32_t)p + 1);
            const uint32_t c1 = (uint32_t)(o.pos - s);
            o.put(',', 1);
            for (uint32_t q = 0; q < bclen; q += 8) {  // the barcode from LDS, 8 bytes at a time
                const uint32_t nq = min(8u, bclen - q);
                uint64_t x = 0;
                for (uint32_t u = 0; u < nq; ++u) x |= (uint64_t)S.bc[q + u] << (8 * u);
                o.put(x, (int)nq);
            }
            const uint32_t c2 = (uint32_t)(o.pos - s);
            o.put(',', 1);
            o.num(v1);
            uint32_t c3 = 0;
            if (f) {
                c3 = (uint32_t)(o.pos - s);
                o.put(',', 1);
                o.num(v2);
            }
            o.put('\n', 1);
            uint32_t* le = lines + 3 * (size_t)k++;
            le[0] = (uint32_t)s;
            le[1] = c1 | (c2 << 16);
            le[2] = c3 | (len << 16);
        }
        o.flush();
    }
    __threadfence_block();
    PROF_STAMP(6);
    __syncthreads();
    // CRC of the segment (raw: init 0, no final xor), four bytes per step (slicing-by-4)
    uint32_t r = 0;
    {
        int i = t0;
        for (; i < t1 && (reinterpret_cast<uintptr_t>(T + i) & 3u); ++i) r = S.crc_tab[0][(r ^ T[i]) & 0xFFu] ^ (r >> 8);
        for (; i + 4 <= t1; i += 4) {
            r ^= *reinterpret_cast<const uint32_t*>(T + i);
            r = S.crc_tab[3][r & 0xFFu] ^ S.crc_tab[2][(r >> 8) & 0xFFu] ^ S.crc_tab[1][(r >> 16) & 0xFFu] ^
                S.crc_tab[0][r >> 24];
        }
        for (; i < t1; ++i) r = S.crc_tab[0][(r ^ T[i]) & 0xFFu] ^ (r >> 8);
    }
    PROF_STAMP(7);
    // the text's CRC-32: raw CRCs are linear, so CRC(S_0 .. S_255) = XOR over t of segment t's
    // CRC shifted past the bytes after it (one shift per thread, no tree of barriers)
    uint32_t x = crc_shift(r, n_text - (uint64_t)t1, S.shift);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x ^= __shfl_xor(x, o, 64);
    if ((t & 63) == 0) S.crc_x[t >> 6] = x;
    __syncthreads();
    if (t == 0) {
        uint32_t raw = 0;
        for (int w = 0; w < kT / 64; ++w) raw ^= S.crc_x[w];
        sc.crc[m] = raw ^ crc_shift(0xFFFFFFFFu, n_text, S.shift) ^ 0xFFFFFFFFu;
    }
    sc.seg[m * (kT + 1) + t] = (uint32_t)t0;
    if (t == kT - 1) sc.seg[m * (kT + 1) + kT] = (uint32_t)t1;
    PROF_STAMP(1);
}

constexpr int kWinLines = 1024;  // line table entries of a window (LDS)

struct MatchLds {
    uint8_t win[kWinBytes];
    uint32_t ln[3 * kWinLines];  // the window's lines (start, field offsets, length)
    int win_k1, win_kb;
};

// Kernel 2 (per member): the match candidates of every position (windows of lines
// staged in LDS, match_window).
__global__ void __launch_bounds__(kT, 4) k_txt_match(Job job, Scratch sc) {
    __shared__ MatchLds S;
    const int t = threadIdx.x;
    const int64_t m = blockIdx.x;
    const int f = (int)(m / job.n);
    const int nf = f ? 4 : 3;
    const uint8_t* const T = sc.text + sc.text_off[m];
    const uint32_t* const lines = sc.lines + 3 * sc.line_off[m];
    uint32_t* const tok = sc.tok + sc.text_off[m];
    const uint64_t n_text = sc.text_n[m];
    if (n_text == 0) return;
    const int n_lines = (int)(sc.line_off[m + 1] - sc.line_off[m]);
    // ---- 2. match candidates, windows of lines staged in LDS ----
    auto line_start = [&](int k) -> int64_t { return k >= n_lines ? (int64_t)n_text : (int64_t)lines[3 * (size_t)k]; };
    for (int k0 = 0; k0 < n_lines;) {
        if (t == 0) {
            // look back up to kJ lines (at most half the window), then as many lines as fit
            // with 64 bytes of look-ahead (a line is at most 4096 + 29 bytes)
            const int64_t s0 = line_start(k0);
            int kb = max(0, k0 - kJ);
            while (kb < k0 && s0 - line_start(kb) > kWinBytes / 2) ++kb;
            const int64_t base = line_start(kb);
            int lo = k0 + 1, hi = min(n_lines, kb + kWinLines);  // largest k1 whose text and lines fit
            while (lo < hi) {
                const int mid = (lo + hi + 1) / 2;
                if (line_start(mid) + 64 - base <= kWinBytes) lo = mid;
                else hi = mid - 1;
            }
            S.win_kb = kb;
            S.win_k1 = lo;
        }
        __syncthreads();
        const int kb = S.win_kb, k1 = S.win_k1;
        const int64_t base = line_start(kb);
        const int64_t wend = min((int64_t)n_text, line_start(k1) + 64);
        for (int64_t x = base + t; x < wend; x += kT) S.win[x - base] = T[x];
        for (int q = t; q < 3 * (k1 - kb); q += kT) S.ln[q] = lines[3 * (size_t)kb + q];
        __syncthreads();
        match_window(S.win, base, wend, S.ln, k0, k1, kb, nf, tok);
        __syncthreads();
        k0 = k1;
    }
    PROF_STAMP(2);
}


// The tokens of every thread (ntok each: literal bytes or l << 16 | d; their
// symbol counts in S.lit_f / S.dist_f) as one final deflate block after the frame's
// header bytes (hdr, hdr_len <= 10) in out, whose region (out_bound(n_text) bytes, room
// for the frame included) is zeroed here: dynamic Huffman codes (length-limited), or
// the fixed codes, or stored blocks of the n_text raw bytes T, whichever is smallest.
// Returns the block's bytes (every thread). All threads call. tok(q): the calling thread's
// q-th token (a functor over the caller's token layout).
template <class Tok>
__device__ uint64_t deflate_block(CodeLds& S, const uint8_t* T, const Tok& tok, uint32_t ntok,
                                  uint64_t n_text, uint32_t* out, const uint8_t* hdr, int hdr_len,
                                  uint64_t* stamps = nullptr) {
    const int t = threadIdx.x;
    auto stamp = [&](int q) {  // (profiling: the wall clock after each phase)
        if (stamps) {
            __syncthreads();
            if (t == 0) stamps[q] = wall_clock64();
        }
    };
    if (t == 0) S.lit_f[256] = 1;  // end of block
    __syncthreads();
    huff_lengths(S.lit_f, kLit, 15, S.lit_len, S.h);
    huff_lengths(S.dist_f, kDist, 15, S.dist_len, S.h);
    // ---- 3. codes and the header ----
    if (t == 0) {
        // a complete distance code: at least two used lengths (one used or none -> codes 0 and 1)
        int used = 0;
        for (int s = 0; s < kDist; ++s) used += S.dist_len[s] != 0;
        if (used < 2) {
            int a = -1;
            for (int s = 0; s < kDist; ++s)
                if (S.dist_len[s]) a = s;
            for (int s = 0; s < kDist; ++s) S.dist_len[s] = 0;
            if (a < 0) a = 0;
            S.dist_len[a] = 1;
            S.dist_len[a == 0 ? 1 : 0] = 1;
        }
        canon(S.lit_len, kLit, S.lit_code);
        canon(S.dist_len, kDist, S.dist_code);
        int hl = 257;
        for (int s = 257; s < kLit; ++s)
            if (S.lit_len[s]) hl = s + 1;
        int hd = 1;
        for (int s = 0; s < kDist; ++s)
            if (S.dist_len[s]) hd = s + 1;
        S.hlit = hl;
        S.hdist = hd;
        // run-length code of the lengths (16: repeat previous 3-6, 17: zeros 3-10, 18: zeros 11-138)
        int nr = 0;
        for (int s = 0; s < 19; ++s) S.cl_f[s] = 0;
        const int na = hl + hd;
        for (int i = 0; i < na;) {
            const int v = i < hl ? S.lit_len[i] : S.dist_len[i - hl];
            int r = 1;
            while (i + r < na && (i + r < hl ? S.lit_len[i + r] : S.dist_len[i + r - hl]) == v) ++r;
            if (v == 0 && r >= 3) {
                const int q = min(r, 138);
                S.rle[nr++] = q >= 11 ? (uint16_t)(18 | (q - 11) << 8) : (uint16_t)(17 | (q - 3) << 8);
                S.cl_f[q >= 11 ? 18 : 17]++;
                i += q;
            } else if (v != 0 && r >= 4) {
                S.rle[nr++] = (uint16_t)v;
                S.cl_f[v]++;
                const int q = min(r - 1, 6);
                S.rle[nr++] = (uint16_t)(16 | (q - 3) << 8);
                S.cl_f[16]++;
                i += 1 + q;
            } else {
                S.rle[nr++] = (uint16_t)v;
                S.cl_f[v]++;
                ++i;
            }
        }
        S.n_rle = nr;
    }
    __syncthreads();
    stamp(0);
    huff_lengths(S.cl_f, 19, 7, S.cl_len, S.h);
    if (t == 0) {
        // (a code-length code with one symbol: add a second so the code is complete)
        int used = 0, a = -1;
        for (int s = 0; s < 19; ++s)
            if (S.cl_len[s]) {
                ++used;
                a = s;
            }
        if (used == 1) S.cl_len[a == 0 ? 1 : 0] = 1;
        canon(S.cl_len, 19, S.cl_code);
        int hc = 4;
        for (int i = 0; i < 19; ++i)
            if (S.cl_len[c_cl_ord[i]]) hc = max(hc, i + 1);
        S.hclen = hc;
        uint64_t hb = 3 + 5 + 5 + 4 + 3 * (uint64_t)hc;
        for (int i = 0; i < S.n_rle; ++i) {
            const int sym = S.rle[i] & 0xFF;
            hb += S.cl_len[sym] + (sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0);
        }
        S.hdr_bits = hb;
    }
    __syncthreads();
    stamp(1);
    // ---- 4. sizes of the three block kinds, then the encoder ----
    uint64_t dyn_b = 0, fix_b = 0;
    for (uint32_t q = 0; q < ntok; ++q) {
        const uint32_t tk = tok(q);
        dyn_b += token_bits(tk, S.lit_len, S.dist_len);
        const uint32_t l = tk >> 16;
        if (!l) fix_b += fixed_len((int)tk);
        else {
            const int cc = len_code((int)l), e = dist_code((int)(tk & 0xFFFFu));
            fix_b += fixed_len(257 + cc) + len_xb(cc) + 5 + dist_xb(e);
        }
    }
    if (t == kT - 1) {
        dyn_b += S.lit_len[256];
        fix_b += 7;
    }
    uint64_t dyn_tot, fix_tot;
    const uint64_t dyn_pre = block_excl_scan(dyn_b, S.wsum, dyn_tot);
    const uint64_t fix_pre = block_excl_scan(fix_b, S.wsum, fix_tot);
    const uint64_t dyn_bytes = (S.hdr_bits + dyn_tot + 7) / 8;
    const uint64_t fix_bytes = (3 + fix_tot + 7) / 8;
    const uint64_t n_blk = n_text / 65535 + 1;
    const uint64_t sto_bytes = n_text + 5 * n_blk;
    const int mode = (dyn_bytes <= fix_bytes && dyn_bytes <= sto_bytes) ? 0 : (fix_bytes <= sto_bytes ? 1 : 2);
    const uint64_t blk_bytes = mode == 0 ? dyn_bytes : mode == 1 ? fix_bytes : sto_bytes;
    stamp(2);
    const uint64_t region = out_bound(n_text) / 4;  // (the bound has room for the frame)
    for (uint64_t q = t; q < region; q += kT) out[q] = 0;
    __threadfence_block();
    __syncthreads();
    uint8_t* const ob = reinterpret_cast<uint8_t*>(out);
    if (t == 0)  // the frame's header bytes (the block's first bits share their last word)
        for (int k = 0; k < hdr_len; ++k) atomicOr(&out[k / 4], (uint32_t)hdr[k] << (8 * (k % 4)));
    if (mode == 0) {
        if (t == 0) {
            BitW bw(out, 8 * (uint64_t)hdr_len);
            bw.put(1, 1);  // BFINAL
            bw.put(2, 2);  // dynamic
            bw.put((uint32_t)(S.hlit - 257), 5);
            bw.put((uint32_t)(S.hdist - 1), 5);
            bw.put((uint32_t)(S.hclen - 4), 4);
            for (int i = 0; i < S.hclen; ++i) bw.put(S.cl_len[c_cl_ord[i]], 3);
            for (int i = 0; i < S.n_rle; ++i) {
                const int sym = S.rle[i] & 0xFF, x = S.rle[i] >> 8;
                bw.put(S.cl_code[sym], S.cl_len[sym]);
                if (sym == 16) bw.put((uint32_t)x, 2);
                else if (sym == 17) bw.put((uint32_t)x, 3);
                else if (sym == 18) bw.put((uint32_t)x, 7);
            }
            bw.done();
        }
        BitW bw(out, 8 * (uint64_t)hdr_len + S.hdr_bits + dyn_pre);
        for (uint32_t q = 0; q < ntok; ++q) put_token(bw, tok(q), S.lit_code, S.lit_len, S.dist_code, S.dist_len);
        if (t == kT - 1) bw.put(S.lit_code[256], S.lit_len[256]);
        bw.done();
    } else if (mode == 1) {
        // the fixed codes (RFC 1951 3.2.6), canonical from their lengths
        if (t == 0) {
            for (int s = 0; s < 288 && s < kLit; ++s) S.lit_len[s] = fixed_len(s);
            for (int s = 0; s < kDist; ++s) S.dist_len[s] = 5;
            canon(S.lit_len, kLit, S.lit_code);
            canon(S.dist_len, kDist, S.dist_code);
            BitW bw(out, 8 * (uint64_t)hdr_len);
            bw.put(1, 1);
            bw.put(1, 2);  // fixed
            bw.done();
        }
        __syncthreads();
        BitW bw(out, 8 * (uint64_t)hdr_len + 3 + fix_pre);
        for (uint32_t q = 0; q < ntok; ++q) put_token(bw, tok(q), S.lit_code, S.lit_len, S.dist_code, S.dist_len);
        if (t == kT - 1) bw.put(S.lit_code[256], S.lit_len[256]);
        bw.done();
    } else {
        // stored blocks of <= 65535 bytes: BFINAL/BTYPE byte, LEN, NLEN, the bytes
        for (uint64_t b = t; b < n_blk; b += kT) {
            const uint64_t o = hdr_len + b * (65535 + 5);
            const uint64_t left = n_text - b * 65535;
            const uint32_t len = (uint32_t)(left < 65535 ? left : 65535);
            ob[o] = b + 1 == n_blk ? 1 : 0;
            ob[o + 1] = (uint8_t)len;
            ob[o + 2] = (uint8_t)(len >> 8);
            ob[o + 3] = (uint8_t)~len;
            ob[o + 4] = (uint8_t)(~len >> 8);
        }
        for (uint64_t x = t; x < n_text; x += kT) ob[hdr_len + 5 * (x / 65535 + 1) + x] = T[x];
    }
    __threadfence_block();
    __syncthreads();
    return blk_bytes;
}

// Kernel 3 (per member): the optimal parse of each segment, the Huffman codes, the
// encoded block (dynamic, fixed or stored: the smallest) and the gzip frame.
__global__ void __launch_bounds__(kT) k_txt_code(Job job, Scratch sc) {
    __shared__ CodeLds S;
    const int t = threadIdx.x;
    const int64_t m = blockIdx.x;
    const uint8_t* const T = sc.text + sc.text_off[m];
    uint32_t* const tok = sc.tok + sc.text_off[m];
    const uint64_t n_text = sc.text_n[m];
    uint32_t* const out = sc.out + sc.out_off[m] / 4;
    if (n_text == 0) {  // no line: no member
        if (t == 0) sc.member_bytes[m] = 0;
        return;
    }
    const int t0 = (int)sc.seg[m * (kT + 1) + t], t1 = (int)sc.seg[m * (kT + 1) + t + 1];
    // ---- 3. optimal parse (one pass at default prices: a second pass at the member's own
    // code lengths gained 0.4-1 % on C4-like text for twice the parse time) ----
    lds_prices_default(S);
    for (int s = t; s < kLit; s += kT) S.lit_f[s] = 0;
    if (t < kDist) S.dist_f[t] = 0;
    __syncthreads();
    dp_segment(T, tok, t0, t1, S);
    // traceback: the chosen tokens, stored over the candidates (compacted), and their counts
    uint32_t ntok = 0;
    for (int i = t0; i < t1;) {
        const uint32_t w = tok[i];
        const uint32_t l = (w >> 22) & 63u;
        if (!l) {
            atomicAdd(&S.lit_f[T[i]], 1u);
            tok[t0 + ntok] = T[i];
            ++i;
        } else {
            const uint32_t d = w & 0xFFFFu;
            atomicAdd(&S.lit_f[257 + len_code((int)l)], 1u);
            atomicAdd(&S.dist_f[dist_code((int)d)], 1u);
            tok[t0 + ntok] = (l << 16) | d;
            i += (int)l;
        }
        ++ntok;
    }
    PROF_STAMP(3);
    const uint8_t gz_hdr[10] = {0x1F, 0x8B, 0x08, 0, 0, 0, 0, 0, 0x02, 0xFF};  // magic, deflate, mtime 0, xfl 2, os 255
    const uint64_t blk_bytes = deflate_block(S, T, [&](uint32_t q) { return tok[t0 + q]; }, ntok, n_text, out, gz_hdr, 10);
    uint8_t* const ob = reinterpret_cast<uint8_t*>(out);
    __threadfence_block();
    __syncthreads();
    if (t == 0) {
        const uint32_t crc = sc.crc[m];
        const uint64_t o = 10 + blk_bytes;
        const uint32_t isz = (uint32_t)n_text;
        for (int q = 0; q < 4; ++q) {
            ob[o + q] = (uint8_t)(crc >> (8 * q));
            ob[o + 4 + q] = (uint8_t)(isz >> (8 * q));
        }
        sc.member_bytes[m] = (uint32_t)(o + 8);
    }
    PROF_STAMP(4);
}

__global__ void __launch_bounds__(kT) k_txt_pack(const uint32_t* __restrict__ out, const uint64_t* __restrict__ out_off,
                                                 const uint32_t* __restrict__ member_bytes,
                                                 const uint64_t* __restrict__ dst_off, uint8_t* __restrict__ dst) {
    const int64_t m = blockIdx.x;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(out) + out_off[m];
    uint8_t* d = dst + dst_off[m];
    const uint32_t n = member_bytes[m];
    for (uint32_t q = threadIdx.x; q < n; q += kT) d[q] = src[q];
}

// ---------------------------------------------------------------------------
// HDF5 chunks: the 11 planes' (crow x ccol) u16 chunks as zlib streams
// ---------------------------------------------------------------------------
// One workgroup per (row chunk, column chunk) of the batch: each position of each column
// read once (a cell's 8 counts as one uint4), the 11 planes' raw chunks written row-major
// (consecutive threads, consecutive columns of a chunk row).
constexpr int kSumRows = 4096;  // chunk rows whose column sums a workgroup gathers in LDS

__global__ void __launch_bounds__(kT) k_h5_gather(H5Job job, H5Scratch sc) {
    __shared__ uint32_t srow[3][kSumRows];  // (<= 100 columns x 65535 per row and plane)
    const bool lsum = job.crow <= kSumRows && (int64_t)job.ccol * 65535 < ((int64_t)1 << 32);
    if (lsum)
        for (int q = threadIdx.x; q < 3 * job.crow; q += kT) srow[q / job.crow][q % job.crow] = 0;
    __syncthreads();
    const int r = blockIdx.x;
    const int rc = r / job.ncc, ccl = r - rc * job.ncc;
    const int cc = job.cc0 + ccl;
    const int n = job.crow * job.ccol;
    uint16_t* const base = reinterpret_cast<uint16_t*>(sc.raw);
    const size_t pstride = (size_t)job.nrc * job.ncc * (sc.raw_stride / 2);  // one plane's chunks (u16)
    const size_t k0 = ((size_t)rc * job.ncc + ccl) * (sc.raw_stride / 2);
    for (int x = threadIdx.x; x < n; x += kT) {
        const int row = x / job.ccol, c = x - row * job.ccol;
        const int p = rc * job.crow + row;
        const int64_t col = (int64_t)cc * job.ccol + c;
        const int cell = (p < job.L && col < job.n_cols) ? job.cell_of_col[col] : -1;
        uint4 a = make_uint4(0, 0, 0, 0);
        uint32_t tt = 0, d = 0;
        if (cell >= 0) {
            const size_t P = (size_t)cell * job.L + p;
            a = job.c16[P];
            tt = job.t16[P];
            d = job.d16[P];
        }
        const uint32_t w[4] = {a.x, a.y, a.z, a.w};
        uint16_t* const o = base + k0 + x;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            o[(2 * q) * pstride] = (uint16_t)(w[q] & 0xFFFFu);
            o[(2 * q + 1) * pstride] = (uint16_t)(w[q] >> 16);
        }
        o[8 * pstride] = (uint16_t)(tt & 0xFFFFu);
        o[9 * pstride] = (uint16_t)(tt >> 16);
        o[10 * pstride] = (uint16_t)d;
        // the report's per-position sums over the columns (writers.py:_report_arrays)
        const uint32_t v3[3] = {d, tt & 0xFFFFu, tt >> 16};
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            if (!v3[q]) continue;
            if (lsum) atomicAdd(&srow[q][row], v3[q]);
            else atomicAdd(&job.sums[(size_t)q * job.L + p], (unsigned long long)v3[q]);
        }
    }
    if (!lsum) return;
    __syncthreads();
    for (int q = threadIdx.x; q < 3 * job.crow; q += kT) {
        const int pl = q / job.crow, row = q - pl * job.crow, p = rc * job.crow + row;
        const uint32_t v = srow[pl][row];
        if (v && p < job.L) atomicAdd(&job.sums[(size_t)pl * job.L + p], (unsigned long long)v);
    }
}

// One workgroup per chunk: a greedy parse into runs (distance 1, lengths 3-258: on C4
// count planes it gives 0.20 of the raw bytes where zlib level 4, the reference's
// compression_opts, gives 0.204, and further distances, same cell one position back or
// the next column, made the streams larger), the block (deflate_block) and the zlib frame
// (header 78 5E, Adler-32). Thread t parses [s_t, s_t+1) where s_t is its nominal start
// moved past the run that continues across it (so the run stays one token of thread t-1).
__global__ void __launch_bounds__(kT) k_h5_code(H5Job job, H5Scratch sc) {
    __shared__ CodeLds S;
    __shared__ uint64_t red[4];
    const int t = threadIdx.x;
    const int64_t k = blockIdx.x;
    const uint8_t* const T = sc.raw + k * sc.raw_stride;
    uint32_t* const tok = sc.tok + k * sc.tok_stride;
    uint32_t* const out = sc.out + k * (sc.out_stride / 4);
    const int n = (int)sc.chunk_raw;
    const int P = h5_seg_bytes(sc.chunk_raw);  // 16-byte aligned nominal segments (kT of them)
    __shared__ int rr[kT];
#define H5_STAMP(q)                                                                   \
    do {                                                                              \
        if (sc.prof) {                                                                \
            __syncthreads();                                                          \
            if (t == 0) sc.prof[k * 8 + (q)] = wall_clock64();                        \
        }                                                                             \
    } while (0)
    H5_STAMP(0);
    // the run continuing across a nominal start belongs to the previous thread's last token
    const int s = min(n, t * P), snext = min(n, s + P);
    int r = 0;
    if (t > 0 && s < n) {
        const uint32_t v = T[s - 1];
        bool go = true;
        for (int i = s; go && i < snext; i += 4) {
            const uint32_t w = *reinterpret_cast<const uint32_t*>(T + i);
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                go = go && i + b < snext && ((w >> (8 * b)) & 0xFFu) == v;
                r += go;
            }
        }
    }
    rr[t] = r;
    for (int q = t; q < kLit; q += kT) S.lit_f[q] = 0;
    if (t < kDist) S.dist_f[t] = 0;
    __syncthreads();
    const int t0 = s + r, t1 = snext + (t + 1 < kT ? rr[t + 1] : 0);
    // one forward pass over the bytes (16 per load, no load waits on a token): a run of
    // bytes equal to the previous one is pending until it breaks or reaches 258 bytes,
    // then it is a match (>= 3 bytes, distance 1) or literals
    uint32_t ntok = 0;
    uint64_t A = 0, W = 0;  // Adler-32 partial sums: sum of bytes, sum of (t1 - i) x byte
    int pend = 0;
    int pv = t0 > 0 ? (int)T[t0 - 1] : -1;
    // the tokens as u16 (a literal byte, or 256 + length - 3 of a distance-1 match), the
    // thread's q-th at tok16[q kT + t]: each wave's loads and stores of its q-th tokens are
    // one contiguous range (the thread-contiguous layout cost 0.6 ms per chunk in each
    // pass over the tokens: 64 lines per wave access)
    uint16_t* const tok16 = reinterpret_cast<uint16_t*>(tok);
    auto put = [&](uint32_t v) { tok16[(size_t)ntok++ * kT + t] = (uint16_t)v; };
    auto flush = [&]() {
        if (pend >= 3) {
            atomicAdd(&S.lit_f[257 + len_code(pend)], 1u);
            atomicAdd(&S.dist_f[0], 1u);
            put(256u + (uint32_t)(pend - 3));
        } else {
            for (int q = 0; q < pend; ++q) {
                atomicAdd(&S.lit_f[pv], 1u);
                put((uint32_t)pv);
            }
        }
    };
    for (int base = t0 & ~15; base < t1; base += 16) {
        const uint4 w4 = *reinterpret_cast<const uint4*>(T + base);
        const uint32_t ws[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int b = 0; b < 16; ++b) {
            const int i = base + b;
            if (i < t0 || i >= t1) continue;
            const int c = (int)((ws[b >> 2] >> (8 * (b & 3))) & 0xFFu);
            A += (uint64_t)c;
            W += (uint64_t)c * (uint64_t)(t1 - i);
            if (c == pv && pend < 258) {
                ++pend;
                continue;
            }
            flush();
            if (c == pv) {  // (a run past 258 bytes goes on)
                pend = 1;
            } else {
                pend = 0;
                atomicAdd(&S.lit_f[c], 1u);
                put((uint32_t)c);
                pv = c;
            }
        }
    }
    flush();
    H5_STAMP(1);
    // Adler-32 of the chunk: s1 = 1 + sum b, s2 = n + sum_i (n - i) b_i
    uint64_t a_tot, w_tot;
    (void)block_excl_scan(A, red, a_tot);
    (void)block_excl_scan(W + (uint64_t)(n - t1) * A, red, w_tot);
    const uint32_t s1 = (uint32_t)((1 + a_tot) % 65521u), s2 = (uint32_t)(((uint64_t)n + w_tot) % 65521u);
    const uint8_t zhdr[2] = {0x78, 0x5E};
    H5_STAMP(2);
    auto tok_of = [&](uint32_t q) -> uint32_t {
        const uint32_t v = tok16[(size_t)q * kT + t];
        return v < 256u ? v : ((v - 253u) << 16) | 1u;  // (length v - 256 + 3, distance 1)
    };
    const uint64_t blk = deflate_block(S, T, tok_of, ntok, (uint64_t)n, out, zhdr, 2, sc.prof ? sc.prof + k * 8 + 4 : nullptr);
    if (t == 0) {
        uint8_t* const ob = reinterpret_cast<uint8_t*>(out);
        const uint32_t ad = (s2 << 16) | s1;
        for (int q = 0; q < 4; ++q) ob[2 + blk + q] = (uint8_t)(ad >> (24 - 8 * q));  // big-endian
        sc.chunk_bytes[k] = (uint32_t)(2 + blk + 4);
    }
    H5_STAMP(3);
#undef H5_STAMP
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
int txt_sizes(const Job& job, uint64_t* sizes, uint64_t* nlines, hipStream_t s) {
    if (job.n <= 0) return 0;
    k_txt_sizes<<<(unsigned)job.n, kT, 0, s>>>(job, sizes, nlines);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int txt_deflate(const Job& job, const Scratch& sc, hipStream_t s) {
    if (job.n <= 0) return 0;
    const unsigned nm = (unsigned)(kFiles * job.n);
    k_txt_format<<<nm, kT, 0, s>>>(job, sc);
    k_txt_match<<<nm, kT, 0, s>>>(job, sc);
    k_txt_code<<<nm, kT, 0, s>>>(job, sc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int txt_pack(const Scratch& sc, int64_t n_members, const uint64_t* dst_off, uint8_t* dst, hipStream_t s) {
    if (n_members <= 0) return 0;
    k_txt_pack<<<(unsigned)n_members, kT, 0, s>>>(sc.out, sc.out_off, sc.member_bytes, dst_off, dst);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int h5_deflate(const H5Job& job, const H5Scratch& sc, hipStream_t s) {
    const unsigned regions = (unsigned)(job.nrc * job.ncc);
    if (!regions) return 0;
    k_h5_gather<<<regions, kT, 0, s>>>(job, sc);
    k_h5_code<<<regions * kPlanes, kT, 0, s>>>(job, sc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int h5_pack(const H5Scratch& sc, int64_t n_chunks, const uint64_t* dst_off, uint8_t* dst, hipStream_t s) {
    if (n_chunks <= 0) return 0;
    k_txt_pack<<<(unsigned)n_chunks, kT, 0, s>>>(sc.out, sc.out_off, sc.chunk_bytes, dst_off, dst);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

void crc_shift_matrices(uint32_t* M) {
    uint32_t tab[256];
    for (uint32_t s = 0; s < 256; ++s) {
        uint32_t r = s;
        for (int b = 0; b < 8; ++b) r = (r >> 1) ^ (0xEDB88320u & (0u - (r & 1u)));
        tab[s] = r;
    }
    for (int k = 0; k < 32; ++k) {  // one zero byte: c -> tab[c & 0xFF] ^ (c >> 8)
        const uint32_t c = 1u << k;
        M[k] = tab[c & 0xFFu] ^ (c >> 8);
    }
    for (int b = 1; b < kShiftPow; ++b) {  // M[b] = M[b-1] o M[b-1]
        const uint32_t* A = M + 32 * (b - 1);
        uint32_t* B = M + 32 * b;
        for (int k = 0; k < 32; ++k) {
            uint32_t v = A[k], r = 0;
            for (int q = 0; q < 32; ++q)
                if ((v >> q) & 1u) r ^= A[q];
            B[k] = r;
        }
    }
}

}  // namespace txtgz
}  // namespace mgp
