// mgp_pack32_host.h — the host producers' 32- and 64-byte record builders (libmgphost.so).
//
// Same bytes as mgp_pack32_record (include/mgpileup.h, the layout's definition, also
// used by the device generator), built without a branch per query position: the
// counted positions as one 64-bit mask (aligned-block ranges of the CIGAR walk of
// pileup.py:55-95, the end-distance window of pileup.py:67-78, int8 quality >= min_baseq
// of pileup.py:80 by SSE2 byte compares, ACGT of pileup.py:83-86 by a byte table), then
// the 3-bit codes deposited into place with BMI2 pdep (three words of 21, 21 and 8
// positions). The per-position loop of the definition cost ~320 ns per read on one
// core (branch mispredictions on the 20 % low-quality bases); this one ~40 ns.
// Checked byte for byte against the Python mirror of the definition
// (tests/test_pack32.py, through mgp_repack32).
#pragma once
#include <immintrin.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "../../../include/mgpileup.h"

namespace mgp_host {

struct Pack32Tables {
    uint8_t base4[256];  // byte of two BAM nibbles -> (base of the high nibble) | (base of the low) << 2
    uint8_t ok2[256];    // -> bit 0: high nibble is A/C/G/T, bit 1: low nibble is
    Pack32Tables() {
        auto b = [](uint32_t n) -> uint32_t { return n == 1 ? 0u : n == 2 ? 1u : n == 4 ? 2u : n == 8 ? 3u : 0u; };
        auto ok = [](uint32_t n) -> uint32_t { return n == 1 || n == 2 || n == 4 || n == 8; };
        for (uint32_t x = 0; x < 256; ++x) {
            base4[x] = (uint8_t)(b(x >> 4) | (b(x & 15) << 2));
            ok2[x] = (uint8_t)(ok(x >> 4) | (ok(x & 15) << 1));
        }
    }
};
inline const Pack32Tables& pack32_tables() {
    static const Pack32Tables t;
    return t;
}

// the repeated 3-bit patterns 001 and 011 over n positions
constexpr uint64_t rep3(uint64_t v, int n) { return n == 0 ? 0ull : (v | (rep3(v, n - 1) << 3)); }

__attribute__((target("bmi2"))) inline void pack32_codes_bmi2(uint64_t counted, uint64_t b0, uint64_t b1,
                                                                uint64_t w[3]) {
    // b0: 2-bit bases of positions 0..31, b1: of positions 32..49
    const uint64_t grp_cnt[3] = {counted & 0x1FFFFFull, (counted >> 21) & 0x1FFFFFull, (counted >> 42) & 0xFFull};
    const uint64_t grp_base[3] = {b0 & ((1ull << 42) - 1), ((b0 >> 42) | (b1 << 22)) & ((1ull << 42) - 1),
                                  (b1 >> 20) & 0xFFFFull};
    const int np[3] = {21, 21, 8};
    for (int g = 0; g < 3; ++g) {
        const uint64_t m1 = rep3(1, np[g]) & ((np[g] == 21) ? ~0ull : ((1ull << (3 * np[g])) - 1));
        const uint64_t m3 = m1 * 3, m4 = m1 << 2;
        const uint64_t full = (1ull << np[g]) - 1;
        const uint64_t c = _pdep_u64(grp_cnt[g], m1) * 3;                // 011 where counted
        const uint64_t b = _pdep_u64(grp_base[g], m3);                   // the base in every slot
        const uint64_t u = _pdep_u64(~grp_cnt[g] & full, m4);            // 100 where not counted
        w[g] = (b & c) | u;
    }
}

inline void pack32_codes_portable(uint64_t counted, uint64_t b0, uint64_t b1, uint64_t w[3]) {
    w[0] = w[1] = w[2] = 0;
    for (int k = 0; k < MGP_PACK_MAX_LEN; ++k) {
        const uint64_t c = (counted >> k) & 1ull;
        const uint64_t base = k < 32 ? (b0 >> (2 * k)) & 3ull : (b1 >> (2 * (k - 32))) & 3ull;
        const uint64_t v = (base & (0ull - c)) | ((c ^ 1ull) << 2);
        w[k / 21] |= v << (3 * (k % 21));
    }
}

// (MGP_NO_BMI2=1 forces the portable code deposit: tests/test_pack32.py checks both)
inline bool cpu_has_bmi2() {
    static const bool has = __builtin_cpu_supports("bmi2") && !std::getenv("MGP_NO_BMI2");
    return has;
}

// mgp_pack32_record's contract: returns 1 and writes out[0..32), or 0 (out untouched).
inline int pack32_record_fast(int32_t start, uint32_t l_seq, uint16_t flag, uint32_t n_cigar, const uint32_t* cigar,
                              const uint8_t* seq, const uint8_t* qual, int32_t min_baseq, int32_t min_dist,
                              uint8_t* out) {
    const int32_t md = min_dist > 0 ? min_dist : 0;
    if ((flag & MGP_FLAG_NOSEQQUAL) || l_seq == 0u || l_seq > MGP_PACK_MAX_LEN || n_cigar > 4u) return 0;
    if (start < 0 || start >= 65536 || min_baseq < -128 || min_baseq > 127 || md > 15) return 0;
    uint64_t inblk = 0;
    uint32_t blocks = 0, q = 0;
    for (uint32_t k = 0; k < n_cigar; ++k) {
        const uint32_t op = cigar[k] & 15u, len = cigar[k] >> 4;
        if (len >= 4096u) return 0;
        const bool aligned = op == 0u || op == 7u || op == 8u;
        if (aligned) {
            ++blocks;
            if (q < l_seq) {
                const uint32_t e = q + len < l_seq ? q + len : l_seq;
                inblk |= ((1ull << (e - q)) - 1ull) << q;
            }
        }
        if (aligned || op == 4u) q += len;
    }
    if (blocks > 2u) return 0;
    const uint64_t lmask = (1ull << l_seq) - 1ull;
    const uint64_t win = (int32_t)l_seq - md > md ? (((1ull << (l_seq - (uint32_t)md)) - 1ull) & ~((1ull << md) - 1ull))
                                                  : 0ull;
    // int8(qual[k]) >= min_baseq, 16 positions per compare (pileup.py Q5: >= 128 wraps)
    uint64_t qm = lmask;
    if (min_baseq > -128) {
        alignas(16) uint8_t qb[64];
        std::memcpy(qb, qual, l_seq);
        const __m128i thr = _mm_set1_epi8((char)(min_baseq - 1));
        qm = 0;
        for (int j = 0; j < 4; ++j) {
            const __m128i v = _mm_load_si128(reinterpret_cast<const __m128i*>(qb + 16 * j));
            qm |= (uint64_t)(uint16_t)_mm_movemask_epi8(_mm_cmpgt_epi8(v, thr)) << (16 * j);
        }
        qm &= lmask;
    }
    // bases: two positions per sequence byte (high nibble first)
    const Pack32Tables& T = pack32_tables();
    uint64_t b0 = 0, b1 = 0, acgt = 0;
    const uint32_t nb = (l_seq + 1u) / 2u;
    for (uint32_t j = 0; j < nb; ++j) {
        const uint8_t x = seq[j];
        acgt |= (uint64_t)T.ok2[x] << (2 * j);
        if (j < 16) b0 |= (uint64_t)T.base4[x] << (4 * j);
        else b1 |= (uint64_t)T.base4[x] << (4 * (j - 16));
    }
    const uint64_t counted = inblk & win & qm & acgt & lmask;
    uint64_t w[3];
    if (cpu_has_bmi2()) pack32_codes_bmi2(counted, b0, b1, w);
    else pack32_codes_portable(counted, b0, b1, w);
    // header (12 bytes), then the codes from bit 96: w0 bits 0..62, w1 from 63, w2 from 126
    out[0] = (uint8_t)start;
    out[1] = (uint8_t)((uint32_t)start >> 8);
    out[2] = (uint8_t)l_seq;
    out[3] = (uint8_t)(n_cigar | ((uint32_t)md << 3) | ((flag & MGP_FLAG_REVERSE) ? 0x80u : 0u));
    for (uint32_t k = 0; k < 4u; ++k) {
        const uint32_t c = k < n_cigar ? cigar[k] : 0u;
        out[4 + 2 * k] = (uint8_t)c;
        out[5 + 2 * k] = (uint8_t)(c >> 8);
    }
    const uint64_t lo = w[0] | (w[1] << 63);
    const uint64_t mid = (w[1] >> 1) | (w[2] << 62);
    const uint64_t hi = w[2] >> 2;
    std::memcpy(out + 12, &lo, 8);
    std::memcpy(out + 20, &mid, 8);
    const uint32_t hi3 = (uint32_t)hi;  // bits 128..151 of the code field: 22 bits used
    out[28] = (uint8_t)hi3;
    out[29] = (uint8_t)(hi3 >> 8);
    out[30] = (uint8_t)(hi3 >> 16);
    out[31] = (uint8_t)(int8_t)min_baseq;
    return 1;
}

// ---- 64-byte records (mgp_pack_record's bytes, include/mgpileup.h) ----
// The definition's per-position loop (nibble, four-way code test, quality shift: ~50
// branches) was most of the BAM decoder's pool pass. Here 16 positions per step with
// SSSE3 byte shuffles: the sequence nibbles spread to one byte per position, the BAM
// code mapped to the base by a 16-entry table (A, C, G, T -> 0..3, any other code ->
// 0xFF, which ORed into qual << 2 gives the definition's 0xFF), positions >= l_seq
// set to 0xFF; the record leaves in four 16-byte stores (non-temporal into aligned
// slots: the decoder never reads the payload back, the device copy does).
// Precondition: the read is packable (bam_packable / mgp_pack_record's tests passed);
// seq32 and qual64 are 32 and 64 readable bytes holding the read's sequence and
// quality first (bytes past them are never used).
__attribute__((target("ssse3"))) inline void pack64_record_ssse3(int32_t start, uint32_t l_seq, uint16_t flag,
                                                                   uint32_t n_cigar, const uint32_t* cigar,
                                                                   const uint8_t* seq32, const uint8_t* qual64,
                                                                   uint8_t* out) {
    const __m128i lut = _mm_setr_epi8(-1, 0, 1, -1, 2, -1, -1, -1, 3, -1, -1, -1, -1, -1, -1, -1);
    const __m128i dup = _mm_setr_epi8(0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7);
    const __m128i odd = _mm_set1_epi16((short)0xFF00);
    const __m128i nib = _mm_set1_epi8(0x0F), fc = _mm_set1_epi8((char)0xFC);
    const __m128i len = _mm_set1_epi8((char)l_seq);
    __m128i idx = _mm_setr_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    __m128i v[4];
    for (int j = 0; j < 4; ++j) {
        const __m128i x = _mm_shuffle_epi8(_mm_loadl_epi64(reinterpret_cast<const __m128i*>(seq32 + 8 * j)), dup);
        const __m128i code = _mm_or_si128(_mm_andnot_si128(odd, _mm_and_si128(_mm_srli_epi16(x, 4), nib)),
                                          _mm_and_si128(odd, _mm_and_si128(x, nib)));
        const __m128i q = _mm_loadu_si128(reinterpret_cast<const __m128i*>(qual64 + 16 * j));
        const __m128i b = _mm_or_si128(_mm_and_si128(_mm_slli_epi16(q, 2), fc), _mm_shuffle_epi8(lut, code));
        v[j] = _mm_or_si128(b, _mm_cmpeq_epi8(_mm_min_epu8(idx, len), len));  // idx >= l_seq -> 0xFF
        idx = _mm_add_epi8(idx, _mm_set1_epi8(16));
    }
    uint64_t c[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < n_cigar && k < 4u; ++k) c[k] = cigar[k] & 0xFFFFu;
    const uint64_t lo = (uint64_t)(uint32_t)start | (uint64_t)l_seq << 32 |
                        (uint64_t)(n_cigar | ((flag & MGP_FLAG_REVERSE) ? 0x80u : 0u)) << 40 | c[0] << 48;
    const uint64_t hi = c[1] | c[2] << 16 | c[3] << 32;
    const __m128i o0 = _mm_or_si128(_mm_set_epi64x((long long)hi, (long long)lo), _mm_slli_si128(v[0], 14));
    const __m128i o1 = _mm_alignr_epi8(v[1], v[0], 2), o2 = _mm_alignr_epi8(v[2], v[1], 2);
    const __m128i o3 = _mm_alignr_epi8(v[3], v[2], 2);
    __m128i* d = reinterpret_cast<__m128i*>(out);
    if (((uintptr_t)out & 15u) == 0) {
        _mm_stream_si128(d, o0);
        _mm_stream_si128(d + 1, o1);
        _mm_stream_si128(d + 2, o2);
        _mm_stream_si128(d + 3, o3);
    } else {
        _mm_storeu_si128(d, o0);
        _mm_storeu_si128(d + 1, o1);
        _mm_storeu_si128(d + 2, o2);
        _mm_storeu_si128(d + 3, o3);
    }
}

// (MGP_NO_SSSE3=1 forces the definition's loop: tests compare both)
inline bool cpu_has_ssse3() {
    static const bool has = __builtin_cpu_supports("ssse3") && !std::getenv("MGP_NO_SSSE3");
    return has;
}

// mgp_pack_record for a packable read whose fields lie in a record ending at `end`
// (the SIMD loads read up to 32 bytes from seq and 64 from qual: shorter tails go
// through a local copy); callers issue _mm_sfence() before publishing the payload.
inline void pack64_record_fast(int32_t start, uint32_t l_seq, uint16_t flag, uint32_t n_cigar, const uint32_t* cigar,
                               const uint8_t* seq, const uint8_t* qual, const uint8_t* end, uint8_t* out) {
    if (!cpu_has_ssse3()) {
        mgp_pack_record(start, l_seq, flag, n_cigar, cigar, seq, qual, out);
        return;
    }
    if (seq + 32 <= end && qual + 64 <= end) {
        pack64_record_ssse3(start, l_seq, flag, n_cigar, cigar, seq, qual, out);
        return;
    }
    alignas(16) uint8_t s[32] = {0}, q[64] = {0};
    std::memcpy(s, seq, (l_seq + 1u) / 2u);
    std::memcpy(q, qual, l_seq);
    pack64_record_ssse3(start, l_seq, flag, n_cigar, cigar, s, q, out);
}

}  // namespace mgp_host
