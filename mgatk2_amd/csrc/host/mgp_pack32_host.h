// mgp_pack32_host.h — the host producers' 32-byte record builder (libmgphost.so).
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

}  // namespace mgp_host
