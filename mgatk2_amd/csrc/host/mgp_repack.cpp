// mgp_repack.cpp — 32-byte records from a batch's full records (host side, libmgphost.so).
//
// The producer-side half of the 32-byte layout (include/mgpileup.h, MGP_FLAG_PACK32):
// the per-base filter of pileup.py:67-88 (end distance, int8 quality >= min_baseq,
// ACGT) and the aligned-block walk of pileup.py:55-95 resolved into one 3-bit code
// per query position for one run's thresholds. The BAM decoder does the same per
// record as it decodes (mgp_bam.cpp, mgp_pack32_record on the BAM fields); this entry
// point does it for a batch already in the full layout (e.g. one built through the
// SimpleRead API), and lets the bench time the per-read cost of the code build.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/mgpileup.h"
#include "../../../include/mgpileup_host.h"
#include "mgp_pack32_host.h"

std::string& mgp_host_err();

extern "C" int64_t mgp_repack32(int64_t n, const uint8_t* payload, int64_t payload_bytes, const uint64_t* rec_off,
                                const uint16_t* flag, int32_t min_baseq, int32_t min_dist, uint8_t* out32,
                                uint16_t* out_flag, int n_threads) {
    if (n < 0 || (n && (!payload || !rec_off || !flag || !out32 || !out_flag))) {
        mgp_host_err() = "mgp_repack32: null or negative arguments";
        return -1;
    }
    if (min_baseq < -128 || min_baseq > 127 || min_dist > 15) {
        mgp_host_err() = "mgp_repack32: 32-byte records need min_baseq in [-128, 127] and min_dist_from_end <= 15";
        return -1;
    }
    const int nt = std::max(1, std::min<int>(n_threads, (int)std::max<int64_t>(1, n / 65536)));
    std::atomic<int64_t> packed{0};
    std::atomic<bool> bad{false};
    auto work = [&](int t) {
        const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
        int64_t k = 0;
        for (int64_t i = lo; i < hi; ++i) {
            uint8_t* o = out32 + (size_t)i * MGP_PACK32_BYTES;
            const uint16_t f = flag[i];
            out_flag[i] = f;
            const uint64_t r = rec_off[i];
            if ((f & (MGP_FLAG_PACKED | MGP_FLAG_PACK32)) || (f & MGP_FLAG_NOSEQQUAL) || r + 16 > (uint64_t)payload_bytes) {
                std::memset(o, 0, MGP_PACK32_BYTES);  // not a full record with SEQ and QUAL: kept as it is
                bad = bad || r + 16 > (uint64_t)payload_bytes;
                continue;
            }
            const uint8_t* rec = payload + r;
            int32_t start;
            uint32_t l_seq, coff;
            uint16_t ncig;
            std::memcpy(&start, rec, 4);
            std::memcpy(&l_seq, rec + 4, 4);
            std::memcpy(&ncig, rec + 8, 2);
            std::memcpy(&coff, rec + 12, 4);
            if (r + (uint64_t)coff + 4ull * ncig > (uint64_t)payload_bytes ||
                r + mgp_seq_offset(l_seq) + (l_seq + 1) / 2 > (uint64_t)payload_bytes) {
                bad = true;
                std::memset(o, 0, MGP_PACK32_BYTES);
                continue;
            }
            uint32_t cw[4] = {0, 0, 0, 0};
            if (ncig <= 4) std::memcpy(cw, rec + coff, 4u * ncig);
            if (ncig <= 4 && mgp_host::pack32_record_fast(start, l_seq, f, ncig, cw, rec + mgp_seq_offset(l_seq), rec + 16,
                                               min_baseq, min_dist, o)) {
                out_flag[i] = (uint16_t)(f | MGP_FLAG_PACK32);
                ++k;
            } else {
                std::memset(o, 0, MGP_PACK32_BYTES);
            }
        }
        packed += k;
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    if (bad) {
        mgp_host_err() = "mgp_repack32: a record lies outside the payload";
        return -1;
    }
    return packed;
}
