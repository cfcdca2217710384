// mgp_shard.cpp — record gather for cell sharding (host side, libmgphost.so).
//
// Cells are split over devices in contiguous whitelist ranges;
// each device's batch holds the records of its cells in BAM order. The SoA
// columns are gathered by index in numpy; the payload records are gathered here:
// sizes and the new offsets in one pass, then a parallel copy. (A numpy byte
// gather needs an 8-byte index per payload byte: 205 GB for the 25.6 GB C4 payload.)
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/mgpileup_host.h"

std::string& mgp_host_err();  // mgp_bam.cpp

extern "C" {

int64_t mgp_gather_offsets(const uint64_t* rec_off, int64_t n_total, int64_t payload_bytes, const int64_t* idx,
                           int64_t m, int32_t rec_align, uint64_t* out_off) {
    mgp_host_err().clear();
    if ((n_total && !rec_off) || (m && (!idx || !out_off)) || m < 0 || n_total < 0 || rec_align < 16 ||
        (rec_align & (rec_align - 1))) {
        mgp_host_err() = "mgp_gather_offsets: bad arguments";
        return -1;
    }
    const uint64_t amask = (uint64_t)rec_align - 1;
    uint64_t off = 0;
    for (int64_t k = 0; k < m; ++k) {
        const int64_t i = idx[k];
        if (i < 0 || i >= n_total) {
            mgp_host_err() = "mgp_gather_offsets: index out of range";
            return -1;
        }
        const uint64_t end = i + 1 < n_total ? rec_off[i + 1] : (uint64_t)payload_bytes;
        if (end < rec_off[i] || end > (uint64_t)payload_bytes) {
            mgp_host_err() = "mgp_gather_offsets: record offsets not increasing";
            return -1;
        }
        out_off[k] = off;
        off += (end - rec_off[i] + amask) & ~amask;
    }
    return (int64_t)off;
}

int mgp_gather_records(const uint8_t* payload, const uint64_t* rec_off, int64_t n_total, int64_t payload_bytes,
                       const int64_t* idx, int64_t m, const uint64_t* out_off, int64_t out_bytes, uint8_t* out,
                       int n_threads) {
    mgp_host_err().clear();
    if (m < 0 || (m && (!payload || !rec_off || !idx || !out_off || !out))) {
        mgp_host_err() = "mgp_gather_records: bad arguments";
        return -1;
    }
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(std::max(n_threads, 1), m / 65536 + 1));
    auto work = [&](int t) {
        const int64_t lo = m * t / nt, hi = m * (t + 1) / nt;
        for (int64_t k = lo; k < hi; ++k) {
            const int64_t i = idx[k];
            const uint64_t end = i + 1 < n_total ? rec_off[i + 1] : (uint64_t)payload_bytes;
            const uint64_t next = k + 1 < m ? out_off[k + 1] : (uint64_t)out_bytes;
            const uint64_t len = end - rec_off[i];
            std::memcpy(out + out_off[k], payload + rec_off[i], len);
            if (next > out_off[k] + len) std::memset(out + out_off[k] + len, 0, next - out_off[k] - len);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    return 0;
}

}  // extern "C"
