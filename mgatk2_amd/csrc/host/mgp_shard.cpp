// mgp_shard.cpp — record gather for cell sharding (host side, libmgphost.so).
//
// Cells are split over devices in contiguous whitelist ranges;
// each device's batch holds the records of its cells in BAM order. The SoA
// columns are gathered by index in numpy; the payload records are gathered here:
// sizes from the record headers (any source placement), the producer placement
// of the subset (mgp_place_records, mgp_place.cpp), then a parallel copy. (A
// numpy byte gather needs an 8-byte index per payload byte: 205 GB for the
// 25.6 GB C4 payload.)
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/mgpileup.h"
#include "../../../include/mgpileup_host.h"

std::string& mgp_host_err();  // mgp_bam.cpp

extern "C" {

int64_t mgp_gather_offsets(const uint8_t* payload, const uint64_t* rec_off, const uint16_t* flag, const int32_t* bc,
                           const int32_t* start, const int32_t* tlen, int64_t n_total, int64_t payload_bytes,
                           const int64_t* idx, int64_t m, int32_t cell_lo, int32_t n_cells, int32_t mode,
                           int32_t rec_align, uint64_t* out_off) {
    mgp_host_err().clear();
    if ((n_total && (!payload || !rec_off || !flag || !bc)) || (m && (!idx || !out_off)) || m < 0 || n_total < 0 ||
        n_cells < 0) {
        mgp_host_err() = "mgp_gather_offsets: bad arguments";
        return -1;
    }
    // the records' sizes from their headers (any source placement), the shard's
    // cell ids rebased to cell_lo, then the producer placement of the subset
    std::vector<int32_t> lbc((size_t)m);
    std::vector<uint16_t> lfl((size_t)m);
    std::vector<uint32_t> sz((size_t)m);
    const bool keyed = start && tlen;
    std::vector<int32_t> lst(keyed ? (size_t)m : 0), ltl(keyed ? (size_t)m : 0);
    for (int64_t k = 0; k < m; ++k) {
        const int64_t i = idx[k];
        if (i < 0 || i >= n_total) {
            mgp_host_err() = "mgp_gather_offsets: index out of range";
            return -1;
        }
        const uint64_t o = rec_off[i];
        if (o + 16 > (uint64_t)payload_bytes) {
            mgp_host_err() = "mgp_gather_offsets: record outside the payload";
            return -1;
        }
        const uint32_t b = mgp_record_bytes(payload + o, flag[i]);
        if (o + b > (uint64_t)payload_bytes) {
            mgp_host_err() = "mgp_gather_offsets: record outside the payload";
            return -1;
        }
        sz[(size_t)k] = b;
        lfl[(size_t)k] = flag[i];
        if (keyed) {
            lst[(size_t)k] = start[i];
            ltl[(size_t)k] = tlen[i];
        }
        const int64_t c = (int64_t)bc[i] - cell_lo;
        lbc[(size_t)k] = (bc[i] >= 0 && c >= 0 && c < n_cells) ? (int32_t)c : -1;
    }
    return mgp_place_records(m, lbc.data(), lfl.data(), keyed ? lst.data() : nullptr, keyed ? ltl.data() : nullptr,
                             sz.data(), n_cells, mode, rec_align, out_off);
}

int mgp_gather_records(const uint8_t* payload, const uint64_t* rec_off, const uint16_t* flag, int64_t n_total,
                       int64_t payload_bytes, const int64_t* idx, int64_t m, const uint64_t* out_off,
                       int64_t out_bytes, uint8_t* out, int n_threads) {
    mgp_host_err().clear();
    if (m < 0 || (m && (!payload || !rec_off || !flag || !idx || !out_off || !out))) {
        mgp_host_err() = "mgp_gather_records: bad arguments";
        return -1;
    }
    for (int64_t k = 0; k < m; ++k) {  // every source and destination inside its buffer
        const int64_t i = idx[k];
        if (i < 0 || i >= n_total || rec_off[i] + 16 > (uint64_t)payload_bytes) {
            mgp_host_err() = "mgp_gather_records: record outside the payload";
            return -1;
        }
        const uint32_t b = mgp_record_bytes(payload + rec_off[i], flag[i]);
        if (rec_off[i] + b > (uint64_t)payload_bytes || out_off[k] + b > (uint64_t)out_bytes) {
            mgp_host_err() = "mgp_gather_records: record outside the payload";
            return -1;
        }
    }
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(std::max(n_threads, 1), m / 65536 + 1));
    auto work = [&](int t) {
        const int64_t lo = m * t / nt, hi = m * (t + 1) / nt;
        for (int64_t k = lo; k < hi; ++k) {
            const int64_t i = idx[k];
            std::memcpy(out + out_off[k], payload + rec_off[i], mgp_record_bytes(payload + rec_off[i], flag[i]));
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    return 0;
}

// Reads by cell range: idx[] = the indices of the reads whose cell lies in [bounds[d],
// bounds[d + 1]), range by range, BAM order inside each; counts[d] = their number. One
// pass to count and one to place (the router of the multi-device stream used one
// numpy scan of the batch per device). Returns the indices written.
int64_t mgp_split_by_range(const int32_t* bc, int64_t n, const int64_t* bounds, int32_t nd, int64_t* counts,
                           int64_t* idx) {
    mgp_host_err().clear();
    if ((!bc && n > 0) || !bounds || nd <= 0 || !counts || (n > 0 && !idx) || n < 0) {
        mgp_host_err() = "mgp_split_by_range: bad arguments";
        return -1;
    }
    for (int32_t d = 0; d < nd; ++d)
        if (bounds[d + 1] < bounds[d]) {
            mgp_host_err() = "mgp_split_by_range: bounds must not decrease";
            return -1;
        }
    const int64_t lo = bounds[0], hi = bounds[nd];
    // a cell's range by table (cells span at most a few 100k): one lookup per read
    std::vector<int32_t> dev((size_t)std::max<int64_t>(0, hi - lo));
    for (int32_t d = 0; d < nd; ++d)
        for (int64_t c = bounds[d]; c < bounds[d + 1]; ++c) dev[(size_t)(c - lo)] = d;
    std::vector<int64_t> cnt((size_t)nd, 0);
    for (int64_t i = 0; i < n; ++i) {
        const int64_t c = bc[i];
        if (c >= lo && c < hi) ++cnt[(size_t)dev[(size_t)(c - lo)]];
    }
    std::vector<int64_t> at((size_t)nd, 0);
    int64_t tot = 0;
    for (int32_t d = 0; d < nd; ++d) {
        counts[d] = cnt[(size_t)d];
        at[(size_t)d] = tot;
        tot += cnt[(size_t)d];
    }
    for (int64_t i = 0; i < n; ++i) {
        const int64_t c = bc[i];
        if (c >= lo && c < hi) idx[at[(size_t)dev[(size_t)(c - lo)]]++] = i;
    }
    return tot;
}

}  // extern "C"
