// mgp_place.cpp — payload placement for producers (host side, libmgphost.so).
//
// The pileup gathers one record per piled read, in each cell's BAM order, and a
// gather costs a whole 128-byte line request whatever the record size
// (profiles/r01/rdreq_v16.txt). A packed record is 64 bytes, so with records in
// BAM order a line carries one read of the cell being piled and one read of a
// random other cell. MGP_PLACE_PAIRED puts two consecutive packed records OF ONE
// CELL into one line (four 32-byte records): the producer keeps, per cell, the line whose first half
// it filled last; the cell's next record takes the second half. Lines are opened
// in BAM order, so the placement is one streaming pass with a table of one
// offset per cell (what a decoder can do as it emits records). Reads the engine
// drops at its filters (readers.py:95-111: no whitelisted barcode, unmapped,
// secondary, supplementary) pair among themselves, and so do, given the start
// and tlen columns, a cell's reads that repeat the start, strand and |tlen| of
// an earlier read of the cell (duplicates, never piled: mgp_place.h); full-layout
// records take their own 128-byte aligned slots. Any placement gives the same
// results: the engine reads every record at its rec_off.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/mgpileup.h"
#include "../../../include/mgpileup_host.h"
#include "mgp_place.h"

std::string& mgp_host_err();  // mgp_bam.cpp

namespace {
constexpr uint64_t kLine = 128;
constexpr uint64_t kNone = ~0ull;
}  // namespace

extern "C" {

int64_t mgp_place_records(int64_t n, const int32_t* bc, const uint16_t* flag, const int32_t* start,
                          const int32_t* tlen, const uint32_t* rec_bytes, int32_t n_cells, int32_t mode,
                          int32_t rec_align, uint64_t* rec_off) {
    mgp_host_err().clear();
    if (n < 0 || (n && (!bc || !flag || !rec_bytes || !rec_off)) || n_cells < 0 || rec_align < 16 ||
        rec_align > 4096 || (rec_align & (rec_align - 1)) || (mode != MGP_PLACE_DENSE && mode != MGP_PLACE_PAIRED)) {
        mgp_host_err() = "mgp_place_records: bad arguments";
        return -1;
    }
    const uint64_t amask = (uint64_t)rec_align - 1;
    uint64_t cur = 0;
    if (mode == MGP_PLACE_DENSE) {
        for (int64_t i = 0; i < n; ++i) {
            rec_off[i] = cur;
            cur += ((uint64_t)rec_bytes[i] + amask) & ~amask;
        }
        return (int64_t)cur;
    }
    // paired: open[k] = the line of key k whose second half is free; 32-byte records go
    // four to a line: open32[k] = the line of key k with free quarters, fill32[k] of them used
    std::vector<uint64_t> open((size_t)n_cells + 1, kNone), open32((size_t)n_cells + 1, kNone);
    std::vector<uint8_t> fill32((size_t)n_cells + 1, 0);
    const uint16_t drop = MGP_FLAG_UNMAPPED | MGP_FLAG_SECONDARY | MGP_FLAG_SUPPLEMENTARY;
    const bool keyed = start && tlen;
    mgp_host::DupTracker dups(keyed ? (size_t)n_cells : 0);
    for (int64_t i = 0; i < n; ++i) {
        const uint16_t f = flag[i];
        const bool p32 = (f & MGP_FLAG_PACK32) && rec_bytes[i] == MGP_PACK32_BYTES;
        if (!p32 && (!(f & MGP_FLAG_PACKED) || (f & MGP_FLAG_PACK32) || rec_bytes[i] != MGP_PACK_BYTES)) {
            cur = (cur + kLine - 1) & ~(kLine - 1);
            rec_off[i] = cur;
            cur += ((uint64_t)rec_bytes[i] + kLine - 1) & ~(kLine - 1);
            continue;
        }
        const int32_t c = bc[i];
        size_t k = (c >= 0 && c < n_cells && !(f & drop)) ? (size_t)c : (size_t)n_cells;
        if (keyed && k < (size_t)n_cells && dups.repeat(k, start[i], (f & MGP_FLAG_REVERSE) != 0, tlen[i]))
            k = (size_t)n_cells;
        if (p32) {
            if (open32[k] == kNone) {
                cur = (cur + kLine - 1) & ~(kLine - 1);
                open32[k] = cur;
                fill32[k] = 0;
                cur += kLine;
            }
            rec_off[i] = open32[k] + (uint64_t)MGP_PACK32_BYTES * fill32[k];
            if (++fill32[k] == kLine / MGP_PACK32_BYTES) open32[k] = kNone;
            continue;
        }
        if (open[k] != kNone) {
            rec_off[i] = open[k] + MGP_PACK_BYTES;
            open[k] = kNone;
        } else {
            cur = (cur + kLine - 1) & ~(kLine - 1);
            rec_off[i] = cur;
            open[k] = cur;
            cur += kLine;
        }
    }
    return (int64_t)cur;
}

}  // extern "C"
