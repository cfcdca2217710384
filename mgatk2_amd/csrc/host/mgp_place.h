// mgp_place.h — the paired placement's duplicate rule, shared by
// mgp_place_records (mgp_place.cpp) and the BAM decoder (mgp_bam.cpp).
//
// A read with the same start, strand and |tlen| as an earlier read of its cell
// is a duplicate under every dedup mode that drops anything (readers.py:118-150:
// the 3-tuple key, and the 2-tuple key it refines), so the pileup never piles
// it. Pairing it with its cell's next read would leave half of that line
// unused, so the paired placement puts such reads on the lines of the dropped
// reads instead. A placement choice only: the engine reads every record at its
// rec_off, and with dedup off the reads are piled from those lines.
#pragma once
#include <cstdint>
#include <vector>

namespace mgp_host {

class DupTracker {
  public:
    explicit DupTracker(size_t n_cells) : cells_(n_cells) {}
    // true iff (start, reverse, |tlen|) repeats a key of an earlier read of cell
    // c; the keys of a cell's current start are kept (up to kKeys), and a cell's
    // reads arrive in coordinate order, so a new start clears them
    bool repeat(size_t c, int32_t start, bool reverse, int32_t tlen) {
        Cell& x = cells_[c];
        const uint64_t at = tlen < 0 ? (uint64_t)(-(int64_t)tlen) : (uint64_t)tlen;
        const uint64_t key = at | (reverse ? 1ull << 32 : 0ull);
        if (x.n == 0 || x.start != start) {
            x.start = start;
            x.n = 1;
            x.key[0] = key;
            return false;
        }
        for (uint32_t k = 0; k < x.n; ++k)
            if (x.key[k] == key) return true;
        if (x.n < kKeys) x.key[x.n++] = key;
        return false;
    }

  private:
    static constexpr uint32_t kKeys = 8;
    // (a cache line of its own: the stream decoder checks disjoint sets of cells on
    // several threads at once)
    struct alignas(64) Cell {
        int32_t start = 0;
        uint32_t n = 0;
        uint64_t key[kKeys];
    };
    std::vector<Cell> cells_;
};

}  // namespace mgp_host
