// mgp_route.cpp — the host side of a streamed batch on its way to the devices
// (libmgphost.so).
//
// * mgp_batch_columns16: the 16-bit barcode / |tlen| columns of a decoded batch
//   (mgp_push_batch16, 7 bytes of columns per read over the host link instead of 11)
//   when the batch allows them: records dense in BAM order at one stride, every
//   |tlen| < 65535, every barcode index < 65535.
// * mgp_route_batch: the multi-device stream's read router ("the host
//   decoder routes each kept read's SoA record to its GPU's pinned ring"). Each read
//   whose cell lies in a device's contiguous whitelist range goes, columns and record,
//   to that device's batch, in BAM order, its barcode rebased to the range; reads the
//   engine's filters drop before anything else (no whitelisted barcode; unmapped /
//   secondary / supplementary, readers.py:96-111) go nowhere: they count only toward
//   total_reads, which the decoder counts. So each device's link and HBM carry only
//   its own cells' reads. The cells' first-seen order (the reference's
//   reads_by_barcode insertion order, readers.py:104-163) is kept on the host as the
//   global index of each cell's first routed read.
// Both are memory-bound passes split over threads in contiguous read ranges: pass 1
// counts (reads and bytes per device and thread), a prefix sum places every thread's
// output, pass 2 copies.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/mgpileup.h"
#include "../../../include/mgpileup_host.h"

std::string& mgp_host_err();  // mgp_bam.cpp

namespace {

int fail(const char* m) {
    mgp_host_err() = m;
    return -1;
}

template <class F>
void parallel(int nt, F&& f) {
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(f, t);
    f(0);
    for (auto& x : th) x.join();
}

inline int threads_for(int64_t n, int n_threads) {
    return (int)std::max<int64_t>(1, std::min<int64_t>(std::max(1, n_threads), n / 65536 + 1));
}

inline uint32_t abs_u32(int32_t t) { return t < 0 ? (uint32_t)(-(int64_t)t) : (uint32_t)t; }

inline bool kept(int32_t bc, uint16_t flag, int64_t lo, int64_t hi) {
    return bc >= lo && bc < hi && !(flag & (MGP_FLAG_UNMAPPED | MGP_FLAG_SECONDARY | MGP_FLAG_SUPPLEMENTARY));
}

// a record's slot in a routed payload: 32-byte records at 32-byte offsets, every other
// record at 64-byte offsets (the engine's gathers read whole 64-byte halves of a line)
inline uint64_t slot_bytes(uint32_t b) { return b <= 32 ? 32 : ((uint64_t)b + 63) & ~uint64_t(63); }

struct Tally {  // one thread's reads of one device
    int64_t n = 0;
    uint64_t bytes = 0;
    uint32_t min_b = UINT32_MAX, max_b = 0, max_tlen = 0;
};

}  // namespace

extern "C" {

int mgp_batch_columns16(int64_t n, const int32_t* bc, const int32_t* tlen, const uint64_t* rec_off,
                        int64_t payload_bytes, int32_t n_cells, uint16_t* bc16, uint16_t* tlen16, int n_threads) {
    mgp_host_err().clear();
    if (n < 0 || (n > 0 && (!bc || !tlen || !bc16 || !tlen16)) || n_cells < 0 || payload_bytes < 0)
        return fail("mgp_batch_columns16: bad arguments");
    if (n == 0) return 3;
    const uint64_t stride = (uint64_t)(payload_bytes / n);
    const bool even = (uint64_t)payload_bytes == stride * (uint64_t)n && stride >= 16 && stride % 16 == 0;
    // every record at stride x i (every offset checked: a paired placement can give the
    // same payload size and last offset with the records permuted), every key in 16
    // bits; the columns are written as the check goes (unused when it fails)
    const int nt = threads_for(n, n_threads);
    std::vector<uint8_t> dense((size_t)nt, 1), keys((size_t)nt, 1);
    parallel(nt, [&](int t) {
        const int64_t a = n * t / nt, b = n * (t + 1) / nt;
        uint32_t wide = 0;
        uint64_t off = 0;
        for (int64_t i = a; i < b; ++i) {
            const int32_t c = bc[i];
            const uint32_t l = abs_u32(tlen[i]);
            wide |= (uint32_t)(c >= 0xFFFF) | (uint32_t)(l >= 0xFFFF);
            if (rec_off) off |= rec_off[i] ^ (stride * (uint64_t)i);
            bc16[i] = c < 0 ? (uint16_t)0xFFFF : (uint16_t)c;
            tlen16[i] = (uint16_t)l;
        }
        keys[(size_t)t] = wide == 0;
        dense[(size_t)t] = off == 0;
    });
    bool d = even, k = n_cells <= 0xFFFF;
    for (int t = 0; t < nt; ++t) {
        d = d && dense[(size_t)t];
        k = k && keys[(size_t)t];
    }
    return (d ? 1 : 0) | (k ? 2 : 0);
}

int mgp_route_batch(int64_t n, const int32_t* bc, const int32_t* tlen, const uint16_t* flag, const uint8_t* mapq,
                    const uint64_t* rec_off, const uint8_t* payload, int64_t payload_bytes, int32_t n_parts,
                    const int32_t* bounds, int64_t first_index, uint32_t* first_seen, mgp_route_part* parts,
                    int n_threads) {
    mgp_host_err().clear();
    if (n < 0 || n_parts <= 0 || !bounds || !parts || (n > 0 && (!bc || !tlen || !flag || !mapq || !payload)))
        return fail("mgp_route_batch: bad arguments");
    for (int32_t d = 0; d < n_parts; ++d) {
        if (bounds[d + 1] < bounds[d] || bounds[d] < 0) return fail("mgp_route_batch: bounds must not decrease");
        const mgp_route_part& p = parts[d];
        if (!p.bc16 || !p.tlen16 || !p.bc32 || !p.tlen32 || !p.flag || !p.mapq || !p.rec_off || !p.payload ||
            p.cap_reads < 0 || p.cap_payload < 256)
            return fail("mgp_route_batch: bad part arrays");
    }
    const int64_t lo = bounds[0], hi = bounds[n_parts];
    if (first_index < 0 || first_index + n > 0xFFFFFFFFll) return fail("mgp_route_batch: read index beyond 2^32 - 1");
    // a cell's device by table (one lookup per read)
    std::vector<int32_t> dev((size_t)(hi - lo));
    for (int32_t d = 0; d < n_parts; ++d)
        for (int64_t c = bounds[d]; c < bounds[d + 1]; ++c) dev[(size_t)(c - lo)] = d;
    const int nt = threads_for(n, n_threads);
    const size_t P = (size_t)n_parts;
    std::vector<Tally> tl((size_t)nt * P);
    std::vector<uint8_t> bad((size_t)nt, 0);
    // record i: at rec_off[i] (any placement), else dense at payload_bytes / n x i
    const uint64_t stride = (rec_off || n == 0) ? 0 : (uint64_t)(payload_bytes / n);
    if (!rec_off && n > 0 && (stride * (uint64_t)n != (uint64_t)payload_bytes || stride < 16))
        return fail("mgp_route_batch: rec_off NULL needs payload_bytes = n x a record stride");
    auto roff = [&](int64_t i) { return rec_off ? rec_off[i] : stride * (uint64_t)i; };
    // pass 1: per thread and device, reads, slot bytes, record sizes, |tlen| range;
    // every record checked inside the payload
    parallel(nt, [&](int t) {
        const int64_t a = n * t / nt, b = n * (t + 1) / nt;
        Tally* my = &tl[(size_t)t * P];
        for (int64_t i = a; i < b; ++i) {
            if (!kept(bc[i], flag[i], lo, hi)) continue;
            const int32_t d = dev[(size_t)(bc[i] - lo)];
            const uint64_t o = roff(i);
            if (o + 16 > (uint64_t)payload_bytes) {
                bad[(size_t)t] = 1;
                return;
            }
            const uint32_t sz = mgp_record_bytes(payload + o, flag[i]);
            if (o + sz > (uint64_t)payload_bytes) {
                bad[(size_t)t] = 1;
                return;
            }
            Tally& x = my[d];
            ++x.n;
            x.bytes += slot_bytes(sz);
            x.min_b = std::min(x.min_b, sz);
            x.max_b = std::max(x.max_b, sz);
            x.max_tlen = std::max(x.max_tlen, abs_u32(tlen[i]));
        }
    });
    for (uint8_t x : bad)
        if (x) return fail("mgp_route_batch: a record lies outside the payload");
    // per device: 16-bit form when every record has one size (32 or 64 bytes: dense at
    // that stride) and every key fits; the threads' output ranges by prefix sums
    std::vector<int64_t> at_n((size_t)nt * P);
    std::vector<uint64_t> at_b((size_t)nt * P);
    std::vector<uint32_t> nstride(P, 0);
    int rc = 0;
    for (size_t d = 0; d < P; ++d) {
        Tally tot;
        for (int t = 0; t < nt; ++t) {
            const Tally& x = tl[(size_t)t * P + d];
            at_n[(size_t)t * P + d] = tot.n;
            at_b[(size_t)t * P + d] = tot.bytes;
            tot.n += x.n;
            tot.bytes += x.bytes;
            tot.min_b = std::min(tot.min_b, x.min_b);
            tot.max_b = std::max(tot.max_b, x.max_b);
            tot.max_tlen = std::max(tot.max_tlen, x.max_tlen);
        }
        mgp_route_part& p = parts[d];
        const bool narrow = tot.n > 0 && tot.min_b == tot.max_b && (tot.min_b == 32 || tot.min_b == 64) &&
                            tot.max_tlen < 0xFFFF && bounds[d + 1] - bounds[d] <= 0xFFFF;
        if (narrow) nstride[d] = tot.min_b;
        p.narrow = narrow ? 1 : 0;
        p.n_reads = tot.n;
        p.payload_bytes = (int64_t)tot.bytes;
        // (256 zeroed bytes after the payload: the kernels read up to 128 past a record)
        if (tot.n > p.cap_reads || (int64_t)tot.bytes + 256 > p.cap_payload) rc = 1;
    }
    if (rc) {
        mgp_host_err() = "mgp_route_batch: a device's batch exceeds its arrays (route fewer reads at once)";
        return 1;
    }
    // pass 2: columns and records into each device's batch
    parallel(nt, [&](int t) {
        const int64_t a = n * t / nt, b = n * (t + 1) / nt;
        std::vector<int64_t> wn(at_n.begin() + (int64_t)t * n_parts, at_n.begin() + (int64_t)(t + 1) * n_parts);
        std::vector<uint64_t> wb(at_b.begin() + (int64_t)t * n_parts, at_b.begin() + (int64_t)(t + 1) * n_parts);
        for (int64_t i = a; i < b; ++i) {
            const int32_t c = bc[i];
            if (!kept(c, flag[i], lo, hi)) continue;
            const int32_t d = dev[(size_t)(c - lo)];
            mgp_route_part& p = parts[d];
            const int64_t k = wn[(size_t)d]++;
            const uint64_t o = roff(i);
            const uint32_t sz = mgp_record_bytes(payload + o, flag[i]);
            const uint64_t dst = wb[(size_t)d];
            wb[(size_t)d] += slot_bytes(sz);
            const int32_t local = c - bounds[d];
            if (p.narrow) {
                p.bc16[k] = (uint16_t)local;
                p.tlen16[k] = (uint16_t)abs_u32(tlen[i]);
            } else {
                p.bc32[k] = local;
                p.tlen32[k] = tlen[i];
                p.rec_off[k] = dst;
            }
            p.flag[k] = flag[i];
            p.mapq[k] = mapq[i];
            std::memcpy(p.payload + dst, payload + o, sz);
            if (slot_bytes(sz) > sz) std::memset(p.payload + dst + sz, 0, slot_bytes(sz) - sz);
            if (first_seen) {
                const uint32_t gi = (uint32_t)(first_index + i);
                uint32_t cur = __atomic_load_n(&first_seen[c - lo], __ATOMIC_RELAXED);
                while (gi < cur &&
                       !__atomic_compare_exchange_n(&first_seen[c - lo], &cur, gi, true, __ATOMIC_RELAXED,
                                                    __ATOMIC_RELAXED)) {
                }
            }
        }
    });
    for (size_t d = 0; d < P; ++d) {
        mgp_route_part& p = parts[d];
        std::memset(p.payload + p.payload_bytes, 0, 256);
    }
    return 0;
}

}  // extern "C"
