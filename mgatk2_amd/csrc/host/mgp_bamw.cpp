// mgp_bamw.cpp — BAM (+ .bai) writer for engine batches (host side, libmgphost.so).
//
// Turns an engine batch (include/mgpileup.h record layout) back into a
// coordinate-sorted BAM: the test and benchmark counterpart of mgp_bam_read_ref,
// used to make synthetic inputs of any size for the end-to-end pipeline
// (BAM -> ingest -> engine -> writers). BGZF blocks are deflated on a thread
// pool; the .bai holds, per reference, bins with merged chunks and the 16 kbp
// linear index (SAM spec §5.2), enough for any indexed reader to seek.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/mgpileup.h"
#include "../../../include/mgpileup_host.h"

std::string& mgp_host_err();  // mgp_bam.cpp

namespace {

int fail(const std::string& m) {
    mgp_host_err() = m;
    return -1;
}

constexpr size_t kBlockData = 0xFF00;  // uncompressed bytes per BGZF block
const uint8_t kEof[28] = {0x1f, 0x8b, 0x08, 0x04, 0, 0, 0, 0, 0, 0xff, 0x06, 0, 0x42, 0x43,
                          0x02, 0,    0x1b, 0,    3, 0, 0, 0, 0, 0, 0, 0,    0, 0};

template <class T>
void put(std::vector<uint8_t>& b, T v) {
    const size_t n = b.size();
    b.resize(n + sizeof(T));
    std::memcpy(b.data() + n, &v, sizeof(T));
}

int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

bool bgzf_block(const uint8_t* src, size_t n, int level, std::vector<uint8_t>& out) {
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return false;
    std::vector<uint8_t> c(deflateBound(&zs, (uLong)n) + 32);
    zs.next_in = const_cast<uint8_t*>(src);
    zs.avail_in = (uInt)n;
    zs.next_out = c.data();
    zs.avail_out = (uInt)c.size();
    const int r = deflate(&zs, Z_FINISH);
    const size_t cl = zs.total_out;
    deflateEnd(&zs);
    if (r != Z_STREAM_END || cl + 26 > 65536) return false;
    out.clear();
    const uint8_t hdr[18] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 0, 0};
    out.insert(out.end(), hdr, hdr + 18);
    const uint16_t bs = (uint16_t)(cl + 25);
    std::memcpy(out.data() + 16, &bs, 2);
    out.insert(out.end(), c.data(), c.data() + cl);
    put<uint32_t>(out, (uint32_t)crc32(0, src, (uInt)n));
    put<uint32_t>(out, (uint32_t)n);
    return true;
}

struct RecPos {
    int64_t beg, end;
    size_t ubeg, uend;  // offsets into the uncompressed stream
};

}  // namespace

extern "C" {

int mgp_bam_write(const char* path, const char* const* ref_names, const int64_t* ref_lens, int n_ref, int tid,
                  const mgp_bam_batch* batch, const char* const* barcodes, int n_barcodes, const char* tag,
                  const char* unlisted, int level, int n_threads, int write_index) {
    mgp_host_err().clear();
    if (!path || !ref_names || !ref_lens || n_ref <= 0 || tid < 0 || tid >= n_ref || !batch || !tag ||
        std::strlen(tag) != 2 || level < 0 || level > 9)
        return fail("bad arguments");
    // ---- uncompressed stream: header, then records -------------------------
    std::vector<uint8_t> u;
    std::string text = "@HD\tVN:1.6\tSO:coordinate\n";
    for (int r = 0; r < n_ref; ++r)
        text += std::string("@SQ\tSN:") + ref_names[r] + "\tLN:" + std::to_string(ref_lens[r]) + "\n";
    u.insert(u.end(), {'B', 'A', 'M', 1});
    put<int32_t>(u, (int32_t)text.size());
    u.insert(u.end(), text.begin(), text.end());
    put<int32_t>(u, n_ref);
    for (int r = 0; r < n_ref; ++r) {
        const size_t ln = std::strlen(ref_names[r]) + 1;
        put<int32_t>(u, (int32_t)ln);
        u.insert(u.end(), ref_names[r], ref_names[r] + ln);
        put<int32_t>(u, (int32_t)ref_lens[r]);
    }
    const size_t header_end = u.size();  // records start in a fresh block
    std::vector<RecPos> pos((size_t)std::max<int64_t>(batch->n_reads, 0));
    char name[32];
    const size_t tag_len_unlisted = unlisted ? std::strlen(unlisted) : 0;
    for (int64_t i = 0; i < batch->n_reads; ++i) {
        const uint8_t* rec = batch->payload + batch->rec_off[i];
        uint8_t full[128];
        if (batch->flag[i] & MGP_FLAG_PACKED) {  // N with quality 0 for its non-ACGT bases
            mgp_unpack_record(rec, full);
            rec = full;
        }
        int32_t start;
        uint32_t lseq, coff;
        uint16_t ncig, flg;
        std::memcpy(&start, rec, 4);
        std::memcpy(&lseq, rec + 4, 4);
        std::memcpy(&ncig, rec + 8, 2);
        std::memcpy(&flg, rec + 10, 2);
        if (batch->flag[i] & MGP_FLAG_PACKED) flg = batch->flag[i];
        std::memcpy(&coff, rec + 12, 4);
        const uint8_t* qual = rec + 16;
        const uint8_t* seq = rec + mgp_seq_offset(lseq);
        const uint8_t* cig = rec + coff;
        const int nl = std::snprintf(name, sizeof(name), "r%lld", (long long)i) + 1;
        int64_t span = 0;
        for (uint32_t k = 0; k < ncig; ++k) {
            uint32_t c;
            std::memcpy(&c, cig + 4 * k, 4);
            const uint32_t op = c & 15u;
            if (op == 0 || op == 2 || op == 3 || op == 7 || op == 8) span += c >> 4;
        }
        const int64_t beg = start, end = start + std::max<int64_t>(span, 1);
        const int32_t b = batch->bc[i];
        const char* tv = b >= 0 && b < n_barcodes ? barcodes[b] : (b < 0 && unlisted && (i % 2 == 0) ? unlisted : nullptr);
        const size_t tl = tv ? (tv == unlisted ? tag_len_unlisted : std::strlen(tv)) : 0;
        const uint32_t block_size =
            32 + (uint32_t)nl + 4 * ncig + (lseq + 1) / 2 + lseq + (tv ? (uint32_t)(3 + tl + 1) : 0u);
        pos[(size_t)i].beg = beg;
        pos[(size_t)i].end = end;
        pos[(size_t)i].ubeg = u.size();
        put<uint32_t>(u, block_size);
        put<int32_t>(u, tid);
        put<int32_t>(u, start);
        u.push_back((uint8_t)nl);
        u.push_back(batch->mapq[i]);
        put<uint16_t>(u, (uint16_t)reg2bin(beg, end));
        put<uint16_t>(u, ncig);
        put<uint16_t>(u, (uint16_t)(flg & 0x0FFF));
        put<uint32_t>(u, lseq);
        put<int32_t>(u, -1);
        put<int32_t>(u, -1);
        put<int32_t>(u, batch->tlen[i]);
        u.insert(u.end(), name, name + nl);
        u.insert(u.end(), cig, cig + 4 * (size_t)ncig);
        u.insert(u.end(), seq, seq + (lseq + 1) / 2);
        u.insert(u.end(), qual, qual + lseq);
        if (tv) {
            u.push_back((uint8_t)tag[0]);
            u.push_back((uint8_t)tag[1]);
            u.push_back('Z');
            u.insert(u.end(), tv, tv + tl + 1);
        }
        pos[(size_t)i].uend = u.size();
    }
    // ---- blocks: [0, header_end) alone, then kBlockData slices ----------------
    std::vector<size_t> cut{0};
    for (size_t o = 0; o < header_end; o += kBlockData) cut.push_back(std::min(header_end, o + kBlockData));
    for (size_t o = header_end; o < u.size(); o += kBlockData) cut.push_back(std::min(u.size(), o + kBlockData));
    const size_t nb = cut.size() - 1;
    std::vector<std::vector<uint8_t>> blk(nb);
    std::atomic<size_t> next{0};
    std::atomic<bool> ok{true};
    auto work = [&]() {
        for (;;) {
            const size_t k = next.fetch_add(1);
            if (k >= nb) break;
            if (!bgzf_block(u.data() + cut[k], cut[k + 1] - cut[k], level, blk[k])) ok = false;
        }
    };
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, nb));
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
    if (!ok) return fail("deflate failed");
    std::vector<uint64_t> coff(nb + 1, 0);
    for (size_t k = 0; k < nb; ++k) coff[k + 1] = coff[k] + blk[k].size();
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(std::string("cannot open ") + path);
    for (size_t k = 0; k < nb; ++k)
        if (std::fwrite(blk[k].data(), 1, blk[k].size(), f) != blk[k].size()) {
            std::fclose(f);
            return fail("write failed");
        }
    std::fwrite(kEof, 1, sizeof(kEof), f);
    if (std::fclose(f) != 0) return fail("close failed");
    if (!write_index) return 0;
    // ---- .bai ---------------------------------------------------------------
    auto voff = [&](size_t uo) -> uint64_t {
        const size_t k = (size_t)(std::upper_bound(cut.begin(), cut.end(), uo) - cut.begin()) - 1;
        if (k >= nb) return coff[nb] << 16;  // end of data
        return (coff[k] << 16) | (uint64_t)(uo - cut[k]);
    };
    std::map<int, std::vector<std::pair<uint64_t, uint64_t>>> bins;
    std::vector<uint64_t> lin;
    for (const RecPos& p : pos) {
        const uint64_t vb = voff(p.ubeg), ve = voff(p.uend);
        auto& ch = bins[reg2bin(std::max<int64_t>(p.beg, 0), std::max<int64_t>(p.end, p.beg + 1))];
        if (!ch.empty() && ch.back().second == vb)
            ch.back().second = ve;
        else
            ch.emplace_back(vb, ve);
        const int64_t w0 = std::max<int64_t>(p.beg, 0) >> 14, w1 = (std::max<int64_t>(p.end, p.beg + 1) - 1) >> 14;
        if ((int64_t)lin.size() <= w1) lin.resize((size_t)w1 + 1, UINT64_MAX);
        for (int64_t wdx = w0; wdx <= w1; ++wdx) lin[(size_t)wdx] = std::min(lin[(size_t)wdx], vb);
    }
    uint64_t last = 0;
    for (auto& v : lin) {
        if (v == UINT64_MAX) v = last;
        last = v;
    }
    std::vector<uint8_t> x{'B', 'A', 'I', 1};
    put<int32_t>(x, n_ref);
    for (int r = 0; r < n_ref; ++r) {
        if (r != tid) {
            put<int32_t>(x, 0);
            put<int32_t>(x, 0);
            continue;
        }
        put<int32_t>(x, (int32_t)bins.size() + (pos.empty() ? 0 : 1));
        for (const auto& kv : bins) {
            put<uint32_t>(x, (uint32_t)kv.first);
            put<int32_t>(x, (int32_t)kv.second.size());
            for (const auto& c : kv.second) {
                put<uint64_t>(x, c.first);
                put<uint64_t>(x, c.second);
            }
        }
        if (!pos.empty()) {  // the metadata pseudo-bin (SAM spec §5.2): extent, mapped / unmapped counts
            uint64_t n_unmapped = 0;
            for (int64_t i = 0; i < batch->n_reads; ++i) n_unmapped += (batch->flag[i] & 0x4) != 0;
            put<uint32_t>(x, 37450u);
            put<int32_t>(x, 2);
            put<uint64_t>(x, voff(pos.front().ubeg));
            put<uint64_t>(x, voff(pos.back().uend));
            put<uint64_t>(x, (uint64_t)batch->n_reads - n_unmapped);
            put<uint64_t>(x, n_unmapped);
        }
        put<int32_t>(x, (int32_t)lin.size());
        for (uint64_t v : lin) put<uint64_t>(x, v);
    }
    const std::string ipath = std::string(path) + ".bai";
    FILE* fi = std::fopen(ipath.c_str(), "wb");
    if (!fi) return fail("cannot open " + ipath);
    const bool wok = std::fwrite(x.data(), 1, x.size(), fi) == x.size();
    if (std::fclose(fi) != 0 || !wok) return fail("index write failed");
    return 0;
}

}  // extern "C"
