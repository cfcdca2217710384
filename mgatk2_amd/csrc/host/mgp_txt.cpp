// mgp_txt.cpp — mgatk txt output at scale (host side, libmgphost.so).
//
// Formats the per-cell count files of IncrementalTextWriter
// (src/file_io/writers.py:430-462, layout in SURVEY.md §3.3) straight from the
// engine's cell-major arrays and deflates them on a thread pool:
//   output.coverage.txt.gz : "pos,barcode,depth"       for depth > 0
//   output.{A,C,G,T}.txt.gz: "pos,barcode,fwd,rev"     for depth > 0 and fwd+rev > 0
// Positions are 1-based; cells are written in the order given. Each group of
// cells becomes one gzip member, so the files are multi-member gzip streams
// whose decompressed bytes equal the reference's text (gzip readers,
// Python's gzip and zcat concatenate members).
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mgp_zcodec.h"
#include "../../../include/mgpileup_host.h"

std::string& mgp_host_err();  // mgp_bam.cpp

namespace {

int fail(const std::string& m) {
    mgp_host_err() = m;
    return -1;
}

inline char* put_u64(char* p, uint64_t v) {
    char tmp[24];
    int n = 0;
    do {
        tmp[n++] = (char)('0' + v % 10);
        v /= 10;
    } while (v);
    while (n) *p++ = tmp[--n];
    return p;
}

// decimal text of 0..9999 (the counts and depths of a position are almost always
// below it): 4 chars + the length, one 8-byte copy per number
struct Digits {
    char s[10000][4];
    uint8_t n[10000];
    Digits() {
        for (int v = 0; v < 10000; ++v) {
            char t[8];
            const int k = std::snprintf(t, sizeof t, "%d", v);
            std::memcpy(s[v], t, 4);
            n[v] = (uint8_t)k;
        }
    }
};
const Digits& digits() {
    static const Digits d;
    return d;
}
inline char* put_num(char* p, uint32_t v, const Digits& D) {
    if (v < 10000u) {
        std::memcpy(p, D.s[v], 4);
        return p + D.n[v];
    }
    return put_u64(p, v);
}

struct Text {
    std::vector<char> b;
    size_t n = 0;
    char* reserve(size_t k) {
        if (n + k > b.size()) b.resize(std::max(b.size() * 2, n + k + (1u << 16)));
        return b.data() + n;
    }
};

bool gzip_member(const char* src, size_t n, mgp_host::Deflator& dz, std::vector<uint8_t>& out) {
    out.clear();
    if (n == 0) return true;
    return dz.gzip(reinterpret_cast<const uint8_t*>(src), n, out);
}

// One group of cells -> 5 texts (coverage, A, C, G, T). T: u32 rows, or the
// engine's exact 16-bit rows (mgp_fetch_rows16 without wide windows).
template <class T>
void format_group(const T* counts, const T* depth, int64_t L, const int64_t* cells, int64_t c0,
                  int64_t c1, const char* const* names, Text* txt) {
    const Digits& D = digits();
    std::vector<char> prebuf(256);  // "pos,barcode," of the current position (every line starts with it)
    for (int64_t k = c0; k < c1; ++k) {
        const int64_t c = cells[k];
        const char* bc = names[k];
        const size_t bl = std::strlen(bc);
        if (prebuf.size() < bl + 32) prebuf.resize(bl + 32);
        char* const pre = prebuf.data();
        const T* d = depth + (size_t)c * (size_t)L;
        const T* q = counts + (size_t)c * (size_t)L * 8;
        for (int64_t p = 0; p < L; ++p) {
            const uint32_t dp = d[p];
            if (!dp) continue;
            char* e0 = put_num(pre, (uint32_t)(p + 1), D);
            *e0++ = ',';
            std::memcpy(e0, bc, bl);
            e0 += bl;
            *e0++ = ',';
            const size_t pl = (size_t)(e0 - pre);
            char* w = txt[0].reserve(pl + 24);
            char* s = w;
            std::memcpy(w, pre, pl);
            w = put_num(w + pl, dp, D);
            *w++ = '\n';
            txt[0].n += (size_t)(w - s);
            const T* e = q + (size_t)p * 8;
            for (int b = 0; b < 4; ++b) {
                const uint32_t fw = e[2 * b], rv = e[2 * b + 1];
                if (!(fw | rv)) continue;
                Text& t = txt[1 + b];
                char* x = t.reserve(pl + 48);
                char* x0 = x;
                std::memcpy(x, pre, pl);
                x = put_num(x + pl, fw, D);
                *x++ = ',';
                x = put_num(x, rv, D);
                *x++ = '\n';
                t.n += (size_t)(x - x0);
            }
        }
    }
}

template <class T>
int write_cells(const char* prefix, const T* counts, const T* depth, int64_t mito_len, const int64_t* cells,
                int64_t n_write, const char* const* names, int level, int n_threads, int append) {
    mgp_host_err().clear();
    if (!prefix || (n_write > 0 && (!counts || !depth || !cells || !names)) || mito_len <= 0 || n_write < 0)
        return fail("bad arguments");
    if (level < 0 || level > 9) return fail("gzip level must be 0..9");
    static const char* kNames[5] = {"coverage", "A", "C", "G", "T"};
    FILE* f[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    for (int i = 0; i < 5; ++i) {
        const std::string path = std::string(prefix) + "." + kNames[i] + ".txt.gz";
        f[i] = std::fopen(path.c_str(), append ? "ab" : "wb");
        if (!f[i]) {
            for (int j = 0; j < i; ++j) std::fclose(f[j]);
            return fail("cannot open " + path);
        }
    }
    // groups of cells sized for ~4 MB of text each (a covered position costs ~30 B per file)
    const int64_t per_group = std::max<int64_t>(1, (int64_t)((4u << 20) / ((size_t)mito_len * 40 + 1)));
    const int64_t n_groups = (n_write + per_group - 1) / per_group;
    const int nt = std::max(1, std::min<int>(n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency(),
                                             (int)std::max<int64_t>(1, n_groups)));
    // One pool over all groups; this thread writes each group's five members in group
    // order as they complete, while the pool works on the groups after it (a ring of
    // `win` groups bounds the buffered output). Until r05 the groups went in rounds of
    // 4 per thread with the members written between rounds: at C4 and gzip level 1 the
    // pool sat idle during ~1.8 GB of serial writes.
    const int64_t win = (int64_t)nt * 4;
    std::vector<std::vector<uint8_t>> out((size_t)win * 5);
    std::vector<int64_t> ready((size_t)win, -1);  // group whose members slot g % win holds
    int64_t written = 0;                           // groups written so far
    std::mutex mu;
    std::condition_variable cv;
    std::atomic<bool> ok{true};
    std::atomic<int64_t> next{0}, ns_fmt{0}, ns_dfl{0}, n_txt{0};
    const bool prof = std::getenv("MGP_TXT_PROFILE") != nullptr;
    auto work = [&]() {
        Text txt[5];
        mgp_host::Deflator dz(level);
        for (;;) {
            const int64_t g = next.fetch_add(1);
            if (g >= n_groups || !ok) break;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return g < written + win || !ok; });
                if (!ok) break;
            }
            const size_t slot = (size_t)(g % win);
            for (auto& t : txt) t.n = 0;
            const int64_t c0 = g * per_group, c1 = std::min(n_write, c0 + per_group);
            const auto a = std::chrono::steady_clock::now();
            format_group(counts, depth, mito_len, cells, c0, c1, names, txt);
            const auto b = std::chrono::steady_clock::now();
            bool good = true;
            for (int i = 0; i < 5; ++i)
                if (!gzip_member(txt[i].b.data(), txt[i].n, dz, out[slot * 5 + i])) good = false;
            if (prof) {
                const auto e = std::chrono::steady_clock::now();
                ns_fmt += std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count();
                ns_dfl += std::chrono::duration_cast<std::chrono::nanoseconds>(e - b).count();
                for (auto& x : txt) n_txt += (int64_t)x.n;
            }
            {
                std::lock_guard<std::mutex> lk(mu);
                if (!good) ok = false;
                ready[slot] = g;
            }
            cv.notify_all();
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(work);
    int rc = 0;
    for (int64_t g = 0; g < n_groups; ++g) {
        const size_t slot = (size_t)(g % win);
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return ready[slot] == g || !ok; });
            if (!ok) break;
        }
        for (int i = 0; i < 5 && rc == 0; ++i) {
            const auto& o = out[slot * 5 + i];
            if (!o.empty() && std::fwrite(o.data(), 1, o.size(), f[i]) != o.size()) rc = fail("write failed");
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            if (rc != 0) ok = false;
            written = g + 1;
        }
        cv.notify_all();
        if (rc != 0) break;
    }
    for (auto& t : th) t.join();
    if (rc == 0 && !ok) rc = fail("deflate failed");
    for (int i = 0; i < 5; ++i)
        if (std::fclose(f[i]) != 0 && rc == 0) rc = fail("close failed");
    if (prof)
        std::fprintf(stderr, "[mgp_txt] %d threads: format %.3f s, deflate %.3f s (thread-summed), text %.1f MB\n",
                     nt, ns_fmt * 1e-9, ns_dfl * 1e-9, n_txt * 1e-6);
    return rc;
}

}  // namespace

extern "C" {

int mgp_txt_write_cells(const char* prefix, const uint32_t* counts, const uint32_t* depth, int64_t mito_len,
                        const int64_t* cells, int64_t n_write, const char* const* names, int level, int n_threads,
                        int append) {
    return write_cells(prefix, counts, depth, mito_len, cells, n_write, names, level, n_threads, append);
}

int mgp_txt_write_cells16(const char* prefix, const uint16_t* counts, const uint16_t* depth, int64_t mito_len,
                          const int64_t* cells, int64_t n_write, const char* const* names, int level, int n_threads,
                          int append) {
    return write_cells(prefix, counts, depth, mito_len, cells, n_write, names, level, n_threads, append);
}

}  // extern "C"
