// mgp_tiles.cpp — parallel deflate of HDF5 chunks (host side, libmgphost.so).
//
// The HDF5 output (IncrementalHDF5Writer, src/file_io/writers.py:60-406)
// stores 11 planes of uint16 [16569, n_cells] with gzip-4 chunks of
// (1000, 100). libhdf5's own filter pipeline deflates one chunk at a time on
// one thread; here every chunk of a plane is compressed on a thread pool in
// the exact form the HDF5 deflate filter (H5Z_DEFLATE: zlib `compress2`
// stream of the chunk, edge chunks padded to full size with the fill value 0)
// produces. The caller writes the chunks with H5Dwrite_chunk.
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mgp_zcodec.h"
#include "../../../include/mgpileup_host.h"

std::string& mgp_host_err();  // mgp_bam.cpp

extern "C" {

int64_t mgp_deflate_tiles(const void* data, int64_t rows, int64_t cols, int32_t elem_size, int64_t crow,
                          int64_t ccol, int level, int n_threads, uint8_t** blob, int64_t* offsets) {
    mgp_host_err().clear();
    if (!data || rows <= 0 || cols <= 0 || crow <= 0 || ccol <= 0 || !blob || !offsets ||
        (elem_size != 1 && elem_size != 2 && elem_size != 4 && elem_size != 8) || level < 0 || level > 9) {
        mgp_host_err() = "bad arguments";
        return -1;
    }
    const int64_t nr = (rows + crow - 1) / crow, nc = (cols + ccol - 1) / ccol, n = nr * nc;
    const size_t chunk_bytes = (size_t)crow * (size_t)ccol * (size_t)elem_size;
    std::vector<std::vector<uint8_t>> out((size_t)n);
    std::atomic<int64_t> next{0};
    std::atomic<bool> ok{true};
    const uint8_t* src = (const uint8_t*)data;
    auto work = [&]() {
        std::vector<uint8_t> tile(chunk_bytes);
        mgp_host::Deflator dz(level);
        for (;;) {
            const int64_t t = next.fetch_add(1);
            if (t >= n) break;
            const int64_t r0 = (t / nc) * crow, c0 = (t % nc) * ccol;
            const int64_t h = std::min(crow, rows - r0), w = std::min(ccol, cols - c0);
            if (h < crow || w < ccol) std::memset(tile.data(), 0, chunk_bytes);
            for (int64_t r = 0; r < h; ++r)
                std::memcpy(tile.data() + (size_t)r * ccol * elem_size,
                            src + ((size_t)(r0 + r) * (size_t)cols + (size_t)c0) * elem_size, (size_t)w * elem_size);
            // the H5Z_DEFLATE form: one zlib stream of the whole (padded) chunk
            if (!dz.zlib(tile.data(), chunk_bytes, out[(size_t)t])) {
                ok = false;
                return;
            }
        }
    };
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n));
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(work);
    work();
    for (auto& x : th) x.join();
    if (!ok) {
        mgp_host_err() = "deflate failed";
        return -1;
    }
    size_t total = 0;
    for (int64_t t = 0; t < n; ++t) {
        offsets[t] = (int64_t)total;
        total += out[(size_t)t].size();
    }
    offsets[n] = (int64_t)total;
    uint8_t* b = (uint8_t*)std::malloc(std::max<size_t>(total, 1));
    if (!b) {
        mgp_host_err() = "out of host memory";
        return -1;
    }
    for (int64_t t = 0; t < n; ++t)
        if (!out[(size_t)t].empty()) std::memcpy(b + offsets[t], out[(size_t)t].data(), out[(size_t)t].size());
    *blob = b;
    return n;
}

}  // extern "C"
