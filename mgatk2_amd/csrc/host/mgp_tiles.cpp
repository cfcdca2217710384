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

// The HDF5 planes of IncrementalHDF5Writer (writers.py:200-218) straight from the
// engine's cell-major result rows, chunked and deflated in one pass: plane e of the
// call (element elems[e] of each row position) is
//   plane[p][j] = min(rows[cell_of_col[j]][p][elems[e]], 65535)   (0 where cell_of_col[j] < 0)
// as a row-major [L][n_cols] u16 array, cut into (crow x ccol) chunks (edge chunks
// padded with 0) and deflated in the H5Z_DEFLATE form. One task per (position chunk,
// column chunk) reads each cell's crow positions once for all planes; no [L][n_cols]
// plane is ever materialised (the numpy transposes cost seconds at C3).
// Chunk t of plane e is blob[offsets[e * n_chunks + t] .. offsets[e * n_chunks + t + 1]),
// chunks row-major over the chunk grid. Returns the chunks per plane, -1 on error.
extern "C" int64_t mgp_h5_plane_tiles(const void* rows, int32_t elem_size, int64_t row_elems, int64_t n_rows,
                                      int64_t L, const int64_t* cell_of_col, int64_t n_cols, const int32_t* elems,
                                      int32_t n_planes, int64_t crow, int64_t ccol, int level, int n_threads,
                                      uint8_t** blob, int64_t* offsets) {
    mgp_host_err().clear();
    if (!rows || !cell_of_col || !elems || !blob || !offsets || (elem_size != 2 && elem_size != 4) || row_elems < 1 ||
        L <= 0 || n_cols <= 0 || n_planes <= 0 || crow <= 0 || ccol <= 0 || level < 0 || level > 9) {
        mgp_host_err() = "mgp_h5_plane_tiles: bad arguments";
        return -1;
    }
    for (int e = 0; e < n_planes; ++e)
        if (elems[e] < 0 || elems[e] >= row_elems) {
            mgp_host_err() = "mgp_h5_plane_tiles: plane element out of range";
            return -1;
        }
    for (int64_t j = 0; j < n_cols; ++j)
        if (cell_of_col[j] >= n_rows) {
            mgp_host_err() = "mgp_h5_plane_tiles: cell index out of range";
            return -1;
        }
    const int64_t nr = (L + crow - 1) / crow, nc = (n_cols + ccol - 1) / ccol, n = nr * nc;
    const size_t tile_elems = (size_t)crow * (size_t)ccol;
    std::vector<std::vector<uint8_t>> out((size_t)n * (size_t)n_planes);
    std::atomic<int64_t> next{0};
    std::atomic<bool> ok{true};
    auto work = [&]() {
        std::vector<uint16_t> tiles(tile_elems * (size_t)n_planes);
        mgp_host::Deflator dz(level);
        for (;;) {
            const int64_t t = next.fetch_add(1);
            if (t >= n || !ok) break;
            const int64_t p0 = (t / nc) * crow, j0 = (t % nc) * ccol;
            const int64_t h = std::min(crow, L - p0), w = std::min(ccol, n_cols - j0);
            if (h < crow || w < ccol) std::fill(tiles.begin(), tiles.end(), (uint16_t)0);
            for (int64_t jj = 0; jj < w; ++jj) {
                const int64_t c = cell_of_col[j0 + jj];
                if (c < 0) {
                    for (int e = 0; e < n_planes; ++e)
                        for (int64_t r = 0; r < h; ++r) tiles[(size_t)e * tile_elems + (size_t)r * ccol + jj] = 0;
                    continue;
                }
                const size_t base = ((size_t)c * (size_t)L + (size_t)p0) * (size_t)row_elems;
                if (elem_size == 2) {
                    const uint16_t* src = static_cast<const uint16_t*>(rows) + base;
                    for (int64_t r = 0; r < h; ++r, src += row_elems)
                        for (int e = 0; e < n_planes; ++e)
                            tiles[(size_t)e * tile_elems + (size_t)r * ccol + jj] = src[elems[e]];
                } else {
                    const uint32_t* src = static_cast<const uint32_t*>(rows) + base;
                    for (int64_t r = 0; r < h; ++r, src += row_elems)
                        for (int e = 0; e < n_planes; ++e)
                            tiles[(size_t)e * tile_elems + (size_t)r * ccol + jj] =
                                (uint16_t)std::min<uint32_t>(src[elems[e]], 65535u);
                }
            }
            for (int e = 0; e < n_planes; ++e)
                if (!dz.zlib(reinterpret_cast<const uint8_t*>(tiles.data() + (size_t)e * tile_elems), tile_elems * 2,
                             out[(size_t)e * (size_t)n + (size_t)t]))
                    ok = false;
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
    const size_t m = (size_t)n * (size_t)n_planes;
    size_t total = 0;
    for (size_t i = 0; i < m; ++i) {
        offsets[i] = (int64_t)total;
        total += out[i].size();
    }
    offsets[m] = (int64_t)total;
    uint8_t* b = (uint8_t*)std::malloc(std::max<size_t>(total, 1));
    if (!b) {
        mgp_host_err() = "out of host memory";
        return -1;
    }
    for (size_t i = 0; i < m; ++i)
        if (!out[i].empty()) std::memcpy(b + offsets[i], out[i].data(), out[i].size());
    *blob = b;
    return n;
}
