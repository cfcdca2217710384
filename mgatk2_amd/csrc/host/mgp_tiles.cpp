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
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "mgp_zcodec.h"
#include "../../../include/mgpileup_host.h"

std::string& mgp_host_err();  // mgp_bam.cpp

namespace {
// The compressed chunks of a parallel deflate: each thread compresses into one scratch
// buffer and appends the result to an arena of its own; the arenas, scratch buffers, tile
// buffers and compressors are all allocated before the threads start, so the threads
// never map or unmap memory (a per-chunk output vector sized to the deflate bound, ~200 KB,
// is above glibc's mmap threshold, so each chunk mapped and unmapped its own buffer).
struct Arena {
    std::vector<uint8_t> buf, scratch;
    std::vector<uint16_t> tiles;
    std::unique_ptr<mgp_host::Deflator> dz;
    void prepare(int level, size_t tile_bytes, size_t expect) {
        dz.reset(new mgp_host::Deflator(level));
        scratch.reserve(tile_bytes + tile_bytes / 8 + 4096);  // (above the deflate bound)
        buf.reserve(expect);
        tiles.resize((tile_bytes + 1) / 2);
    }
};
struct Piece {
    int32_t th = 0;
    uint64_t off = 0, len = 0;
};
// the pieces, in order, into one malloc'd blob with offsets[0..m] (offsets[m] = total)
bool gather_pieces(const std::vector<Piece>& pc, const std::vector<Arena>& ar, uint8_t** blob, int64_t* offsets) {
    size_t total = 0;
    for (size_t i = 0; i < pc.size(); ++i) {
        offsets[i] = (int64_t)total;
        total += pc[i].len;
    }
    offsets[pc.size()] = (int64_t)total;
    uint8_t* b = (uint8_t*)std::malloc(std::max<size_t>(total, 1));
    if (!b) return false;
    for (size_t i = 0; i < pc.size(); ++i)
        if (pc[i].len) std::memcpy(b + offsets[i], ar[(size_t)pc[i].th].buf.data() + pc[i].off, pc[i].len);
    *blob = b;
    return true;
}
// one chunk through the thread's scratch into its arena
bool deflate_piece(mgp_host::Deflator& dz, const uint8_t* src, size_t n, Arena& a, int32_t th, Piece& out) {
    if (!dz.zlib(src, n, a.scratch)) return false;
    out.th = th;
    out.off = a.buf.size();
    out.len = a.scratch.size();
    a.buf.insert(a.buf.end(), a.scratch.begin(), a.scratch.end());
    return true;
}
}  // namespace

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
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n));
    std::vector<Piece> pc((size_t)n);
    std::vector<Arena> ar((size_t)nt);
    std::atomic<int64_t> next{0};
    std::atomic<bool> ok{true};
    const uint8_t* src = (const uint8_t*)data;
    for (auto& a : ar) a.prepare(level, chunk_bytes, chunk_bytes * (size_t)((n + nt - 1) / nt) / 3);
    auto work = [&](int32_t ti) {
        Arena& a = ar[(size_t)ti];
        uint8_t* tile = reinterpret_cast<uint8_t*>(a.tiles.data());
        for (;;) {
            const int64_t t = next.fetch_add(1);
            if (t >= n) break;
            const int64_t r0 = (t / nc) * crow, c0 = (t % nc) * ccol;
            const int64_t h = std::min(crow, rows - r0), w = std::min(ccol, cols - c0);
            if (h < crow || w < ccol) std::memset(tile, 0, chunk_bytes);
            for (int64_t r = 0; r < h; ++r)
                std::memcpy(tile + (size_t)r * ccol * elem_size,
                            src + ((size_t)(r0 + r) * (size_t)cols + (size_t)c0) * elem_size, (size_t)w * elem_size);
            // the H5Z_DEFLATE form: one zlib stream of the whole (padded) chunk
            if (!deflate_piece(*a.dz, tile, chunk_bytes, a, ti, pc[(size_t)t])) {
                ok = false;
                return;
            }
        }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(work, (int32_t)i);
    work(0);
    for (auto& x : th) x.join();
    if (!ok) {
        mgp_host_err() = "deflate failed";
        return -1;
    }
    if (!gather_pieces(pc, ar, blob, offsets)) {
        mgp_host_err() = "out of host memory";
        return -1;
    }
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
    int nt = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n));
    std::vector<Piece> pc((size_t)n * (size_t)n_planes);
    std::vector<Arena> ar((size_t)nt);
    std::atomic<int64_t> next{0};
    std::atomic<bool> ok{true};
    for (auto& a : ar)
        a.prepare(level, tile_elems * 2 * (size_t)n_planes, tile_elems * 2 * (size_t)n_planes * (size_t)((n + nt - 1) / nt) / 3);
    auto work = [&](int32_t ti) {
        Arena& a = ar[(size_t)ti];
        std::vector<uint16_t>& tiles = a.tiles;
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
                if (!deflate_piece(*a.dz, reinterpret_cast<const uint8_t*>(tiles.data() + (size_t)e * tile_elems),
                                   tile_elems * 2, a, ti, pc[(size_t)e * (size_t)n + (size_t)t]))
                    ok = false;
        }
    };
    std::vector<std::thread> th;
    for (int i = 1; i < nt; ++i) th.emplace_back(work, (int32_t)i);
    work(0);
    for (auto& x : th) x.join();
    if (!ok) {
        mgp_host_err() = "deflate failed";
        return -1;
    }
    if (!gather_pieces(pc, ar, blob, offsets)) {
        mgp_host_err() = "out of host memory";
        return -1;
    }
    return n;
}
