// mgp_txtgz.h — the engine's txt writer on the device (internal interface between
// mgp_engine.hip and mgp_txtgz.hip; the C-ABI is mgp_txt_gz* in include/mgpileup.h).
//
// IncrementalTextWriter (src/file_io/writers.py:430-486) formats, per passing cell,
//   output.coverage.txt: "pos,barcode,depth\n"   for every position with depth > 0
//   output.{A,C,G,T}.txt: "pos,barcode,fwd,rev\n" for those with fwd + rev > 0
// (1-based positions, cells in first-seen order) and then gzips each file at
// compresslevel=9. Here one workgroup per (cell, file) formats the cell's lines from
// the count rows resident in HBM and deflates them into one gzip member (a dynamic-
// Huffman block from an optimal parse over line-aligned match candidates, or a fixed
// or stored block when smaller), so only the compressed members cross the host link
// and a file is its members concatenated in cell order (gzip readers, Python's gzip
// and zcat read multi-member files as one stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mgp {
namespace txtgz {

constexpr int kFiles = 5;  // coverage, A, C, G, T (member m of cell k is file m % 5 ... see Members)

// The count rows the lines are made from: the engine's 16-bit rows (u16 (fwd, rev)
// pairs per base as one uint4 per position, u16 depth) with the exact u32 rows of its
// drained windows (wide flag per (cell, window)), or plain u32 rows (c16 == nullptr).
struct Rows {
    const uint4* c16;
    const uint16_t* d16;
    const uint8_t* wide;
    const uint32_t* c32;  // [cells][L][8]
    const uint32_t* d32;  // [cells][L]
    int L, W, nwin;
};

// One batch of cells (the caller's order) and their barcodes (device arrays).
struct Job {
    Rows rows;
    int64_t n;                 // cells of the batch
    const int32_t* cells;      // row index of each
    const char* names;         // barcodes, concatenated
    const int64_t* name_off;   // n + 1
};

// Device scratch of a batch; every array is sized by the caller from txt_sizes().
struct Scratch {
    uint64_t* text_off;   // [5n + 1] member text offsets (member = file * n + cell), 16-byte aligned
    const uint64_t* text_n;  // [5n] member text bytes (txt_sizes)
    uint64_t* line_off;   // [5n + 1]
    uint64_t* out_off;    // [5n + 1] member output regions (bounds)
    uint8_t* text;        // text_off[5n] bytes
    uint32_t* tok;        // text_off[5n] words: the parse's choices, then the tokens
    uint32_t* lines;      // line_off[5n] x 3 words: start, c1 | c2 << 16, c3 | len << 16
    uint32_t* out;        // out_off[5n] / 4 words (member outputs)
    uint32_t* member_bytes;  // [5n] compressed bytes of each member
    const uint32_t* crc_shift;  // [kShiftPow][32]: one-zero-byte CRC operator to the powers 2^b (GF(2) matrices)
    uint32_t* seg;              // [5n][257] each thread's segment start in its member's text (and the end)
    uint32_t* crc;              // [5n] CRC-32 of each member's text
    uint64_t* prof;             // MGP_TXT_PROF: [5n][8] kernel stamps (100 MHz wall clock), else null
};

// member text bytes and lines of every (file, cell) of the batch -> sizes[5n], nlines[5n]
int txt_sizes(const Job& job, uint64_t* sizes, uint64_t* nlines, hipStream_t s);
// the members (gzip) into scratch.out at out_off; member_bytes filled
int txt_deflate(const Job& job, const Scratch& sc, hipStream_t s);
// members packed back to back in member order (file-major) from out_off into dst at dst_off[5n]
int txt_pack(const Scratch& sc, int64_t n_members, const uint64_t* dst_off, uint8_t* dst, hipStream_t s);
// the CRC shift matrices (host): texts up to 2^kShiftPow bytes (a member of 16569 lines
// of 4096-byte barcodes is ~68 MB)
constexpr int kShiftPow = 28;
void crc_shift_matrices(uint32_t* m /* kShiftPow x 32 */);
// ---- HDF5 chunks (IncrementalHDF5Writer's count datasets, writers.py:60-131) ----
// The 11 u16 planes [L][n_cols] (A_fwd, A_rev, ..., T_rev, tn5_cuts_fwd, tn5_cuts_rev,
// coverage; min(v, 65535) of the run's values, which its 16-bit rows hold; a column is a
// cell of the rows or zeros) cut into (crow x ccol) chunks, edge chunks padded with 0,
// each deflated on the device into one zlib stream, the H5Z_DEFLATE filter's form.
constexpr int kPlanes = 11;
struct H5Job {
    const uint4* c16;           // [cells][L]: 8 x u16 (A_fwd, A_rev, ..., T_rev)
    const uint32_t* t16;        // [cells][L]: tn5 fwd | rev << 16
    const uint16_t* d16;        // [cells][L]
    int L;
    const int32_t* cell_of_col;  // [n_cols]: a cell of the rows, -1: a zero column
    int64_t n_cols;
    int crow, ccol;             // chunk shape
    int nrc;                    // row chunks, ceil(L / crow)
    int cc0, ncc;               // this batch: column chunks [cc0, cc0 + ncc)
    unsigned long long* sums;   // [3][L]: per-position sums over the batch's columns of the
                                // coverage, tn5 fwd and tn5 rev planes (zeroed by the caller)
};
// Batch chunk k = (plane * nrc + rc) * ncc + (cc - cc0): its raw bytes at raw + k raw_stride,
// its output region at out + k out_stride (out_off[k]).
struct H5Scratch {
    uint8_t* raw;
    uint32_t* tok;           // tok_stride words per chunk (h5_tok_words)
    uint32_t* out;
    const uint64_t* out_off;
    uint32_t* chunk_bytes;   // [chunks] zlib stream bytes
    uint64_t chunk_raw, out_stride;
    uint64_t raw_stride;     // chunk_raw rounded up to 16 bytes (the parse loads 16 at a time)
    uint64_t tok_stride;     // h5_tok_words(chunk_raw)
    uint64_t* prof;          // MGP_H5_PROF: [chunks][4] phase stamps (100 MHz wall clock), else null
};
// a chunk's parse segment (bytes per thread, 16-aligned) and its token words (u16 tokens,
// at most two segments' worth per thread)
__host__ __device__ inline int h5_seg_bytes(uint64_t chunk_raw) { return (int)((((chunk_raw + 255) / 256) + 15) & ~uint64_t(15)); }
__host__ __device__ inline uint64_t h5_tok_words(uint64_t chunk_raw) { return (uint64_t)h5_seg_bytes(chunk_raw) * 256; }
// the planes' raw chunks of the batch, then their zlib streams (chunk_bytes filled)
int h5_deflate(const H5Job& job, const H5Scratch& sc, hipStream_t s);
// the streams packed back to back (chunk order) into dst at dst_off[chunks]
int h5_pack(const H5Scratch& sc, int64_t n_chunks, const uint64_t* dst_off, uint8_t* dst, hipStream_t s);

// bound of a member's output region for `text` bytes
__host__ __device__ inline uint64_t out_bound(uint64_t text) { return ((text + 5 * (text / 65535 + 1) + 64 + 31) & ~uint64_t(31)); }

}  // namespace txtgz
}  // namespace mgp
