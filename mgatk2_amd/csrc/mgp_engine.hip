// mgp_engine.hip — MI355X (gfx950) per-barcode chrM pileup engine + its C-ABI.
//
// Hot path (one mgp_run over the HBM-resident read set), restating the
// reference's per-read Python loops (paths relative to the reference root):
//
//   k_bin_count     per (start bin, cell slice): bin bounds by binary search,
//                   coordinate-order check (pysam's fetch() order, readers.py:87-92),
//                   flag/barcode filters (readers.py:95-111) and the per-cell read
//                   histogram in LDS
//   k_scan_*        exclusive scan of the histogram in (cell, start-bin) order: the
//                   cell-major layout of `reads_by_barcode` (readers.py:69,164)
//   k_group_a/b     two-pass stable grouping: per start bin into (bin, 64-cell group)
//                   buckets, then per cell group into cell-major order; one 16-byte
//                   grouping element per valid read at
//                   its cell-major slot, BAM order kept inside each cell (stable)
//   k_pileup        per (cell chunk, position window): duplicate marking by a short
//                   walk back over equal starts (readers.py:118-150, first in BAM
//                   order wins), kept-read counts (processors.py:22,34), MAPQ gate
//                   (pileup.py:33), Tn5 cuts + CIGAR walk + end-distance / base
//                   quality / base filters (pileup.py:32-95) into an LDS count tile,
//                   then strand-bias filter, depth, Tn5 masking (pileup.py:128-154),
//                   per-cell depth statistics (processors.py:36-39, writers.py:187-197)
//                   and per-workgroup reference-allele partial tallies
//                   (writers.py:221-222) at the tile flush
//   k_gate_fixup    min-reads gate (processors.py:22) when min_reads > 1
//   k_median        np.median of covered depths per cell (writers.py:190)
//   k_tally_reduce  sum of the partial tallies (writers.py:340-349 input)
//   RCCL allreduce  tallies over ranks when cells are sharded over GPUs
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <rccl/rccl.h>

#include <algorithm>
#include <type_traits>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mgpileup.h"
#include "mgp_kernels.h"
#include "mgp_txtgz.h"

using namespace mgp;

// ---------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------
static thread_local std::string g_err;

static int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e__ = (expr);                                                        \
        if (e__ != hipSuccess) {                                                        \
            return set_err(e__ == hipErrorOutOfMemory ? MGP_E_OOM : MGP_E_HIP,          \
                           std::string(#expr) + ": " + hipGetErrorString(e__));         \
        }                                                                               \
    } while (0)

#define MGP_TRY(expr)             \
    do {                          \
        int r__ = (expr);         \
        if (r__ != MGP_OK) return r__; \
    } while (0)

// ---------------------------------------------------------------------------
// device buffers
// ---------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    int ensure(size_t bytes, bool preserve = false, size_t used = 0, hipStream_t s = 0) {
        if (bytes <= cap) return MGP_OK;
        size_t ncap = std::max(bytes, cap + cap / 2);
        ncap = (ncap + 255) & ~size_t(255);
        void* np = nullptr;
        hipError_t e = hipMalloc(&np, ncap);
        if (e != hipSuccess) {
            ncap = (bytes + 255) & ~size_t(255);
            e = hipMalloc(&np, ncap);
            if (e != hipSuccess)
                return set_err(MGP_E_OOM, "hipMalloc(" + std::to_string(ncap) + ") failed: " +
                                              hipGetErrorString(e));
        }
        if (preserve && p && used) {
            HIP_TRY(hipMemcpyAsync(np, p, used, hipMemcpyDeviceToDevice, s));
            HIP_TRY(hipStreamSynchronize(s));
        }
        if (p) (void)hipFree(p);
        p = np;
        cap = ncap;
        return MGP_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

// mgp_txt_gz: the device txt writer's buffers (mgp_txtgz.hip), kept for the next call
struct TxtState {
    DevBuf cells, names, name_off, sizes, nlines, offs, text, tok, lines, out, member_bytes, crc_shift, dst_off, packed;
    DevBuf rows_c, rows_d;  // (mgp_txt_gz_rows: the caller's u32 rows)
    DevBuf prof;            // MGP_TXT_PROF
    DevBuf seg, crc;
    bool shift_ready = false;
    int64_t n = 0;
    uint64_t total = 0;
};

// mgp_h5_tiles: the HDF5 chunk deflate's buffers (mgp_txtgz.hip), kept for the next call
struct H5State {
    DevBuf coc, raw, tok, out, out_off, chunk_bytes, dst_off, packed, sums, prof;
    uint64_t total = 0;
};

enum Stage { ST_HIST, ST_SCAN, ST_GROUP_A, ST_GROUP_B, ST_PILEUP, ST_GATE, ST_MEDIAN, ST_TALLY, ST_COMM, ST_N };
static const char* kStageNames = "hist,scan,group_a,group_b,pileup,gate,median,tally,comm";

struct mgp_ctx {
    mgp_config cfg{};
    int dev = 0;
    hipStream_t s_comp = nullptr, s_copy = nullptr;
    hipStream_t s_side = nullptr;  // the tally reduction, concurrent with the medians
    // mgp_set_rows16_target: the 16-bit rows of each segment's windows go to these pinned
    // host arrays on their own stream as soon as the segment's pileup ends
    hipStream_t s_d2h = nullptr;
    hipEvent_t ev_rows = nullptr;
    mgp_rows16 rows_tgt{};
    bool rows_on = false;
    mgp_rows8 rows8_tgt{};  // mgp_set_rows_target: the 8-bit target of the windows that fit (ABI 7)
    bool rows8_on = false;
    bool rows_pending = false;  // the run's last segment's rows: copied by run_finish
    int rows_p0 = 0, rows_p1 = 0;
    hipEvent_t ev_copy = nullptr, ev_fork = nullptr, ev_join = nullptr;
    int seg_min_win = 1;     // a streaming push queues a segment once this many windows are complete (MGP_SEG_MIN_WIN)
    int rows_wg = 256;       // workgroups of a segment's k_rows_to_host (MGP_ROWS_WG)
    int32_t cell_lo = 0;     // mgp_set_cell_range: the context's cells in the pushed batches' barcode indices
    bool cell_range = false;
    int pile_wg_stream = 0;  // a streaming run's pileup workgroups per window (set_pile_chunks; 0: the default)
    int pile_min_cpb_stream = 1;  // a streaming run's least cells per pileup chunk (MGP_PILE_MIN_CPB_STREAM)
    // on-device pairing of dense 64-byte batches (mgp_push_batch): two staging buffers
    // the H2D copies land in, the event after the pairing kernels that last read each
    // Off by default since round 6: the pairing copy (k_pair_rank + k_pair_place, ~10 ms of
    // GPU time per C4 step) saved ~1.3 ms of pileup, and the streamed step is link-bound
    // with or without it (profiles/r06/tail_r6i.txt); MGP_DEV_PAIR=1 turns it on
    bool dev_pair = false;
    int stage_i = 0;
    DevBuf stage[2], pair_rank, pair_cnt, pair_lines;
    DevBuf col16[2];  // a 16-bit batch's barcode and |tlen| columns (mgp_push_batch16), before widening
    hipEvent_t ev_stage[2] = {nullptr, nullptr};
    hipEvent_t ev_bits = nullptr;  // the run's input check words have reached h_bits
    uint32_t* h_bits = nullptr;    // pinned host copy of the input check words (roff_irregular)
    static constexpr int kRing = 64;   // per-run event slots (timing over many runs without syncs)
    hipEvent_t ev[kRing][ST_N][2];
    bool stage_ran[kRing][ST_N]{};
    // a streaming run's segment pileups (each mgp_push_batch that completes windows
    // launches one): HIP event pairs per run slot, created on the first streaming
    // segment; seg_n = segments recorded for the slot's run (kSegEv + 1: more than
    // kSegEv, the run's pileup is then untimed)
    static constexpr int kSegEv = 24;
    std::vector<hipEvent_t> seg_ev;
    int seg_n[kRing]{};
    int64_t runs = 0;                  // completed mgp_run calls
    Geom g{};
    int lds_hist_max_cells = 0;
    int hist_slice_cells = 0;  // > 0: cap on the histogram's cells per slice (MGP_HIST_SLICE_CELLS)
    bool hist_xcd = true;      // several slices: a bin's slices dealt to one XCD (MGP_HIST_XCD)
    int hist_narrow = -1;      // 8-bit histogram counters: -1 when 32-bit ones need several slices (MGP_HIST_NARROW)
    int64_t ga_wide_min = 8192;   // reads per pass-A workgroup from which it runs 512 threads (MGP_GA_WIDE_MIN)
    int hist_bounds = 1;       // bin bounds by k_bin_bounds (MGP_HIST_BOUNDS=0: searched by each histogram workgroup)
    bool group_wide = false;   // MGP_GROUP_WIDE=1: 16-byte grouping elements always (tests, A/B)

    // resident inputs (BAM order)
    int64_t n = 0, pay = 0;
    DevBuf start, bc, tlen, flag, mapq, span, roff, payload;
    DevBuf roff32;          // u32 rec_off >> 6 (grouping pass A reads it when every offset fits, kOffR32)
    DevBuf roff_irregular;  // u32 words of the input check (k_bin_count): CHK_* bits, largest kept span
    DevBuf order_bad;       // u32: a streaming push found reads out of coordinate order (k_check_order)
    int roff_mode = -1;     // pass A's offset source (kOffDense / kOffR32 / kOffR64), from the run's input check
    uint32_t read_bits = 0; // the input check's CHK_* bits of the resident reads
    bool no_spec = false;   // the speculative compact grouping failed on the resident reads (ERR_RESPEC)
    // the input check's flag bits of the last run over the same resident reads (no push,
    // reset or generation since): the next run picks its variants from them without the
    // mid-run host wait, and check_stats (pass B) verifies them on the device (ERR_RESPEC)
    bool bits_cached = false;
    uint32_t cached_bits = 0;
    bool stage_all = true;  // HIP events around every stage (false: the pileup's only, mgp_set_stage_timing)

    // run scratch
    DevBuf bin_start, H, P, cell_cnt, cell_base, bin_valid, bin_base, bucket_off, gel2, PG, F;
    DevBuf chunk_perm;  // the pileup's cell chunks, largest first (k_scan_cells)
    DevBuf pel, tally_part, tally, dup_part;
    DevBuf n_reads, any_paired, passed, covered, dsum, dmax, med_lo, med_hi, first_read;
    DevBuf counts, tn5, depth, stats;  // u32 rows: drained windows, and mgp_fetch's widened copy
    DevBuf counts16, tn5_16, depth16, wide, fit8;  // the run's 16-bit result rows (Out16)

    bool ran = false;
    int last_status = MGP_OK;
    DevStats* host_stats = nullptr;  // pinned: the run's stats copy stays asynchronous

    ncclComm_t comm = nullptr;
    int nranks = 1;
    unsigned long long* h_respec = nullptr;  // pinned: the ranks' all-reduced ERR_RESPEC count
    bool rerunning = false;                  // mgp_sync is running the fallback rerun

    // streaming runs (MGP_CFG_STREAM): pushes run the complete windows as segments
    bool stream = false;
    bool stream_off = false;   // the resident reads cannot stream (payload too large for compact elements)
    bool seg_open = false;     // segments of the current run are queued (mgp_run finishes it)
    int w_done = 0;            // windows [0, w_done) of the current run are queued
    int stream_layout = 1;     // kLayP64 / kLayP32: the packed layout the run's segments assume
    int64_t segments = 0;      // segments queued by pushes (all runs)
    bool last_streamed = false;

    TxtState txt;  // mgp_txt_gz
    H5State h5;    // mgp_h5_tiles
};

// ---------------------------------------------------------------------------
// kernels
// ---------------------------------------------------------------------------

__device__ __forceinline__ bool read_valid(int c, uint16_t f, int nc) {
    return c >= 0 && c < nc && !(f & (MGP_FLAG_UNMAPPED | MGP_FLAG_SECONDARY | MGP_FLAG_SUPPLEMENTARY));
}

// first index i in [0, n) with start[i] >= t (start[] is coordinate-sorted). (A
// workgroup-wide search with blockDim probes per step, ~4 dependent steps at 200M
// starts, measured slower: its barriers cost more than these dependent loads, which
// the other resident workgroups hide; r03 v48.)
__device__ __forceinline__ int64_t lower_bound_start(const int32_t* __restrict__ start, int64_t n, int64_t t) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)start[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// smallest start of bin b (bin_of() inverse)
__device__ __forceinline__ int64_t bin_threshold(int b, const Geom& g) {
    if (b <= 0) return INT64_MIN;
    if (b >= g.nbins) return INT64_MAX;
    if (b == g.nb_reg) return g.L;
    return (int64_t)b * g.G;
}

// Streaming runs (MGP_CFG_STREAM) process the resident reads in segments of
// complete position windows [seg_w0, seg_w1) while later batches are still on
// their way (mgp_push_batch). A segment's start bins are [seg_lo_bin, seg_bhi):
// the bins of its windows plus the halo bins of window seg_w0, i.e. the bins
// whose reads can reach seg_w0 given the largest declared span of the reads of
// the earlier segments (st->max_span when the segment starts: every read before
// seg_w0 x W was checked by an earlier segment). Other bins count as empty.
__device__ __forceinline__ int seg_lo_bin(int seg_w0, const Geom& g, const DevStats* st) {
    if (seg_w0 <= 0) return 0;
    const uint32_t ms = st->max_span;
    const int R = (int)((ms + g.G - 1) / g.G) * g.G;
    return win_lo_bin(seg_w0, R, g);
}

constexpr int kGroup = 64;  // cells per grouping bucket (pass A) and per pass-B workgroup

// Start bins are split into kParts parts (equal read-index ranges) so that
// grouping pass A runs on kParts x nbins workgroups: a grid of ~2 slot-rounds
// (4 workgroups per CU) would leave a long tail.
#ifndef MGP_PARTS
#define MGP_PARTS 4
#endif
constexpr int kParts = MGP_PARTS;
__device__ __forceinline__ void part_range(int64_t lo, int64_t hi, int p, int64_t& plo, int64_t& phi) {
    const int64_t len = hi - lo;
    plo = lo + len * p / kParts;
    phi = lo + len * (p + 1) / kParts;
}

#ifndef MGP_HIST_U
#define MGP_HIST_U 6  // reads per thread per histogram step (r03 A/B: 4 and 8 slower)
#endif
#ifndef MGP_HIST_BLOCK
#define MGP_HIST_BLOCK 512
#endif
constexpr uint64_t kRecStride = MGP_PACK_BYTES;  // record stride of a dense packed payload
constexpr uint32_t kCompactTlen = 1u << 16;       // |tlen| below this fits the compact grouping element
// The input check's words (ck[0] bits, ck[1] the largest declared span of the reads
// the run keeps at its filters: the pileup's window halo). Bit 1: some record offset
// is not kRecStride x its read index (else the payload is dense and grouping pass A
// computes the offsets); bit 2: some offset is not a multiple of 64 below 2^38 (else
// pass A reads the u32 column roff32 = rec_off >> 6, written by the check).
// Where the bits come from (mgp_run): the start-bin histogram takes the flag bits
// (CHK_PAIRED, CHK_UNPAIRED, CHK_NOSEQ, CHK_FULL) from the flags it reads anyway.
// When they allow compact grouping elements, grouping pass A checks the rest on the
// reads it loads anyway (coordinate order, span, key widths, 64-byte offsets) and
// raises ERR_RESPEC if an element does not fit: mgp_sync then runs the run again on
// the fallback path, whose standalone check (k_check_inputs) takes every bit first.
// CHK_PAIRED / CHK_UNPAIRED / CHK_NOSEQ: some read is paired / unpaired / lacks SEQ
// or QUAL (pass B tracks pairedness and SEQ per read only when the reads mix or lack
// them). CHK_FULL / CHK_P64 / CHK_P32: some record is in the full / packed 64-byte /
// 32-byte layout (include/mgpileup.h; a flag word with both packed bits is a 32-byte
// record). CHK_WIDEKEY: some start lies
// outside [0, mito_len) or some |tlen| >= kCompactTlen (no compact grouping element).
// CHK_UNSORTED: a start below its predecessor's (pysam's fetch order, readers.py:87-92).
constexpr uint32_t CHK_PAIRED = 4u, CHK_UNPAIRED = 8u, CHK_NOSEQ = 16u, CHK_FULL = 32u, CHK_WIDEKEY = 64u,
                   CHK_UNSORTED = 128u, CHK_P64 = 256u, CHK_P32 = 512u;
__device__ __forceinline__ uint32_t layout_bit(uint32_t f) {
    return (f & MGP_FLAG_PACK32) ? CHK_P32 : (f & MGP_FLAG_PACKED) ? CHK_P64 : CHK_FULL;
}
// Record layouts (include/mgpileup.h) and the pileup's instantiations: every record of
// one packed layout (the fast paths), or any mix (kLayAny: the layout per read)
enum { kLayFull = 0, kLayP64 = 1, kLayP32 = 2, kLayAny = 3 };

// One workgroup (8 waves) per (start bin, cell slice): bin bounds by binary
// search in the starts, flag/barcode filters (readers.py:95-111) and the LDS
// histogram of the slice's cells over the bin's reads (6 bytes read per read). A
// slice is as many 64-cell groups as the LDS holds (one slice up to ~24k cells;
// more cells scan the bin once per slice). The bin's parts are counted one after
// the other; after each part the per-64-cell-group totals are snapshotted, giving
// the per-(bin, part, group) counts of pass A. Slice 0 writes the bin's bounds and
// valid count, and ORs the flag bits of the input check into ck[0].
constexpr int kHistBlock = MGP_HIST_BLOCK;
// kNarrow: 8-bit counters, four cells per LDS word (a slice of up to ~144k cells in
// 150 KiB: C5's 100k cells in one pass over the bin instead of three). Every add
// returns the word it found; an add that finds its byte at 255 wraps it (and carries
// into the next cell's byte), so the workgroup then counts its cells again with 32-bit
// counters in sub-slices that fit the same LDS (a cell with more than 255 reads
// starting in one bin: rare, exact either way).
#ifndef MGP_HIST_NBLOCK
// the 8-bit form's threads per workgroup and reads per thread per step: its slices fill a
// CU's LDS (one workgroup per CU), so more waves and more loads in flight per workgroup
// (r04 A/B at C5: 512 x 6 4.12 ms, 512 x 12 3.56, 1024 x 6 2.64, 1024 x 12 2.49)
#define MGP_HIST_NBLOCK 1024
#endif
#ifndef MGP_HIST_NU
#define MGP_HIST_NU 12
#endif
template <bool kNarrow, int kHB = kNarrow ? MGP_HIST_NBLOCK : kHistBlock, int kU = kNarrow ? MGP_HIST_NU : MGP_HIST_U>
__global__ void __launch_bounds__(kHB) k_bin_count(const int32_t* __restrict__ start,
                                                          const int32_t* __restrict__ bc,
                                                          const uint16_t* __restrict__ flag, int64_t n, Geom g,
                                                          int slice_cells, uint32_t* __restrict__ H,
                                                          uint32_t* __restrict__ PG, int ngroups,
                                                          uint32_t* __restrict__ bin_lo,
                                                          uint32_t* __restrict__ bin_valid, uint32_t* __restrict__ ck,
                                                          DevStats* st, int seg_w0, int seg_bhi, int nslices,
                                                          int pre_bounds) {
    extern __shared__ uint32_t hist[];  // [slice cells] counts (kNarrow: bytes), then cum[slice groups]
    __shared__ int64_t s_range[2];
    __shared__ uint32_t s_nvalid, s_bits;
    // grid: (bins, slices), or with several slices a 1-D grid that deals the slices of
    // one bin to one XCD back to back (workgroups go round-robin over the 8 XCDs: ids
    // x, x + 8, ... share one), so the slices' re-reads of the bin's barcodes and flags
    // hit that XCD's L2 instead of HBM (slice-major order re-read every bin ~2000
    // workgroups later)
    int b = blockIdx.x, sl = blockIdx.y;
    if (nslices < 0) {
        const int ns = -nslices, j = (int)(blockIdx.x >> 3);
        b = 8 * (j / ns) + (int)(blockIdx.x & 7u);
        sl = j % ns;
        if (b >= g.nbins) return;
    }
    const bool first = sl == 0;
    const int nc = g.nc;
    const int c_lo = sl * slice_cells, c_hi = min(nc, c_lo + slice_cells);
    const int ncs = c_hi - c_lo;
    const int lane = threadIdx.x & 63;
    uint32_t* row = H + (size_t)b * nc;
    // the bin's bounds: searched here, or (pre_bounds) by k_bin_bounds into bin_lo
    if (threadIdx.x < 2)
        s_range[threadIdx.x] = pre_bounds ? (int64_t)bin_lo[b + threadIdx.x]
                                          : lower_bound_start(start, n, bin_threshold(b + threadIdx.x, g));
    if (threadIdx.x == 0) s_nvalid = 0, s_bits = 0;
    __syncthreads();
    // a bin outside the segment counts no read (its bounds are still written: pass A
    // takes a bin's upper bound from the next bin's lower one)
    const bool in_seg = b < seg_bhi && b >= seg_lo_bin(seg_w0, g, st);
    const int64_t blo = s_range[0], bhi = in_seg ? max(s_range[1], blo) : blo;
    if (first && threadIdx.x == 0) {
        if (!pre_bounds) {
            bin_lo[b] = (uint32_t)blo;
            if (b == g.nbins - 1) bin_lo[g.nbins] = (uint32_t)n;
        }
        // sorted starts give monotone bounds, and monotone bounds partition the reads
        // (each counted once, whatever the order inside); otherwise a read may be in
        // two bins' ranges and the grouping slots would outgrow their buffers
        if (s_range[1] < s_range[0]) atomicOr(&st->err, ERR_BOUNDS | ERR_UNSORTED);
    }
    unsigned long long nvalid = 0;
    bool badbc = false;
    uint32_t bits = 0;  // the input check's flag bits (slice 0)
    uint32_t* pg = PG + (size_t)b * kParts * ngroups;
    // count the cells [s_lo, s_hi) over the bin's parts; after each part the per-group
    // totals are snapshotted (pass A's per-(bin, part, group) counts); the rows go out at
    // the end. primary: the slice's own pass (the run's counts and check bits are taken
    // once). Returns whether an 8-bit counter wrapped (workgroup-uniform).
    auto count = [&](const int s_lo, const int s_hi, const bool narrow, const bool primary) -> bool {
        const int ns = s_hi - s_lo;
        const int nw = narrow ? (ns + 3) >> 2 : ns;
        const int gs_lo = s_lo / kGroup, ngss = (ns + kGroup - 1) / kGroup;
        uint32_t* cum = hist + nw;
        auto value = [&](int c) -> uint32_t { return narrow ? (hist[c >> 2] >> (8 * (c & 3))) & 0xFFu : hist[c]; };
        for (int x = threadIdx.x; x < nw; x += blockDim.x) hist[x] = 0;
        __syncthreads();
        bool wrap = false;
        for (int part = 0; part < kParts; ++part) {
            int64_t lo, hi;
            part_range(blo, bhi, part, lo, hi);
            // kU reads per thread per step, loads issued together (clamped index, no branches)
            for (int64_t i0 = lo + threadIdx.x; i0 < hi; i0 += kU * kHB) {
                int cc[kU];
                uint32_t ff[kU];
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const int64_t i = i0 + u * kHB;
                    const int64_t j = i < hi ? i : hi - 1;
                    cc[u] = bc[j];
                    ff[u] = flag[j];
                }
                if (primary) {
#pragma unroll
                    for (int u = 0; u < kU; ++u) {
                        const uint32_t f = ff[u];
                        if (i0 + u * kHB < hi)
                            bits |= (f & MGP_FLAG_PAIRED ? CHK_PAIRED : CHK_UNPAIRED) |
                                    (f & MGP_FLAG_NOSEQQUAL ? CHK_NOSEQ : 0u) | layout_bit(f);
                    }
                }
#pragma unroll
                for (int u = 0; u < kU; ++u) {
                    const int64_t i = i0 + u * kHB;
                    const int c = cc[u];
                    const bool in = i < hi;
                    if (primary) badbc |= in && (c >= nc);
                    if (in && read_valid(c, (uint16_t)ff[u], nc)) {
                        if (c >= s_lo && c < s_hi) {
                            const int x = c - s_lo;
                            if (narrow) {
                                const uint32_t sh = 8u * (uint32_t)(x & 3);
                                const uint32_t old = atomicAdd(&hist[x >> 2], 1u << sh);
                                wrap |= ((old >> sh) & 0xFFu) == 0xFFu;
                            } else {
                                atomicAdd(&hist[x], 1u);
                            }
                        }
                        if (primary) ++nvalid;
                    }
                }
            }
            __syncthreads();
            // group totals so far; this part's counts are the growth since the last part
            // (a group is always handled by the same wave, so `cum` needs no barrier)
            uint32_t* pgp = pg + (size_t)part * ngroups + gs_lo;
            for (int gi = threadIdx.x >> 6; gi < ngss; gi += kHB / kWave) {
                const int c = gi * kGroup + lane;
                const uint32_t h = wave_sum(c < ns ? value(c) : 0u);
                if (lane == 0) {
                    pgp[gi] = h - (part ? cum[gi] : 0u);
                    cum[gi] = h;
                }
            }
            __syncthreads();  // the snapshot is complete before the next part counts
        }
        for (int c = threadIdx.x; c < ns; c += blockDim.x) row[s_lo + c] = value(c);
        return narrow && __syncthreads_or(wrap) != 0;
    };
    if (count(c_lo, c_hi, kNarrow, true)) {
        // a wrapped 8-bit counter: 32-bit counts of the same cells, as many as the LDS
        // holds at a time (whole groups)
        const int words = (ncs + 3) / 4 + (ncs + kGroup - 1) / kGroup;
        const int sub = max(kGroup, words / (kGroup + 1) * kGroup);
        for (int s0 = c_lo; s0 < c_hi; s0 += sub) count(s0, min(c_hi, s0 + sub), false, false);
    }
    if (!first) return;
    nvalid = wave_sum(nvalid);
    const bool anybad = __ballot(badbc) != 0ull;
    bits = wave_or(bits);
    // the bin's valid count and check words (a global atomic per wave on one word
    // serialises at the memory side: one per workgroup)
    if (lane == 0) {
        if (nvalid) atomicAdd(&s_nvalid, (uint32_t)nvalid);
        if (bits) atomicOr(&s_bits, bits);
        if (anybad) atomicOr(&st->err, ERR_BADBC);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        bin_valid[b] = s_nvalid;
        if (s_bits && (__atomic_load_n(ck, __ATOMIC_RELAXED) & s_bits) != s_bits) atomicOr(ck, s_bits);
    }
}

// The start bins' bounds, one thread per bin (bin_lo[b] = first read of bin b,
// bin_lo[nbins] = n), for histograms whose workgroups would each wait on their own
// ~30 dependent loads with no other workgroup of the CU to hide them (one per CU).
__global__ void k_bin_bounds(const int32_t* __restrict__ start, int64_t n, Geom g, uint32_t* __restrict__ bin_lo) {
    const int b = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (b <= g.nbins) bin_lo[b] = (uint32_t)lower_bound_start(start, n, bin_threshold(b, g));
}

// Scan step a: column sums over blocks of RB rows, and the cells' totals (zeroed by
// k_run_init). grid (ceil(nc/256), nrb)
__global__ void k_scan_colsum(const uint32_t* __restrict__ H, int nrows, int nc, int RB,
                              uint32_t* __restrict__ P, uint32_t* __restrict__ cnt) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    int rb = blockIdx.y;
    if (c >= nc) return;
    int r0 = rb * RB, r1 = min(nrows, r0 + RB);
    uint32_t acc = 0;
    for (int r = r0; r < r1; ++r) acc += H[(size_t)r * nc + c];
    P[(size_t)rb * nc + c] = acc;
    if (acc) atomicAdd(&cnt[c], acc);
}

// (Scan step b, before r03 v55: the exclusive scan over row blocks per cell and the
// cells' totals in a kernel of its own; k_scan_apply now sums its row-block prefix.)
// Exclusive scan of cnt[0, n) into base by one workgroup of 1024; returns the total.
__device__ uint32_t block_exclusive_scan(const uint32_t* __restrict__ cnt, int n, uint32_t* __restrict__ base,
                                         uint32_t* wsum /* [16] LDS */, uint32_t* carry /* LDS */) {
    if (threadIdx.x == 0) *carry = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int c0 = 0; c0 < n; c0 += 1024) {
        int c = c0 + threadIdx.x;
        uint32_t v = c < n ? cnt[c] : 0;
        uint32_t x = v;  // inclusive wave scan
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wid] = x;
        __syncthreads();
        if (threadIdx.x < 16) {
            uint32_t w = wsum[threadIdx.x];
            uint32_t xs = w;
            for (int o = 1; o < 16; o <<= 1) {
                uint32_t y = __shfl_up(xs, o, 64);
                if ((int)threadIdx.x >= o) xs += y;
            }
            wsum[threadIdx.x] = xs - w;  // exclusive
        }
        __syncthreads();
        uint32_t excl = *carry + wsum[wid] + x - v;
        if (c < n) base[c] = excl;
        __syncthreads();
        if (threadIdx.x == 1023) *carry = excl + v;
        __syncthreads();
    }
    return *carry;
}

// Scan step c (single workgroup of 1024): exclusive scan over cells, and over the
// start bins' valid counts (bin_valid -> bin_base, grouping pass A's bucket bases;
// nbins = 0: none). Then it orders the pileup's cell chunks of cpb cells by size,
// largest first (a counting sort over 64 size classes): the pileup takes its
// workgroups' chunks in that order, so the largest chunks are not the grid's tail
// (lognormal cells: a chunk of 4 cells can hold twice the mean).
__global__ void __launch_bounds__(1024) k_scan_cells(const uint32_t* __restrict__ cnt, int nc,
                                                     uint32_t* __restrict__ base, int cpb, int nchunks,
                                                     uint32_t* __restrict__ perm,
                                                     const uint32_t* __restrict__ bin_valid, int nbins,
                                                     uint32_t* __restrict__ bin_base) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry;
    const int lane = threadIdx.x & 63;
    if (nbins > 0) (void)block_exclusive_scan(bin_valid, nbins, bin_base, wsum, &carry);
    const uint32_t total = block_exclusive_scan(cnt, nc, base, wsum, &carry);
    // chunk sizes from the cell bases this workgroup just wrote (visible to it behind
    // the barriers above); the last chunk ends at the total
    __shared__ uint32_t cls[64], s_max;
    auto size_of = [&](int ch) {
        const int c0 = ch * cpb, c1 = min(nc, c0 + cpb);
        return (c1 < nc ? base[c1] : total) - base[c0];
    };
    if (threadIdx.x < 64) cls[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_max = 0;
    __syncthreads();
    uint32_t mx = 0;
    for (int ch = threadIdx.x; ch < nchunks; ch += 1024) mx = max(mx, size_of(ch));
    mx = wave_max(mx);
    if (lane == 0 && mx) atomicMax(&s_max, mx);
    __syncthreads();
    const uint64_t m1 = (uint64_t)s_max + 1;
    auto key_of = [&](int ch) { return 63u - (uint32_t)((uint64_t)size_of(ch) * 64u / m1); };
    for (int ch = threadIdx.x; ch < nchunks; ch += 1024) atomicAdd(&cls[key_of(ch)], 1u);
    __syncthreads();
    if (threadIdx.x < 64) {  // exclusive scan of the class counts (one wave)
        const uint32_t v = cls[threadIdx.x];
        uint32_t x = v;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        cls[threadIdx.x] = x - v;
    }
    __syncthreads();
    for (int ch = threadIdx.x; ch < nchunks; ch += 1024) perm[atomicAdd(&cls[key_of(ch)], 1u)] = (uint32_t)ch;
}

// Scan step d: H[r][c] <- exclusive (cell-major) offset; row nrows <- cell end;
// F[r] bit c <- r is the first bin holding reads of c.
__global__ void k_scan_apply(uint32_t* __restrict__ H, const uint32_t* __restrict__ P,
                             const uint32_t* __restrict__ base, const uint32_t* __restrict__ cnt, int nrows,
                             int nc, int RB, int nrb, uint32_t* __restrict__ F) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    int rb = blockIdx.y;
    if (c >= nc) return;
    const uint32_t b0 = base[c];
    // the cell's reads in the row blocks before this one (independent loads)
    uint32_t pre = 0;
#pragma unroll 8
    for (int q = 0; q < rb; ++q) pre += P[(size_t)q * nc + c];
    uint32_t acc = b0 + pre;
    int r0 = rb * RB, r1 = min(nrows, r0 + RB);
    const size_t fw = (size_t)(nc + 31) / 32;
    for (int r = r0; r < r1; ++r) {
        size_t k = (size_t)r * nc + c;
        uint32_t h = H[k];
        if (h && acc == b0) atomicOr(&F[(size_t)r * fw + (c >> 5)], 1u << (c & 31));
        H[k] = acc;
        acc += h;
    }
    if (rb == nrb - 1) H[(size_t)nrows * nc + c] = b0 + cnt[c];
}

// Grouping element (16 bytes, cell-major, BAM order inside a cell):
//   w = record byte offset | meta << 56, start, |tlen|
struct __align__(16) GElem {
    unsigned long long w;
    int32_t start;
    uint32_t tlen;
};
constexpr unsigned long long GM_REV = 1ull << 56, GM_PAIRED = 2ull << 56, GM_MAPQ_OK = 4ull << 56,
                             GM_BAD = 8ull << 56, GM_PACKED = 16ull << 56, GM_P32 = 32ull << 56;

// Grouping in two passes (a single pass that writes each 16-byte element straight
// to its cell-major slot is bound by ~200M scattered partial-line stores):
//   A, per (start bin, part): valid reads -> buckets (bin, group of 64 cells), BAM
//      order kept inside each bucket; a bucket receives a contiguous run per step,
//      so its lines fill in L2 before they go to HBM;
//   B, per (cell group, bin range): bucket elements -> cell-major slots through
//      an LDS stage, duplicate marking, 8-byte pileup elements out; a cell's
//      slots over consecutive bins are contiguous, so a step writes 64 runs.
// The 6-bit cell id inside the group rides in bits 50..55 of GElem.w between
// the passes (record offsets stay below 2^50).
constexpr unsigned long long GM_LCELL_SHIFT = 50, GM_LCELL = 63ull << GM_LCELL_SHIFT;
// where grouping pass A takes the record offsets from (the input check in k_bin_count):
//   kOffDense  every offset is kRecStride x the read index: computed, nothing read
//   kOffR32    every offset is a multiple of 64 below 2^38: the u32 column roff32 = rec_off >> 6
//   kOffR64    otherwise: the u64 rec_off column
//   kOffSpec   the u64 column, with the input check's remaining tests on the loaded
//              reads (compact elements only; a read that does not fit raises ERR_RESPEC)
enum { kOffDense = 0, kOffR32 = 1, kOffR64 = 2, kOffSpec = 3 };

// Pileup element values (see k_group_b)
constexpr uint32_t PE_DUP = 0xFFFFFFFFu, PE_KEEP = 0xFFFFFFFEu, PE_PACKED = 0x80000000u, PE_OFF = 0x7FFFFFFFu;
// the wide (any-layout) path's pileup elements: PE_PACKED | PE_P32 for a 32-byte record,
// PE_PACKED alone for a packed 64-byte one, and a 30-bit offset (below PE_KEEP's)
constexpr uint32_t PE_P32 = 0x40000000u, PE_OFF30 = 0x3FFFFFFFu;

// Compact grouping element (8 bytes), used when every resident record is packed
// at a 64-byte multiple below 2^37 (dense or u32 offsets), the reads do not mix
// paired and unpaired ones and all have SEQ/QUAL, every start lies in
// [0, mito_len) and every |tlen| < 2^16 (the input check's bits):
//   low word   the pileup element of the read if it is kept: record offset / 64
//              (bits 0..30) | PE_PACKED when MAPQ >= min_mapq; 0 in bit 31 otherwise
//   high word  |tlen| (bits 0..15), start mod 256 (16..23), reverse (24), cell in
//              group (25..30): every duplicate-key field, so pass B compares one word
// Pass B compares starts mod 256: its steps span fewer than 32 start bins (256
// positions), and a cell's elements of one step are in start order, so equal
// starts mod 256 inside a cell's run of a step are equal starts.
constexpr int GC_START_SHIFT = 16, GC_LCELL_SHIFT = 25;
constexpr uint32_t GC_TLEN = 0xFFFFu, GC_START = 0xFFu << GC_START_SHIFT, GC_REV = 1u << 24,
                   GC_LCELL = 63u << GC_LCELL_SHIFT;
constexpr int kCompactBins = 32;             // start bins per pass-B step (compact elements)

#ifndef MGP_GA_AHEAD
#define MGP_GA_AHEAD 8  // reads per lane per pass-A step (A/B: 2, 3, 4, 6 slower)
#endif
#ifndef MGP_GA_WAVES
#define MGP_GA_WAVES 1
#endif
#ifndef MGP_ABL_A
#define MGP_ABL_A 0  // pass-A ablations (experiments only): 1 no element stores, 2 no ranking (slot = read index),
                     // 3 no span column (the C4 generator's 53 assumed)
#endif
#ifndef MGP_GA_DB
#define MGP_GA_DB 1  // pass A: next step's loads in flight during this step (double buffer)
#endif
#ifndef MGP_GA_BLOCK
#define MGP_GA_BLOCK 512  // threads per pass-A workgroup (r04 A/B: 256 2.06, 768 1.85, 1024 1.85 against 1.78 ms at C4)
#endif
constexpr int kGABlock = MGP_GA_BLOCK;
#ifndef MGP_GA_NBLOCK
#define MGP_GA_NBLOCK 128  // pass A's threads per workgroup for small sets / many cells (r04 A/B at 1250 cells: 256 0.262, 128 0.219 ms)
#endif
constexpr int kGANBlock = MGP_GA_NBLOCK;
// kCompact: 8-byte elements (GCompact, below; kOff is then dense or u32). kBlk: threads
// per workgroup. run_segment launches kGABlock (512) when its per-wave group counters
// fit the LDS and a (bin, part) workgroup gets at least MGP_GA_WIDE_MIN reads, else
// kGANBlock (128): small sets (the multi-GPU shares) and more than ~140k cells
template <int kOff, bool kCompact, int kBlk>
__global__ void __launch_bounds__(kBlk, MGP_GA_WAVES) k_group_a(int64_t n, const int32_t* __restrict__ start,
                                                    const int32_t* __restrict__ bc, const int32_t* __restrict__ tlen,
                                                    const uint16_t* __restrict__ flag, const uint8_t* __restrict__ mapq,
                                                    const uint64_t* __restrict__ roff,
                                                    const uint32_t* __restrict__ roff32,
                                                    const uint32_t* __restrict__ span,
                                                    const uint32_t* __restrict__ bin_lo,
                                                    const uint32_t* __restrict__ PG, const uint32_t* __restrict__ F,
                                                    const uint32_t* __restrict__ binbase,
                                                    Geom g, int ngroups, int gbits, int min_mapq,
                                                    uint32_t* __restrict__ bucket_off, GElem* __restrict__ gel2,
                                                    uint32_t* __restrict__ first_read, uint32_t* __restrict__ ck,
                                                    DevStats* st, int seg_w0, int seg_bhi, int spec_unit) {
    static_assert(kOff != kOffSpec || kCompact, "the speculative check writes compact elements");
    constexpr bool kSpec = kOff == kOffSpec;
    if (__atomic_load_n(&st->err, __ATOMIC_RELAXED) & ERR_BOUNDS) return;  // unsorted input (k_bin_count)
    extern __shared__ uint32_t sm[];
    uint32_t* gcnt = sm;             // [ngroups] next free slot of each bucket (this part)
    uint32_t* fbits = sm + ngroups;  // [ceil(nc/32)] cell's first read is in this bin
    // [2][waves][ngroups]: a step's per-wave group counts, then each wave's first slot
    // (two sets, alternating per step, so a set is rewritten only behind a barrier)
    uint32_t* wc = fbits + (g.nc + 31) / 32;
    const int b = blockIdx.x, part = blockIdx.y;
    const int nc = g.nc;
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (scalar)
    const unsigned long long lt = lanemask_lt();
    // exclusive scan over groups (wave 0, 64 at a time) of the bin's bucket sizes
    // (the parts' sums), based at the bin's first slot; this part's slots follow the
    // earlier parts' in every bucket
    const uint32_t* pg = PG + (size_t)b * kParts * ngroups;
    if (wid == 0) {
        uint32_t carry = binbase[b];
        for (int g0 = 0; g0 < ngroups; g0 += kWave) {
            const int gi = g0 + lane;
            uint32_t v = 0, before = 0;
            if (gi < ngroups) {
#pragma unroll
                for (int p = 0; p < kParts; ++p) {
                    const uint32_t x = pg[(size_t)p * ngroups + gi];
                    v += x;
                    before += p < part ? x : 0u;
                }
            }
            uint32_t x = v;
            for (int o = 1; o < kWave; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, kWave);
                if (lane >= o) x += y;
            }
            if (gi < ngroups) {
                gcnt[gi] = carry + x - v + before;
                if (part == 0) bucket_off[(size_t)b * (ngroups + 1) + gi] = carry + x - v;
            }
            carry += __shfl(x, kWave - 1, kWave);
        }
        if (lane == 0 && part == 0) bucket_off[(size_t)b * (ngroups + 1) + ngroups] = carry;
    }
    // a bin outside the segment: empty buckets (written above), no reads
    if (b >= seg_bhi || b < seg_lo_bin(seg_w0, g, st)) return;
    // cells whose first read is in this bin (k_scan_apply)
    const size_t fw = (size_t)(nc + 31) / 32;
    uint32_t fany = 0u;
    for (int x = threadIdx.x; x < (int)fw; x += blockDim.x) {
        const uint32_t f = F[(size_t)b * fw + x];
        fbits[x] = f;
        fany |= f;
    }
    int64_t lo, hi;
    part_range(bin_lo[b], max((int64_t)bin_lo[b + 1], (int64_t)bin_lo[b]), part, lo, hi);
    // no cell has its first read in this bin (most bins): no per-read first-read test
    const bool any_first = __syncthreads_or(fany != 0u) != 0;
    // each wave owns a contiguous run of kAhead*64 reads per step (BAM order = wave
    // order, then round order); waves claim bucket slots in wave order
    constexpr int kAhead = MGP_GA_AHEAD;
    constexpr int kStep = kAhead * kBlk;
    // per read: barcode, start, tlen, flag | mapq << 16 and the record offset
    // (its 64-byte unit or read index for the dense / u32 sources: 32 bits)
    using OffT = typename std::conditional<kOff == kOffR64 || kSpec, uint64_t, uint32_t>::type;
    struct Pre {
        int c[kAhead], s[kAhead], t[kAhead];
        uint32_t fm[kAhead];
        OffT o[kAhead];
    };
    // loads issued unconditionally (index clamped into the bin) so every path has
    // the same number in flight and the waits stay counted. A wave's reads of a step
    // are i0 + k (k = u * 64 + lane): the column pointers at the clamped run start
    // are wave-uniform and k a 32-bit lane offset (scalar base + vector offset loads).
    // the record offset: from the index (dense), the u32 column or the u64 column (kOff)
    auto wave_i0 = [&](int64_t base0) { return base0 + wid * (kAhead * kWave); };
    auto load = [&](Pre& P, int64_t base0) {
        const int64_t ib = min(wave_i0(base0), hi - 1);           // (uniform; hi > lo here)
        const uint32_t lim = (uint32_t)(hi - 1 - ib);
        const int32_t* bcw = bc + ib;
        const uint16_t* flw = flag + ib;
        const uint8_t* mqw = mapq + ib;
        const int32_t* stw = start + ib;
        const int32_t* tlw = tlen + ib;
#pragma unroll
        for (int u = 0; u < kAhead; ++u) {
            const uint32_t k = min((uint32_t)(u * kWave + lane), lim);
            P.c[u] = bcw[k];
            P.fm[u] = (uint32_t)flw[k] | (uint32_t)mqw[k] << 16;
            P.s[u] = stw[k];
            P.t[u] = tlw[k];
            if constexpr (kOff == kOffDense) P.o[u] = (OffT)(ib + k);
            else if constexpr (kOff == kOffR32) P.o[u] = roff32[ib + k];
            else P.o[u] = roff[ib + k];
        }
    };
    // A step: each wave ranks its own reads by group (ballot peers, the leader of a
    // group bumps the wave's LDS counter), then per group the waves' counts become
    // consecutive slot ranges after the bucket's cursor, in wave order = BAM order.
    // Two barriers per step, no wave waits for another's ranking.
    int set = 0;
    // the speculative check (kSpec): coordinate order over every read; span, key
    // widths and 64-byte offsets over the valid reads (the ones pass A stores)
    bool ck_uns = false, ck_bad = false;
    uint32_t ck_span = 0;
    auto process = [&](const Pre& P, int64_t base0) {
        // the check's extra loads go out first and land behind the ranking: the span,
        // and the start before the wave's run (a read's predecessor is the lane below,
        // or lane 63 of the previous slot)
        uint32_t spn[kSpec ? kAhead : 1];
        int prev0 = 0;
        if constexpr (kSpec) {
            const int64_t ib = min(wave_i0(base0), hi - 1);
            const uint32_t lim = (uint32_t)(hi - 1 - ib);
            const uint32_t* spw = span + ib;
#pragma unroll
            for (int u = 0; u < kAhead; ++u)
                spn[u] = MGP_ABL_A == 3 ? 53u : spw[min((uint32_t)(u * kWave + lane), lim)];
            const int64_t w0 = wave_i0(base0);
            prev0 = start[w0 > 0 ? (w0 <= hi ? w0 - 1 : hi - 1) : 0];
        }
        uint32_t* my = wc + ((size_t)set * (kBlk / kWave) + wid) * ngroups;
        for (int x = lane; x < ngroups; x += kWave) my[x] = 0;
        __builtin_amdgcn_wave_barrier();
        bool valid[kAhead];
        uint32_t rk[kAhead];
        const int64_t i0 = wave_i0(base0);
        const int64_t nleft = hi - i0;  // reads of the bin from i0 on (uniform)
#pragma unroll
        for (int u = 0; u < kAhead; ++u) {
            const uint32_t k = (uint32_t)(u * kWave + lane);
            const int c = P.c[u];
            valid[u] = (int64_t)k < nleft && read_valid(c, (uint16_t)P.fm[u], nc);
            const uint32_t gi = (uint32_t)c >> 6;
            // peers: same cell group (first 8 group-id bits unrolled; interleaving the
            // reads' chains measured no faster)
            const unsigned long long pm = peer_mask<8>(valid[u], gi, gbits);
            if (any_first && valid[u] && (fbits[c >> 5] >> (c & 31)) & 1u)
                atomicMin(&first_read[c], (uint32_t)(i0 + k));
            // every peer reads the group's counter in one LDS read, before its leader
            // (lowest peer) stores the bumped value: no cross-lane broadcast needed
            const uint32_t bef = valid[u] ? my[gi] : 0u;
            __builtin_amdgcn_wave_barrier();
            if (valid[u] && (pm & lt) == 0ull) my[gi] = bef + (uint32_t)__popcll(pm);
            rk[u] = bef + (uint32_t)__popcll(pm & lt);
            __builtin_amdgcn_wave_barrier();
        }
        if (MGP_ABL_A == 2) {  // ablation: no ranking, every element at its read index
#pragma unroll
            for (int u = 0; u < kAhead; ++u) rk[u] = 0;
        }
        bool fit[kAhead];
#pragma unroll
        for (int u = 0; u < kAhead; ++u) {
            fit[u] = true;
            if constexpr (kSpec) {
                const int64_t i = i0 + u * kWave + lane;
                const int t = P.t[u];
                const uint32_t at = t < 0 ? (uint32_t)(-(int64_t)t) : (uint32_t)t;
                // the previous read's start: DPP wave_shr:1 (lane - 1), lane 0 from the slot before
                const int below = __builtin_amdgcn_update_dpp(0, P.s[u], 0x138, 0xf, 0xf, false);
                const int first = u ? __builtin_amdgcn_readlane(P.s[u > 0 ? u - 1 : 0], kWave - 1) : prev0;
                const int pv = lane ? below : first;
                ck_uns |= i < hi && i > 0 && P.s[u] < pv;
                // the record's offset in units of its layout's size (64 or 32 bytes)
                fit[u] = (P.o[u] & ((1ull << spec_unit) - 1ull)) == 0ull && P.s[u] >= 0 && P.s[u] < g.L &&
                         at < kCompactTlen;
                if (valid[u]) {
                    ck_span = max(ck_span, spn[u]);
                    ck_bad |= !fit[u];
                }
            }
        }
        __syncthreads();
        for (int gi = threadIdx.x; gi < ngroups; gi += kBlk) {
            uint32_t run = gcnt[gi];
#pragma unroll
            for (int w = 0; w < kBlk / kWave; ++w) {
                uint32_t* r = wc + ((size_t)set * (kBlk / kWave) + w) * ngroups;
                const uint32_t x = r[gi];
                r[gi] = run;
                run += x;
            }
            gcnt[gi] = run;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kAhead; ++u) {
            if (!valid[u]) continue;
            const uint32_t dest = MGP_ABL_A == 2 ? (uint32_t)(i0 + u * kWave + lane) : my[P.c[u] >> 6] + rk[u];
            if (MGP_ABL_A == 1 && dest != 0xFFFFFFFFu) continue;  // ablation: no stores
            const uint16_t f = (uint16_t)P.fm[u];
            const int t = P.t[u];
            const unsigned long long off = kOff == kOffDense ? (unsigned long long)P.o[u] * kRecStride
                                           : kOff == kOffR32 ? (unsigned long long)P.o[u] << 6
                                                             : (unsigned long long)P.o[u];
            const uint32_t at = t < 0 ? (uint32_t)(-(int64_t)t) : (uint32_t)t;
            const bool mq = (int)(P.fm[u] >> 16) >= min_mapq;
            if ((int64_t)dest >= n) {  // never: counts and slots come from one histogram
                atomicOr(&st->err, ERR_OVERFLOW);
            } else if constexpr (kCompact) {
                // the record's 64-byte unit (dense: the read index; u32 column: rec_off >> 6);
                // a read that does not fit (kSpec) piles nothing: the run is redone
                const uint32_t unit64 = kSpec ? (uint32_t)(P.o[u] >> spec_unit) : (uint32_t)P.o[u];
                const uint32_t lo = fit[u] ? unit64 | (mq ? PE_PACKED : 0u) : 0u;
                const uint32_t hi = at | ((uint32_t)(P.s[u] & 255) << GC_START_SHIFT) |
                                    (f & MGP_FLAG_REVERSE ? GC_REV : 0u) |
                                    ((uint32_t)(P.c[u] & (kGroup - 1)) << GC_LCELL_SHIFT);
                const unsigned long long e = (unsigned long long)hi << 32 | lo;
                reinterpret_cast<unsigned long long*>(gel2)[dest] = e;
            } else {
                GElem e;
                e.w = off | (f & MGP_FLAG_REVERSE ? GM_REV : 0ull) | (f & MGP_FLAG_PAIRED ? GM_PAIRED : 0ull) |
                      (mq ? GM_MAPQ_OK : 0ull) | (f & MGP_FLAG_NOSEQQUAL ? GM_BAD : 0ull) |
                      (f & (MGP_FLAG_PACKED | MGP_FLAG_PACK32) ? GM_PACKED : 0ull) |
                      (f & MGP_FLAG_PACK32 ? GM_P32 : 0ull) |
                      ((unsigned long long)(P.c[u] & (kGroup - 1)) << GM_LCELL_SHIFT);
                e.start = P.s[u];
                e.tlen = at;
                gel2[dest] = e;
            }
        }
        set ^= 1;
    };
    if (lo >= hi) return;
#if MGP_GA_DB
    Pre A, B;
    load(A, lo);
    for (int64_t base0 = lo; base0 < hi; base0 += 2 * kStep) {
        load(B, base0 + kStep);
        process(A, base0);
        load(A, base0 + 2 * kStep);
        if (base0 + kStep < hi) process(B, base0 + kStep);
    }
#else
    for (int64_t base0 = lo; base0 < hi; base0 += kStep) {
        Pre A;
        load(A, base0);
        process(A, base0);
    }
#endif
    if constexpr (kSpec) {
        const bool uns = __ballot(ck_uns) != 0ull, bad = __ballot(ck_bad) != 0ull;
        const uint32_t sp = wave_max(ck_span);
        if (lane == 0) {
            if (uns) atomicOr(ck, CHK_UNSORTED);
            if (bad) atomicOr(&st->err, ERR_RESPEC);
            if (sp > __atomic_load_n(ck + 1, __ATOMIC_RELAXED)) atomicMax(ck + 1, sp);
        }
    }
}

// The input check's words into the run's stats (grouping pass B's first workgroup,
// behind pass A): the pileup's halo span and the order check. spec_layout: 0, or the
// one CHK_P64 / CHK_P32 layout a streaming segment assumed without the host's look at
// the flag bits; reads it cannot serve make the run rerun resident. max_span is a
// running maximum (a streaming run's segments accumulate it).
__device__ __forceinline__ void check_stats(const uint32_t* __restrict__ ck, DevStats* st, uint32_t spec_layout) {
    if (threadIdx.x == 0) {
        const uint32_t b = ck[0];
        st->max_span = max(st->max_span, ck[1]);
        if (b & CHK_UNSORTED) atomicOr(&st->err, ERR_UNSORTED);
        if (spec_layout && ((b & (CHK_FULL | CHK_P64 | CHK_P32 | CHK_NOSEQ) & ~spec_layout) ||
                            ((b & CHK_PAIRED) && (b & CHK_UNPAIRED))))
            atomicOr(&st->err, ERR_RESPEC);
    }
}

// Pass B: workgroup = (cell group, bin range). A step takes the group's buckets
// of as many consecutive bins as fit the LDS stage; each wave ranks the elements
// of its bins (one bin at a time, stable: ballot peers + per-cell counters) and
// drops them at their place inside the step's per-cell runs in LDS; a cell's
// slots over consecutive bins are contiguous in the output, so the stage is then
// written out as a few long runs (full lines) instead of 64 scattered 16-byte
// stores per instruction. A bucket larger than the stage goes straight out.
//
// Duplicate marking happens here (readers.py:118-150): every read that can be a
// duplicate of a read shares its start, hence its start bin, hence its bucket,
// and inside a cell's staged run equal starts are adjacent and in BAM order (the
// input is coordinate-sorted and both passes are stable). So a read is a
// duplicate iff a read before it in the run, among the equal starts, has the
// same strand (and the same |tlen|): first in BAM order wins. Both duplicate
// counters (readers.py:141-144) are taken here, each read being seen exactly
// once. The output is one 4-byte pileup element per read (PE_*): the record's
// offset when the read is piled (kept and MAPQ >= min_mapq, pileup.py:33),
// PE_KEEP or PE_DUP otherwise.
#ifndef MGP_GB_STAGE
#define MGP_GB_STAGE 2048
#endif
constexpr int kStageB = MGP_GB_STAGE;
constexpr int kMaxRbB = 256;  // bins per pass-B workgroup (bucket sizes kept in LDS; 4 workgroups per CU)
#ifndef MGP_GB_WG
#define MGP_GB_WG 8192  // target pass-B grid size
#endif
// Pileup element (4 bytes, cell-major): a read to pile (kept by the duplicate
// marking, MAPQ >= min_mapq, pileup.py:33) is its record offset in units of
// 2^unit bytes (unit 6, or 4 for 16-byte aligned placements) | PE_PACKED; a kept
// read below min_mapq is PE_KEEP, a duplicate PE_DUP (the pileup counts the
// kept reads, processors.py:22). Offsets stay below PE_KEEP's (mgp_run checks).
constexpr unsigned long long GM_OFF = (1ull << GM_LCELL_SHIFT) - 1;

struct DedupAcc {  // per-thread duplicate counters of pass B
    unsigned long long d2 = 0, d3 = 0;
};


#ifndef MGP_GB_WAVES
#define MGP_GB_WAVES 3  // wide elements: the LDS stage (32 KB) and the deferred-walk lists allow 3
#endif
#ifndef MGP_GB_WAVES_C
#define MGP_GB_WAVES_C 5
#endif
// Element access for the two grouping element forms (pass B).
struct GWide {
    using T = GElem;
    static constexpr int kWaves = MGP_GB_WAVES;  // pass-B waves per SIMD
    static __device__ __forceinline__ T zero() {
        T e;
        e.w = 0;
        e.start = 0;
        e.tlen = 0;
        return e;
    }
    static __device__ __forceinline__ int lcell(const T& e) { return (int)((e.w >> GM_LCELL_SHIFT) & (kGroup - 1)); }
    // same cell and start (the run of equal starts), then same strand, then same |tlen|
    static __device__ __forceinline__ bool run_eq(const T& a, const T& b) {
        return ((a.w ^ b.w) & GM_LCELL) == 0ull && a.start == b.start;
    }
    static __device__ __forceinline__ bool start_eq(const T& a, const T& b) { return a.start == b.start; }
    static __device__ __forceinline__ bool strand_eq(const T& a, const T& b) { return ((a.w ^ b.w) & GM_REV) == 0ull; }
    static __device__ __forceinline__ bool tlen_eq(const T& a, const T& b) { return a.tlen == b.tlen; }
    static __device__ __forceinline__ bool mapq_ok(const T& e) { return (e.w & GM_MAPQ_OK) != 0ull; }
    static __device__ __forceinline__ uint32_t pile(const T& e, int unit) {
        return (uint32_t)((e.w & GM_OFF) >> unit) | (e.w & GM_PACKED ? PE_PACKED : 0u) | (e.w & GM_P32 ? PE_P32 : 0u);
    }
    // a predecessor's duplicate key, read from the LDS stage, against element x:
    // same run (cell and start), then also strand, then also |tlen|
    using P = GElem;
    static __device__ __forceinline__ P pred(const T* stage, uint32_t i) { return stage[i]; }
    static __device__ __forceinline__ void match(const P& p, const T& x, bool& run, bool& strand, bool& tl) {
        run = run_eq(p, x);
        strand = strand_eq(p, x);
        tl = tlen_eq(p, x);
    }
    static __device__ __forceinline__ bool paired(const T& e) { return (e.w & GM_PAIRED) != 0ull; }
    static __device__ __forceinline__ bool bad(const T& e) { return (e.w & GM_BAD) != 0ull; }
};
struct GCompact {
    using T = unsigned long long;
    static constexpr int kWaves = MGP_GB_WAVES_C;  // fewer registers: 5 waves per SIMD (A/B: 4 slower)
    static __device__ __forceinline__ uint32_t key(const T& e) { return (uint32_t)(e >> 32); }
    static __device__ __forceinline__ T zero() { return 0ull; }
    static __device__ __forceinline__ int lcell(const T& e) { return (int)((key(e) >> GC_LCELL_SHIFT) & (kGroup - 1)); }
    static __device__ __forceinline__ bool run_eq(const T& a, const T& b) {
        return ((key(a) ^ key(b)) & (GC_LCELL | GC_START)) == 0u;
    }
    static __device__ __forceinline__ bool start_eq(const T& a, const T& b) { return ((key(a) ^ key(b)) & GC_START) == 0u; }
    static __device__ __forceinline__ bool strand_eq(const T& a, const T& b) { return ((key(a) ^ key(b)) & GC_REV) == 0u; }
    static __device__ __forceinline__ bool tlen_eq(const T& a, const T& b) { return ((key(a) ^ key(b)) & GC_TLEN) == 0u; }
    static __device__ __forceinline__ bool mapq_ok(const T& e) { return ((uint32_t)e & PE_PACKED) != 0u; }
    static __device__ __forceinline__ uint32_t pile(const T& e, int) { return (uint32_t)e; }
    using P = uint32_t;  // the high word only (a 4-byte LDS read)
    static __device__ __forceinline__ P pred(const T* stage, uint32_t i) {
        return reinterpret_cast<const uint32_t*>(stage)[2 * i + 1];
    }
    static __device__ __forceinline__ void match(P p, const T& x, bool& run, bool& strand, bool& tl) {
        const uint32_t d = p ^ key(x);
        run = (d & (GC_LCELL | GC_START)) == 0u;
        strand = (d & GC_REV) == 0u;
        tl = (d & GC_TLEN) == 0u;
    }
    static __device__ __forceinline__ bool paired(const T&) { return true; }
    static __device__ __forceinline__ bool bad(const T&) { return false; }
};

// The pileup element of one read given its duplicate flags; keep = the read
// survives the duplicate marking (counted in n_reads, processors.py:22).
template <class Tr>
__device__ __forceinline__ uint32_t group_b_emit(const typename Tr::T& e, bool dup2, bool dup3, int mode, int unit,
                                                 DedupAcc& acc, bool& keep, bool cnt = true) {
    keep = mode == MGP_DEDUP_NONE ? true : mode == MGP_DEDUP_START ? !dup2 : !dup3;
    acc.d2 += cnt & dup2;
    acc.d3 += cnt & dup3;
    if (!keep) return PE_DUP;
    if (!Tr::mapq_ok(e)) return PE_KEEP;
    return Tr::pile(e, unit);
}

// Per-cell flags of pass B when the resident reads mix paired and unpaired ones,
// or some read lacks SEQ/QUAL (kTrack; the input check's CHK_* bits): the cell
// has a kept paired read (processors.py:34) iff it has more kept reads (its
// elements in the workgroup's bin range, the cbase advance, minus its
// duplicates) than kept unpaired ones, both counted here into the workgroup's
// per-cell LDS counters; a kept read without SEQ/QUAL sets ERR_BADREAD.
// Otherwise every kept read is paired (or none is), which the pileup applies
// with its kept-read counts, and no read lacks SEQ/QUAL.
template <bool kTrack, class Tr>
__device__ __forceinline__ void cell_tally(bool act, int lc, bool keep, const typename Tr::T& e, uint32_t* s_ndup,
                                           uint32_t* s_nunp, DevStats* st) {
    if (kTrack) {
        if (act && !keep) atomicAdd(&s_ndup[lc], 1u);
        if (act && keep && !Tr::paired(e)) atomicAdd(&s_nunp[lc], 1u);
        if (act && keep && Tr::bad(e)) atomicOr(&st->err, ERR_BADREAD);
    }
}

template <class Tr>
__device__ __forceinline__ bool same_key(const typename Tr::T& p, const typename Tr::T& e, bool& dup3) {
    if (!Tr::strand_eq(p, e)) return false;
    if (Tr::tlen_eq(p, e)) dup3 = true;
    return true;
}

// kStage: rank into the LDS stage. Otherwise (a bucket larger than the stage):
// rank, mark duplicates by walking back over the bucket's equal starts (BAM
// order, other cells skipped) and store the pileup elements directly.
template <bool kStage, class Tr>
__device__ __forceinline__ void group_b_rank(const typename Tr::T* __restrict__ gel2, uint32_t k0, uint32_t k1,
                                             uint32_t* cnt, int lane, unsigned long long lt, typename Tr::T* stage,
                                             const uint32_t* cbase, const uint32_t* cstart, int mode, int unit,
                                             uint32_t* __restrict__ pel, DedupAcc& acc, uint32_t* s_ndup,
                                             uint32_t* s_nunp, DevStats* st, bool count_dups) {
    using T = typename Tr::T;
    for (uint32_t k = k0; k < k1; k += kWave) {
        const uint32_t j = k + lane;
        const bool act = j < k1;
        T e = Tr::zero();
        if (act) e = gel2[j];
        const int lc = Tr::lcell(e);
        const unsigned long long peers = peer_mask<6>(act, (uint32_t)lc);
        const uint32_t base = act ? cnt[lc] : 0u;
        __builtin_amdgcn_wave_barrier();
        if (act && (peers & lt) == 0ull) cnt[lc] = base + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        if (act) {
            const uint32_t dest = base + (uint32_t)__popcll(peers & lt);
            if (kStage) {
                stage[cstart[lc] + (dest - cbase[lc])] = e;
            } else {
                bool dup2 = false, dup3 = false;
                if (mode != MGP_DEDUP_NONE) {
                    // one bucket = one start bin (starts within 8 positions, so equal
                    // starts mod 256 are equal starts); equal starts are adjacent
                    for (uint32_t m = j; m-- > k0;) {
                        const T p = gel2[m];
                        if (!Tr::start_eq(p, e)) break;
                        if (Tr::lcell(p) == lc && same_key<Tr>(p, e, dup3)) {
                            dup2 = true;
                            if (dup3) break;
                        }
                    }
                }
                bool keep;
                pel[dest] = group_b_emit<Tr>(e, dup2, dup3, mode, unit, acc, keep, count_dups);
                cell_tally<true, Tr>(true, lc, keep, e, s_ndup, s_nunp, st);
            }
        }
    }
}

// A step: the group's buckets of consecutive bins [b, be) that fit the stage, taken
// as one flat sequence (bin order, BAM order inside a bucket = start order). Each
// wave loads its quarter of the sequence at once (8 independent 16-byte loads per
// lane) and ranks it by cell (ballot peers, per-wave per-cell counters); the
// waves' counts give every cell its run in the stage and every wave its place in
// the run, so the stage fills in (cell, bin, BAM) order. A cell's run is then
// written to its slots, which continue where the previous step's ended (cbase).
#ifndef MGP_GB_BLOCK
#define MGP_GB_BLOCK 256  // pass-B threads per workgroup
#endif
constexpr int kGBBlock = MGP_GB_BLOCK;
constexpr int kBPer = kStageB / kGBBlock;  // elements per lane per step
#ifndef MGP_GB_NT
#define MGP_GB_NT 1  // pass B's element loads non-temporal: L2 keeps the partial pel lines (r05: write traffic 1.20 -> 1.06 GB, time equal)
#endif
#ifndef MGP_GB_XCD
#define MGP_GB_XCD 0  // pass B's workgroups dealt to the XCDs in contiguous (group, range) runs (A/B)
#endif
#ifndef MGP_ABL_B
#define MGP_ABL_B 0  // pass-B ablations (experiments only): 1 no dedup walk, 2 no pel stores, 3 no loads
#endif
#ifndef MGP_GB_CARRY
// A cell's elements of a step end mid-way through a 64-byte granule of pel; the next
// step (~16 us later, other lines meanwhile through the XCD's L2) writes the rest, so
// the granule reached HBM twice (r04-r05: 1.06-1.20 GB written per C4 launch for 0.65 GB
// of elements). With the carry, a step's incomplete tail granule stays in LDS
// (carry[cell]) until a later step completes it, and every granule is written once
// except at the workgroup's first and last (its bin range's ends). Off: it takes the
// writes from 1.06 to 0.86-0.89 GB but pass B from 1.02 to 1.13 ms, and pass B without
// any pel store (MGP_ABL_B=2) takes 1.045 ms, so its stores, amplified or not, cost it
// no time (profiles/r05/ab_carry_r5x.txt).
#define MGP_GB_CARRY 0
#endif

#ifndef MGP_GB_LOOK
#define MGP_GB_LOOK 3  // predecessors compared branch-free before a deferred walk (v42 A/B: 2, 4, 6 slower)
#endif
template <bool kTrack, class Tr>
__global__ void __launch_bounds__(kGBBlock, Tr::kWaves) k_group_b(const typename Tr::T* __restrict__ gel2,
                                                    const uint32_t* __restrict__ bucket_off,
                                                    const uint32_t* __restrict__ O, Geom g, int ngroups, int rb,
                                                    int mode, int unit, uint32_t* __restrict__ pel,
                                                    uint8_t* __restrict__ any_paired,
                                                    unsigned long long* __restrict__ dup_part, DevStats* st,
                                                    int cnt_lo, const uint32_t* __restrict__ ck,
                                                    uint32_t spec_layout) {
    using T = typename Tr::T;
    constexpr bool kCompact = sizeof(T) == 8;
    // the workgroup's (cell group, bin range): blockIdx as launched, or with MGP_GB_XCD a
    // 1-D grid whose dispatch index i (XCD i mod 8) is dealt so that each XCD takes a
    // contiguous run of (group, range) pairs, ranges fastest: the neighbouring ranges
    // of a group, whose cell runs share their boundary lines in pel, then write them
    // through one L2 at about the same time
#if MGP_GB_XCD
    const int nrg = (g.nbins + rb - 1) / rb;
    const unsigned per = gridDim.x / 8u, li = (blockIdx.x & 7u) * per + (blockIdx.x >> 3);
    if (li >= (unsigned)(ngroups * nrg)) return;
    const int gx = (int)(li / (unsigned)nrg), gy = (int)(li % (unsigned)nrg);
    const size_t wg_lin = (size_t)gy * ngroups + gx;
#else
    const int gx = blockIdx.x, gy = blockIdx.y;
    const size_t wg_lin = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
#endif
    if (gx == 0 && gy == 0) check_stats(ck, st, spec_layout);
    if (__atomic_load_n(&st->err, __ATOMIC_RELAXED) & ERR_BOUNDS) return;  // unsorted input (k_bin_count)
    __shared__ T stage[kStageB];
    __shared__ uint32_t wcnt[kGBBlock / kWave][kGroup];
    __shared__ uint32_t cbase[kGroup], cstart[kGroup + 1];
    __shared__ uint32_t bst[kMaxRbB], bsz[kMaxRbB], spre[kMaxRbB + 1];
    __shared__ int s_be;
    __shared__ uint32_t s_ndup[kGroup], s_nunp[kGroup];  // the group's duplicates / kept unpaired reads in this bin range
    __shared__ uint16_t wpend[kGBBlock / kWave][kBPer * kWave];  // per wave: stage indices of deferred walks
    // MGP_GB_CARRY: per cell, the elements [carry_lo, cbase & 15) of the granule holding
    // cbase (written by earlier steps, not yet to pel)
    __shared__ uint32_t carry[MGP_GB_CARRY ? kGroup : 1][16];
    __shared__ uint32_t carry_lo[kGroup];
    const int gi = gx;
    const int B0 = gy * rb, B1 = min(g.nbins, B0 + rb);
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (scalar)
    const int nc = g.nc;
    const int c = gi * kGroup + lane;
    const unsigned long long lt = lanemask_lt();
    const size_t bo = (size_t)ngroups + 1;
    const bool dedup = mode != MGP_DEDUP_NONE;
    DedupAcc acc;
    for (int x = threadIdx.x; x < B1 - B0; x += kGBBlock) {
        const uint32_t o0 = bucket_off[(size_t)(B0 + x) * bo + gi];
        bst[x] = o0;
        bsz[x] = bucket_off[(size_t)(B0 + x) * bo + gi + 1] - o0;
    }
    if (wid == 0) {
        cbase[lane] = c < nc ? O[(size_t)B0 * nc + c] : 0u;  // each cell's next slot
        carry_lo[lane] = cbase[lane] & 15u;                  // (nothing carried)
        s_ndup[lane] = 0u;
        s_nunp[lane] = 0u;
    }
    __syncthreads();
    // a pileup element to pel, or to its cell's carry when it falls in the step's
    // incomplete tail granule (stage index t of cell lc's run)
    auto put = [&](int lc, uint32_t t, uint32_t pv) {
        const uint32_t p = cbase[lc] + (t - cstart[lc]);
        const uint32_t e = cbase[lc] + (cstart[lc + 1] - cstart[lc]);
        if (MGP_GB_CARRY && (p >> 4) == (e >> 4) && (e & 15u)) carry[lc][p & 15u] = pv;
        else pel[p] = pv;
    };
    // every cell's carried elements to pel (full = false: only the cells whose carried
    // granule this step completes; before the step's tail elements reuse the slots)
    auto flush = [&](bool full) {
        for (int x = threadIdx.x; x < kGroup * 16; x += kGBBlock) {
            const int lc = x >> 4;
            const uint32_t k = (uint32_t)x & 15u, cb = cbase[lc];
            const bool done = full || ((cb + (cstart[lc + 1] - cstart[lc])) >> 4) != (cb >> 4);
            if (done && k >= carry_lo[lc] && k < (cb & 15u)) pel[(cb & ~15u) + k] = carry[lc][k];
        }
    };
    // bins [b, s_be) of the step starting at b: as many as fit the stage (one if its
    // bucket alone is larger: direct path); spre = prefix of their bucket sizes
    auto plan = [&](int b) {
        if (threadIdx.x == 0) {
            uint32_t tot = 0;
            int be = b;
            spre[0] = 0;
            while (be < B1) {
                // a streaming segment's halo bins (below cnt_lo, counted by an earlier
                // segment) never share a step with its own bins
                if (be == cnt_lo && be > b) break;
                const uint32_t sz = bsz[be - B0];
                if (tot + sz > (uint32_t)kStageB) break;
                if (kCompact && be - b >= kCompactBins) break;  // starts compared mod 256
                tot += sz;
                ++be;
                spre[be - b] = tot;
            }
            s_be = be;
        }
        __syncthreads();
        return s_be;
    };
    // this wave's quarter of the step's flat sequence (all loads issued together)
    T e[kBPer];
    auto load = [&](int b, int be) {
        const int nb = be - b;
        const uint32_t tot = spre[nb];
#pragma unroll
        for (int u = 0; u < kBPer; ++u) {
            const uint32_t t = (uint32_t)(wid * (kBPer * kWave) + u * kWave + lane);
            e[u] = Tr::zero();
            if (t < tot) {
                int lo = 0, hi = nb;  // bin k of t: spre[k] <= t < spre[k + 1]
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (spre[mid] <= t) lo = mid;
                    else hi = mid;
                }
                if constexpr (MGP_ABL_B == 3 && !kCompact) {
                    e[u].w = (unsigned long long)((t * 37u) & 63u) << GM_LCELL_SHIFT;
                    e[u].start = (int)(bst[b - B0 + lo] + t);
                } else if constexpr (MGP_GB_NT && kCompact) {  // (A/B: the stream's lines evict-first in L2)
                    e[u] = __builtin_nontemporal_load(&gel2[bst[b - B0 + lo] + (t - spre[lo])]);
                } else {
                    e[u] = gel2[bst[b - B0 + lo] + (t - spre[lo])];
                }
            }
        }
        return tot;
    };
    int b = B0;
    int be = b < B1 ? plan(b) : b;
    uint32_t tot = be > b ? load(b, be) : 0u;
    while (b < B1) {
        if (be == b) {  // one bucket larger than the stage: direct stores (wave 0)
            if (MGP_GB_CARRY) {
                flush(true);
                __syncthreads();
            }
            if (wid == 0) {
                wcnt[0][lane] = cbase[lane];
                __builtin_amdgcn_wave_barrier();
                group_b_rank<false, Tr>(gel2, bst[b - B0], bst[b - B0] + bsz[b - B0], wcnt[0], lane, lt, nullptr,
                                    nullptr, nullptr, mode, unit, pel, acc, s_ndup, s_nunp, st, b >= cnt_lo);
                __builtin_amdgcn_wave_barrier();
                cbase[lane] = wcnt[0][lane];
                carry_lo[lane] = cbase[lane] & 15u;
            }
            __syncthreads();
            ++b;
            be = b < B1 ? plan(b) : b;
            tot = be > b ? load(b, be) : 0u;
            continue;
        }
        // rank by cell inside the wave's quarter (stable)
        wcnt[wid][lane] = 0;
        __builtin_amdgcn_wave_barrier();
        uint32_t rk[kBPer];
#pragma unroll
        for (int u = 0; u < kBPer; ++u) {
            const uint32_t t = (uint32_t)(wid * (kBPer * kWave) + u * kWave + lane);
            const bool act = t < tot;
            const int lc = Tr::lcell(e[u]);
            // (one element's peers at a time: interleaving the elements' chains spills at
            // this kernel's 5 waves per SIMD)
            const unsigned long long peers = peer_mask<6>(act, (uint32_t)lc);
            const uint32_t base = act ? wcnt[wid][lc] : 0u;
            __builtin_amdgcn_wave_barrier();
            if (act && (peers & lt) == 0ull) wcnt[wid][lc] = base + (uint32_t)__popcll(peers);
            __builtin_amdgcn_wave_barrier();
            rk[u] = base + (uint32_t)__popcll(peers & lt);
        }
        __syncthreads();
        if (wid == 0) {  // per cell: the waves' places in its run, and the run in the stage
            uint32_t run = 0;
#pragma unroll
            for (int w = 0; w < kGBBlock / kWave; ++w) {
                const uint32_t x = wcnt[w][lane];
                wcnt[w][lane] = run;
                run += x;
            }
            uint32_t x = run;
            for (int o = 1; o < kWave; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, kWave);
                if (lane >= o) x += y;
            }
            cstart[lane] = x - run;
            if (lane == kWave - 1) cstart[kGroup] = x;
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < kBPer; ++u) {
            const uint32_t t = (uint32_t)(wid * (kBPer * kWave) + u * kWave + lane);
            if (t < tot) {
                const int lc = Tr::lcell(e[u]);
                stage[cstart[lc] + wcnt[wid][lc] + rk[u]] = e[u];
            }
        }
        // the next step's loads go out now and land while this step is written out
        const uint32_t cur = tot;
        const int nb0 = be;
        // granules carried from earlier steps that this step completes, before the barrier
        // below (the step's tail elements then reuse the carry slots)
        if (MGP_GB_CARRY) flush(false);
        const int nbe = nb0 < B1 ? plan(nb0) : nb0;  // (its barrier also completes the stage)
        if (nb0 >= B1) __syncthreads();
        const uint32_t ntot = nbe > nb0 ? load(nb0, nbe) : 0u;
        const bool cnt = b >= cnt_lo;  // the step's duplicates count (not a halo step)
        // write-out with duplicate marking: equal starts of a cell's run sit just
        // before t, in BAM order; a cell has one run in the stage, so an element of
        // another cell ends the walk. The element and its kLook predecessors are
        // loaded for 2 elements at once and compared branch-free; a walk further
        // back is needed only behind kLook + 1 equal starts.
        constexpr int kWo = 2;
        constexpr int kLook = MGP_GB_LOOK;
        uint32_t npend = 0;  // the wave's deferred walks this step (wave-uniform)

#pragma unroll
        for (int h = 0; h < kBPer; h += kWo) {
            T xs[kWo];
            bool d2[kWo], d3[kWo], wk[kWo];
#pragma unroll
            for (int q = 0; q < kWo; ++q) {
                const uint32_t t = threadIdx.x + (uint32_t)(h + q) * kGBBlock;
                const uint32_t tc = t < cur ? t : 0u;
                const T x = stage[tc];
                typename Tr::P pk[kLook];
#pragma unroll
                for (int k = 0; k < kLook; ++k) pk[k] = Tr::pred(stage, tc >= (uint32_t)(k + 1) ? tc - (uint32_t)(k + 1) : 0u);
                bool r = true, s2 = false, t3 = false;  // r: the k nearest predecessors are all in x's run
#pragma unroll
                for (int k = 0; k < kLook; ++k) {
                    bool rk, sk, tk;
                    Tr::match(pk[k], x, rk, sk, tk);
                    r = r & (tc >= (uint32_t)(k + 1)) & rk;
                    s2 |= r & sk;
                    t3 |= r & sk & tk;
                }
                xs[q] = x;
                d2[q] = dedup & s2;
                d3[q] = dedup & t3;
                wk[q] = dedup & r & !t3 & (tc >= (uint32_t)(kLook + 1)) & (t < cur);
            }
#pragma unroll
            for (int q = 0; q < kWo; ++q) {
                const uint32_t t = threadIdx.x + (uint32_t)(h + q) * kGBBlock;
                // an element behind kLook + 1 equal starts without a full-key match waits
                // for the wave's deferred walks (one divergent loop per step, not per element)
                const bool defer = MGP_ABL_B != 1 && wk[q];
                const unsigned long long dm = __ballot(defer);
                if (defer) wpend[wid][npend + (uint32_t)__popcll(dm & lt)] = (uint16_t)t;
                npend += (uint32_t)__popcll(dm);
                const bool act = t < cur && !defer;
                const int lc = Tr::lcell(xs[q]);
                bool keep = false;
                if (act) {
                    const uint32_t pv = group_b_emit<Tr>(xs[q], d2[q], d3[q], mode, unit, acc, keep, cnt);
                    if (MGP_ABL_B < 2 || pv == 7u) put(lc, t, pv);
                }
                cell_tally<kTrack, Tr>(act, lc, keep, xs[q], s_ndup, s_nunp, st);
            }
        }
        // the deferred walks, one element per lane: every predecessor back to the
        // run's start (kLook key words loaded together) or a full-key match
        __builtin_amdgcn_wave_barrier();
        for (uint32_t p0 = 0; p0 < npend; p0 += kWave) {
            const bool act = p0 + (uint32_t)lane < npend;
            const uint32_t t = act ? (uint32_t)wpend[wid][p0 + lane] : 0u;
            const T x = stage[t];
            bool dup2 = false, dup3 = false;
            for (uint32_t m = act ? t : 0u; !dup3 && m > 0; m -= m < (uint32_t)kLook ? m : kLook) {
                typename Tr::P pk[kLook];
#pragma unroll
                for (int k = 0; k < kLook; ++k) pk[k] = Tr::pred(stage, m >= (uint32_t)(k + 1) ? m - (uint32_t)(k + 1) : 0u);
                bool r = true;
#pragma unroll
                for (int k = 0; k < kLook; ++k) {
                    bool rk, sk, tk;
                    Tr::match(pk[k], x, rk, sk, tk);
                    r = r & (m >= (uint32_t)(k + 1)) & rk;
                    dup2 |= r & sk;
                    dup3 |= r & sk & tk;
                }
                if (!r) break;
            }
            const int lc = Tr::lcell(x);
            bool keep = false;
            if (act) {
                const uint32_t pv = group_b_emit<Tr>(x, dup2, dup3, mode, unit, acc, keep, cnt);
                if (MGP_ABL_B < 2 || pv == 7u) put(lc, t, pv);
            }
            cell_tally<kTrack, Tr>(act, lc, keep, x, s_ndup, s_nunp, st);
        }
        __syncthreads();
        if (wid == 0) {
            const uint32_t cb = cbase[lane], e = cb + (cstart[lane + 1] - cstart[lane]);
            if ((e >> 4) != (cb >> 4)) carry_lo[lane] = 0u;  // the carry now holds e's granule from its start
            cbase[lane] = e;
        }
        __syncthreads();
        b = nb0;
        be = nbe;
        tot = ntot;
    }
    if (MGP_GB_CARRY) flush(true);  // the last granules (the bin range's end)
    // the group's per-cell paired flags over this bin range (kTrack)
    if (kTrack && wid == 0 && c < nc) {
        const uint32_t kept = cbase[lane] - O[(size_t)B0 * nc + c] - s_ndup[lane];
        if (kept > s_nunp[lane]) any_paired[c] = 1;  // benign race: every writer stores 1
    }
    // per-workgroup duplicate counts (k_run_stats sums them)
    const unsigned long long d2 = wave_sum(acc.d2), d3 = wave_sum(acc.d3);
    __shared__ unsigned long long s_dup[2][kGBBlock / kWave];
    if (lane == 0) {
        s_dup[0][wid] = d2;
        s_dup[1][wid] = d3;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        unsigned long long t = 0;
        for (int w = 0; w < kGBBlock / kWave; ++w) t += s_dup[threadIdx.x][w];
        dup_part[2 * wg_lin + threadIdx.x] = t;
    }
}

struct PileCfg {
    int min_baseq, min_dist, min_reads, dedup_mode;
    double max_bias;
    bool bias_active;  // max_bias < 1 (max/total <= 1 otherwise)
    bool keep_tn5;     // MGP_CFG_KEEP_TN5
};

__device__ __forceinline__ int base_index(uint32_t code) {
    // BAM 4-bit codes: 1=A, 2=C, 4=G, 8=T; everything else is skipped (pileup.py:83-86)
    return code == 1 ? 0 : code == 2 ? 1 : code == 4 ? 2 : code == 8 ? 3 : -1;
}

struct Win {
    int w0, wlen, Wp;
};

#ifndef MGP_ROW_OPAQUE
#define MGP_ROW_OPAQUE 1
#endif
// LDS tile, plane-major: planes 0..3 count A, C, G, T, plane 4 is a trash plane
// (never read: where the 32-byte path adds the bases it does not count), plane 5
// counts Tn5 cuts; every u32 packs the forward count in its low 16 bits and the
// reverse count in its high 16 bits (a window is processed in segments of < 65536
// reads, so no half can carry). A plane is kTilePitch words: kTileGuard guard words,
// the window's positions, guard words (never read either: positions just outside
// the window). The pointer the pile functions get is position 0 of plane 0. A
// count's address is the read's row + plane x plane stride + the query offset (in
// the instruction's immediate). Plane-major puts consecutive positions in
// consecutive banks: the reads of a wave, a few dozen consecutive starts apart, add
// to distinct banks (position-major 16-byte rows spread only position mod 8 over
// the banks: 4-way conflicts on every add, profiles/r03).
constexpr int kTileGuard = 64;
constexpr int kPlaneTrash = 4, kPlaneTn5 = 5, kTilePlanes = 6;
#ifndef MGP_WIN
#define MGP_WIN 1280  // target window width (positions); W <= kMaxPosPerThread * 256 (A/B: 768-2048)
#endif
constexpr int kMaxPosPerThread = MGP_WIN / 256;
// words per plane: guards + the window (>= W) + MGP_TILE_PAD
#ifndef MGP_TILE_PAD
#define MGP_TILE_PAD 0
#endif
constexpr int kTilePitch = MGP_WIN + 2 * kTileGuard + MGP_TILE_PAD;
constexpr uint32_t kPlaneBytes = 4u * kTilePitch;
__device__ __forceinline__ uint32_t strand_inc(int strand) { return strand ? 0x10000u : 1u; }

__device__ __forceinline__ void tn5_cut(bool has, int32_t start, uint32_t lseq, int strand, const Win& w,
                                        uint32_t* t5) {
    // pileup.py:43-50: reverse reads cut at start + len(seq) - 1. Branch-free: a
    // lane whose cut is elsewhere adds 0 to a guard word of its own
    const int64_t cut = strand ? (int64_t)start + lseq - 1 : (int64_t)start;
    const bool in = has && cut >= w.w0 && cut < (int64_t)w.w0 + w.wlen;
    atomicAdd(&t5[in ? (int)(cut - w.w0) : -1 - (int)(threadIdx.x & 63)], in ? strand_inc(strand) : 0u);
}

// Generic path (any read): CIGAR walk with byte loads (pileup.py:55-95).
// Returns whether the read's reach exceeds max_span.
__device__ bool pile_slow(const uint8_t* __restrict__ rec, int32_t start, uint32_t lseq, uint32_t ncig,
                          uint32_t coff, int strand, const Win& w, const PileCfg& pc, uint32_t* tile,
                          uint32_t max_span) {
    const uint32_t* cig = reinterpret_cast<const uint32_t*>(rec + coff);
    const uint8_t* qual = rec + 16;
    const uint8_t* seq = rec + mgp_seq_offset(lseq);
    const int64_t wend = (int64_t)w.w0 + w.wlen;
    const int64_t vq0 = pc.min_dist > 0 ? pc.min_dist : 0;
    const int64_t vq1 = pc.min_dist > 0 ? (int64_t)lseq - pc.min_dist : (int64_t)lseq;
    int64_t ref = start, q = 0;
    const uint32_t inc = strand_inc(strand);
    for (uint32_t o = 0; o < ncig; ++o) {
        const uint32_t cg = cig[o];
        const uint32_t op = cg & 15u;
        const int64_t len = cg >> 4;
        if (op == 0 || op == 7 || op == 8) {
            const int64_t klo = max((int64_t)0, max((int64_t)w.w0 - ref, vq0 - q));
            const int64_t khi = min(len, min(wend - ref, min(vq1, (int64_t)lseq) - q));
            for (int64_t k = klo; k < khi; ++k) {
                const int64_t qq = q + k;
                if ((int)(int8_t)qual[qq] < pc.min_baseq) continue;
                const uint8_t sb = seq[qq >> 1];
                const int bi = base_index((qq & 1) ? (sb & 15u) : (sb >> 4));
                if (bi < 0) continue;
                atomicAdd(&tile[bi * kTilePitch + (int)(ref + k - w.w0)], inc);
            }
            q += len;
            ref += len;
        } else if (op == 2 || op == 3) {
            ref += len;
        } else if (op == 4) {
            q += len;
        }
    }
    return max(ref - (int64_t)start, (int64_t)lseq) > (int64_t)max_span;
}

constexpr int kFastLen = 64;   // reads up to 64 bases with <= 4 CIGAR ops and <= 2 aligned blocks
constexpr int kFastCig = 4;
constexpr uint32_t kValid = 0x0116u;   // codes 1, 2, 4, 8 are counted (pileup.py:83-86)

// One read per lane, entered by EVERY lane of the wave (has = lane holds a read):
// the unrolled loop bounds are wave reductions, so no lane may be absent.
//
// Register path (l_seq <= 64, <= 4 CIGAR ops, <= 2 aligned blocks): the CIGAR
// becomes two blocks; for block k the counted query positions are
// [a_k, b_k) = [qs_k, qe_k) intersected with the end-distance window [vq0, vq1)
// and with the reference window (r = q + d_k in [w0, w0 + wlen)). Insertions do
// not move q (pileup.py Q1: no branch for op 1). qual sits 16-byte aligned at +16
// and is loaded together with the header; the per-base loop is unrolled so every
// register index is static. Other reads take the generic byte-load path.
#ifndef MGP_ABL
#define MGP_ABL 0  // ablation switch for experiments: 0 = real kernel (11: flush only zeroes the tile, 12: 11 and no piling)
#endif
// The first 128-byte line of a record in registers: header, qual (+16), seq (+80)
// and CIGAR (+112) of a read of <= 64 bases with <= 4 operations
// (include/mgpileup.h); no load depends on another. A packed record is the
// first 64 bytes only (h, qv[0..2]): header, CIGAR and base bytes from +14.
struct RecLine {
    uint4 h, qv[4], sv[2], cv;
};

__device__ __forceinline__ void load_line(bool has, int lay, const uint8_t* __restrict__ rec, const Win& w,
                                          RecLine& R) {
    R.h = make_uint4(0, 0, 0, 0);
    R.cv = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 4; ++k) R.qv[k] = make_uint4(0, 0, 0, 0);
    R.sv[0] = R.sv[1] = make_uint4(0, 0, 0, 0);
    if (MGP_ABL == 3) {
        // synthetic read from the record address only: no payload loads
        const uint32_t x = (uint32_t)(reinterpret_cast<uintptr_t>(rec) >> 4);
        R.h = make_uint4((uint32_t)w.w0 + (x * 7u) % (uint32_t)w.wlen, 50u,
                         1u | (x & 1u ? (MGP_FLAG_REVERSE << 16) : 0u), 112u);
#pragma unroll
        for (int k = 0; k < 4; ++k) R.qv[k] = make_uint4(0x25252525u, 0x25252525u, 0x25252525u, 0x25252525u);
#pragma unroll
        for (int k = 0; k < 2; ++k) R.sv[k] = make_uint4(0x12481248u, 0x24812481u, 0x48124812u, 0x81248124u);
        R.cv.x = 50u << 4;
    } else if (has) {
        // a 32-byte record is 2 loads, a packed 64-byte one 4, a full line 8
        const uint4* r4 = reinterpret_cast<const uint4*>(rec);
        R.h = r4[0];
        R.qv[0] = r4[1];
        if (lay != kLayP32) {
            R.qv[1] = r4[2];
            R.qv[2] = r4[3];
        }
        if (lay == kLayFull) {
            R.qv[3] = r4[4];
            R.sv[0] = r4[5];
            R.sv[1] = r4[6];
            R.cv = r4[7];
        }
    }
}

__device__ __forceinline__ void pile_line(bool has, int lay, const uint8_t* __restrict__ rec, const RecLine& R,
                                          const Win& w, const PileCfg& pc, uint32_t* tile, uint32_t* t5,
                                          uint32_t max_span, bool& span_err, bool& pk_err);

__device__ __forceinline__ void pile_read(bool has, int lay, const uint8_t* __restrict__ rec, const Win& w,
                                          const PileCfg& pc, uint32_t* tile, uint32_t* t5, uint32_t max_span,
                                          bool& span_err, bool& pk_err) {
    if (MGP_ABL == 1 || MGP_ABL == 12) return;
    if (MGP_ABL == 3) lay = kLayFull;  // the synthetic reads are in the full layout
    RecLine R;
    load_line(has, lay, rec, w, R);
    pile_line(has, lay, rec, R, w, pc, tile, t5, max_span, span_err, pk_err);
}

__device__ __forceinline__ uint32_t byte_at(const uint32_t* wd, int j) { return (wd[j >> 2] >> (8 * (j & 3))) & 0xFFu; }

// The counted bases of the register-path reads of a wave (act: the lane takes
// part). Block k of a read counts query positions [a_k, b_k) at reference q +
// d_k. kPacked: base bytes qual << 2 | b at +14 of the packed layout; otherwise
// qual bytes at +16 and 4-bit codes at +80. Every lane of the wave enters: the
// unrolled loop bounds are wave reductions.
template <bool kPacked>
__device__ __forceinline__ void pile_bases(bool act, int a0, int b0, int a1, int b1, int qs1, int dl0, int dl1,
                                           const RecLine& R, const Win& w, const PileCfg& pc, uint32_t* tile,
                                           uint32_t inc) {
    constexpr int kLen = kPacked ? MGP_PACK_MAX_LEN : kFastLen;
    int qlo = 1 << 30, qhi = 0;
    if (act) {
        if (a0 < b0) {
            qlo = a0;
            qhi = b0;
        }
        if (a1 < b1) {
            qlo = min(qlo, a1);
            qhi = max(qhi, b1);
        }
    }
    // wave-uniform bounds of the unrolled loop (every lane participates)
    const int wq_lo = __builtin_amdgcn_readfirstlane(wave_min(qlo));
    const int wq_hi = __builtin_amdgcn_readfirstlane(wave_max(qhi));
    if (wq_lo >= wq_hi) return;
    if (!act) a0 = b0 = a1 = b1 = 0;
    uint32_t qw[16];  // packed: the 64 record bytes; else the qual bytes
    if (kPacked) {
        const uint4 v[4] = {R.h, R.qv[0], R.qv[1], R.qv[2]};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            qw[4 * k] = v[k].x;
            qw[4 * k + 1] = v[k].y;
            qw[4 * k + 2] = v[k].z;
            qw[4 * k + 3] = v[k].w;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            qw[4 * k] = R.qv[k].x;
            qw[4 * k + 1] = R.qv[k].y;
            qw[4 * k + 2] = R.qv[k].z;
            qw[4 * k + 3] = R.qv[k].w;
        }
    }
    const uint32_t sw[8] = {R.sv[0].x, R.sv[0].y, R.sv[0].z, R.sv[0].w, R.sv[1].x, R.sv[1].y, R.sv[1].z, R.sv[1].w};
    // one count at rowp[qq] when ok, branch-free: a lane that does not count adds at
    // its own word + qq of the trash plane, so 4 qq bytes become the atomic's
    // immediate offset and the row select is one pointer select
    uint32_t* const own = tile + kPlaneTrash * kTilePitch + (threadIdx.x & 63);
    auto count_q = [&](uint32_t ok, uint32_t* rowp, int qq) {
        uint32_t* const p = ok ? rowp : own;
        atomicAdd(p + qq, inc);
    };
    const int minbq = pc.min_baseq;
    // packed: counted iff qual << 2 | b lies in [4 * max(min_baseq, 0), 252) (0xFF and
    // anything >= 252 are never counted; packed quals are <= 62)
    const uint32_t lo4 = 4u * (uint32_t)min(max(minbq, 0), 63);
    const uint32_t span4 = 252u - lo4;
    // base index = log2(code) for the counted codes 1, 2, 4, 8 (A, C, G, T); the
    // plane offset is base index x the compile-time pitch
    // ok / plane of query position qq (static register indices)
    auto decode = [&](int qq, uint32_t& plane) -> uint32_t {
        if (kPacked) {
            const uint32_t x = byte_at(qw, 14 + qq);
            plane = x & 3u;
            return (uint32_t)(x - lo4 < span4);
        } else {
            const int qb = (int)(int8_t)byte_at(qw, qq);
            const uint32_t code = (sw[qq >> 3] >> (8 * ((qq >> 1) & 3) + ((qq & 1) ? 0 : 4))) & 15u;
            plane = (uint32_t)__builtin_ctz(code | 16u);
            return (uint32_t)(qb >= minbq) & ((kValid >> code) & 1u);
        }
    };
    const bool one_block = __ballot(act && a1 < b1) == 0ull;
    // common case: every lane of the wave has the same single counted range
    // [a0, b0) (all reads inside the window, same length): no range test
    const int ua0 = __builtin_amdgcn_readfirstlane(a0), ub0 = __builtin_amdgcn_readfirstlane(b0);
    const bool uniform = one_block && __ballot(!(act && a0 == ua0 && b0 == ub0)) == 0ull;
    // iterations run: a wave-uniform 64-bit mask (one scalar bit test per base)
    // (bounds clamped into [0, 64] before any shift: a block right of the window
    // has a negative hi, and a shift by a negative amount is undefined)
    auto range_mask = [](int lo, int hi) -> unsigned long long {
        lo = min(max(lo, 0), 64);
        hi = min(max(hi, 0), 64);
        const unsigned long long h = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
        const unsigned long long l = lo >= 64 ? ~0ull : ((1ull << lo) - 1ull);
        return lo < hi ? (h & ~l) : 0ull;
    };
    // the core [kC0, kC1) of the usual range [min_dist, l_seq - min_dist) of full
    // length reads runs with no per-base range test when the wave's range covers
    // it; bases outside it only behind a scalar bit test of the wave's range
    constexpr int kC0 = 5, kC1 = kLen - 5;
    auto run = [&](int lo, int hi, auto&& body) {
        const unsigned long long smask = range_mask(lo, hi);
        if (lo <= kC0 && hi >= kC1) {
            if (lo < kC0) {
#pragma unroll
                for (int qq = 0; qq < kC0; ++qq)
                    if ((smask >> qq) & 1ull) body(qq);
            }
#pragma unroll
            for (int qq = kC0; qq < kC1; ++qq) body(qq);
            if (hi > kC1) {
#pragma unroll
                for (int qq = kC1; qq < kLen; ++qq)
                    if ((smask >> qq) & 1ull) body(qq);
            }
        } else {
#pragma unroll
            for (int qq = 0; qq < kLen; ++qq)
                if ((smask >> qq) & 1ull) body(qq);
        }
    };
    // LDS rows of the read's blocks (u32 index of query offset 0)
    uint32_t* const r0p = tile + (dl0 - w.w0);
    uint32_t* const r1p = tile + (dl1 - w.w0);
    if (uniform) {
        run(ua0, ub0, [&](int qq) {
            uint32_t plane;
            const uint32_t ok = decode(qq, plane);
            count_q(ok, r0p + plane * kTilePitch, qq);
        });
    } else {
        // the lane's counted query positions as a 64-bit mask: one bit test per base
        const unsigned long long vm = range_mask(a0, b0) | range_mask(a1, b1);
        const uint32_t vlo = (uint32_t)vm, vhi = (uint32_t)(vm >> 32);
        auto counted = [&](int qq) -> uint32_t { return ((qq < 32 ? vlo : vhi) >> (qq & 31)) & 1u; };
        if (one_block) {
            run(wq_lo, wq_hi, [&](int qq) {
                uint32_t plane;
                const uint32_t ok = decode(qq, plane) & counted(qq);
                count_q(ok, r0p + plane * kTilePitch, qq);
            });
        } else {
            run(wq_lo, wq_hi, [&](int qq) {
                // a block's row: the second block starts at query offset qs1
                uint32_t* const rowp = qq >= qs1 ? r1p : r0p;
                uint32_t plane;
                const uint32_t ok = decode(qq, plane) & counted(qq);
                count_q(ok, rowp + plane * kTilePitch, qq);
            });
        }
    }
}

#ifndef MGP_QQ_STRIDE
#define MGP_QQ_STRIDE 1  // query positions per pass of the per-base core loops (A/B)
#endif
constexpr int kQS = MGP_QQ_STRIDE;

// LDS byte addresses: the packed loop computes a count's address as integer
// arithmetic (row | plane * 4) and adds through an LDS-qualified pointer, so the
// query offset still folds into the atomic's immediate.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
__device__ __forceinline__ uint32_t lds_addr(uint32_t* p) { return (uint32_t)(uintptr_t)(lds_u32*)p; }
__device__ __forceinline__ void lds_add(uint32_t addr, uint32_t v) {
    __hip_atomic_fetch_add((lds_u32*)(uintptr_t)addr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The counted bases of the packed register-path reads of a wave. The record's
// base bytes (qual << 2 | b at +14) outside the lane's counted ranges [a_k, b_k)
// are first set to 0xFF (never counted: one v_perm per word), so every wave
// shape runs one loop whose body is a range test on the byte, the count's
// address (the block's row | plane * 4, or the lane's own scratch word when the
// base is not counted) and an LDS add; two-block waves also pick the block's row
// per base. Every lane of the wave enters: the unrolled loop bounds are wave
// reductions.
__device__ __forceinline__ void pile_bases_packed(bool act, int a0, int b0, int a1, int b1, int qs1, int dl0,
                                                  int dl1, const RecLine& R, const Win& w, const PileCfg& pc,
                                                  uint32_t* tile, uint32_t inc) {
    constexpr int kLen = MGP_PACK_MAX_LEN;
    auto range_mask = [](int lo, int hi) -> unsigned long long {
        lo = min(max(lo, 0), 64);
        hi = min(max(hi, 0), 64);
        const unsigned long long h = hi >= 64 ? ~0ull : ((1ull << hi) - 1ull);
        const unsigned long long l = lo >= 64 ? ~0ull : ((1ull << lo) - 1ull);
        return lo < hi ? (h & ~l) : 0ull;
    };
    const unsigned long long vm = act ? (range_mask(a0, b0) | range_mask(a1, b1)) : 0ull;
    int qlo = 1 << 30, qhi = 0;
    if (vm) {
        qlo = __builtin_ctzll(vm);
        qhi = 64 - __builtin_clzll(vm);
    }
    const int wq_lo = __builtin_amdgcn_readfirstlane(wave_min(qlo));
    const int wq_hi = __builtin_amdgcn_readfirstlane(wave_max(qhi));
    if (wq_lo >= wq_hi) return;
    uint32_t qw[16];
    {
        const uint4 v[4] = {R.h, R.qv[0], R.qv[1], R.qv[2]};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            qw[4 * k] = v[k].x;
            qw[4 * k + 1] = v[k].y;
            qw[4 * k + 2] = v[k].z;
            qw[4 * k + 3] = v[k].w;
        }
    }
    // uncounted positions -> 0xFF: word j holds query positions 4j - 14 .. 4j - 11,
    // bits 4j - 12 .. 4j - 9 of u = ~vm << 2 (its bits 0, 1 are the header bytes
    // 12, 13, left alone); a set bit i selects byte i + 4 of {0xFFFFFFFF, word}
    const unsigned long long u = ~vm << 2;
    const uint32_t ulo = (uint32_t)u, uhi = (uint32_t)(u >> 32);
#pragma unroll
    for (int j = 3; j < 16; ++j) {
        const int s = 4 * j - 12;
        const uint32_t b4 = ((s < 32 ? ulo : uhi) >> (s & 31)) & 15u;
        const uint32_t sel = 0x03020100u | ((b4 * 0x810204u) & 0x04040404u);
        qw[j] = __builtin_amdgcn_perm(0xFFFFFFFFu, qw[j], sel);
    }
    // counted iff qual << 2 | b lies in [4 * max(min_baseq, 0), 252)
    const uint32_t lo4 = 4u * (uint32_t)min(max(pc.min_baseq, 0), 63);
    const uint32_t span4 = 252u - lo4;
    const uint32_t tb = lds_addr(tile);
    const uint32_t own = tb + kPlaneTrash * kPlaneBytes + 4u * (threadIdx.x & 63);  // (trash plane)
    // rows: byte address of query offset 0 of each block (4 bytes per position)
    const uint32_t r0 = tb + 4u * (uint32_t)(dl0 - w.w0), r1 = tb + 4u * (uint32_t)(dl1 - w.w0);
    auto count = [&](int qq, uint32_t row) {
        const uint32_t x = (qw[(14 + qq) >> 2] >> (8 * ((14 + qq) & 3))) & 0xFFu;
        const uint32_t a = row + (x & 3u) * kPlaneBytes;
        lds_add((x - lo4 < span4 ? a : own) + 4u * (uint32_t)qq, inc);
    };
    const bool two = __ballot(act && a1 < b1) != 0ull;
    // the wave's range [wq_lo, wq_hi): the core [kC0, kC1) without a test when
    // covered, positions outside it behind a scalar bit test of the range
    const unsigned long long smask = range_mask(wq_lo, wq_hi);
    constexpr int kC0 = 5, kC1 = kLen - 5;
    auto run = [&](auto&& body) {
        if (wq_lo <= kC0 && wq_hi >= kC1) {
            if (wq_lo < kC0) {
#pragma unroll
                for (int qq = 0; qq < kC0; ++qq)
                    if ((smask >> qq) & 1ull) body(qq);
            }
            // the core in MGP_QQ_STRIDE interleaved passes (consecutive adds of a lane
            // kQS positions apart, not 1)
#pragma unroll
            for (int j = 0; j < kQS; ++j)
#pragma unroll
                for (int qq = kC0 + j; qq < kC1; qq += kQS) body(qq);
            if (wq_hi > kC1) {
#pragma unroll
                for (int qq = kC1; qq < kLen; ++qq)
                    if ((smask >> qq) & 1ull) body(qq);
            }
        } else {
#pragma unroll
            for (int qq = 0; qq < kLen; ++qq)
                if ((smask >> qq) & 1ull) body(qq);
        }
    };
    if (two) run([&](int qq) { count(qq, qq >= qs1 ? r1 : r0); });
    else run([&](int qq) { count(qq, r0); });
}

// The counted bases of the 32-byte register-path reads of a wave. A record's codes
// already say which query positions count (include/mgpileup.h: 0..3 the counted
// base, 4 not counted), so a base is its 3-bit code (a static bit-field extract, a
// funnel shift where it straddles two words) and one LDS add at the block's row +
// code x plane stride + the query offset: code 4 adds to the trash plane. The loop
// runs over the wave's counted query range [min a_k, max b_k); a lane's positions
// there outside the window land in the tile's guard words (never read) when every
// row of the wave stays within kTileGuard positions of the window, else each base
// is tested. Lanes without a register-path read add all-4 codes (the trash plane).
__device__ __forceinline__ void pile_bases_p32(bool act, int a0, int b0, int a1, int b1, int qs1, int dl0, int dl1,
                                               const RecLine& R, const Win& w, uint32_t* tile, uint32_t inc) {
    constexpr int kLen = MGP_PACK_MAX_LEN;
    int qlo = 1 << 30, qhi = 0;
    if (act && a0 < b0) {
        qlo = a0;
        qhi = b0;
    }
    if (act && a1 < b1) {
        qlo = min(qlo, a1);
        qhi = max(qhi, b1);
    }
    const int wq_lo = __builtin_amdgcn_readfirstlane(wave_min(qlo));
    const int wq_hi = __builtin_amdgcn_readfirstlane(wave_max(qhi));
    if (wq_lo >= wq_hi) return;
    // a lane counting nothing in the window takes code 4 in every 3-bit field (word
    // by word: fields straddle words) at a row of its own, so such lanes add to
    // distinct trash words (one shared word would serialize their atomics)
    const bool live = qlo < qhi;
    constexpr uint32_t kAll4[5] = {0x24924924u, 0x49249249u, 0x92492492u, 0x24924924u, 0x49249249u};
    const uint32_t cw[6] = {live ? R.h.w : kAll4[0], live ? R.qv[0].x : kAll4[1], live ? R.qv[0].y : kAll4[2],
                            live ? R.qv[0].z : kAll4[3], live ? R.qv[0].w : kAll4[4], 0u};
    // row offsets (window positions of query offset 0): block 1 from qs1 on (a lane
    // with one block has qs1 past the read)
    const bool two = __ballot(live && qs1 < kLen) != 0ull;
    const int e0 = live ? dl0 - w.w0 : (int)(threadIdx.x & 63);
    const int e1 = live && qs1 < kLen ? dl1 - w.w0 : e0;
    const int plo = min(e0, e1) + wq_lo, phi = max(e0, e1) + wq_hi - 1;
    const bool guarded = __ballot(plo < -kTileGuard || phi >= kTilePitch - kTileGuard) == 0ull;
    const uint32_t tb = lds_addr(tile);
    uint32_t r0 = tb + 4u * (uint32_t)e0, r1 = tb + 4u * (uint32_t)e1;
#if MGP_ROW_OPAQUE
    // the rows as opaque VGPRs: otherwise the compiler splits the uniform tile base
    // out of them and keeps tile base + 4 x query offset as one SGPR per offset (50 of
    // them, spilled to VGPR lanes: a v_readlane + s_nop + v_add3 per base) instead of
    // folding the query offset into the LDS add's immediate (v_mad_u32_u24 + ds_add)
    asm volatile("" : "+v"(r0), "+v"(r1));
#endif
    auto code = [&](int qq) -> uint32_t {
        const int bit = 3 * qq, j = bit >> 5, sh = bit & 31;
        return sh <= 29 ? __builtin_amdgcn_ubfe(cw[j], sh, 3) : (__builtin_amdgcn_alignbit(cw[j + 1], cw[j], sh) & 7u);
    };
    const unsigned long long smask = (wq_hi >= 64 ? ~0ull : ((1ull << wq_hi) - 1ull)) & ~((1ull << wq_lo) - 1ull);
    constexpr int kC0 = 5, kC1 = kLen - 5;
    auto run = [&](auto&& body) {
        if (wq_lo <= kC0 && wq_hi >= kC1) {
            if (wq_lo < kC0) {
#pragma unroll
                for (int qq = 0; qq < kC0; ++qq)
                    if ((smask >> qq) & 1ull) body(qq);
            }
            // the core in MGP_QQ_STRIDE interleaved passes (consecutive adds of a lane
            // kQS positions apart, not 1)
#pragma unroll
            for (int j = 0; j < kQS; ++j)
#pragma unroll
                for (int qq = kC0 + j; qq < kC1; qq += kQS) body(qq);
            if (wq_hi > kC1) {
#pragma unroll
                for (int qq = kC1; qq < kLen; ++qq)
                    if ((smask >> qq) & 1ull) body(qq);
            }
        } else {
#pragma unroll
            for (int qq = 0; qq < kLen; ++qq)
                if ((smask >> qq) & 1ull) body(qq);
        }
    };
    if (MGP_ABL == 10) {  // ablation (counts meaningless): every lane of a half on its own bank
        const uint32_t lr = tb + 4u * (threadIdx.x & 63);
        run([&](int qq) { lds_add(lr + code(qq) * kPlaneBytes + 4u * (uint32_t)qq, inc); });
    } else if (guarded) {
        if (two) run([&](int qq) { lds_add((qq >= qs1 ? r1 : r0) + code(qq) * kPlaneBytes + 4u * (uint32_t)qq, inc); });
        else run([&](int qq) { lds_add(r0 + code(qq) * kPlaneBytes + 4u * (uint32_t)qq, inc); });
    } else {
        const uint32_t own = tb + kPlaneTrash * kPlaneBytes + 4u * (threadIdx.x & 63);
        run([&](int qq) {
            const int p = (qq >= qs1 ? e1 : e0) + qq;
            const bool in = (unsigned)p < (unsigned)w.wlen;
            lds_add(in ? tb + code(qq) * kPlaneBytes + 4u * (uint32_t)p : own, inc);
        });
    }
}

__device__ __forceinline__ void pile_line(bool has, int lay, const uint8_t* __restrict__ rec, const RecLine& R,
                                          const Win& w, const PileCfg& pc, uint32_t* tile, uint32_t* t5,
                                          uint32_t max_span, bool& span_err, bool& pk_err) {
    if (MGP_ABL == 1 || MGP_ABL == 12) return;
    const uint4 h = R.h, cv = R.cv;
    const bool packed = lay != kLayFull, p32 = lay == kLayP32;
    // header fields of the three layouts (include/mgpileup.h)
    const int32_t start = p32 ? (int32_t)(h.x & 0xFFFFu) : (int32_t)h.x;
    const uint32_t lseq = p32 ? ((h.x >> 16) & 0xFFu) : packed ? (h.y & 0xFFu) : h.y;
    const uint32_t ncig = p32 ? ((h.x >> 24) & 7u) : packed ? ((h.y >> 8) & 0x7Fu) : (h.z & 0xFFFFu);
    const uint32_t coff = h.w;
    const int strand = p32 ? (int)(h.x >> 31) : packed ? (int)((h.y >> 15) & 1u)
                                                     : (((h.z >> 16) & MGP_FLAG_REVERSE) ? 1 : 0);
    const uint32_t cigw[4] = {p32 ? (h.y & 0xFFFFu) : packed ? (h.y >> 16) : cv.x,
                              p32 ? (h.y >> 16) : packed ? (h.z & 0xFFFFu) : cv.y,
                              p32 ? (h.z & 0xFFFFu) : packed ? (h.z >> 16) : cv.z,
                              p32 ? (h.z >> 16) : packed ? (h.w & 0xFFFFu) : cv.w};
    // a 32-byte record's codes were made for one (min_baseq, min_dist) pair (bytes 31, 3)
    if (has && p32 &&
        ((int)(int8_t)(R.qv[0].w >> 24) != pc.min_baseq || (int)((h.x >> 27) & 15u) != max(pc.min_dist, 0)))
        pk_err = true;
    tn5_cut(has, start, lseq, strand, w, t5);

    bool fast = has && lseq <= (uint32_t)(packed ? MGP_PACK_MAX_LEN : kFastLen) && ncig <= (uint32_t)kFastCig &&
                start >= -(1 << 28) && start < (1 << 28);
    // The CIGAR as at most two aligned blocks, straight-line code (per-lane
    // branches on the operation would be exec-mask branches for every op of every
    // read). Block k covers query [qs_k, qe_k) at reference q + d_k. An aligned op
    // that continues the last block (same q and reference offset: after an I,
    // which moves neither, pileup.py Q1) extends it; a third block leaves the
    // register path.
    int qs0 = 0, qe0 = 0, d0 = 0, qs1 = 1 << 30, qe1 = 1 << 30, d1 = 0;
    int nb = 0, ref = start, q = 0;
    bool over = false;
#pragma unroll
    for (int o = 0; o < kFastCig; ++o) {
        const bool live = (uint32_t)o < ncig;
        const uint32_t cg = cigw[o];
        const uint32_t op = cg & 15u;
        const int len = (int)min(cg >> 4, (uint32_t)(1 << 26));
        const bool isM = live && (op == 0 || op == 7 || op == 8);
        const bool isD = live && (op == 2 || op == 3);
        const bool isS = live && op == 4;
        const int dl = ref - q;
        const bool ext0 = isM && nb == 1 && q == qe0 && dl == d0;
        const bool ext1 = isM && nb == 2 && q == qe1 && dl == d1;
        const bool new0 = isM && nb == 0;
        const bool new1 = isM && nb == 1 && !ext0;
        over = over || (isM && nb == 2 && !ext1);
        qs0 = new0 ? q : qs0;
        d0 = new0 ? dl : d0;
        qe0 = (new0 || ext0) ? q + len : qe0;
        qs1 = new1 ? q : qs1;
        d1 = new1 ? dl : d1;
        qe1 = (new1 || ext1) ? q + len : qe1;
        nb += (new0 || new1) ? 1 : 0;
        q += (isM || isS) ? len : 0;
        ref += (isM || isD) ? len : 0;
    }
    fast = fast && !over;
    span_err = span_err || (fast && max(ref - start, (int)lseq) > (int)max_span);
    const int vq0 = pc.min_dist > 0 ? pc.min_dist : 0;
    const int vq1 = min((int)lseq, pc.min_dist > 0 ? (int)lseq - pc.min_dist : (int)lseq);
    const int wlo = w.w0, whi = w.w0 + w.wlen;
    int a0 = max(max(qs0, vq0), wlo - d0);
    int b0 = min(min(qe0, vq1), whi - d0);
    int a1 = max(max(qs1, vq0), wlo - d1);
    int b1 = min(min(qe1, vq1), whi - d1);
    b0 = (fast && nb >= 1) ? b0 : a0;
    b1 = (fast && nb >= 2) ? b1 : a1;
    const int dl0 = d0, dl1 = d1;
    const uint32_t inc = strand_inc(strand);
    if (MGP_ABL == 8) {  // records loaded, no per-base work (experiments only)
        const uint32_t x = R.h.x ^ R.h.y ^ R.h.z ^ R.h.w ^ R.qv[0].x ^ R.qv[0].y ^ R.qv[0].z ^ R.qv[0].w ^
                           R.qv[1].x ^ R.qv[1].y ^ R.qv[1].z ^ R.qv[1].w ^ R.qv[2].x ^ R.qv[2].y ^ R.qv[2].z ^
                           R.qv[2].w;
        if (x == 0x9e3779b9u) atomicAdd(&tile[0], 1u);
        return;
    }
    // one register pass per layout present in the wave (mixed waves are rare:
    // producers pack every read that fits)
    if (__ballot(fast && !packed) != 0ull)
        pile_bases<false>(fast && !packed, a0, b0, a1, b1, qs1, dl0, dl1, R, w, pc, tile, inc);
    if (__ballot(fast && packed && !p32) != 0ull)
        pile_bases_packed(fast && packed && !p32, a0, b0, a1, b1, qs1, dl0, dl1, R, w, pc, tile, inc);
    if (__ballot(fast && p32) != 0ull) pile_bases_p32(fast && p32, a0, b0, a1, b1, qs1, dl0, dl1, R, w, tile, inc);
    const bool slow = has && !fast;
    pk_err = pk_err || (slow && packed);  // a packed record outside the layout's limits
    bool se = false;
    if (slow && !packed) se = pile_slow(rec, start, lseq, ncig, coff, strand, w, pc, tile, max_span);
    span_err = span_err || se;
}

#ifndef MGP_LANE_PERM
#define MGP_LANE_PERM 1
#endif
#ifndef MGP_STREAM_U
#define MGP_STREAM_U 2
#endif
constexpr int kStreamU = MGP_STREAM_U;  // pileup elements per lane per stream step
// per-wave ring of reads waiting to be piled (LDS, a power of two holding the
// < 64 left over plus one stream step)
constexpr int kWaveQ = kStreamU <= 1 ? 2 * kWave : kStreamU <= 3 ? 4 * kWave : 8 * kWave;
static_assert(kWaveQ >= kWave * (kStreamU + 1) && kStreamU <= 7, "pileup ring too small");

// record byte offset of a pileup element (MGP_ABL 6, experiments only: every
// record read from the first 256 MiB of the payload, to time the pileup with a
// small gather footprint; the counts are then meaningless)
__device__ __forceinline__ unsigned long long rec_at(uint32_t qe, int unit, uint32_t pe_off) {
    const unsigned long long off = (unsigned long long)(qe & pe_off) << unit;
    return MGP_ABL == 6 ? off & ((256ull << 20) - 128) : off;
}
constexpr uint32_t kSeg = 65535;     // elements per tile segment (16-bit halves cannot carry)

// the record layout of a pileup element (kLayAny: from its PE_PACKED / PE_P32 bits)
template <int kLayout>
__device__ __forceinline__ int elem_layout(uint32_t qe) {
    if (kLayout != kLayAny) return kLayout;
    return (qe & PE_PACKED) ? ((qe & PE_P32) ? kLayP32 : kLayP64) : kLayFull;
}

// grid (nchunks, nwin): workgroup = (cell chunk, position window). For each cell
// of the chunk, the cell's pileup elements with start bin in [window start -
// reach, window end) are taken by the 4 waves independently, in interleaved
// blocks of 128 (the next step's elements loaded while the current one is
// queued); the reads to pile (kept by pass B's duplicate marking, MAPQ passed)
// go to the wave's LDS ring and are piled 64 at a time, one read per lane.
// Workgroup barriers only at cell boundaries; the packed tile is then
// strand-filtered and flushed.
#ifndef MGP_PILEUP_WAVES
#define MGP_PILEUP_WAVES 4
#endif

// Output (Out16): the strand-filtered counts as u16 pairs, exactly the tile's
// packed words (fwd low, rev high), Tn5 as one u32 pair word and depth as u16.
// A cell window with at most 65535 elements cannot hold a larger value, so these
// are exact; a drained window (more elements) keeps its exact u32 rows in the
// 32-bit arrays and is flagged in `wide` (the u16 copy is saturated, the HDF5
// form writers.py:205-218). mgp_fetch expands the 16-bit form into the caller's
// u32 arrays.
struct Out16 {
    uint4* counts;     // [cells][L]: 8 x u16 A_fwd, A_rev, ... T_rev
    uint32_t* tn5;     // [cells][L]: fwd | rev << 16
    uint16_t* depth;   // [cells][L]
    uint8_t* wide;     // [cells][nwin]: 1 = exact values in the u32 arrays
    uint8_t* fit8;     // [cells][nwin]: 1 = every value of the window's rows is <= 255 (the 8-bit target)
};

__device__ __forceinline__ uint32_t sat16(uint32_t v) { return v > 0xFFFFu ? 0xFFFFu : v; }

// kPacked: every resident record is packed (the input check's CHK_FULL clear):
// no full-layout path, and the records of a wave's next 64 queued reads are
// loaded before the current 64 are piled (one batch of gathers in flight
// behind the per-base work; the registers the full-layout path would hold pay
// for the second record set).
#ifndef MGP_PILE_PREFETCH
#define MGP_PILE_PREFETCH 1
#endif
// kLayout: kLayP64 / kLayP32 when every resident record has that packed layout (the
// next batch's records loaded ahead), kLayAny otherwise (the layout from the element's
// PE_PACKED / PE_P32 bits). pe_off: the element's offset bits (30 for the wide
// grouping elements, which carry the layout; 31 for the compact ones).
template <int kLayout>
__global__ void __launch_bounds__(kBlock, MGP_PILEUP_WAVES) k_pileup(
    Geom g, PileCfg pc, const uint8_t* __restrict__ payload, const uint32_t* __restrict__ pel, int unit,
    uint32_t pe_off,
    const uint32_t* __restrict__ O, Out16 o16, uint32_t* __restrict__ counts, uint32_t* __restrict__ tn5,
    uint32_t* __restrict__ depth, uint32_t* __restrict__ n_reads, uint8_t* __restrict__ any_paired, int pair_mode,
    uint32_t* __restrict__ covered, unsigned long long* __restrict__ dsum,
    uint32_t* __restrict__ dmax, uint32_t* __restrict__ tally_part, DevStats* st, int w_base,
    const uint32_t* __restrict__ ck, const uint32_t* __restrict__ chunk_perm) {
    // the tile: kTilePlanes planes of kTilePitch words (A, C, G, T, trash, Tn5; fwd | rev << 16)
    extern __shared__ __align__(16) uint32_t tile_planes[];
    uint32_t* const tile = tile_planes + kTileGuard;  // position 0 of plane 0
    uint32_t* const t5 = tile + kPlaneTn5 * kTilePitch;
    if (__atomic_load_n(&st->err, __ATOMIC_RELAXED) & ERR_BOUNDS) return;  // unsorted input (k_bin_count)
    __shared__ uint32_t wq_all[kBlock / kWave][kWaveQ];
    __shared__ uint32_t r_cov[4], r_max[4], r_keep[4], r_big[4];
    __shared__ unsigned long long r_sum[4];

    // the workgroups take the chunks largest first (chunk_perm, k_scan_cells), all
    // windows of a chunk in a row; a streaming segment's windows start at w_base
    const uint32_t nw = gridDim.y, lin = blockIdx.y * gridDim.x + blockIdx.x;
    const int chunk = (int)chunk_perm[lin / nw];
    const int k = w_base + (int)(lin % nw);  // window
    // pair_mode < 0 (streaming): every read paired iff the input check saw only paired
    // reads (a mix reruns the run resident, ERR_RESPEC)
    if (pair_mode < 0) pair_mode = (ck[0] & CHK_PAIRED) && !(ck[0] & CHK_UNPAIRED) ? 1 : 0;
    Win w;
    w.w0 = k * g.W;
    w.wlen = min(g.W, g.L - w.w0);
    w.Wp = g.Wp;
    const int L = g.L;
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // (scalar)
    uint32_t* wq = wq_all[wid];
    // the queued read a lane piles: even queue slots in lanes 0..31, odd in 32..63. The
    // queue is in coordinate order and LDS atomics conflict per 32-lane half, so
    // reads with the same start (same count address) are split over the halves.
    const uint32_t qlane = MGP_LANE_PERM ? (uint32_t)(((lane & 31) << 1) | (lane >> 5)) : (uint32_t)lane;
    const uint32_t max_span = st->max_span;
    const int R = (int)((max_span + g.G - 1) / g.G) * g.G;
    const int lo_bin = win_lo_bin(k, R, g);
    const int own_bin = (int)((long long)k * g.W / g.G);
    const int hi_bin = k == g.nwin - 1 ? g.nbins : win_hi_bin(k, g);
    const int nc = g.nc;
    const unsigned long long lt = lanemask_lt();
    bool span_err = false;
    bool pk_err = false;  // a packed record outside the packed layout's limits

    uint32_t tal[kMaxPosPerThread][4];
#pragma unroll
    for (int m = 0; m < kMaxPosPerThread; ++m)
#pragma unroll
        for (int b = 0; b < 4; ++b) tal[m][b] = 0;

    const int c0 = chunk * g.cpb, c1 = min(nc, c0 + g.cpb);
    // element ranges of the next cell are loaded one cell ahead
    uint32_t n_lo = c0 < c1 ? O[(size_t)lo_bin * nc + c0] : 0u;
    uint32_t n_own = c0 < c1 ? O[(size_t)own_bin * nc + c0] : 0u;
    uint32_t n_hi = c0 < c1 ? O[(size_t)hi_bin * nc + c0] : 0u;
    // the tile starts zeroed; each flush zeroes what it read, so the next cell
    // starts from zero behind the flush's barrier
    for (int x = threadIdx.x; x < kTilePlanes * kTilePitch; x += blockDim.x) tile_planes[x] = 0;
    __syncthreads();
    for (int c = c0; c < c1; ++c) {
        const uint32_t lo = n_lo, own = n_own, hi = n_hi;
        if (c + 1 < c1) {
            n_lo = O[(size_t)lo_bin * nc + c + 1];
            n_own = O[(size_t)own_bin * nc + c + 1];
            n_hi = O[(size_t)hi_bin * nc + c + 1];
        }
        // kept reads, counted once: by the window owning the start bin
        uint32_t nkeep = 0;
        const bool drained = hi - lo > kSeg;  // tile drained into the output rows between segments
        for (uint32_t seg = lo; seg < hi; seg += kSeg) {
            const uint32_t seg_hi = min(hi, seg + kSeg);
            // the wave's ring of queued reads: [qh, qh + qn), wave-uniform
            uint32_t qh = 0, qn = 0;
            constexpr bool kPacked = kLayout == kLayP64 || kLayout == kLayP32;
            RecLine Rp;         // kPacked: the loaded batch waiting to be piled
            bool pend = false;  // (wave-uniform)
            // a stream step: each wave takes kStreamU x 64 consecutive elements (the
            // waves' blocks interleaved), the next step's loaded while this one is
            // queued and piled
            constexpr uint32_t kStepW = kStreamU * kWave, kStepB = kStepW * (kBlock / kWave);
            uint32_t cb = seg + kStepW * wid;
            uint32_t pe[kStreamU];
#pragma unroll
            for (int u = 0; u < kStreamU; ++u) {
                const uint32_t j = cb + u * kWave + lane;
                pe[u] = j < seg_hi ? pel[j] : PE_DUP;
            }
            for (; cb < seg_hi; cb += kStepB) {
                uint32_t cur[kStreamU];
#pragma unroll
                for (int u = 0; u < kStreamU; ++u) {
                    cur[u] = pe[u];
                    const uint64_t j = (uint64_t)cb + kStepB + u * kWave + lane;
                    pe[u] = j < seg_hi ? pel[j] : PE_DUP;
                }
#pragma unroll
                for (int u = 0; u < kStreamU; ++u) {
                    nkeep += (cb + u * kWave + lane >= own) & (cur[u] != PE_DUP);  // PE_DUP past seg_hi
                    const bool piled = cur[u] < PE_KEEP;
                    const unsigned long long bal = __ballot(piled);
                    if (piled) wq[(qh + qn + (uint32_t)__popcll(bal & lt)) & (kWaveQ - 1)] = cur[u];
                    qn += (uint32_t)__popcll(bal);
                }
                __builtin_amdgcn_wave_barrier();
                while (qn >= (uint32_t)kWave) {
                    const uint32_t qe = wq[(qh + qlane) & (kWaveQ - 1)];
                    qh += kWave;
                    qn -= kWave;
                    if constexpr (kPacked && MGP_PILE_PREFETCH) {
                        RecLine Rn;  // this batch's records load while the pending batch is piled
                        load_line(true, kLayout, payload + rec_at(qe, unit, pe_off), w, Rn);
                        if (pend) pile_line(true, kLayout, nullptr, Rp, w, pc, tile, t5, max_span, span_err, pk_err);
                        Rp = Rn;
                        pend = true;
                    } else {
                        pile_read(true, elem_layout<kLayout>(qe), payload + rec_at(qe, unit, pe_off), w, pc, tile,
                                  t5, max_span, span_err, pk_err);
                    }
                }
            }
            {   // tail: every lane of the wave enters, lanes past qn hold no read
                const bool has = qlane < qn;
                const uint32_t qe = has ? wq[(qh + qlane) & (kWaveQ - 1)] : 0u;
                if constexpr (kPacked && MGP_PILE_PREFETCH) {
                    RecLine Rn;
                    load_line(has, kLayout, payload + rec_at(qe, unit, pe_off), w, Rn);
                    if (pend) pile_line(true, kLayout, nullptr, Rp, w, pc, tile, t5, max_span, span_err, pk_err);
                    pend = false;
                    pile_line(has, kLayout, nullptr, Rn, w, pc, tile, t5, max_span, span_err, pk_err);
                } else {
                    pile_read(has, elem_layout<kLayout>(qe), payload + rec_at(qe, unit, pe_off), w, pc, tile, t5,
                              max_span, span_err, pk_err);
                }
            }
            if (drained) {  // add this segment's packed tile into the 32-bit output rows
                __syncthreads();
                for (int p = threadIdx.x; p < w.wlen; p += blockDim.x) {
                    const size_t P = (size_t)c * L + w.w0 + p;
                    uint4* cp = reinterpret_cast<uint4*>(counts + P * 8);
                    uint4 a = seg == lo ? make_uint4(0, 0, 0, 0) : cp[0];
                    uint4 b = seg == lo ? make_uint4(0, 0, 0, 0) : cp[1];
                    uint2 t = seg == lo ? make_uint2(0, 0) : reinterpret_cast<uint2*>(tn5)[P];
                    const uint32_t x0 = tile[p], x1 = tile[kTilePitch + p], x2 = tile[2 * kTilePitch + p],
                                   x3 = tile[3 * kTilePitch + p], x4 = t5[p];
                    a.x += x0 & 0xFFFFu; a.y += x0 >> 16; a.z += x1 & 0xFFFFu; a.w += x1 >> 16;
                    b.x += x2 & 0xFFFFu; b.y += x2 >> 16; b.z += x3 & 0xFFFFu; b.w += x3 >> 16;
                    t.x += x4 & 0xFFFFu; t.y += x4 >> 16;
                    cp[0] = a;
                    cp[1] = b;
                    reinterpret_cast<uint2*>(tn5)[P] = t;
#pragma unroll
                    for (int b = 0; b < 4; ++b) tile[b * kTilePitch + p] = 0;
                    t5[p] = 0;
                }
                __syncthreads();
            }
        }
        nkeep = wave_sum(nkeep);
        __syncthreads();
        uint32_t cov = 0, mx = 0, big = 0;  // big: a value of the rows above 255
        unsigned long long sum = 0;
#pragma unroll
        for (int m = 0; m < kMaxPosPerThread; ++m) {
            const int p = threadIdx.x + m * kBlock;
            if ((MGP_ABL == 11 || MGP_ABL == 12) && p < w.wlen) {  // ablation: the flush only zeroes the tile
#pragma unroll
                for (int x = 0; x < 4; ++x) tile[x * kTilePitch + p] = 0u;
                t5[p] = 0u;
                continue;
            }
            if (p < w.wlen) {
                const size_t P = (size_t)c * L + w.w0 + p;
                uint32_t v[8], tf, tr;
                uint32_t pk4[4] = {0u, 0u, 0u, 0u}, pk5 = 0u;  // the packed words (not drained)
                if (drained) {
                    const uint4 a = reinterpret_cast<const uint4*>(counts + P * 8)[0];
                    const uint4 b = reinterpret_cast<const uint4*>(counts + P * 8)[1];
                    const uint2 t = reinterpret_cast<const uint2*>(tn5)[P];
                    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
                    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
                    tf = t.x;
                    tr = t.y;
                } else {
#pragma unroll
                    for (int x = 0; x < 4; ++x) {
                        pk4[x] = tile[x * kTilePitch + p];
                        tile[x * kTilePitch + p] = 0u;
                        v[2 * x] = pk4[x] & 0xFFFFu;
                        v[2 * x + 1] = pk4[x] >> 16;
                    }
                    pk5 = t5[p];
                    t5[p] = 0u;
                    tf = pk5 & 0xFFFFu;
                    tr = pk5 >> 16;
                }
                uint32_t d = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t fw = v[2 * b], rv = v[2 * b + 1];
                    const uint32_t tot = fw + rv;
                    if (pc.bias_active && tot > 0) {
                        const double bias = (double)(fw > rv ? fw : rv) / (double)tot;
                        if (bias > pc.max_bias) {
                            v[2 * b] = 0;
                            v[2 * b + 1] = 0;
                            pk4[b] = 0u;
                        }
                    }
                    const uint32_t t2 = v[2 * b] + v[2 * b + 1];
                    tal[m][b] += t2;
                    d += t2;
                }
                if (d == 0 && !pc.keep_tn5) {
                    tf = tr = 0;
                    pk5 = 0u;
                }
                if (MGP_ABL != 4 || (v[0] == 0xFFFFFFFFu && d == 7u)) {
                    if (drained) {  // exact u32 rows, saturated u16 copy
                        uint4* cp = reinterpret_cast<uint4*>(counts + P * 8);
                        cp[0] = make_uint4(v[0], v[1], v[2], v[3]);
                        cp[1] = make_uint4(v[4], v[5], v[6], v[7]);
                        reinterpret_cast<uint2*>(tn5)[P] = make_uint2(tf, tr);
                        depth[P] = d;
#pragma unroll
                        for (int b = 0; b < 4; ++b) pk4[b] = sat16(v[2 * b]) | sat16(v[2 * b + 1]) << 16;
                        pk5 = sat16(tf) | sat16(tr) << 16;
                    }
                    o16.counts[P] = make_uint4(pk4[0], pk4[1], pk4[2], pk4[3]);
                    o16.tn5[P] = pk5;
                    o16.depth[P] = (uint16_t)sat16(d);
                }
                cov += d > 0;
                sum += d;
                mx = d > mx ? d : mx;
                big |= (d | tf | tr) > 0xFFu;  // (every count is at most d)
            }
        }
        const bool anybig = __ballot(big != 0u) != 0ull;
        cov = wave_sum(cov);
        sum = wave_sum(sum);
        mx = wave_max(mx);
        if (lane == 0) {
            r_cov[wid] = cov;
            r_sum[wid] = sum;
            r_max[wid] = mx;
            r_keep[wid] = nkeep;
            r_big[wid] = anybig;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            o16.wide[(size_t)c * g.nwin + k] = drained ? 1u : 0u;
            o16.fit8[(size_t)c * g.nwin + k] = (drained || r_big[0] || r_big[1] || r_big[2] || r_big[3]) ? 0u : 1u;
            uint32_t C = 0, M = 0, K = 0;
            unsigned long long S = 0;
            for (int q = 0; q < 4; ++q) {
                C += r_cov[q];
                S += r_sum[q];
                M = max(M, r_max[q]);
                K += r_keep[q];
            }
            if (C) {
                atomicAdd(&covered[c], C);
                atomicAdd(&dsum[c], S);
                atomicMax(&dmax[c], M);
            }
            if (K) {
                atomicAdd(&n_reads[c], K);
                if (pair_mode) any_paired[c] = 1;  // benign race: every writer stores 1
            }
        }
    }
#pragma unroll
    for (int m = 0; m < kMaxPosPerThread; ++m) {
        const int p = threadIdx.x + m * kBlock;
        if (p < w.wlen) {
            uint4* tp = reinterpret_cast<uint4*>(tally_part + ((size_t)chunk * L + w.w0 + p) * 4);
            *tp = make_uint4(tal[m][0], tal[m][1], tal[m][2], tal[m][3]);
        }
    }
    const bool anyspan = __ballot(span_err) != 0ull;
    if (lane == 0 && anyspan) atomicOr(&st->err, ERR_SPAN);
    const bool anypk = __ballot(pk_err) != 0ull;
    if (lane == 0 && anypk) atomicOr(&st->err, ERR_PACKED);
}

// min-reads gate (processors.py:22) for min_reads > 1: a cell with fewer kept
// reads produces no result; remove its counts and its tally contribution.
__global__ void __launch_bounds__(kBlock) k_gate_fixup(Geom g, int min_reads, const uint32_t* __restrict__ n_reads,
                                                       Out16 o16, uint32_t* __restrict__ counts,
                                                       uint32_t* __restrict__ tn5, uint32_t* __restrict__ depth,
                                                       uint32_t* __restrict__ covered,
                                                       unsigned long long* __restrict__ dsum,
                                                       uint32_t* __restrict__ dmax, uint32_t* __restrict__ tally_part,
                                                       uint4* __restrict__ hc, uint32_t* __restrict__ ht,
                                                       uint16_t* __restrict__ hd, uint2* __restrict__ hc8,
                                                       uint16_t* __restrict__ ht8, uint8_t* __restrict__ hd8) {
    // hc/ht/hd (mgp_set_rows16_target, else null): the pinned host rows, which the
    // segments' k_rows_to_host already wrote: the dropped cell's rows are zeroed there too
    const int c = blockIdx.x;
    const uint32_t nr = n_reads[c];
    if (nr == 0 || nr >= (uint32_t)min_reads || covered[c] == 0) return;
    const int L = g.L;
    uint32_t* tp = tally_part + (size_t)(c / g.cpb) * L * 4;
    for (int p = threadIdx.x; p < L; p += blockDim.x) {
        const size_t P = (size_t)c * L + p;
        const bool wide = o16.wide[(size_t)c * g.nwin + p / g.W] != 0;
        if ((wide ? depth[P] : (uint32_t)o16.depth[P]) == 0u) continue;
        uint32_t t[4];
        if (wide) {
            uint4* cp = reinterpret_cast<uint4*>(counts + P * 8);
            const uint4 a = cp[0], b = cp[1];
            t[0] = a.x + a.y;
            t[1] = a.z + a.w;
            t[2] = b.x + b.y;
            t[3] = b.z + b.w;
            cp[0] = make_uint4(0, 0, 0, 0);
            cp[1] = make_uint4(0, 0, 0, 0);
            reinterpret_cast<uint2*>(tn5)[P] = make_uint2(0, 0);
            depth[P] = 0;
        } else {
            const uint4 a = o16.counts[P];
            const uint32_t w4[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) t[q] = (w4[q] & 0xFFFFu) + (w4[q] >> 16);
        }
        for (int q = 0; q < 4; ++q)
            if (t[q]) atomicSub(&tp[(size_t)p * 4 + q], t[q]);
        o16.counts[P] = make_uint4(0, 0, 0, 0);
        o16.tn5[P] = 0u;
        o16.depth[P] = 0;
        if (hc) {
            hc[P] = make_uint4(0, 0, 0, 0);
            ht[P] = 0u;
            hd[P] = 0;
        }
        if (hc8) {  // (the 8-bit target, ABI 7: whichever of the two holds the window)
            hc8[P] = make_uint2(0, 0);
            ht8[P] = 0;
            hd8[P] = 0;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        covered[c] = 0;
        dsum[c] = 0;
        dmax[c] = 0;
    }
}
// One workgroup per cell: pass flag and the two middle order statistics of the
// covered depths (np.median, writers.py:190). Each order statistic is found by a
// binary search over the value range [1, max depth]: count(depth > x) per thread,
// one block reduction per step, both statistics searched in the same steps. No
// atomics and no histogram, whatever the depths. The 16-bit depth row sits in
// registers as packed pairs (36 words per thread at L <= 18432: 8 waves per SIMD,
// so twice the cells in flight of a u32 row), counted with packed 16-bit
// saturating subtracts; a cell with a drained window (exact u32 depths) counts
// from memory instead.
constexpr int kMedRegs = 72;  // register-resident depths per thread (L < 18432), two per word
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// The depth of position p of cell c: the u16 row, or the u32 row in a drained window.
__device__ __forceinline__ uint32_t depth_at(const Geom& g, int c, int p, const uint16_t* __restrict__ d16,
                                            const uint32_t* __restrict__ d32, const uint8_t* __restrict__ wide,
                                            bool anyw) {
    const size_t P = (size_t)c * g.L + p;
    if (anyw && wide[(size_t)c * g.nwin + p / g.W]) return d32[P];
    return d16[P];
}

template <bool kRegs>
__global__ void __launch_bounds__(kBlock) k_median(Geom g, int min_reads, const uint16_t* __restrict__ depth16,
                                                   const uint32_t* __restrict__ depth32,
                                                   const uint8_t* __restrict__ wide,
                                                   const uint32_t* __restrict__ n_reads,
                                                   const uint32_t* __restrict__ covered,
                                                   const uint32_t* __restrict__ dmax,
                                                   uint32_t* __restrict__ med_lo, uint32_t* __restrict__ med_hi,
                                                   uint8_t* __restrict__ passed, DevStats* st) {
    __shared__ uint32_t red[2][2][kBlock / kWave];  // [iteration parity][lo, hi][wave]
    const int c = blockIdx.x;
    const uint32_t n = covered[c];
    const uint32_t nr = n_reads[c];
    const bool pass = n > 0 && nr >= (uint32_t)max(1, min_reads);
    if (!pass) {
        if (threadIdx.x == 0) {
            med_lo[c] = 0;
            med_hi[c] = 0;
            passed[c] = 0;
        }
        return;
    }
    const int L = g.L;
    bool anyw = false;  // a drained window: its depths are in the u32 row
    for (int k = 0; k < g.nwin; ++k) anyw |= wide[(size_t)c * g.nwin + k] != 0;
    // the register path: no drained window (every depth fits 16 bits) and depths below
    // 2^15 (the packed counting's sign-bit compare); otherwise count from memory
    const bool regs = kRegs && !anyw && dmax[c] < 0x8000u;  // (uniform)
    const uint16_t* drow = depth16 + (size_t)c * g.L;
    constexpr int kW = kRegs ? kMedRegs / 2 : 1;
    // 4-byte loads from the 4-byte aligned address at or below the row's start: word j
    // holds positions 2j - s and 2j + 1 - s (s = 1 when the row starts mid-word);
    // halves outside the row are zeroed (a zero is never above a threshold >= 1)
    u16x2 v[kW];
    if (regs) {
        const int s = (int)((reinterpret_cast<uintptr_t>(drow) >> 1) & 1u);  // (uniform)
        const uint32_t* wrow = reinterpret_cast<const uint32_t*>(drow - s);
        const uint32_t jmax = (uint32_t)(L - 1 + s) >> 1;  // the row's last word
        uint32_t w[kW];
#pragma unroll
        for (int k = 0; k < kW; ++k) w[k] = wrow[min((uint32_t)(threadIdx.x + k * kBlock), jmax)];  // (clamped)
#pragma unroll
        for (int k = 0; k < kW; ++k) {
            const int p0 = 2 * (int)(threadIdx.x + k * kBlock) - s;
            const uint32_t keep = (p0 >= 0 && p0 < L ? 0xFFFFu : 0u) | (p0 + 1 < L ? 0xFFFF0000u : 0u);
            const uint32_t x = w[k] & keep;
            v[k] = __builtin_bit_cast(u16x2, x);
        }
    }
    // the k-th smallest covered depth: zero depths sort first, so it is the smallest x
    // with count(depth <= x) >= zeros + k, i.e. count(depth > x) <= L - zeros - k = n - k
    const uint32_t g_lo = n - ((n - 1) / 2 + 1), g_hi = n - (n / 2 + 1);  // counts above to reach
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    // count(depth > m1), count(depth > m2) and, in the last pass, min{depth > m1}
    auto count_pass = [&](int it, uint32_t m1, uint32_t m2, bool want_min, uint32_t& s1, uint32_t& s2) {
        uint32_t c1 = 0, c2 = 0, mn = 0xFFFFFFFFu;
        if (regs) {
            // depths and thresholds are below 2^15 here (regs), so depth > m iff the
            // 16-bit difference m - depth has its top bit set
            const u16x2 M1 = {(uint16_t)m1, (uint16_t)m1}, M2 = {(uint16_t)m2, (uint16_t)m2};
            u16x2 a1 = {0, 0}, a2 = {0, 0};
            if (want_min) {
                u16x2 lo = {0xFFFF, 0xFFFF};
#pragma unroll
                for (int k = 0; k < kW; ++k) {
                    const u16x2 gt = (u16x2)(M1 - v[k]) >> (uint16_t)15;  // 1 where depth > m1
                    a1 += gt;
                    lo = __builtin_elementwise_min(lo, v[k] | (u16x2)(gt - (uint16_t)1));  // 0xFFFF where not
                }
                mn = min((uint32_t)lo.x, (uint32_t)lo.y);
            } else {
#pragma unroll
                for (int k = 0; k < kW; ++k) {
                    a1 += (u16x2)(M1 - v[k]) >> (uint16_t)15;
                    a2 += (u16x2)(M2 - v[k]) >> (uint16_t)15;
                }
            }
            c1 = (uint32_t)a1.x + a1.y;
            c2 = (uint32_t)a2.x + a2.y;
        } else {
            for (int p = threadIdx.x; p < L; p += kBlock) {
                const uint32_t d = depth_at(g, c, p, depth16, depth32, wide, anyw);
                c1 += d > m1;
                c2 += d > m2;
                if (d > m1) mn = min(mn, d);
            }
        }
        c1 = wave_sum(c1);
        const uint32_t x = want_min ? wave_min(mn) : wave_sum(c2);
        if (lane == 0) {
            red[it][0][wid] = c1;
            red[it][1][wid] = x;
        }
        __syncthreads();
        s1 = 0;
        s2 = want_min ? 0xFFFFFFFFu : 0u;
#pragma unroll
        for (int w = 0; w < kBlock / kWave; ++w) {
            s1 += red[it][0][w];
            s2 = want_min ? min(s2, red[it][1][w]) : s2 + red[it][1][w];
        }
    };
    // the lower middle value by a three-way search over [1, max depth] (two thresholds per
    // block reduction); one barrier per step: the partial sums alternate between two LDS
    // sets, and a set is rewritten two steps later, behind the next step's barrier
    uint32_t x0 = 1, x1 = dmax[c];  // the answer lies in [x0, x1]
    int it = 0;
    for (; x0 < x1; it ^= 1) {
        const uint32_t span = x1 - x0, m1 = x0 + span / 3, m2 = x0 + (2 * span) / 3;
        uint32_t s1, s2;
        count_pass(it, m1, m2, false, s1, s2);
        if (s1 <= g_lo) x1 = m1;
        else if (s2 <= g_lo) x0 = m1 + 1, x1 = m2;
        else x0 = m2 + 1;
    }
    const uint32_t lo0 = x0;
    // the upper middle: the lower one when as few depths lie above it as the upper one
    // allows (n odd, or a run of equal values), else the next larger depth
    uint32_t above, next;
    count_pass(it, lo0, lo0, true, above, next);
    const uint32_t hi0 = above <= g_hi ? lo0 : next;
    if (threadIdx.x == 0) {
        med_lo[c] = lo0;
        med_hi[c] = hi0;
        passed[c] = 1;
    }
}

// Run statistics from per-workgroup / per-cell partials (one workgroup of 1024
// threads) at the end of a run: kept reads, barcodes with a kept read, passing
// cells and the two duplicate counters (readers.py:141-144,193-199,
// processors.py:22).
__global__ void __launch_bounds__(1024) k_run_stats(const uint32_t* __restrict__ n_reads,
                                                    const uint8_t* __restrict__ passed, int nc,
                                                    const unsigned long long* __restrict__ dup_part, int nparts,
                                                    DevStats* st, int with_dups,
                                                    const uint32_t* __restrict__ order_bad) {
    __shared__ unsigned long long red[5][1024 / kWave];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    unsigned long long a = 0, b = 0, c = 0, d = 0, e = 0;
    for (int i = threadIdx.x; i < nc; i += 1024) {
        const uint32_t r = n_reads[i];
        a += r;
        b += r != 0u;
        c += passed[i] != 0;
    }
    for (int i = threadIdx.x; i < nparts; i += 1024) {
        d += dup_part[2 * (size_t)i];
        e += dup_part[2 * (size_t)i + 1];
    }
    a = wave_sum(a);
    b = wave_sum(b);
    c = wave_sum(c);
    d = wave_sum(d);
    e = wave_sum(e);
    if (lane == 0) {
        red[0][wid] = a;
        red[1][wid] = b;
        red[2][wid] = c;
        red[3][wid] = d;
        red[4][wid] = e;
    }
    __syncthreads();
    // a streaming push found reads out of coordinate order (k_check_order)
    if (threadIdx.x == 5 && *order_bad) atomicOr(&st->err, ERR_UNSORTED);
    if (threadIdx.x < 5) {
        unsigned long long t = 0;
        for (int w = 0; w < 1024 / kWave; ++w) t += red[threadIdx.x][w];
        if (threadIdx.x == 0) st->filtered = t;
        else if (threadIdx.x == 1) st->n_barcodes = t;
        else if (threadIdx.x == 2) st->cells_passed = t;
        else if (!with_dups) (void)0;  // a streaming run's segments accumulated them (k_dup_accum)
        else if (threadIdx.x == 3) st->dup_pos = t;
        else st->dup_len = t;
    }
}

// Sum of the pileup's per-chunk tally partials: grid (L / 256, Y), thread x sums the 4
// bases of position x over chunks y, y + Y, ... (16-byte loads, four chunks in flight per
// thread) and adds its sums to the zeroed tally. Y is small (tens of chunks per thread):
// the u64 atomics on the same 66k words, Y per word, cost more than the loads (32 per
// word took 0.13 ms at any size).
__global__ void k_tally_reduce(const uint32_t* __restrict__ part, int nchunks, int L4,
                               unsigned long long* __restrict__ tally) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;  // position: 4 u32 partials
    const int L = L4 / 4;
    if (x >= L) return;
    const uint4* p4 = reinterpret_cast<const uint4*>(part);
    const int Y = gridDim.y;
    unsigned long long a[4] = {0, 0, 0, 0};
    auto add = [&](const uint4 v) {
        a[0] += v.x;
        a[1] += v.y;
        a[2] += v.z;
        a[3] += v.w;
    };
    int ch = blockIdx.y;
    for (; ch + 3 * Y < nchunks; ch += 4 * Y) {
        const uint4 v0 = p4[(size_t)ch * L + x], v1 = p4[(size_t)(ch + Y) * L + x];
        const uint4 v2 = p4[(size_t)(ch + 2 * Y) * L + x], v3 = p4[(size_t)(ch + 3 * Y) * L + x];
        add(v0);
        add(v1);
        add(v2);
        add(v3);
    }
    for (; ch < nchunks; ch += Y) add(p4[(size_t)ch * L + x]);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (a[k]) atomicAdd(&tally[(size_t)x * 4 + k], a[k]);
}

// mgp_fetch: the 16-bit result rows widened into the u32 arrays the caller
// receives (drained windows already hold their exact u32 rows). One thread per
// (cell, position).
__global__ void __launch_bounds__(kBlock) k_expand(Geom g, int64_t p0, int64_t npos, Out16 o16,
                                                   uint32_t* __restrict__ counts, uint32_t* __restrict__ tn5,
                                                   uint32_t* __restrict__ depth) {
    const int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (x >= npos) return;
    const int64_t P = p0 + x;  // (cell, position) index of the cell range's first position p0
    const int64_t c = P / g.L, p = P - c * g.L;
    if (o16.wide[c * g.nwin + p / g.W]) return;
    if (counts) {
        const uint4 a = o16.counts[P];
        uint4* cp = reinterpret_cast<uint4*>(counts + P * 8);
        cp[0] = make_uint4(a.x & 0xFFFFu, a.x >> 16, a.y & 0xFFFFu, a.y >> 16);
        cp[1] = make_uint4(a.z & 0xFFFFu, a.z >> 16, a.w & 0xFFFFu, a.w >> 16);
    }
    if (tn5) {
        const uint32_t t = o16.tn5[P];
        reinterpret_cast<uint2*>(tn5)[P] = make_uint2(t & 0xFFFFu, t >> 16);
    }
    if (depth) depth[P] = o16.depth[P];
}

// mgp_set_rows16_target: positions [p0, p1) of every cell's 16-bit rows into the pinned
// host target (device-mapped: vector stores over PCIe, consecutive lanes consecutive
// addresses, so they leave as full-width writes)
__global__ void __launch_bounds__(kBlock) k_rows_to_host(int L, int nc, int p0, int p1, const uint4* __restrict__ c16,
                                                         const uint32_t* __restrict__ t16,
                                                         const uint16_t* __restrict__ d16, uint4* __restrict__ hc,
                                                         uint32_t* __restrict__ ht, uint16_t* __restrict__ hd) {
    const int p = p0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= p1) return;
    for (int c = blockIdx.y; c < nc; c += gridDim.y) {
        const size_t P = (size_t)c * L + p;
        hc[P] = c16[P];
        ht[P] = t16[P];
        hd[P] = d16[P];
    }
}

// the low bytes of the four u16 halves of x, y (x's first)
__device__ __forceinline__ uint32_t low_bytes(uint32_t x, uint32_t y) {
    return (x & 0xFFu) | ((x >> 8) & 0xFF00u) | ((y & 0xFFu) << 16) | ((y << 8) & 0xFF000000u);
}

// The same with the 8-bit target beside (mgp_set_rows_target, ABI 7): a position of a
// (cell, window) whose values all fit a byte (fit8, set by the pileup's flush) leaves as
// 11 bytes instead of 22
__global__ void __launch_bounds__(kBlock) k_rows_to_host8(int L, int nc, int p0, int p1, int W, int nwin,
                                                          const uint4* __restrict__ c16, const uint32_t* __restrict__ t16,
                                                          const uint16_t* __restrict__ d16,
                                                          const uint8_t* __restrict__ fit8, uint4* __restrict__ hc,
                                                          uint32_t* __restrict__ ht, uint16_t* __restrict__ hd,
                                                          uint2* __restrict__ hc8, uint16_t* __restrict__ ht8,
                                                          uint8_t* __restrict__ hd8) {
    const int p = p0 + (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (p >= p1) return;
    const int k = p / W;
    for (int c = blockIdx.y; c < nc; c += gridDim.y) {
        const size_t P = (size_t)c * L + p;
        const uint4 a = c16[P];
        const uint32_t t = t16[P];
        const uint16_t d = d16[P];
        if (fit8[(size_t)c * nwin + k]) {  // (u16 pairs -> bytes: the low byte of each half)
            hc8[P] = make_uint2(low_bytes(a.x, a.y), low_bytes(a.z, a.w));
            ht8[P] = (uint16_t)((t & 0xFFu) | ((t >> 8) & 0xFF00u));
            hd8[P] = (uint8_t)d;
        } else {
            hc[P] = a;
            ht[P] = t;
            hd[P] = d;
        }
    }
}

// mgp_set_cell_range: a pushed batch's barcode indices rebased to the context's cells
// [lo, lo + nc); the others -1 (read_valid drops them like reads without a barcode)
__global__ void k_rebase_bc(int32_t* __restrict__ bc, int64_t n, int32_t lo, int32_t nc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const int32_t v = bc[i];
        bc[i] = (v >= lo && v - lo < nc) ? v - lo : -1;
    }
}

// ---- on-device pairing of a dense batch of 64-byte records (mgp_push_batch) ----
// A streaming producer's batch holds its records in BAM order: a 128-byte line then
// carries two reads of unrelated cells, and the pileup, which gathers each cell's
// reads, fetches every line twice (the resident step on such records: pileup 5.2 ms
// at C4 against 3.5 ms with a cell's records two per line, profiles/r05). After the
// batch lands in a staging buffer, three kernels put the records of one cell two per
// line, the rule of mgp_place_records applied per workgroup range: each workgroup
// ranks its range's reads per cell with LDS atomics (reads the engine drops, and
// reads without a cell of this context, pair among themselves), the ranges' line
// counts are scanned, and the records are copied to line base + rank / 2, half rank & 1.
// Atomic ranks follow the waves' progress, so a line's two reads are near each
// other in the cell's order, not always adjacent; the results never depend on where
// a record sits (every read is found through its rec_off).
constexpr int kPairBlock = 1024;
constexpr int64_t kPairReads = 1 << 18;  // reads of a pairing workgroup's range
#ifndef MGP_PAIR_SPLIT
// copy workgroups per range: a 16M-read batch has only 61 ranges, and one workgroup per
// range left three CUs in four idle (k_pair_place 17.2 ms per C4 step, r5aa trace)
#define MGP_PAIR_SPLIT 16
#endif
constexpr int kPairSplit = MGP_PAIR_SPLIT;
#ifndef MGP_PAIR_NT
#define MGP_PAIR_NT 0  // the record copy's loads and stores non-temporal (A/B)
#endif
constexpr int kPairMaxKeys = 32768;      // cells + 1 whose counters fit a workgroup's LDS

__device__ __forceinline__ int pair_key(int32_t c, uint16_t f, int nc) {
    const uint16_t drop = MGP_FLAG_UNMAPPED | MGP_FLAG_SECONDARY | MGP_FLAG_SUPPLEMENTARY;
    return (c >= 0 && c < nc && !(f & drop)) ? c : nc;
}

__global__ void __launch_bounds__(kPairBlock) k_pair_rank(const int32_t* __restrict__ bc,
                                                          const uint16_t* __restrict__ flag, int64_t n, int nc,
                                                          uint32_t* __restrict__ rank, uint32_t* __restrict__ cntw,
                                                          uint32_t* __restrict__ lines_w) {
    extern __shared__ uint32_t pcnt[];  // [nc + 1]
    __shared__ uint32_t tot;
    const int64_t lo = (int64_t)blockIdx.x * kPairReads, hi = min(n, lo + kPairReads);
    for (int k = threadIdx.x; k <= nc; k += blockDim.x) pcnt[k] = 0u;
    if (threadIdx.x == 0) tot = 0u;
    __syncthreads();
    for (int64_t i = lo + threadIdx.x; i < hi; i += blockDim.x) rank[i] = atomicAdd(&pcnt[pair_key(bc[i], flag[i], nc)], 1u);
    __syncthreads();
    uint32_t lines = 0;
    for (int k = threadIdx.x; k <= nc; k += blockDim.x) {
        const uint32_t x = pcnt[k];
        cntw[(size_t)blockIdx.x * (nc + 1) + k] = x;
        lines += (x + 1u) >> 1;
    }
    lines = wave_sum(lines);
    if ((threadIdx.x & 63) == 0) atomicAdd(&tot, lines);
    __syncthreads();
    if (threadIdx.x == 0) lines_w[blockIdx.x] = tot;
}

// the ranges' first lines (exclusive scan of their line counts, in place)
__global__ void __launch_bounds__(1024) k_pair_scan(uint32_t* __restrict__ lines_w, int nw) {
    __shared__ uint32_t wsum[16], carry;
    block_exclusive_scan(lines_w, nw, lines_w, wsum, &carry);
}

// every record to its line half; rec_off = pay0 + line x 128 + half x 64. Four lanes
// copy a record (16 bytes each); blockIdx.y takes 1 / kPairSplit of range blockIdx.x
// (each workgroup scans the range's key counts into line bases itself).
__global__ void __launch_bounds__(kPairBlock) k_pair_place(const uint4* __restrict__ src, const int32_t* __restrict__ bc,
                                                           const uint16_t* __restrict__ flag, int64_t n, int nc,
                                                           const uint32_t* __restrict__ rank,
                                                           const uint32_t* __restrict__ cntw,
                                                           const uint32_t* __restrict__ wline, uint64_t pay0,
                                                           uint8_t* __restrict__ payload, uint64_t* __restrict__ roff) {
    extern __shared__ uint32_t lbase[];  // [nc + 1]: each key's first line in the range
    __shared__ uint32_t wsum[16], carry;
    const int64_t r0 = (int64_t)blockIdx.x * kPairReads, part = kPairReads / kPairSplit;
    const int64_t lo = r0 + (int64_t)blockIdx.y * part, hi = min(n, lo + part);
    if (lo >= hi) return;
    for (int k = threadIdx.x; k <= nc; k += blockDim.x) lbase[k] = (cntw[(size_t)blockIdx.x * (nc + 1) + k] + 1u) >> 1;
    __syncthreads();
    block_exclusive_scan(lbase, nc + 1, lbase, wsum, &carry);
    const uint32_t w0 = wline[blockIdx.x];
    for (int64_t t = lo * 4 + threadIdx.x; t < hi * 4; t += blockDim.x) {
        const int64_t i = t >> 2;
        const uint32_t r = rank[i];
        const uint64_t line = (uint64_t)w0 + lbase[pair_key(bc[i], flag[i], nc)] + (r >> 1);
        const uint64_t off = pay0 + line * 128u + (uint64_t)(r & 1u) * 64u;
#if MGP_PAIR_NT
        // (A/B: the copy's lines streamed past the caches, the pileup's data left in them)
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + t);
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(payload + off) + (t & 3));
#else
        reinterpret_cast<uint4*>(payload + off)[t & 3] = src[t];
#endif
        if ((t & 3) == 0) roff[i] = off;
    }
}

// mgp_push_batch16: the batch's 16-bit barcode (0xFFFF: none) and |tlen| columns widened
// into the resident 32-bit ones
__global__ void k_widen16(const uint16_t* __restrict__ c16, int64_t n, int32_t* __restrict__ bc,
                          int32_t* __restrict__ tlen) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint32_t b = c16[i];
        bc[i] = b == 0xFFFFu ? -1 : (int32_t)b;
        tlen[i] = (int32_t)c16[n + i];
    }
}

// mgp_push_batch without rec_off: dense records in BAM order, record i at base + i x stride
__global__ void k_dense_off(uint64_t* __restrict__ roff, int64_t n, uint64_t base, uint64_t stride) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) roff[i] = base + (uint64_t)i * stride;
}

// Every pushed batch: each record (offset, header and, for the full layout, its CIGAR)
// must lie inside the batch's payload [pay_lo, pay_hi) (a bad offset, CIGAR offset or a
// dense stride shorter than a full record sets bit 2 of *bad: the run then reports
// MGP_E_INVALID and no kernel reads a record; k_run_init). span != nullptr (a batch
// without span, ABI v3.1): max(reference span of the CIGAR, l_seq) of each read from its
// record (include/mgpileup.h, the three layouts), as the BAM decoder computes it (M, D,
// N, =, X consume the reference). start != nullptr (a batch without start, ABI 4): the
// record's start.
__global__ void k_check_records(const uint8_t* __restrict__ payload, const uint64_t* __restrict__ roff,
                                const uint16_t* __restrict__ flag, int64_t n, uint64_t pay_lo, uint64_t pay_hi,
                                uint32_t* __restrict__ span, int32_t* __restrict__ start,
                                uint32_t* __restrict__ bad) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool err = false;
    if (i < n) {
        const uint64_t r = roff[i];
        const uint32_t f = flag[i];
        const bool p32 = (f & MGP_FLAG_PACK32) != 0, packed = (f & (MGP_FLAG_PACKED | MGP_FLAG_PACK32)) != 0;
        const uint64_t fixed = p32 ? MGP_PACK32_BYTES : packed ? MGP_PACK_BYTES : 16u;
        if (r < pay_lo || (r & 15ull) != 0ull || r + fixed > pay_hi) {
            err = true;
            if (span) span[i] = 0u;
            if (start) start[i] = 0;
        } else {
            const uint8_t* rec = payload + r;
            const uint4 h = *reinterpret_cast<const uint4*>(rec);
            // (a batch without a start column: the record's; every layout holds it)
            if (start) start[i] = p32 ? (int32_t)(h.x & 0xFFFFu) : (int32_t)h.x;
            const uint32_t lseq = p32 ? ((h.x >> 16) & 0xFFu) : packed ? (h.y & 0xFFu) : h.y;
            const uint32_t ncig = p32 ? ((h.x >> 24) & 7u) : packed ? ((h.y >> 8) & 0x7Fu) : (h.z & 0xFFFFu);
            // a full record: qual at +16 and seq at mgp_seq_offset(l_seq) (both read by the
            // pileup for every query position), then the CIGAR at exactly
            // mgp_cigar_offset(l_seq) (include/mgpileup.h), all inside the payload. The
            // CIGAR follows qual and seq, so its end bounds the whole record
            err = !packed && (lseq > (1u << 28) || h.w != mgp_cigar_offset(lseq) || r + h.w + 4ull * ncig > pay_hi);
            if (span) {
                auto consumes = [](uint32_t op) { return op == 0u || op == 2u || op == 3u || op == 7u || op == 8u; };
                uint64_t ref = 0;
                if (packed) {
                    const uint32_t cw[4] = {p32 ? (h.y & 0xFFFFu) : (h.y >> 16), p32 ? (h.y >> 16) : (h.z & 0xFFFFu),
                                            p32 ? (h.z & 0xFFFFu) : (h.z >> 16), p32 ? (h.z >> 16) : (h.w & 0xFFFFu)};
#pragma unroll
                    for (int o = 0; o < 4; ++o)
                        if ((uint32_t)o < ncig && consumes(cw[o] & 15u)) ref += cw[o] >> 4;
                } else if (!err) {
                    const uint32_t* cig = reinterpret_cast<const uint32_t*>(rec + h.w);
                    for (uint32_t o = 0; o < ncig; ++o)
                        if (consumes(cig[o] & 15u)) ref += cig[o] >> 4;
                }
                span[i] = (uint32_t)max<uint64_t>(min<uint64_t>(ref, 0xFFFFFFFFull), lseq);
            }
        }
    }
    if (__ballot(err) && (threadIdx.x & 63) == 0) atomicOr(bad, 2u);
}

__global__ void k_add_u64(uint64_t* __restrict__ a, int64_t n, uint64_t add) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) a[i] += add;
}

// A run's zeroed state (one launch instead of a memset per buffer): per-cell
// counters, first reads (all ones), the first-bin bits F, the check words, stats.
__global__ void k_run_init(int nc, int64_t nF, uint32_t* __restrict__ covered, unsigned long long* __restrict__ dsum,
                           uint32_t* __restrict__ dmax, uint32_t* __restrict__ n_reads, uint8_t* __restrict__ any_paired,
                           uint32_t* __restrict__ first_read, uint32_t* __restrict__ F, uint32_t* __restrict__ ck,
                           DevStats* st, int what, uint32_t* __restrict__ cell_cnt,
                           const uint32_t* __restrict__ order_bad) {
    // what: 1 the run's state (per-cell counters, check words, stats), 2 the first-bin
    // bits F and the scan's cell totals (every segment of a streaming run; the run state
    // only at its first)
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, step = (int64_t)gridDim.x * blockDim.x;
    if (what & 2) {
        for (int64_t i = i0; i < nF; i += step) F[i] = 0u;
        for (int64_t i = i0; i < nc; i += step) cell_cnt[i] = 0u;
    }
    if (what & 1) {
        for (int64_t i = i0; i < nc; i += step) {
            covered[i] = 0u;
            dsum[i] = 0ull;
            dmax[i] = 0u;
            n_reads[i] = 0u;
            any_paired[i] = 0u;
            first_read[i] = 0xFFFFFFFFu;
        }
        if (i0 == 0) {
            ck[0] = 0u;
            ck[1] = 0u;
            *st = DevStats{};
        }
    }
    // a pushed record outside its batch's payload (k_check_records): no kernel of this
    // run reads a record (ERR_BOUNDS stops grouping and pileup at entry)
    if (i0 == 0 && (*order_bad & 2u)) st->err |= ERR_BOUNDS | ERR_BADOFF;
}

// The run's view of the input check: the pileup's halo span and the order check.
// The standalone input check (the fallback path of mgp_run): every bit and the span
// over all resident reads, and the u32 offset column roff32 = rec_off >> 6.
__global__ void k_check_inputs(const uint64_t* __restrict__ roff, const uint16_t* __restrict__ flag,
                               const int32_t* __restrict__ start, const int32_t* __restrict__ tlen,
                               const int32_t* __restrict__ bc, const uint32_t* __restrict__ span, int mito_len,
                               int n_cells, int64_t n, uint32_t* __restrict__ ck, uint32_t* __restrict__ roff32) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = i < n;
    const uint64_t r = in ? roff[i] : 0ull;
    const uint32_t f = in ? flag[i] : 0u;
    const int32_t s0 = in ? start[i] : 0, t0 = in ? tlen[i] : 0;
    const bool uns = in && i > 0 && s0 < start[i - 1];
    const uint32_t sp = in && read_valid(bc[i], (uint16_t)f, n_cells) ? span[i] : 0u;
    const uint32_t at = t0 < 0 ? (uint32_t)(-(int64_t)t0) : (uint32_t)t0;
    if (in) roff32[i] = (uint32_t)(r >> 6);
    uint32_t bits = 0;
    if (in)
        bits = (r != (uint64_t)i * kRecStride ? 1u : 0u) | ((r & 63ull) != 0ull || (r >> 38) != 0ull ? 2u : 0u) |
               (f & MGP_FLAG_PAIRED ? CHK_PAIRED : CHK_UNPAIRED) | (f & MGP_FLAG_NOSEQQUAL ? CHK_NOSEQ : 0u) |
               layout_bit(f) |
               (s0 < 0 || s0 >= mito_len || at >= kCompactTlen ? CHK_WIDEKEY : 0u) | (uns ? CHK_UNSORTED : 0u);
    bits = wave_or(bits);
    const uint32_t msp = wave_max(sp);
    // one atomic per wave at most, and none once the bits are set
    if ((threadIdx.x & 63) == 0) {
        if (msp > __atomic_load_n(ck + 1, __ATOMIC_RELAXED)) atomicMax(ck + 1, msp);
        if (bits && (__atomic_load_n(ck, __ATOMIC_RELAXED) & bits) != bits) atomicOr(ck, bits);
    }
}

// a streaming segment's duplicate counts into the run's stats (k_run_stats takes
// them from the partials of a resident run's one pass B)
__global__ void __launch_bounds__(256) k_dup_accum(const unsigned long long* __restrict__ dup_part, int nparts,
                                                    DevStats* st) {
    __shared__ unsigned long long red[2][256 / kWave];
    unsigned long long d = 0, e = 0;
    for (int i = threadIdx.x; i < nparts; i += 256) {
        d += dup_part[2 * (size_t)i];
        e += dup_part[2 * (size_t)i + 1];
    }
    d = wave_sum(d);
    e = wave_sum(e);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red[0][wid] = d;
        red[1][wid] = e;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        unsigned long long t = 0;
        for (int w = 0; w < 256 / kWave; ++w) t += red[threadIdx.x][w];
        if (t) atomicAdd(threadIdx.x == 0 ? &st->dup_pos : &st->dup_len, t);
    }
}

// Streaming pushes: coordinate order of a pushed batch, and against the batch before
// (a segment sees only the start bins it runs, so a read out of order outside them
// would go unnoticed); the flag stays set until the resident set is replaced.
__global__ void k_check_order(const int32_t* __restrict__ start, int64_t i0, int64_t i1, uint32_t* __restrict__ bad) {
    const int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool uns = i < i1 && i > 0 && start[i] < start[i - 1];
    if (__ballot(uns) && (threadIdx.x & 63) == 0) atomicOr(bad, 1u);
}

__global__ void k_order_err(const uint32_t* __restrict__ bad, DevStats* st) {
    if (threadIdx.x == 0 && *bad) atomicOr(&st->err, ERR_UNSORTED);
}

// the run's ERR_RESPEC as a count in the all-reduced buffer (slot after the
// tallies): every rank then sees whether any rank has to rerun, and all do
__global__ void k_respec_slot(const DevStats* st, unsigned long long* slot) {
    if (threadIdx.x == 0) *slot = (st->err & ERR_RESPEC) ? 1ull : 0ull;
}

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// r03 v52 re-sweep with the chunks taken largest first (ab_geo_v52.txt): fewer, larger
// chunks now cost the pileup little and halve the tally partials the reduction reads
// beside the medians (C4 6.63 -> 6.60 ms at 8192 workgroups; 1250 cells 1.022 -> 0.992
// ms at 8 cells per chunk)
#ifndef MGP_PILE_WG
#define MGP_PILE_WG 8192
#endif
#ifndef MGP_PILE_MIN_CPB
#define MGP_PILE_MIN_CPB 8
#endif
#ifndef MGP_PILE_WG_STREAM
#define MGP_PILE_WG_STREAM 2048  // a streaming run's pileup workgroups per window (MGP_PILE_WG_STREAM env too)
#endif
// Cells per pileup chunk. A resident run launches every window at once: ~MGP_PILE_WG
// workgroups over the windows, at least MGP_PILE_MIN_CPB cells: each (chunk, window)
// workgroup writes a tally partial row (16 B per position) that k_tally_reduce reads
// back, so at few cells per chunk the partials, not the cells, set the cost (1250
// cells at 1 per chunk: 331 MB, the same as C4's 10k cells at 8; at 4 per chunk the
// 1250-cell step is 11 % shorter). A streaming run launches the pileup per segment,
// about one window each: there the chunks are sized for ~wg_stream workgroups per
// window (C4: 2000 chunks of 5 cells instead of 625 of 16, which left 40 % of the
// 1024 workgroup slots of a one-window launch empty). Chunks of one cell are allowed
// there (r05, `abs_r5ad.txt`): the 8-GPU share of C4 (1250 cells) had 625 workgroups per
// launch at 2 cells each, the pileup 1.19 -> 0.95 ms per step at 1 (the step unchanged).
static void set_pile_chunks(Geom& g, bool stream, int wg_stream, int min_cpb_stream = 1) {
    int64_t cpb;
    if (stream) {
        cpb = std::max<int64_t>(min_cpb_stream, ((int64_t)g.nc + wg_stream - 1) / std::max(1, wg_stream));
    } else {
        const int64_t target = MGP_PILE_WG;
        cpb = std::max<int64_t>(MGP_PILE_MIN_CPB, ((int64_t)g.nc * g.nwin + target - 1) / target);
    }
    g.cpb = (int)std::min<int64_t>(cpb, 64);
    g.nchunks = g.nc > 0 ? (g.nc + g.cpb - 1) / g.cpb : 0;
}
static inline unsigned blocks_for(int64_t n, int bs = kBlock) { return (unsigned)((n + bs - 1) / bs); }

static int configure_geometry(mgp_ctx* ctx) {
    const mgp_config& c = ctx->cfg;
    Geom& g = ctx->g;
    g.L = c.mito_len;
    g.G = 8;
    g.nb_reg = (g.L + g.G - 1) / g.G;
    g.nbins = g.nb_reg + 1;
    g.nwin = (g.L + MGP_WIN - 1) / MGP_WIN;  // ~MGP_WIN positions per window
    g.W = (g.L + g.nwin - 1) / g.nwin;
    g.W = ((g.W + g.G - 1) / g.G) * g.G;   // multiple of the bin width
    g.nwin = (g.L + g.W - 1) / g.W;
    if (g.W > kMaxPosPerThread * kBlock) return set_err(MGP_E_INVALID, "window too wide");
    // plane pitch of the pileup tile: a compile-time power of two, so a base's plane
    // offset is a shift folded into the address add (A/B: no bank-conflict cost)
    g.Wp = kTilePitch;
    g.nc = c.n_cells;
    // cells per pileup chunk (a resident run's; a streaming run sets its own)
    set_pile_chunks(g, false, MGP_PILE_WG_STREAM);
    return MGP_OK;
}

extern "C" {

int mgp_abi_version(void) { return MGP_ABI_VERSION; }
const char* mgp_last_error(void) { return g_err.c_str(); }

int mgp_device_count(int* out) {
    if (!out) return set_err(MGP_E_INVALID, "null out");
    HIP_TRY(hipGetDeviceCount(out));
    return MGP_OK;
}

int mgp_host_alloc(int64_t bytes, void** out) {
    if (!out || bytes < 0) return set_err(MGP_E_INVALID, "bad args");
    HIP_TRY(hipHostMalloc(out, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault));
    return MGP_OK;
}
int mgp_host_free(void* p) {
    if (p) HIP_TRY(hipHostFree(p));
    return MGP_OK;
}

int mgp_open(const mgp_config* cfg, int hip_device, mgp_ctx** out) {
    if (!cfg || !out) return set_err(MGP_E_INVALID, "null config/out");
    if (cfg->mito_len <= 0 || cfg->mito_len > (1 << 24)) return set_err(MGP_E_INVALID, "mito_len out of range");
    if (cfg->n_cells < 0) return set_err(MGP_E_INVALID, "n_cells < 0");
    if (cfg->dedup_mode < 0 || cfg->dedup_mode > 2) return set_err(MGP_E_INVALID, "dedup_mode out of range");
    if (cfg->flags & ~(MGP_CFG_KEEP_TN5 | MGP_CFG_STREAM)) return set_err(MGP_E_INVALID, "unknown config.flags bits");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (hip_device < 0 || hip_device >= ndev)
        return set_err(MGP_E_INVALID, "hip_device " + std::to_string(hip_device) + " not present (" +
                                          std::to_string(ndev) + " devices)");
    HIP_TRY(hipSetDevice(hip_device));
    mgp_ctx* ctx = new mgp_ctx();
    ctx->cfg = *cfg;
    ctx->dev = hip_device;
    ctx->stream = (cfg->flags & MGP_CFG_STREAM) != 0;
    int r = configure_geometry(ctx);
    if (r != MGP_OK) {
        delete ctx;
        return r;
    }
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, hip_device));
    // the histogram's LDS per workgroup (one workgroup of 8 waves per CU either way): up to
    // 150 KiB, ~37k cells per slice (C5's 100k cells in 3 slices, not 5 at 96 KiB);
    // MGP_HIST_LDS_KB / MGP_HIST_XCD=0 for A/B. The same budget bounds grouping pass A's
    // per-group counters (its 512-thread form when they fit and a workgroup gets at least
    // MGP_GA_WIDE_MIN reads; kGANBlock = 128 threads otherwise: beyond ~140k cells and for
    // the small multi-GPU shares)
    size_t hist_kb = 150;
    if (const char* e = std::getenv("MGP_HIST_LDS_KB")) hist_kb = (size_t)std::max(4L, std::strtol(e, nullptr, 10));
    ctx->lds_hist_max_cells = (int)std::min<size_t>(prop.sharedMemPerBlock, hist_kb * 1024) / 4;
    if (const char* e = std::getenv("MGP_HIST_XCD")) ctx->hist_xcd = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("MGP_HIST_NARROW")) ctx->hist_narrow = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("MGP_HIST_BOUNDS")) ctx->hist_bounds = std::strtol(e, nullptr, 10) != 0;
    if (const char* e = std::getenv("MGP_GA_WIDE_MIN")) ctx->ga_wide_min = std::strtoll(e, nullptr, 10);
    if (const char* e = std::getenv("MGP_HIST_SLICE_CELLS")) {  // tests: force several histogram slices
        const long v = std::strtol(e, nullptr, 10);
        if (v >= kGroup) ctx->hist_slice_cells = (int)(v / kGroup * kGroup);
    }
    if (const char* e = std::getenv("MGP_GROUP_WIDE")) ctx->group_wide = std::strtol(e, nullptr, 10) != 0;
    // kernels whose dynamic LDS may exceed 64 KiB (gfx950: up to 160 KiB per workgroup);
    // best effort: the runtime may already allow it without the attribute
    {
        const int lds_max = (int)prop.sharedMemPerBlock;
        (void)hipFuncSetAttribute((const void*)k_bin_count<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  lds_max);
        (void)hipFuncSetAttribute((const void*)k_bin_count<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  lds_max);
        for (const void* f : {(const void*)k_group_a<kOffDense, false, kGABlock>, (const void*)k_group_a<kOffR32, false, kGABlock>,
                              (const void*)k_group_a<kOffR64, false, kGABlock>, (const void*)k_group_a<kOffDense, true, kGABlock>,
                              (const void*)k_group_a<kOffR32, true, kGABlock>, (const void*)k_group_a<kOffSpec, true, kGABlock>,
                              (const void*)k_group_a<kOffDense, false, kGANBlock>, (const void*)k_group_a<kOffR32, false, kGANBlock>,
                              (const void*)k_group_a<kOffR64, false, kGANBlock>, (const void*)k_group_a<kOffDense, true, kGANBlock>,
                              (const void*)k_group_a<kOffR32, true, kGANBlock>, (const void*)k_group_a<kOffSpec, true, kGANBlock>})
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
        (void)hipFuncSetAttribute((const void*)k_pileup<kLayAny>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
        (void)hipFuncSetAttribute((const void*)k_pileup<kLayP64>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
        (void)hipFuncSetAttribute((const void*)k_pileup<kLayP32>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
        (void)hipFuncSetAttribute((const void*)k_pair_rank, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
        (void)hipFuncSetAttribute((const void*)k_pair_place, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max);
        (void)hipGetLastError();
        if ((size_t)ctx->g.L * 4 + 2048 > prop.sharedMemPerBlock) {
            delete ctx;
            return set_err(MGP_E_INVALID, "mito_len too large for the per-cell median LDS buffer");
        }
    }
    HIP_TRY(hipStreamCreateWithFlags(&ctx->s_comp, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&ctx->s_copy, hipStreamNonBlocking));
    if (const char* e = std::getenv("MGP_DEV_PAIR")) ctx->dev_pair = std::atoi(e) != 0;
    for (int i = 0; i < 2; ++i) HIP_TRY(hipEventCreateWithFlags(&ctx->ev_stage[i], hipEventDisableTiming));
    if (const char* e = std::getenv("MGP_SEG_MIN_WIN")) ctx->seg_min_win = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("MGP_ROWS_WG")) ctx->rows_wg = std::max(1, std::atoi(e));
    ctx->pile_wg_stream = MGP_PILE_WG_STREAM;
    if (const char* e = std::getenv("MGP_PILE_WG_STREAM")) ctx->pile_wg_stream = std::max(1, std::atoi(e));
    if (const char* e = std::getenv("MGP_PILE_MIN_CPB_STREAM")) ctx->pile_min_cpb_stream = std::max(1, std::atoi(e));
    HIP_TRY(hipStreamCreateWithFlags(&ctx->s_side, hipStreamNonBlocking));
    // the rows target's kernel stores into pinned host memory: each store waits on the
    // host link, and a CU with a queue of them serves other kernels' loads late (the
    // streamed run's last medians and tally ran 20-30x slower beside it, round 5).
    // MGP_D2H_CUS=N keeps that stream's kernels on N CUs spread over the XCDs (0: any)
    {
        int d2h_cus = 0;
        if (const char* e = std::getenv("MGP_D2H_CUS")) d2h_cus = std::max(0, std::atoi(e));
        hipDeviceProp_t prop{};
        if (d2h_cus > 0 && hipGetDeviceProperties(&prop, hip_device) == hipSuccess &&
            d2h_cus < prop.multiProcessorCount) {
            const int ncu = prop.multiProcessorCount;
            std::vector<uint32_t> mask((size_t)(ncu + 31) / 32, 0u);
            // every (ncu / N)-th CU: the CU ids interleave the XCDs, so the set covers each
            const int step = std::max(1, ncu / d2h_cus);
            for (int k = 0; k < d2h_cus; ++k) {
                const int cu = (k * step) % ncu;
                mask[(size_t)cu / 32] |= 1u << (cu % 32);
            }
            HIP_TRY(hipExtStreamCreateWithCUMask(&ctx->s_d2h, (uint32_t)mask.size(), mask.data()));
        } else {
            HIP_TRY(hipStreamCreateWithFlags(&ctx->s_d2h, hipStreamNonBlocking));
        }
    }
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_rows, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_copy, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&ctx->ev_bits, hipEventDisableTiming));
    HIP_TRY(hipHostMalloc((void**)&ctx->h_bits, 8, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&ctx->host_stats, sizeof(DevStats), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&ctx->h_respec, 8, hipHostMallocDefault));
    *ctx->h_respec = 0ull;
    *ctx->host_stats = DevStats{};
    MGP_TRY(ctx->roff_irregular.ensure(8));
    MGP_TRY(ctx->order_bad.ensure(4));
    HIP_TRY(hipMemsetAsync(ctx->order_bad.p, 0, 4, ctx->s_copy));
    HIP_TRY(hipEventRecord(ctx->ev_copy, ctx->s_copy));
    for (int r = 0; r < mgp_ctx::kRing; ++r)
        for (int s = 0; s < ST_N; ++s) {
            HIP_TRY(hipEventCreate(&ctx->ev[r][s][0]));
            HIP_TRY(hipEventCreate(&ctx->ev[r][s][1]));
        }
    if (cfg->reserve_reads > 0) {
        const size_t n = (size_t)cfg->reserve_reads;
        MGP_TRY(ctx->start.ensure(n * 4));
        MGP_TRY(ctx->bc.ensure(n * 4));
        MGP_TRY(ctx->tlen.ensure(n * 4));
        MGP_TRY(ctx->flag.ensure(n * 2));
        MGP_TRY(ctx->mapq.ensure(n));
        MGP_TRY(ctx->span.ensure(n * 4));
        MGP_TRY(ctx->roff.ensure(n * 8));
        MGP_TRY(ctx->roff32.ensure(n * 4));
    }
    if (cfg->reserve_payload > 0) MGP_TRY(ctx->payload.ensure((size_t)cfg->reserve_payload));
    *out = ctx;
    return MGP_OK;
}

void mgp_close(mgp_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->dev);
    (void)hipStreamSynchronize(ctx->s_comp);
    (void)hipStreamSynchronize(ctx->s_copy);
    (void)hipStreamSynchronize(ctx->s_side);
    (void)hipStreamSynchronize(ctx->s_d2h);
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    DevBuf* bufs[] = {&ctx->start,     &ctx->bc,        &ctx->tlen,     &ctx->flag,       &ctx->mapq,
                      &ctx->span,      &ctx->roff,      &ctx->payload,  &ctx->bin_start,  &ctx->gel2,
                      &ctx->roff32,    &ctx->roff_irregular, &ctx->dup_part, &ctx->order_bad,
                      &ctx->H,         &ctx->P,         &ctx->cell_cnt, &ctx->cell_base,  &ctx->pel,
                      &ctx->PG,        &ctx->F,         &ctx->chunk_perm,
                      &ctx->tally_part, &ctx->tally,   &ctx->n_reads,    &ctx->any_paired,
                      &ctx->passed,    &ctx->covered,   &ctx->dsum,     &ctx->dmax,       &ctx->med_lo,
                      &ctx->med_hi,    &ctx->first_read, &ctx->counts,  &ctx->tn5,        &ctx->depth,
                      &ctx->stats,     &ctx->counts16,  &ctx->tn5_16,  &ctx->depth16,    &ctx->wide,
                      &ctx->fit8};
    for (DevBuf* b : bufs) b->release();
    for (auto e : ctx->seg_ev) (void)hipEventDestroy(e);
    for (int r = 0; r < mgp_ctx::kRing; ++r)
        for (int s = 0; s < ST_N; ++s) {
            (void)hipEventDestroy(ctx->ev[r][s][0]);
            (void)hipEventDestroy(ctx->ev[r][s][1]);
        }
    (void)hipEventDestroy(ctx->ev_copy);
    (void)hipEventDestroy(ctx->ev_fork);
    (void)hipEventDestroy(ctx->ev_join);
    (void)hipEventDestroy(ctx->ev_bits);
    if (ctx->h_bits) (void)hipHostFree(ctx->h_bits);
    if (ctx->host_stats) (void)hipHostFree(ctx->host_stats);
    if (ctx->h_respec) (void)hipHostFree(ctx->h_respec);
    (void)hipStreamDestroy(ctx->s_comp);
    (void)hipStreamDestroy(ctx->s_copy);
    (void)hipStreamDestroy(ctx->s_side);
    (void)hipStreamDestroy(ctx->s_d2h);
    for (int i = 0; i < 2; ++i) {
        if (ctx->ev_stage[i]) (void)hipEventDestroy(ctx->ev_stage[i]);
        ctx->stage[i].release();
        ctx->col16[i].release();
    }
    ctx->pair_rank.release();
    ctx->pair_cnt.release();
    ctx->pair_lines.release();
    (void)hipEventDestroy(ctx->ev_rows);
    delete ctx;
}

// Finish what the compute streams have queued (buffers are about to be replaced).
static int drain_compute(mgp_ctx* ctx) {
    HIP_TRY(hipSetDevice(ctx->dev));
    HIP_TRY(hipStreamSynchronize(ctx->s_comp));
    HIP_TRY(hipStreamSynchronize(ctx->s_side));
    return MGP_OK;
}

// A streaming run in progress is abandoned (the resident set is replaced).
static int drain_stream(mgp_ctx* ctx) {
    MGP_TRY(drain_compute(ctx));
    ctx->seg_open = false;
    ctx->w_done = 0;
    ctx->stream_off = false;
    return MGP_OK;
}

static int ensure_inputs(mgp_ctx* ctx, int64_t n_total, int64_t pay_total, bool preserve) {
    const size_t n = (size_t)n_total;
    const size_t used = preserve ? (size_t)ctx->n : 0;
    hipStream_t s = ctx->s_copy;
    // growing replaces a buffer that queued kernels (a streaming run's segments) may read
    if (ctx->start.cap < n * 4 || ctx->payload.cap < (size_t)pay_total + 256) MGP_TRY(drain_compute(ctx));
    MGP_TRY(ctx->start.ensure(n * 4, preserve, used * 4, s));
    MGP_TRY(ctx->bc.ensure(n * 4, preserve, used * 4, s));
    MGP_TRY(ctx->tlen.ensure(n * 4, preserve, used * 4, s));
    MGP_TRY(ctx->flag.ensure(n * 2, preserve, used * 2, s));
    MGP_TRY(ctx->mapq.ensure(n, preserve, used, s));
    MGP_TRY(ctx->span.ensure(n * 4, preserve, used * 4, s));
    MGP_TRY(ctx->roff.ensure(n * 8, preserve, used * 8, s));
    MGP_TRY(ctx->roff32.ensure(n * 4, preserve, used * 4, s));
    MGP_TRY(ctx->payload.ensure((size_t)pay_total + 256, preserve, preserve ? (size_t)ctx->pay : 0, s));
    return MGP_OK;
}

static int stream_segments(mgp_ctx* ctx, int64_t last_start, uint16_t last_flag);

// A batch's copies and kernels (mgp_push_batch, mgp_push_batch16: c16 = the 16-bit
// barcode and |tlen| columns, then b->bc / b->tlen are unused)
static int push_impl(mgp_ctx* ctx, const mgp_batch* b, const uint16_t* bc16, const uint16_t* tlen16);

int mgp_push_batch(mgp_ctx* ctx, const mgp_batch* b) {
    if (!ctx || !b) return set_err(MGP_E_INVALID, "null ctx/batch");
    if (b->n_reads < 0 || b->payload_bytes < 0) return set_err(MGP_E_INVALID, "negative sizes");
    if (b->n_reads == 0) return MGP_OK;
    if (!b->bc || !b->tlen || !b->flag || !b->mapq || !b->payload) return set_err(MGP_E_INVALID, "null batch array");
    return push_impl(ctx, b, nullptr, nullptr);
}

int mgp_push_batch16(mgp_ctx* ctx, const mgp_batch16* b) {
    if (!ctx || !b) return set_err(MGP_E_INVALID, "null ctx/batch");
    if (b->n_reads < 0 || b->payload_bytes < 0) return set_err(MGP_E_INVALID, "negative sizes");
    if (b->n_reads == 0) return MGP_OK;
    if (!b->bc || !b->abs_tlen || !b->flag || !b->mapq || !b->payload)
        return set_err(MGP_E_INVALID, "null batch array");
    if (ctx->g.nc > 0xFFFF) return set_err(MGP_E_INVALID, "16-bit barcode indices need n_cells <= 65535");
    // with a cell range the columns hold whole-whitelist indices up to cell_hi - 1, and
    // 0xFFFF is the no-barcode sentinel
    if (ctx->cell_range && (int64_t)ctx->cell_lo + ctx->g.nc > 0xFFFF)
        return set_err(MGP_E_INVALID, "16-bit barcode indices with a cell range need cell_hi <= 65535");
    mgp_batch w{};
    w.n_reads = b->n_reads;
    w.flag = b->flag;
    w.mapq = b->mapq;
    w.payload = b->payload;
    w.payload_bytes = b->payload_bytes;
    return push_impl(ctx, &w, b->bc, b->abs_tlen);
}

static int push_impl(mgp_ctx* ctx, const mgp_batch* b, const uint16_t* bc16, const uint16_t* tlen16) {
    // rec_off NULL: dense records in BAM order (record i at i x payload_bytes / n_reads);
    // span NULL: the spans come from the records' CIGARs on the device
    const bool dense = b->rec_off == nullptr;
    const int64_t stride = dense ? b->payload_bytes / b->n_reads : 0;
    if (dense && (stride * b->n_reads != b->payload_bytes || stride < 16 || stride % 16 != 0))
        return set_err(MGP_E_INVALID, "rec_off NULL needs payload_bytes = n_reads x a record stride that is a "
                                      "multiple of 16");
    if (ctx->n + b->n_reads > (int64_t)0xFFFFFFFEll)
        return set_err(MGP_E_INVALID, "more than 2^32-2 resident reads per context; shard or batch the run");
    HIP_TRY(hipSetDevice(ctx->dev));
    const int64_t n0 = ctx->n, nb = b->n_reads;
    const int64_t pay0 = (ctx->pay + 255) & ~int64_t(255);  // keeps the batch's record alignment
    const int nc = ctx->g.nc;
    // a dense batch of 64-byte slots lands in a staging buffer and is paired on the device
    const bool pair = dense && stride == 64 && ctx->dev_pair && nb >= 65536 && nc + 1 <= kPairMaxKeys;
    const int npw = pair ? (int)((nb + kPairReads - 1) / kPairReads) : 0;
    // paired: at most one line per two reads plus one half-empty line per key and range
    const int64_t pay_b = pair ? 64 * (nb + (int64_t)npw * (nc + 2)) : b->payload_bytes;
    MGP_TRY(ensure_inputs(ctx, n0 + nb, pay0 + pay_b, true));
    hipStream_t s = ctx->s_copy, sp = ctx->s_comp;
    // the copy stream only copies (the link never waits on a kernel); the batch's
    // kernels follow on the compute stream, ahead of the segments it completes
    const int j = ctx->stage_i;
    const bool staged = pair || bc16;  // (the staging slot j is used: wait for its last readers)
    if (pair) {
        MGP_TRY(ctx->stage[j].ensure((size_t)b->payload_bytes));
        MGP_TRY(ctx->pair_rank.ensure((size_t)nb * 4));
        MGP_TRY(ctx->pair_cnt.ensure((size_t)npw * (nc + 1) * 4));
        MGP_TRY(ctx->pair_lines.ensure((size_t)npw * 4));
    }
    if (bc16) MGP_TRY(ctx->col16[j].ensure((size_t)nb * 4));
    if (staged) HIP_TRY(hipStreamWaitEvent(s, ctx->ev_stage[j], 0));  // the kernels that read slot j last
    if (b->start) HIP_TRY(hipMemcpyAsync(ctx->start.as<int32_t>() + n0, b->start, nb * 4, hipMemcpyHostToDevice, s));
    if (bc16) {
        HIP_TRY(hipMemcpyAsync(ctx->col16[j].as<uint16_t>(), bc16, nb * 2, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(ctx->col16[j].as<uint16_t>() + nb, tlen16, nb * 2, hipMemcpyHostToDevice, s));
    } else {
        HIP_TRY(hipMemcpyAsync(ctx->bc.as<int32_t>() + n0, b->bc, nb * 4, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(ctx->tlen.as<int32_t>() + n0, b->tlen, nb * 4, hipMemcpyHostToDevice, s));
    }
    HIP_TRY(hipMemcpyAsync(ctx->flag.as<uint16_t>() + n0, b->flag, nb * 2, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(ctx->mapq.as<uint8_t>() + n0, b->mapq, nb, hipMemcpyHostToDevice, s));
    if (b->span)
        HIP_TRY(hipMemcpyAsync(ctx->span.as<uint32_t>() + n0, b->span, nb * 4, hipMemcpyHostToDevice, s));
    if (!dense)
        HIP_TRY(hipMemcpyAsync(ctx->roff.as<uint64_t>() + n0, b->rec_off, nb * 8, hipMemcpyHostToDevice, s));
    if (b->payload_bytes)
        HIP_TRY(hipMemcpyAsync(pair ? ctx->stage[j].as<uint8_t>() : ctx->payload.as<uint8_t>() + pay0, b->payload,
                               b->payload_bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipEventRecord(ctx->ev_copy, s));
    HIP_TRY(hipStreamWaitEvent(sp, ctx->ev_copy, 0));
    if (bc16) {
        k_widen16<<<blocks_for(nb), kBlock, 0, sp>>>(ctx->col16[j].as<uint16_t>(), nb, ctx->bc.as<int32_t>() + n0,
                                                     ctx->tlen.as<int32_t>() + n0);
        HIP_TRY(hipGetLastError());
    }
    if (ctx->cell_range) {
        k_rebase_bc<<<blocks_for(nb), kBlock, 0, sp>>>(ctx->bc.as<int32_t>() + n0, nb, ctx->cell_lo, nc);
        HIP_TRY(hipGetLastError());
    }
    if (pair) {
        const size_t lds = (size_t)(nc + 1) * 4;
        k_pair_rank<<<npw, kPairBlock, lds, sp>>>(ctx->bc.as<int32_t>() + n0, ctx->flag.as<uint16_t>() + n0, nb, nc,
                                                  ctx->pair_rank.as<uint32_t>(), ctx->pair_cnt.as<uint32_t>(),
                                                  ctx->pair_lines.as<uint32_t>());
        HIP_TRY(hipGetLastError());
        k_pair_scan<<<1, 1024, 0, sp>>>(ctx->pair_lines.as<uint32_t>(), npw);
        HIP_TRY(hipGetLastError());
        k_pair_place<<<dim3((unsigned)npw, (unsigned)kPairSplit), kPairBlock, lds, sp>>>(
            ctx->stage[j].as<uint4>(), ctx->bc.as<int32_t>() + n0, ctx->flag.as<uint16_t>() + n0, nb, nc,
            ctx->pair_rank.as<uint32_t>(), ctx->pair_cnt.as<uint32_t>(), ctx->pair_lines.as<uint32_t>(),
            (uint64_t)pay0, ctx->payload.as<uint8_t>(), ctx->roff.as<uint64_t>() + n0);
        HIP_TRY(hipGetLastError());
    } else if (dense) {
        k_dense_off<<<blocks_for(nb), kBlock, 0, sp>>>(ctx->roff.as<uint64_t>() + n0, nb, (uint64_t)pay0,
                                                       (uint64_t)stride);
        HIP_TRY(hipGetLastError());
    } else if (pay0) {
        k_add_u64<<<blocks_for(nb), kBlock, 0, sp>>>(ctx->roff.as<uint64_t>() + n0, nb, (uint64_t)pay0);
        HIP_TRY(hipGetLastError());
    }
    if (staged) {  // slot j's readers are queued: the next batch that uses it waits for them
        HIP_TRY(hipEventRecord(ctx->ev_stage[j], sp));
        ctx->stage_i ^= 1;
    }
    // every record inside the batch's payload (and, without a span / start column, its
    // span / start from the record)
    k_check_records<<<blocks_for(nb), kBlock, 0, sp>>>(
        ctx->payload.as<uint8_t>(), ctx->roff.as<uint64_t>() + n0, ctx->flag.as<uint16_t>() + n0, nb, (uint64_t)pay0,
        (uint64_t)(pay0 + pay_b), b->span ? nullptr : ctx->span.as<uint32_t>() + n0,
        b->start ? nullptr : ctx->start.as<int32_t>() + n0, ctx->order_bad.as<uint32_t>());
    HIP_TRY(hipGetLastError());
    if (ctx->stream) {
        k_check_order<<<blocks_for(nb), kBlock, 0, sp>>>(ctx->start.as<int32_t>(), n0, n0 + nb,
                                                         ctx->order_bad.as<uint32_t>());
        HIP_TRY(hipGetLastError());
    }
    ctx->n = n0 + nb;
    ctx->pay = pay0 + pay_b;
    ctx->ran = false;
    ctx->no_spec = false;
    ctx->bits_cached = false;
    // streaming: the windows this batch completes go through the hot path now,
    // behind its copies, while the caller pushes the next batch
    if (ctx->stream) {
        // the batch's last start: from its column, or from its last record on the host
        int64_t last = 0;
        if (b->start) {
            last = b->start[nb - 1];
        } else {
            const uint64_t ro = dense ? (uint64_t)(nb - 1) * (uint64_t)stride : b->rec_off[nb - 1];
            const uint16_t f = b->flag[nb - 1];
            if (ro + 4 <= (uint64_t)b->payload_bytes) {
                const uint8_t* r = b->payload + ro;
                if (f & MGP_FLAG_PACK32) {
                    last = (int64_t)((uint32_t)r[0] | ((uint32_t)r[1] << 8));
                } else {
                    int32_t v;
                    std::memcpy(&v, r, 4);
                    last = v;
                }
            }
        }
        MGP_TRY(stream_segments(ctx, last, b->flag[nb - 1]));
    }
    return MGP_OK;
}

int mgp_reset(mgp_ctx* ctx) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    HIP_TRY(hipSetDevice(ctx->dev));
    HIP_TRY(hipStreamSynchronize(ctx->s_copy));
    HIP_TRY(hipStreamSynchronize(ctx->s_comp));
    HIP_TRY(hipStreamSynchronize(ctx->s_d2h));  // (a rows target's copies read rows the next run rewrites)
    HIP_TRY(hipMemsetAsync(ctx->order_bad.p, 0, 4, ctx->s_copy));
    HIP_TRY(hipEventRecord(ctx->ev_copy, ctx->s_copy));
    ctx->n = 0;
    ctx->pay = 0;
    ctx->ran = false;
    ctx->no_spec = false;
    ctx->bits_cached = false;
    ctx->seg_open = false;
    ctx->w_done = 0;
    ctx->stream_off = false;
    return MGP_OK;
}

int mgp_resident(mgp_ctx* ctx, int64_t* n_reads, int64_t* payload_bytes) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    if (n_reads) *n_reads = ctx->n;
    if (payload_bytes) *payload_bytes = ctx->pay;
    return MGP_OK;
}

static int ensure_run_buffers(mgp_ctx* ctx) {
    const Geom& g = ctx->g;
    // a streaming run sizes the per-read scratch for the announced read count at once
    // (growing it between segments would wait for the queued ones)
    const size_t n = (size_t)std::max<int64_t>(std::max<int64_t>(ctx->n, ctx->stream ? ctx->cfg.reserve_reads : 0), 1);
    if (ctx->pel.cap < n * 4 || ctx->gel2.cap < n * sizeof(GElem)) MGP_TRY(drain_compute(ctx));
    const size_t nc = (size_t)std::max(g.nc, 1);
    const size_t L = (size_t)g.L;
    MGP_TRY(ctx->bin_start.ensure((size_t)(g.nbins + 1) * 4));
    MGP_TRY(ctx->H.ensure((size_t)(g.nbins + 1) * nc * 4));
    MGP_TRY(ctx->PG.ensure((size_t)g.nbins * kParts * ((nc + kGroup - 1) / kGroup) * 4));
    MGP_TRY(ctx->F.ensure((size_t)g.nbins * ((nc + 31) / 32) * 4));
    MGP_TRY(ctx->P.ensure((size_t)((g.nbins + 31) / 32 + 1) * nc * 4));
    MGP_TRY(ctx->cell_cnt.ensure(nc * 4));
    MGP_TRY(ctx->cell_base.ensure(nc * 4));
    MGP_TRY(ctx->chunk_perm.ensure((size_t)std::max(g.nchunks, 1) * 4));
    MGP_TRY(ctx->pel.ensure(n * 4));
    MGP_TRY(ctx->gel2.ensure(n * sizeof(GElem)));
    MGP_TRY(ctx->bin_valid.ensure((size_t)(g.nbins + 1) * 4));
    MGP_TRY(ctx->bin_base.ensure((size_t)(g.nbins + 1) * 4));
    MGP_TRY(ctx->bucket_off.ensure((size_t)g.nbins * ((nc + kGroup - 1) / kGroup + 1) * 4));
    MGP_TRY(ctx->tally_part.ensure((size_t)std::max(g.nchunks, 1) * L * 16));
    MGP_TRY(ctx->tally.ensure(L * 4 * 8 + 8));  // + the all-reduced ERR_RESPEC slot
    MGP_TRY(ctx->n_reads.ensure(nc * 4));
    MGP_TRY(ctx->any_paired.ensure(nc));
    MGP_TRY(ctx->passed.ensure(nc));
    MGP_TRY(ctx->covered.ensure(nc * 4));
    MGP_TRY(ctx->dsum.ensure(nc * 8));
    MGP_TRY(ctx->dmax.ensure(nc * 4));
    MGP_TRY(ctx->med_lo.ensure(nc * 4));
    MGP_TRY(ctx->med_hi.ensure(nc * 4));
    MGP_TRY(ctx->first_read.ensure(nc * 4));
    MGP_TRY(ctx->counts.ensure(nc * L * 32));
    MGP_TRY(ctx->tn5.ensure(nc * L * 8));
    MGP_TRY(ctx->depth.ensure(nc * L * 4));
    MGP_TRY(ctx->counts16.ensure(nc * L * 16));
    MGP_TRY(ctx->tn5_16.ensure(nc * L * 4));
    MGP_TRY(ctx->depth16.ensure(nc * L * 2));
    MGP_TRY(ctx->wide.ensure(nc * (size_t)std::max(g.nwin, 1)));
    MGP_TRY(ctx->fit8.ensure(nc * (size_t)std::max(g.nwin, 1)));
    MGP_TRY(ctx->stats.ensure(sizeof(DevStats)));
    return MGP_OK;
}

static Out16 out16_of(mgp_ctx* ctx) {
    Out16 o;
    o.counts = ctx->counts16.as<uint4>();
    o.tn5 = ctx->tn5_16.as<uint32_t>();
    o.depth = ctx->depth16.as<uint16_t>();
    o.wide = ctx->wide.as<uint8_t>();
    o.fit8 = ctx->fit8.as<uint8_t>();
    return o;
}

// Stage events: each is a marker between two kernels of the stream (about 11 us
// of idle GPU at a stage boundary on MI355X), so mgp_set_stage_timing can keep the
// pileup's only. A streaming segment (slot < 0) records none.
#define STAGE_ON(st) (slot >= 0 && (ctx->stage_all || (st) == ST_PILEUP))
#define STAGE_BEGIN(st) \
    if (STAGE_ON(st)) { HIP_TRY(hipEventRecord(ctx->ev[slot][st][0], s)); ctx->stage_ran[slot][st] = true; }
#define STAGE_END(st) \
    if (STAGE_ON(st)) HIP_TRY(hipEventRecord(ctx->ev[slot][st][1], s))

// One segment of a run: the resident reads whose start bins lie in the segment
// through the input check, the histogram, the scan, both grouping passes and the
// pileup of windows [w0, w1). A resident run is one segment over every window.
struct Seg {
    int w0, w1;   // pileup windows
    int bhi;      // start bins [seg_lo_bin(w0), bhi) (nbins: through the overflow bin)
    bool first;   // the run's first segment: zero the run's state
    bool stream;  // a streaming segment: speculative compact grouping, no host wait
    bool last;    // the run's last segment: its rows leave after the medians (run_finish)
};

// k_rows_to_host (or k_rows_to_host8 with an 8-bit target) over positions [p0, p1) on the
// D2H stream
static int rows_launch(mgp_ctx* ctx, dim3 gr, int p0, int p1) {
    const Geom& g = ctx->g;
    const mgp_rows16& t = ctx->rows_tgt;
    if (ctx->rows8_on) {
        const mgp_rows8& t8 = ctx->rows8_tgt;
        k_rows_to_host8<<<gr, kBlock, 0, ctx->s_d2h>>>(
            g.L, g.nc, p0, p1, g.W, g.nwin, ctx->counts16.as<uint4>(), ctx->tn5_16.as<uint32_t>(),
            ctx->depth16.as<uint16_t>(), ctx->fit8.as<uint8_t>(), reinterpret_cast<uint4*>(t.counts),
            reinterpret_cast<uint32_t*>(t.tn5), t.depth, reinterpret_cast<uint2*>(t8.counts),
            reinterpret_cast<uint16_t*>(t8.tn5), t8.depth);
    } else {
        k_rows_to_host<<<gr, kBlock, 0, ctx->s_d2h>>>(g.L, g.nc, p0, p1, ctx->counts16.as<uint4>(),
                                                    ctx->tn5_16.as<uint32_t>(), ctx->depth16.as<uint16_t>(),
                                                    reinterpret_cast<uint4*>(t.counts),
                                                    reinterpret_cast<uint32_t*>(t.tn5), t.depth);
    }
    HIP_TRY(hipGetLastError());
    return MGP_OK;
}

// The rows of windows' positions [p0, p1) of every cell to the host target, on the D2H
// stream behind the compute stream's work so far (mgp_set_rows16_target): written by a
// kernel into the mapped pinned target (a strided 2D copy of 10k rows per segment runs as
// row-by-row DMA transfers: 4x slower overall)
static int rows_copy(mgp_ctx* ctx, int p0, int p1) {
    const Geom& g = ctx->g;
    const int nc = g.nc;
    HIP_TRY(hipEventRecord(ctx->ev_rows, ctx->s_comp));
    HIP_TRY(hipStreamWaitEvent(ctx->s_d2h, ctx->ev_rows, 0));
    // a few hundred workgroups looping over the cells: the stores wait on the host
    // link, and a grid of one workgroup per (cell, 256 positions) held every CU
    // slot of the device while they drained, starving the kernels of the next
    // segment and the run's medians (MGP_ROWS_WG)
    const unsigned gx = (unsigned)((p1 - p0 + kBlock - 1) / kBlock);
    dim3 gr(gx, (unsigned)std::max(1, std::min(std::min(nc, 65535), ctx->rows_wg / (int)gx)));
    return rows_launch(ctx, gr, p0, p1);
}

static int run_segment(mgp_ctx* ctx, const Seg& sg, int slot, int& dup_parts, int& pair_mode) {
    const Geom g = ctx->g;
    const int64_t n = ctx->n;
    const int nc = g.nc;
    hipStream_t s = ctx->s_comp;
    HIP_TRY(hipStreamWaitEvent(s, ctx->ev_copy, 0));
    DevStats* st = ctx->stats.as<DevStats>();
    dup_parts = 0;
    pair_mode = 0;
    if (nc > 0) {  // the run's per-cell counters, stats, check words and first-bin bits in one launch
        const int64_t nF = (int64_t)g.nbins * ((nc + 31) / 32);
        k_run_init<<<std::max(1u, std::min(1024u, blocks_for(std::max<int64_t>(nc, nF)))), kBlock, 0, s>>>(
            nc, nF, ctx->covered.as<uint32_t>(), ctx->dsum.as<unsigned long long>(), ctx->dmax.as<uint32_t>(),
            ctx->n_reads.as<uint32_t>(), ctx->any_paired.as<uint8_t>(), ctx->first_read.as<uint32_t>(),
            ctx->F.as<uint32_t>(), ctx->roff_irregular.as<uint32_t>(), st, sg.first ? 3 : 2,
            ctx->cell_cnt.as<uint32_t>(), ctx->order_bad.as<uint32_t>());
        HIP_TRY(hipGetLastError());
    } else {
        if (sg.first) HIP_TRY(hipMemsetAsync(st, 0, sizeof(DevStats), s));
        return MGP_OK;
    }
    const int ngroups = (nc + kGroup - 1) / kGroup;
    // 1. per (start bin, cell) histogram + per (bin, part, group) counts + bin bounds, and
    // the flag bits of the input check (pairedness / SEQ mix, record layout). They travel
    // to pinned host memory while the scan runs; the host picks the grouping and pileup
    // variants from them below (a streaming segment takes the speculative variants and
    // leaves the check to the device).
    STAGE_BEGIN(ST_HIST);
    if (n == 0) HIP_TRY(hipMemsetAsync(ctx->H.p, 0, (size_t)(g.nbins + 1) * nc * 4, s));
    if (n == 0) HIP_TRY(hipMemsetAsync(ctx->bin_start.p, 0, (size_t)(g.nbins + 1) * 4, s));
    if (n > 0) {
        // cells per slice: whole 64-cell groups, counts + group totals within the LDS budget
        // (32-bit counters: 65 words per group; 8-bit: 17). 8-bit counters when the cells
        // need more than one 32-bit slice (MGP_HIST_NARROW=0/1 forces the choice)
        const int wide_cells = ctx->lds_hist_max_cells / (kGroup + 1) * kGroup;
        const bool narrow = ctx->hist_narrow >= 0 ? ctx->hist_narrow != 0 : nc > wide_cells;
        int lds_cells = narrow ? ctx->lds_hist_max_cells / (kGroup / 4 + 1) * kGroup : wide_cells;
        if (ctx->hist_slice_cells > 0) lds_cells = std::min(lds_cells, ctx->hist_slice_cells);
        const int slice = nc <= lds_cells ? nc : lds_cells;
        const int nslices = (nc + slice - 1) / slice;
        const size_t lds_words = narrow ? (size_t)(slice + 3) / 4 + (slice + kGroup - 1) / kGroup
                                        : (size_t)slice + (slice + kGroup - 1) / kGroup;
        // (the narrow kernel's 32-bit recount takes at least one group: 65 words)
        const size_t lds = std::max<size_t>(lds_words, narrow ? kGroup + 1 : 0) * 4;
        const bool xcd = nslices > 1 && ctx->hist_xcd;
        const dim3 gh = xcd ? dim3((unsigned)(8 * nslices * ((g.nbins + 7) / 8))) : dim3((unsigned)g.nbins, (unsigned)nslices);
        // the bins' bounds searched up front, one thread per bin, instead of by two lanes of
        // each histogram workgroup (r04 A/B: C5 hist 2.54 -> 2.44 ms, C4 0.298 -> 0.293, the
        // 1250-cell share 0.070 -> 0.066; MGP_HIST_BOUNDS=0 searches per workgroup)
        const bool pre = ctx->hist_bounds != 0;
        if (pre) {
            k_bin_bounds<<<(g.nbins + 1 + 255) / 256, 256, 0, s>>>(ctx->start.as<int32_t>(), n, g,
                                                                   ctx->bin_start.as<uint32_t>());
            HIP_TRY(hipGetLastError());
        }
        auto kern = narrow ? k_bin_count<true> : k_bin_count<false>;
        kern<<<gh, narrow ? MGP_HIST_NBLOCK : kHistBlock, lds, s>>>(
            ctx->start.as<int32_t>(), ctx->bc.as<int32_t>(), ctx->flag.as<uint16_t>(), n, g, slice,
            ctx->H.as<uint32_t>(), ctx->PG.as<uint32_t>(), ngroups, ctx->bin_start.as<uint32_t>(),
            ctx->bin_valid.as<uint32_t>(), ctx->roff_irregular.as<uint32_t>(), st, sg.w0, sg.bhi,
            xcd ? -nslices : nslices, pre ? 1 : 0);
        HIP_TRY(hipGetLastError());
        // (a rerun on an unchanged resident set takes the cached bits: no copy, no wait)
        if (!sg.stream && !(ctx->bits_cached && !ctx->no_spec)) {
            HIP_TRY(hipMemcpyAsync(ctx->h_bits, ctx->roff_irregular.p, 8, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipEventRecord(ctx->ev_bits, s));
        }
    }
    STAGE_END(ST_HIST);

    // 2. cell-major exclusive scan of the histogram
    STAGE_BEGIN(ST_SCAN);
    const int RB = 32;
    const int nrb = (g.nbins + RB - 1) / RB;
    dim3 g2((nc + kBlock - 1) / kBlock, nrb);
    k_scan_colsum<<<g2, kBlock, 0, s>>>(ctx->H.as<uint32_t>(), g.nbins, nc, RB, ctx->P.as<uint32_t>(),
                                        ctx->cell_cnt.as<uint32_t>());
    k_scan_cells<<<1, 1024, 0, s>>>(ctx->cell_cnt.as<uint32_t>(), nc, ctx->cell_base.as<uint32_t>(), g.cpb,
                                    g.nchunks, ctx->chunk_perm.as<uint32_t>(), ctx->bin_valid.as<uint32_t>(),
                                    n > 0 ? g.nbins : 0, ctx->bin_base.as<uint32_t>());
    k_scan_apply<<<g2, kBlock, 0, s>>>(ctx->H.as<uint32_t>(), ctx->P.as<uint32_t>(),
                                       ctx->cell_base.as<uint32_t>(), ctx->cell_cnt.as<uint32_t>(), g.nbins, nc,
                                       RB, nrb, ctx->F.as<uint32_t>());
    HIP_TRY(hipGetLastError());
    STAGE_END(ST_SCAN);

    // The input check's flag bits (the GPU runs the scan meanwhile). When they allow
    // compact grouping elements, pass A checks the rest on the reads it loads (kOffSpec);
    // otherwise, or once that failed on the resident reads (no_spec, ERR_RESPEC), the
    // standalone check takes every bit first (k_check_inputs, then a host wait).
    STAGE_BEGIN(ST_GROUP_A);
    int unit = 6;  // the pileup element's record offset unit: 64 bytes (32 for 32-byte records on the
                   // speculative path), or 16 bytes when some record is not 64-byte aligned
    bool spec = false, track = false;
    uint32_t check_layout = 0;  // the one packed layout the variants assume, verified on the device
    int layout = kLayP64;  // the pileup's instantiation (the record layouts present)
    ctx->roff_mode = kOffR64;
    ctx->read_bits = 0;
    constexpr uint32_t kLayBits = CHK_FULL | CHK_P64 | CHK_P32;
    if (n > 0 && sg.stream) {
        // the layout the run's first batch showed; check_stats (pass B) makes the run rerun
        // resident if another one turns up
        spec = true;
        ctx->roff_mode = kOffSpec;
        layout = ctx->stream_layout;
        unit = layout == kLayP32 ? 5 : 6;
    } else if (n > 0) {
        const bool cached = ctx->bits_cached && !ctx->no_spec;
        if (!cached) HIP_TRY(hipEventSynchronize(ctx->ev_bits));
        const uint32_t fb = cached ? ctx->cached_bits : ctx->h_bits[0];
        const uint32_t lb = fb & kLayBits;
        const int su = lb == CHK_P32 ? 5 : 6;
        track = ((fb & CHK_PAIRED) && (fb & CHK_UNPAIRED)) || (fb & CHK_NOSEQ);
        spec = !ctx->no_spec && !ctx->group_wide && !track && (lb == CHK_P64 || lb == CHK_P32) &&
               (uint64_t)ctx->pay < ((uint64_t)(PE_KEEP & PE_OFF) << su);
        // only the speculative choice is cached: it needs nothing but these bits
        ctx->bits_cached = spec;
        ctx->cached_bits = fb;
        if (spec) {
            ctx->roff_mode = kOffSpec;
            ctx->read_bits = fb;
            unit = su;
            check_layout = cached ? lb : 0u;
        } else {
            k_check_inputs<<<blocks_for(n), kBlock, 0, s>>>(
                ctx->roff.as<uint64_t>(), ctx->flag.as<uint16_t>(), ctx->start.as<int32_t>(),
                ctx->tlen.as<int32_t>(), ctx->bc.as<int32_t>(), ctx->span.as<uint32_t>(), ctx->cfg.mito_len,
                ctx->cfg.n_cells, n, ctx->roff_irregular.as<uint32_t>(), ctx->roff32.as<uint32_t>());
            HIP_TRY(hipGetLastError());
            HIP_TRY(hipMemcpyAsync(ctx->h_bits, ctx->roff_irregular.p, 8, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipEventRecord(ctx->ev_bits, s));
            HIP_TRY(hipEventSynchronize(ctx->ev_bits));
            const uint32_t irr = ctx->h_bits[0];
            ctx->roff_mode = !(irr & 1u) ? kOffDense : !(irr & 2u) ? kOffR32 : kOffR64;
            ctx->read_bits = irr;
            unit = ctx->roff_mode == kOffR64 ? 4 : 6;
        }
        const uint32_t rl = ctx->read_bits & kLayBits;
        layout = rl == CHK_P32 ? kLayP32 : (rl == 0u || rl == CHK_P64) ? kLayP64 : kLayAny;
    }

    // 3. stable grouping into cell-major order (two passes), duplicate marking in pass B;
    // 8-byte elements when the resident reads allow them (GCompact: one packed layout)
    const uint32_t rbits = ctx->read_bits;
    const bool compact = spec || (!ctx->group_wide && ctx->roff_mode != kOffR64 && unit == 6 && !track &&
                                  layout != kLayAny && !(rbits & CHK_WIDEKEY));
    // pileup elements: 31 offset bits (compact) or 30 and the layout bits (wide), below PE_KEEP
    const uint32_t pe_off = compact ? PE_OFF : PE_OFF30;
    if (n > 0 && (uint64_t)ctx->pay >= ((uint64_t)(PE_KEEP & pe_off) << unit))
        return set_err(MGP_E_INVALID, "payload of " + std::to_string(ctx->pay) + " bytes above the " +
                                          std::to_string((uint64_t)(PE_KEEP & pe_off) << unit) +
                                          "-byte limit of one context for this record placement; shard the "
                                          "cells or place records at 64-byte offsets");
    if (n > 0) {
        int gbits = 0;
        while (gbits < 31 && (1 << gbits) < ngroups) ++gbits;
        auto a_lds_for = [&](int blk) {
            return (size_t)ngroups * (1 + 2 * (blk / kWave)) * 4 + (size_t)((nc + 31) / 32) * 4;
        };
        // the 512-thread form pays with two or more 4096-read steps per (bin, part) workgroup;
        // smaller sets (the 4- and 8-GPU shares of C4) run the 128-thread form (r04 A/B at
        // 1250 / 2500 / 5000 cells: 0.39 / 0.60 / 0.93 ms at 512 threads, 0.22 / 0.47 / 1.07 at 128)
        const int64_t per_wg = n / std::max<int64_t>(1, (int64_t)g.nbins * kParts);
        const bool a_wide = a_lds_for(kGABlock) <= (size_t)ctx->lds_hist_max_cells * 4 && per_wg >= ctx->ga_wide_min;
        const size_t a_lds = a_lds_for(a_wide ? kGABlock : kGANBlock);
        if (a_lds > (size_t)ctx->lds_hist_max_cells * 4)
            return set_err(MGP_E_INVALID, "too many cells for one context (grouping LDS)");
        if (gbits > 16) return set_err(MGP_E_INVALID, "too many cells for one context (cell groups)");
        if ((uint64_t)ctx->pay >= (1ull << GM_LCELL_SHIFT))
            return set_err(MGP_E_INVALID, "payload too large (record offsets must stay below 2^50)");
        dim3 ga((unsigned)g.nbins, kParts);
        auto launch_a = [&](auto kern_wide, auto kern_256) {
            auto kern = a_wide ? kern_wide : kern_256;
            kern<<<ga, a_wide ? kGABlock : kGANBlock, a_lds, s>>>(
                n, ctx->start.as<int32_t>(), ctx->bc.as<int32_t>(), ctx->tlen.as<int32_t>(),
                ctx->flag.as<uint16_t>(), ctx->mapq.as<uint8_t>(), ctx->roff.as<uint64_t>(),
                ctx->roff32.as<uint32_t>(), ctx->span.as<uint32_t>(), ctx->bin_start.as<uint32_t>(),
                ctx->PG.as<uint32_t>(), ctx->F.as<uint32_t>(), ctx->bin_base.as<uint32_t>(), g, ngroups, gbits,
                ctx->cfg.min_mapq, ctx->bucket_off.as<uint32_t>(), ctx->gel2.as<GElem>(),
                ctx->first_read.as<uint32_t>(), ctx->roff_irregular.as<uint32_t>(), st, sg.w0, sg.bhi, unit);
        };
        if (spec) {
            launch_a(k_group_a<kOffSpec, true, kGABlock>, k_group_a<kOffSpec, true, kGANBlock>);
        } else if (compact) {
            if (ctx->roff_mode == kOffDense) launch_a(k_group_a<kOffDense, true, kGABlock>, k_group_a<kOffDense, true, kGANBlock>);
            else launch_a(k_group_a<kOffR32, true, kGABlock>, k_group_a<kOffR32, true, kGANBlock>);
        } else if (ctx->roff_mode == kOffDense) {
            launch_a(k_group_a<kOffDense, false, kGABlock>, k_group_a<kOffDense, false, kGANBlock>);
        } else if (ctx->roff_mode == kOffR32) {
            launch_a(k_group_a<kOffR32, false, kGABlock>, k_group_a<kOffR32, false, kGANBlock>);
        } else {
            launch_a(k_group_a<kOffR64, false, kGABlock>, k_group_a<kOffR64, false, kGANBlock>);
        }
        HIP_TRY(hipGetLastError());
    }
    STAGE_END(ST_GROUP_A);
    STAGE_BEGIN(ST_GROUP_B);
    if (MGP_ABL_A == 1) HIP_TRY(hipMemsetAsync(ctx->gel2.p, 0, (size_t)n * sizeof(GElem), s));  // ablation
    if (MGP_ABL_B >= 2) HIP_TRY(hipMemsetAsync(ctx->pel.p, 0xFF, (size_t)n * 4, s));  // ablation: nothing piles
    if (n > 0) {
        // about MGP_GB_WG workgroups (many per slot: 4 fit a CU, so a grid of a few
        // slot-rounds leaves a tail); bins per workgroup at most kMaxRbB, whose
        // bucket sizes the workgroup keeps in LDS
        const int64_t tgt = MGP_GB_WG;
        const int rb = std::min(kMaxRbB, std::max(1, (int)(((int64_t)ngroups * g.nbins + tgt - 1) / tgt)));
#if MGP_GB_XCD
        const unsigned nwg_b = (unsigned)ngroups * (unsigned)((g.nbins + rb - 1) / rb);
        dim3 gb(8u * ((nwg_b + 7u) / 8u));
#else
        dim3 gb((unsigned)ngroups, (unsigned)((g.nbins + rb - 1) / rb));
#endif
        dup_parts = ngroups * ((g.nbins + rb - 1) / rb);  // (one partial per (group, range) workgroup)
        MGP_TRY(ctx->dup_part.ensure((size_t)dup_parts * 16));
        // duplicates of the halo bins of a streaming segment were counted by an earlier one
        const int cnt_lo = sg.w0 > 0 ? (int)((int64_t)sg.w0 * g.W / g.G) : 0;
        // per-read pairedness / SEQ tracking only when the reads mix paired and
        // unpaired ones or some read lacks SEQ/QUAL
        // pass B's first workgroup also takes the input check's span and order bits into
        // the run's stats (the pileup's halo); a streaming segment also checks there the
        // flag bits its variants assume (check_stats)
        const uint32_t spec_layout = sg.stream ? (layout == kLayP32 ? CHK_P32 : CHK_P64) : check_layout;
        auto launch_b = [&](auto kern, auto* gel) {
            kern<<<gb, kGBBlock, 0, s>>>(gel, ctx->bucket_off.as<uint32_t>(), ctx->H.as<uint32_t>(),
                                       g, ngroups, rb, ctx->cfg.dedup_mode, unit, ctx->pel.as<uint32_t>(),
                                       ctx->any_paired.as<uint8_t>(), ctx->dup_part.as<unsigned long long>(), st,
                                       cnt_lo, ctx->roff_irregular.as<uint32_t>(), spec_layout);
        };
        if (compact) launch_b(k_group_b<false, GCompact>, ctx->gel2.as<unsigned long long>());
        else if (track) launch_b(k_group_b<true, GWide>, ctx->gel2.as<GElem>());
        else launch_b(k_group_b<false, GWide>, ctx->gel2.as<GElem>());
        pair_mode = sg.stream ? -1 : track ? 0 : (rbits & CHK_PAIRED) ? 1 : 0;
        HIP_TRY(hipGetLastError());
        if (sg.stream) {
            k_dup_accum<<<1, 256, 0, s>>>(ctx->dup_part.as<unsigned long long>(), dup_parts, st);
            HIP_TRY(hipGetLastError());
        }
    }
    STAGE_END(ST_GROUP_B);

    // 5. dedup + pileup + strand filter + stats
    STAGE_BEGIN(ST_PILEUP);
    PileCfg pc;
    pc.min_baseq = ctx->cfg.min_baseq;
    pc.min_dist = ctx->cfg.min_dist_from_end;
    pc.min_reads = ctx->cfg.min_reads;
    pc.dedup_mode = ctx->cfg.dedup_mode;
    pc.max_bias = ctx->cfg.max_strand_bias;
    pc.bias_active = ctx->cfg.max_strand_bias < 1.0;
    pc.keep_tn5 = (ctx->cfg.flags & MGP_CFG_KEEP_TN5) != 0;
    // a streaming segment (slot < 0) times its pileup launch into the coming run's
    // segment events (that run's slot is runs % kRing: mgp_run takes it)
    hipEvent_t* sev = nullptr;
    if (slot < 0 && sg.stream && sg.w1 > sg.w0) {
        const int rs = (int)(ctx->runs % mgp_ctx::kRing);
        if (sg.first) ctx->seg_n[rs] = 0;
        if (ctx->seg_ev.empty()) {
            ctx->seg_ev.assign((size_t)mgp_ctx::kRing * mgp_ctx::kSegEv * 2, nullptr);
            for (auto& e : ctx->seg_ev) HIP_TRY(hipEventCreate(&e));
        }
        if (ctx->seg_n[rs] < mgp_ctx::kSegEv) sev = &ctx->seg_ev[((size_t)rs * mgp_ctx::kSegEv + ctx->seg_n[rs]) * 2];
        ctx->seg_n[rs] = std::min(ctx->seg_n[rs] + 1, mgp_ctx::kSegEv + 1);
    }
    if (sg.w1 > sg.w0) {
        dim3 gp(g.nchunks, sg.w1 - sg.w0);
        const size_t psm = (size_t)kTilePlanes * kTilePitch * 4;
        if (sev) HIP_TRY(hipEventRecord(sev[0], s));
        auto pile_kern = layout == kLayP32 ? k_pileup<kLayP32> : layout == kLayP64 ? k_pileup<kLayP64>
                                                                                    : k_pileup<kLayAny>;
        pile_kern<<<gp, kBlock, psm, s>>>(g, pc, ctx->payload.as<uint8_t>(), ctx->pel.as<uint32_t>(), unit, pe_off,
                                         ctx->H.as<uint32_t>(), out16_of(ctx), ctx->counts.as<uint32_t>(),
                                         ctx->tn5.as<uint32_t>(), ctx->depth.as<uint32_t>(),
                                         ctx->n_reads.as<uint32_t>(), ctx->any_paired.as<uint8_t>(), pair_mode,
                                         ctx->covered.as<uint32_t>(), ctx->dsum.as<unsigned long long>(),
                                         ctx->dmax.as<uint32_t>(), ctx->tally_part.as<uint32_t>(), st, sg.w0,
                                         ctx->roff_irregular.as<uint32_t>(), ctx->chunk_perm.as<uint32_t>());
        HIP_TRY(hipGetLastError());
        if (sev) HIP_TRY(hipEventRecord(sev[1], s));
        // the windows' rows are final now (all cells): to the host target behind them,
        // while later batches are still being copied in (mgp_set_rows16_target). The
        // run's last segment leaves its rows to run_finish: host-bound stores queued in
        // the memory system slowed every kernel beside them, and the medians and tallies
        // of the run's tail ran 20-30x slower under them (round 5)
        if (ctx->rows_on) {
            const int p0 = sg.w0 * g.W, p1 = std::min(g.L, sg.w1 * g.W);
            if (sg.last) {
                ctx->rows_p0 = p0;
                ctx->rows_p1 = p1;
                ctx->rows_pending = true;
            } else {
                MGP_TRY(rows_copy(ctx, p0, p1));
            }
        }
    }
    STAGE_END(ST_PILEUP);
    return MGP_OK;
}

// The end of a run: min-reads gate, tallies, medians and pass flags, run statistics,
// the tally all-reduce, and the stats' copy to pinned host memory.
static int run_finish(mgp_ctx* ctx, int slot, int dup_parts, bool streamed) {
    const Geom g = ctx->g;
    const int nc = g.nc;
    hipStream_t s = ctx->s_comp;
    DevStats* st = ctx->stats.as<DevStats>();
    unsigned long long* tally = ctx->tally.as<unsigned long long>();
    if (nc > 0) {
        // 6. min-reads gate
        if (ctx->cfg.min_reads > 1) {
            STAGE_BEGIN(ST_GATE);
            // with a rows target, the rows already sent (the last segment's copies run on
            // the D2H stream) are final before the gate rewrites the dropped cells there
            const bool tgt = ctx->rows_on, tgt8 = tgt && ctx->rows8_on;
            if (tgt) {
                HIP_TRY(hipEventRecord(ctx->ev_rows, ctx->s_d2h));
                HIP_TRY(hipStreamWaitEvent(s, ctx->ev_rows, 0));
            }
            k_gate_fixup<<<nc, kBlock, 0, s>>>(g, ctx->cfg.min_reads, ctx->n_reads.as<uint32_t>(),
                                               out16_of(ctx), ctx->counts.as<uint32_t>(), ctx->tn5.as<uint32_t>(),
                                               ctx->depth.as<uint32_t>(), ctx->covered.as<uint32_t>(),
                                               ctx->dsum.as<unsigned long long>(), ctx->dmax.as<uint32_t>(),
                                               ctx->tally_part.as<uint32_t>(),
                                               tgt ? reinterpret_cast<uint4*>(ctx->rows_tgt.counts) : nullptr,
                                               tgt ? reinterpret_cast<uint32_t*>(ctx->rows_tgt.tn5) : nullptr,
                                               tgt ? ctx->rows_tgt.depth : nullptr,
                                               tgt8 ? reinterpret_cast<uint2*>(ctx->rows8_tgt.counts) : nullptr,
                                               tgt8 ? reinterpret_cast<uint16_t*>(ctx->rows8_tgt.tn5) : nullptr,
                                               tgt8 ? ctx->rows8_tgt.depth : nullptr);
            HIP_TRY(hipGetLastError());
            STAGE_END(ST_GATE);
        }

        // 7. tallies on the side stream, concurrent with the medians (both only read
        // the pileup's outputs); joined before the stats and the all-reduce
        {
            hipStream_t s2 = ctx->s_side;
            HIP_TRY(hipEventRecord(ctx->ev_fork, s));
            HIP_TRY(hipStreamWaitEvent(s2, ctx->ev_fork, 0));
            if (STAGE_ON(ST_TALLY)) {
                HIP_TRY(hipEventRecord(ctx->ev[slot][ST_TALLY][0], s2));
                ctx->stage_ran[slot][ST_TALLY] = true;
            }
            HIP_TRY(hipMemsetAsync(tally, 0, (size_t)g.L * 32, s2));
            dim3 gt(blocks_for((int64_t)g.L), (unsigned)std::max(1, std::min(g.nchunks / 16, 16)));
            k_tally_reduce<<<gt, kBlock, 0, s2>>>(ctx->tally_part.as<uint32_t>(), g.nchunks, g.L * 4, tally);
            HIP_TRY(hipGetLastError());
            if (STAGE_ON(ST_TALLY)) HIP_TRY(hipEventRecord(ctx->ev[slot][ST_TALLY][1], s2));
            HIP_TRY(hipEventRecord(ctx->ev_join, s2));
        }

        // 8. medians + pass flags, run statistics
        STAGE_BEGIN(ST_MEDIAN);
        if (g.L < kMedRegs * kBlock)
            k_median<true><<<nc, kBlock, 0, s>>>(g, ctx->cfg.min_reads, ctx->depth16.as<uint16_t>(),
                                                 ctx->depth.as<uint32_t>(), ctx->wide.as<uint8_t>(),
                                                 ctx->n_reads.as<uint32_t>(), ctx->covered.as<uint32_t>(),
                                                 ctx->dmax.as<uint32_t>(), ctx->med_lo.as<uint32_t>(),
                                                 ctx->med_hi.as<uint32_t>(), ctx->passed.as<uint8_t>(), st);
        else
            k_median<false><<<nc, kBlock, 0, s>>>(g, ctx->cfg.min_reads, ctx->depth16.as<uint16_t>(),
                                                  ctx->depth.as<uint32_t>(), ctx->wide.as<uint8_t>(),
                                                  ctx->n_reads.as<uint32_t>(), ctx->covered.as<uint32_t>(),
                                                  ctx->dmax.as<uint32_t>(), ctx->med_lo.as<uint32_t>(),
                                                  ctx->med_hi.as<uint32_t>(), ctx->passed.as<uint8_t>(), st);
        HIP_TRY(hipGetLastError());
        k_run_stats<<<1, 1024, 0, s>>>(ctx->n_reads.as<uint32_t>(), ctx->passed.as<uint8_t>(), nc,
                                       ctx->dup_part.as<unsigned long long>(), streamed ? 0 : dup_parts, st,
                                       streamed ? 0 : 1, ctx->order_bad.as<uint32_t>());
        HIP_TRY(hipGetLastError());
        STAGE_END(ST_MEDIAN);
        HIP_TRY(hipStreamWaitEvent(s, ctx->ev_join, 0));
        // the last segment's rows, now that the medians and tallies are done
        if (ctx->rows_pending && ctx->rows_on) MGP_TRY(rows_copy(ctx, ctx->rows_p0, ctx->rows_p1));
        ctx->rows_pending = false;
    } else {
        ctx->rows_pending = false;
        HIP_TRY(hipMemsetAsync(tally, 0, (size_t)g.L * 32, s));
        // (with cells, k_run_stats takes the streaming order check)
        k_order_err<<<1, 64, 0, s>>>(ctx->order_bad.as<uint32_t>(), st);
        HIP_TRY(hipGetLastError());
    }

    // the wide flags of the rows target (the pileups of every segment are behind)
    if (ctx->rows_on && nc > 0) {
        HIP_TRY(hipEventRecord(ctx->ev_rows, s));
        HIP_TRY(hipStreamWaitEvent(ctx->s_d2h, ctx->ev_rows, 0));
        HIP_TRY(hipMemcpyAsync(ctx->rows_tgt.wide, ctx->wide.p, (size_t)nc * g.nwin, hipMemcpyDeviceToHost,
                               ctx->s_d2h));
        if (ctx->rows8_on)
            HIP_TRY(hipMemcpyAsync(ctx->rows8_tgt.narrow, ctx->fit8.p, (size_t)nc * g.nwin, hipMemcpyDeviceToHost,
                                   ctx->s_d2h));
    }

    // 9. tallies over ranks; the slot after them carries the ranks' ERR_RESPEC so that
    // every rank reruns when one has to (the reruns' all-reduces then match up)
    if (ctx->comm) {
        STAGE_BEGIN(ST_COMM);
        k_respec_slot<<<1, 64, 0, s>>>(st, tally + (size_t)g.L * 4);
        HIP_TRY(hipGetLastError());
        ncclResult_t r = ncclAllReduce(tally, tally, (size_t)g.L * 4 + 1, ncclUint64, ncclSum, ctx->comm, s);
        if (r != ncclSuccess) return set_err(MGP_E_COMM, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        HIP_TRY(hipMemcpyAsync(ctx->h_respec, tally + (size_t)g.L * 4, 8, hipMemcpyDeviceToHost, s));
        STAGE_END(ST_COMM);
    }
    HIP_TRY(hipMemcpyAsync(ctx->host_stats, st, sizeof(DevStats), hipMemcpyDeviceToHost, s));
    return MGP_OK;
}

// Streaming (MGP_CFG_STREAM): after a push, the windows whose reads have all arrived
// (every start below the window's end: the input is coordinate-sorted, so the last
// pushed start says which) go through the hot path as one segment, queued behind the
// batch's copies while the next batches are still being copied. The last window
// (it also takes the overflow bin) waits for mgp_run.
static int stream_segments(mgp_ctx* ctx, int64_t last_start, uint16_t last_flag) {
    const Geom& g = ctx->g;
    if (ctx->stream_off || g.nc <= 0 || last_start < 0) return MGP_OK;
    const int64_t wc = std::min<int64_t>(last_start / g.W, g.nwin - 1);  // windows [0, wc) are complete
    if (wc - ctx->w_done < ctx->seg_min_win) return MGP_OK;
    if (!ctx->seg_open) ctx->stream_layout = (last_flag & MGP_FLAG_PACK32) ? kLayP32 : kLayP64;
    const int unit = ctx->stream_layout == kLayP32 ? 5 : 6;
    if ((uint64_t)ctx->pay >= ((uint64_t)(PE_KEEP & PE_OFF) << unit)) {  // not for compact elements: run resident
        ctx->stream_off = true;
        return MGP_OK;
    }
    if (!ctx->seg_open) set_pile_chunks(ctx->g, true, ctx->pile_wg_stream, ctx->pile_min_cpb_stream);  // (the whole run's chunks)
    MGP_TRY(ensure_run_buffers(ctx));
    int dup_parts = 0, pair_mode = 0;
    const Seg sg{ctx->w_done, (int)wc, (int)(wc * g.W / g.G), !ctx->seg_open, true};
    MGP_TRY(run_segment(ctx, sg, -1, dup_parts, pair_mode));
    ctx->seg_open = true;
    ctx->w_done = (int)wc;
    ctx->segments++;
    return MGP_OK;
}

int mgp_run(mgp_ctx* ctx) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    HIP_TRY(hipSetDevice(ctx->dev));
    ctx->ran = false;  // (until this run is queued: an error below leaves no results)
    // a run not begun by streaming segments is one resident launch of every window
    const bool streamed_run = ctx->seg_open && !ctx->no_spec && !ctx->stream_off;
    if (!streamed_run) set_pile_chunks(ctx->g, false, ctx->pile_wg_stream);
    MGP_TRY(ensure_run_buffers(ctx));
    const Geom g = ctx->g;
    const int slot = (int)(ctx->runs % mgp_ctx::kRing);
    for (int i = 0; i < ST_N; ++i) ctx->stage_ran[slot][i] = false;
    int dup_parts = 0, pair_mode = 0;
    // a streaming run whose pushes already ran segments: the rest of the windows;
    // otherwise (or on the fallback path) one resident segment over everything
    const bool streamed = ctx->seg_open && !ctx->no_spec && !ctx->stream_off;
    if (!streamed) ctx->seg_n[slot] = 0;  // (no segment pileups of this run to time)
    const Seg sg = streamed ? Seg{ctx->w_done, g.nwin, g.nbins, false, true, true}
                            : Seg{0, g.nwin, g.nbins, true, false, true};
    ctx->seg_open = false;
    ctx->w_done = 0;
    MGP_TRY(run_segment(ctx, sg, slot, dup_parts, pair_mode));
    MGP_TRY(run_finish(ctx, slot, dup_parts, streamed));
    ctx->last_streamed = streamed;
    ctx->ran = true;
    ctx->runs++;
    ctx->last_status = MGP_OK;
    return MGP_OK;
}

int mgp_sync(mgp_ctx* ctx) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    if (!ctx->ran) return set_err(MGP_E_STATE, "no run to wait for");
    HIP_TRY(hipSetDevice(ctx->dev));
    HIP_TRY(hipStreamSynchronize(ctx->s_comp));
    if (ctx->rows_on) HIP_TRY(hipStreamSynchronize(ctx->s_d2h));
    const uint32_t e = ctx->host_stats->err;
    // some read did not fit the speculative grouping (on any rank, with a communicator):
    // run again on the fallback path, once
    const bool respec = ctx->comm ? *ctx->h_respec != 0ull : (e & ERR_RESPEC) != 0u;
    if (respec && !ctx->rerunning) {
        ctx->no_spec = true;
        ctx->bits_cached = false;
        ctx->rerunning = true;
        int r = mgp_run(ctx);
        if (r == MGP_OK) r = mgp_sync(ctx);
        ctx->rerunning = false;
        return r;
    }
    if (e & ERR_BADOFF)
        return set_err(MGP_E_INVALID, "a pushed record (rec_off, its header or its CIGAR) lies outside its batch's "
                                      "payload, or a dense stride is shorter than a full record");
    if (e & ERR_RESPEC) return set_err(MGP_E_STATE, "speculative grouping failed on the fallback path");
    if (e & ERR_UNSORTED) return set_err(MGP_E_UNSORTED, "records are not in coordinate order");
    if (e & ERR_BADBC) return set_err(MGP_E_INVALID, "barcode index >= n_cells");
    if (e & ERR_OVERFLOW) return set_err(MGP_E_INVALID, "inconsistent grouping (unsorted input?)");
    if (e & ERR_BADREAD)
        return set_err(MGP_E_BADREAD, "a kept read has no SEQ or QUAL (pysam would return None)");
    if (e & ERR_SPAN) return set_err(MGP_E_SPAN, "a read's CIGAR reach exceeds the declared span");
    if (e & ERR_PACKED)
        return set_err(MGP_E_INVALID, "a packed record (MGP_FLAG_PACKED / MGP_FLAG_PACK32) does not fit its layout's "
                                      "limits, or a 32-byte record was made for other thresholds than the run's "
                                      "(its min_baseq in byte 31 and min_distance_from_end in byte 3 must equal "
                                      "the run's min_baseq and min_dist_from_end)");
    return MGP_OK;
}

int mgp_fetch_cells(mgp_ctx* ctx, int32_t lo, int32_t hi, mgp_result* out) {
    if (!ctx || !out) return set_err(MGP_E_INVALID, "null ctx/out");
    if (lo < 0 || hi < lo || hi > ctx->g.nc) return set_err(MGP_E_INVALID, "cell range outside [0, n_cells)");
    MGP_TRY(mgp_sync(ctx));
    const Geom& g = ctx->g;
    const size_t nc = (size_t)(hi - lo), L = (size_t)g.L, c0 = (size_t)lo;
    auto d2h = [&](void* dst, const DevBuf& src, size_t off, size_t bytes) -> int {
        if (dst && bytes) HIP_TRY(hipMemcpy(dst, src.as<uint8_t>() + off, bytes, hipMemcpyDeviceToHost));
        return MGP_OK;
    };
    if (nc && (out->counts || out->tn5 || out->depth)) {  // widen the 16-bit rows (drained windows are exact already)
        const int64_t npos = (int64_t)nc * (int64_t)L;
        k_expand<<<blocks_for(npos), kBlock, 0, ctx->s_comp>>>(
            g, (int64_t)c0 * (int64_t)L, npos, out16_of(ctx), out->counts ? ctx->counts.as<uint32_t>() : nullptr,
            out->tn5 ? ctx->tn5.as<uint32_t>() : nullptr, out->depth ? ctx->depth.as<uint32_t>() : nullptr);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(ctx->s_comp));
    }
    MGP_TRY(d2h(out->counts, ctx->counts, c0 * L * 32, nc * L * 32));
    MGP_TRY(d2h(out->tn5, ctx->tn5, c0 * L * 8, nc * L * 8));
    MGP_TRY(d2h(out->depth, ctx->depth, c0 * L * 4, nc * L * 4));
    MGP_TRY(d2h(out->n_reads, ctx->n_reads, c0 * 4, nc * 4));
    MGP_TRY(d2h(out->any_paired, ctx->any_paired, c0, nc));
    MGP_TRY(d2h(out->passed, ctx->passed, c0, nc));
    MGP_TRY(d2h(out->covered, ctx->covered, c0 * 4, nc * 4));
    MGP_TRY(d2h(out->depth_sum, ctx->dsum, c0 * 8, nc * 8));
    MGP_TRY(d2h(out->depth_max, ctx->dmax, c0 * 4, nc * 4));
    MGP_TRY(d2h(out->median_lo, ctx->med_lo, c0 * 4, nc * 4));
    MGP_TRY(d2h(out->median_hi, ctx->med_hi, c0 * 4, nc * 4));
    MGP_TRY(d2h(out->first_read, ctx->first_read, c0 * 4, nc * 4));
    MGP_TRY(d2h(out->ref_tally, ctx->tally, 0, L * 4 * 8));
    if (out->stats) {
        const DevStats& h = *ctx->host_stats;
        mgp_stats* o = out->stats;
        o->total_reads = ctx->n;
        o->filtered_reads = (int64_t)h.filtered;
        o->n_barcodes = (int64_t)h.n_barcodes;
        o->duplicate_reads_with_length = (int64_t)h.dup_len;
        o->duplicate_reads_position_only = (int64_t)h.dup_pos;
        o->cells_passed = (int64_t)h.cells_passed;
        o->max_span = (int32_t)h.max_span;
        o->error_bits = (int32_t)h.err;
    }
    return MGP_OK;
}

int mgp_fetch(mgp_ctx* ctx, mgp_result* out) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    return mgp_fetch_cells(ctx, 0, ctx->g.nc, out);
}

int mgp_fetch_rows16(mgp_ctx* ctx, int32_t lo, int32_t hi, mgp_rows16* out) {
    if (!ctx || !out) return set_err(MGP_E_INVALID, "null ctx/out");
    if (lo < 0 || hi < lo || hi > ctx->g.nc) return set_err(MGP_E_INVALID, "cell range outside [0, n_cells)");
    MGP_TRY(mgp_sync(ctx));
    const Geom& g = ctx->g;
    const size_t nc = (size_t)(hi - lo), L = (size_t)g.L, c0 = (size_t)lo, nw = (size_t)g.nwin;
    auto d2h = [&](void* dst, const DevBuf& src, size_t off, size_t bytes) -> int {
        if (dst && bytes) HIP_TRY(hipMemcpyAsync(dst, src.as<uint8_t>() + off, bytes, hipMemcpyDeviceToHost, ctx->s_comp));
        return MGP_OK;
    };
    // the pileup's 16-bit rows as they are: u16 pairs (fwd, rev) per base, Tn5 (fwd, rev), depth
    MGP_TRY(d2h(out->counts, ctx->counts16, c0 * L * 16, nc * L * 16));
    MGP_TRY(d2h(out->tn5, ctx->tn5_16, c0 * L * 4, nc * L * 4));
    MGP_TRY(d2h(out->depth, ctx->depth16, c0 * L * 2, nc * L * 2));
    MGP_TRY(d2h(out->wide, ctx->wide, c0 * nw, nc * nw));
    HIP_TRY(hipStreamSynchronize(ctx->s_comp));
    return MGP_OK;
}

int mgp_windows(mgp_ctx* ctx, int32_t* n_windows, int32_t* window_width) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    if (n_windows) *n_windows = ctx->g.nwin;
    if (window_width) *window_width = ctx->g.W;
    return MGP_OK;
}

// the device's mapping of a pinned host array (the rows targets)
static int mapped(void* host, void** dev) {
    void* dp = nullptr;
    if (!host || hipHostGetDevicePointer(&dp, host, 0) != hipSuccess || !dp) {
        (void)hipGetLastError();
        return set_err(MGP_E_INVALID, "rows target not in pinned host memory (mgp_host_alloc)");
    }
    *dev = dp;
    return MGP_OK;
}

int mgp_set_rows_target(mgp_ctx* ctx, const mgp_rows16* rows, const mgp_rows8* rows8) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    // (set during a streaming run: the windows piled so far are copied at once, below;
    // replacing or clearing a target mid-run is not allowed)
    if (ctx->seg_open && (!rows || ctx->rows_on))
        return set_err(MGP_E_STATE, "a streaming run is in progress (mgp_run or mgp_reset first)");
    HIP_TRY(hipSetDevice(ctx->dev));
    HIP_TRY(hipStreamSynchronize(ctx->s_d2h));
    if (!rows) {
        ctx->rows_on = false;
        ctx->rows8_on = false;
        return MGP_OK;
    }
    if (!rows->counts || !rows->tn5 || !rows->depth || !rows->wide) return set_err(MGP_E_INVALID, "null rows array");
    if (rows8 && (!rows8->counts || !rows8->tn5 || !rows8->depth || !rows8->narrow))
        return set_err(MGP_E_INVALID, "null rows8 array");
    // the kernel writes the rows through the device's mapping of the pinned arrays
    mgp_rows16 d{};
    void* dp = nullptr;
    MGP_TRY(mapped(rows->counts, &dp));
    d.counts = static_cast<uint16_t*>(dp);
    MGP_TRY(mapped(rows->tn5, &dp));
    d.tn5 = static_cast<uint16_t*>(dp);
    MGP_TRY(mapped(rows->depth, &dp));
    d.depth = static_cast<uint16_t*>(dp);
    d.wide = rows->wide;  // (an async copy: the host pointer)
    mgp_rows8 d8{};
    if (rows8) {
        MGP_TRY(mapped(rows8->counts, &dp));
        d8.counts = static_cast<uint8_t*>(dp);
        MGP_TRY(mapped(rows8->tn5, &dp));
        d8.tn5 = static_cast<uint8_t*>(dp);
        MGP_TRY(mapped(rows8->depth, &dp));
        d8.depth = static_cast<uint8_t*>(dp);
        d8.narrow = rows8->narrow;  // (an async copy: the host pointer)
    }
    ctx->rows_tgt = d;
    ctx->rows8_tgt = d8;
    ctx->rows_on = true;
    ctx->rows8_on = rows8 != nullptr;
    if (ctx->seg_open && ctx->w_done > 0) {  // catch up: the rows of the windows piled before
        const Geom& g = ctx->g;
        const int p1 = std::min(g.L, ctx->w_done * g.W);
        HIP_TRY(hipEventRecord(ctx->ev_rows, ctx->s_comp));
        HIP_TRY(hipStreamWaitEvent(ctx->s_d2h, ctx->ev_rows, 0));
        MGP_TRY(rows_launch(ctx, dim3((unsigned)((p1 + kBlock - 1) / kBlock), (unsigned)std::min(g.nc, 65535)), 0, p1));
    }
    return MGP_OK;
}

int mgp_set_rows16_target(mgp_ctx* ctx, const mgp_rows16* rows) { return mgp_set_rows_target(ctx, rows, nullptr); }

int mgp_copy_wait(mgp_ctx* ctx) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    HIP_TRY(hipSetDevice(ctx->dev));
    HIP_TRY(hipEventSynchronize(ctx->ev_copy));
    return MGP_OK;
}

int mgp_set_streaming(mgp_ctx* ctx, int on) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    if (ctx->seg_open) return set_err(MGP_E_STATE, "a streaming run is in progress (mgp_run or mgp_reset first)");
    ctx->stream = on != 0;
    return MGP_OK;
}

int mgp_set_cell_range(mgp_ctx* ctx, int32_t cell_lo, int32_t cell_hi) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    if (cell_lo < 0 || cell_hi < cell_lo || cell_hi - cell_lo != ctx->g.nc)
        return set_err(MGP_E_INVALID, "cell range [lo, hi) must have n_cells cells, lo >= 0");
    if (ctx->n > 0) return set_err(MGP_E_STATE, "set the cell range before the first push of a run (mgp_reset)");
    ctx->cell_lo = cell_lo;
    ctx->cell_range = true;
    return MGP_OK;
}

int mgp_stream_info(mgp_ctx* ctx, int64_t* segments, int32_t* last_streamed) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    if (segments) *segments = ctx->segments;
    if (last_streamed) *last_streamed = ctx->last_streamed ? 1 : 0;
    return MGP_OK;
}

int mgp_finish(mgp_ctx* ctx, mgp_result* out) {
    MGP_TRY(mgp_run(ctx));
    return mgp_fetch(ctx, out);
}

int mgp_kernel_times(mgp_ctx* ctx, int last_runs, float* ms, int max_n, int* n_out, char* names, int names_len) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    if (!ctx->ran || ctx->runs == 0) return set_err(MGP_E_STATE, "no run");
    if (last_runs < 1) last_runs = 1;
    if (last_runs > mgp_ctx::kRing) return set_err(MGP_E_INVALID, "last_runs > 64");
    if (last_runs > ctx->runs) last_runs = (int)ctx->runs;
    HIP_TRY(hipSetDevice(ctx->dev));
    HIP_TRY(hipStreamSynchronize(ctx->s_comp));
    int k = 0;
    for (int st = 0; st < ST_N && k < max_n; ++st, ++k) {
        double acc = 0.0;
        int timed = 0;  // runs that recorded this stage (mgp_set_stage_timing)
        for (int r = 0; r < last_runs; ++r) {
            const int slot = (int)((ctx->runs - 1 - r) % mgp_ctx::kRing);
            float t = 0.f;
            const int sn = st == ST_PILEUP ? ctx->seg_n[slot] : 0;
            if (sn > mgp_ctx::kSegEv) continue;  // (a streamed run with more segments than events)
            if (ctx->stage_ran[slot][st]) {
                HIP_TRY(hipEventElapsedTime(&t, ctx->ev[slot][st][0], ctx->ev[slot][st][1]));
                ++timed;
            }
            // the pileup of a streamed run: its segments' launches, then the run's own
            for (int k = 0; k < sn; ++k) {
                float ts = 0.f;
                const hipEvent_t* e = &ctx->seg_ev[((size_t)slot * mgp_ctx::kSegEv + k) * 2];
                HIP_TRY(hipEventElapsedTime(&ts, e[0], e[1]));
                t += ts;
            }
            if (sn > 0 && !ctx->stage_ran[slot][st]) ++timed;
            acc += t;
        }
        if (ms) ms[k] = timed ? (float)(acc / timed) : 0.f;
    }
    if (n_out) *n_out = k;
    if (names && names_len > 0) {
        std::strncpy(names, kStageNames, (size_t)names_len - 1);
        names[names_len - 1] = 0;
    }
    return MGP_OK;
}

int mgp_set_stage_timing(mgp_ctx* ctx, int all_stages) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    ctx->stage_all = all_stages != 0;
    return MGP_OK;
}

int mgp_comm_unique_id(uint8_t* out128) {
    if (!out128) return set_err(MGP_E_INVALID, "null out");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return set_err(MGP_E_COMM, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(out128, &id, 128);
    return MGP_OK;
}

int mgp_comm_init(mgp_ctx* ctx, const uint8_t* uid128, int nranks, int rank) {
    if (!ctx || !uid128 || nranks < 1 || rank < 0 || rank >= nranks) return set_err(MGP_E_INVALID, "bad comm args");
    HIP_TRY(hipSetDevice(ctx->dev));
    ncclUniqueId id;
    std::memcpy(&id, uid128, 128);
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    ctx->comm = nullptr;
    ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        ctx->comm = nullptr;
        return set_err(MGP_E_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    ctx->nranks = nranks;
    return MGP_OK;
}

int mgp_download_inputs(mgp_ctx* ctx, int32_t* start, int32_t* bc, int32_t* tlen, uint16_t* flag, uint8_t* mapq,
                        uint32_t* span, uint64_t* rec_off, uint8_t* payload) {
    if (!ctx) return set_err(MGP_E_INVALID, "null ctx");
    HIP_TRY(hipSetDevice(ctx->dev));
    HIP_TRY(hipStreamSynchronize(ctx->s_copy));
    HIP_TRY(hipStreamSynchronize(ctx->s_comp));
    const size_t n = (size_t)ctx->n;
    if (!n) return MGP_OK;
    if (start) HIP_TRY(hipMemcpy(start, ctx->start.p, n * 4, hipMemcpyDeviceToHost));
    if (bc) HIP_TRY(hipMemcpy(bc, ctx->bc.p, n * 4, hipMemcpyDeviceToHost));
    if (tlen) HIP_TRY(hipMemcpy(tlen, ctx->tlen.p, n * 4, hipMemcpyDeviceToHost));
    if (flag) HIP_TRY(hipMemcpy(flag, ctx->flag.p, n * 2, hipMemcpyDeviceToHost));
    if (mapq) HIP_TRY(hipMemcpy(mapq, ctx->mapq.p, n, hipMemcpyDeviceToHost));
    if (span) HIP_TRY(hipMemcpy(span, ctx->span.p, n * 4, hipMemcpyDeviceToHost));
    if (rec_off) HIP_TRY(hipMemcpy(rec_off, ctx->roff.p, n * 8, hipMemcpyDeviceToHost));
    if (payload && ctx->pay) HIP_TRY(hipMemcpy(payload, ctx->payload.p, (size_t)ctx->pay, hipMemcpyDeviceToHost));
    return MGP_OK;
}

// implemented in mgp_synth.hip
int mgp_synth_fill(void* stream, uint64_t seed, int64_t n, int read_len, int n_cells, int mito_len,
                   const uint32_t* d_cdf, const uint8_t* d_ref, int32_t* start, int32_t* bc, int32_t* tlen,
                   uint16_t* flag, uint8_t* mapq, uint32_t* span, uint64_t* roff, uint8_t* payload,
                   int64_t* payload_bytes, int rec_align, int pack, int placed, int cell_lo, int cell_hi,
                   int shard_rank, int shard_world, uint64_t* d_map, int64_t* n_out, int p32_minq, int p32_dist);

int mgp_synth_generate(mgp_ctx* ctx, const mgp_synth_params* p) {
    if (!ctx || !p || !p->cell_cdf || !p->ref_codes) return set_err(MGP_E_INVALID, "null synth args");
    const bool shard = p->cell_hi > p->cell_lo;
    if (shard) {
        if (p->cell_lo < 0 || p->cell_hi > p->n_cells || p->shard_world < 0 ||
            (p->shard_world > 0 && (p->shard_rank < 0 || p->shard_rank >= p->shard_world)))
            return set_err(MGP_E_INVALID, "synth cell shard out of range");
        if (p->cell_hi - p->cell_lo != ctx->cfg.n_cells)
            return set_err(MGP_E_INVALID, "synth shard cells != context n_cells");
    } else if (p->n_cells != ctx->cfg.n_cells) {
        return set_err(MGP_E_INVALID, "synth n_cells != context n_cells");
    }
    if (p->n_reads < 0 || p->n_reads > (int64_t)0xFFFFFFFEll || p->read_len < 12 || p->read_len > 4096)
        return set_err(MGP_E_INVALID, "synth sizes out of range");
    if (ctx->cfg.mito_len < p->read_len) return set_err(MGP_E_INVALID, "mito_len < read_len");
    const int align = p->rec_align ? p->rec_align : 16;
    if (align < 16 || align > 4096 || (align & (align - 1))) return set_err(MGP_E_INVALID, "rec_align must be a power of two in [16, 4096]");
    MGP_TRY(drain_stream(ctx));
    HIP_TRY(hipSetDevice(ctx->dev));
    HIP_TRY(hipStreamSynchronize(ctx->s_comp));
    HIP_TRY(hipStreamSynchronize(ctx->s_copy));
    HIP_TRY(hipMemsetAsync(ctx->order_bad.p, 0, 4, ctx->s_copy));
    ctx->n = 0;
    ctx->pay = 0;
    const int64_t n = p->n_reads;
    const int L = ctx->cfg.mito_len;
    const int nc = p->n_cells;
    // bytes the generator writes per record: a packed record (read_len <= MGP_PACK_MAX_LEN),
    // else the full layout of up to 3 CIGAR operations, at the placement's alignment
    const int64_t max_rec = ((int64_t)mgp_cigar_offset((uint32_t)p->read_len) + 16 + align - 1) & ~(int64_t)(align - 1);
    if (p->pack < 0 || p->pack > 2 ||
        (p->pack == 2 && (p->pack_min_baseq < -128 || p->pack_min_baseq > 127 || p->pack_min_dist > 15)))
        return set_err(MGP_E_INVALID, "synth pack must be 0, 1 or 2 (32-byte records for a min_baseq in [-128, 127] "
                                      "and a min_dist_from_end <= 15)");
    const bool packed = p->pack && p->read_len <= MGP_PACK_MAX_LEN;
    const int64_t rec_bytes = packed ? (int64_t)(p->pack == 2 ? MGP_PACK32_BYTES : MGP_PACK_BYTES) : max_rec;
    const bool placed = p->rec_off != nullptr;
    if (placed && p->payload_bytes < 0) return set_err(MGP_E_INVALID, "synth payload_bytes out of range");
    DevBuf cdf, ref, map;
    MGP_TRY(cdf.ensure((size_t)std::max(nc, 1) * 4));
    MGP_TRY(ref.ensure((size_t)L));
    hipStream_t s = ctx->s_copy;
    if (nc) HIP_TRY(hipMemcpyAsync(cdf.p, p->cell_cdf, (size_t)nc * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(ref.p, p->ref_codes, (size_t)L, hipMemcpyHostToDevice, s));
    // a shard counts its reads first (keep scan only), then allocates for them
    int64_t n_out = n;
    int r = MGP_OK;
    int64_t pay = placed ? p->payload_bytes : 0;
    if (shard) {
        MGP_TRY(map.ensure((size_t)std::max<int64_t>(n, 1) * 8));
        r = mgp_synth_fill(s, p->seed, n, p->read_len, nc, L, cdf.as<uint32_t>(), ref.as<uint8_t>(), nullptr,
                           nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &pay, align, p->pack, -1,
                           p->cell_lo, p->cell_hi, p->shard_rank, p->shard_world, map.as<uint64_t>(), &n_out,
                           p->pack_min_baseq, p->pack_min_dist);
        if (r != MGP_OK) return set_err(r, "synth: keep scan failed");
        pay = placed ? p->payload_bytes : 0;
    }
    if (placed && p->payload_bytes > n_out * std::max<int64_t>(max_rec, 128) + 128)
        return set_err(MGP_E_INVALID, "synth payload_bytes out of range");
    MGP_TRY(ensure_inputs(ctx, std::max<int64_t>(n_out, 1), placed ? p->payload_bytes : n_out * rec_bytes, false));
    // placed: rec_off has one entry per kept read (n_rec_off of them)
    if (placed && p->n_rec_off != n_out)
        return set_err(MGP_E_INVALID, "synth rec_off has " + std::to_string(p->n_rec_off) + " entries for " +
                                          std::to_string(n_out) + " generated reads");
    if (placed && n_out) {
        for (int64_t i = 0; i < n_out; ++i)
            if ((p->rec_off[i] & 15u) || (int64_t)p->rec_off[i] + rec_bytes > pay)
                return set_err(MGP_E_INVALID, "synth rec_off outside the payload or not 16-byte aligned");
        HIP_TRY(hipMemcpyAsync(ctx->roff.p, p->rec_off, (size_t)n_out * 8, hipMemcpyHostToDevice, s));
    }
    r = mgp_synth_fill(s, p->seed, n, p->read_len, nc, L, cdf.as<uint32_t>(), ref.as<uint8_t>(),
                       ctx->start.as<int32_t>(), ctx->bc.as<int32_t>(), ctx->tlen.as<int32_t>(),
                       ctx->flag.as<uint16_t>(), ctx->mapq.as<uint8_t>(), ctx->span.as<uint32_t>(),
                       ctx->roff.as<uint64_t>(), ctx->payload.as<uint8_t>(), &pay, align, p->pack, placed,
                       shard ? p->cell_lo : 0, shard ? p->cell_hi : 0, p->shard_rank, p->shard_world,
                       map.as<uint64_t>(), &n_out, p->pack_min_baseq, p->pack_min_dist);
    if (r != MGP_OK) return r == MGP_E_INVALID ? set_err(r, "synth: invalid arguments") : set_err(r, "synth failed");
    HIP_TRY(hipStreamSynchronize(s));
    cdf.release();
    ref.release();
    map.release();
    HIP_TRY(hipEventRecord(ctx->ev_copy, s));
    ctx->n = n_out;
    ctx->pay = pay;
    ctx->ran = false;
    ctx->no_spec = false;
    ctx->bits_cached = false;
    return MGP_OK;
}

// ---------------------------------------------------------------------------
// mgp_txt_gz: the txt count files formatted and deflated on the device
// (IncrementalTextWriter.write_cell + finalize's gzip -9, writers.py:430-486)
// ---------------------------------------------------------------------------
static int txt_run(TxtState& st, hipStream_t s, const txtgz::Rows& rows, int32_t n_rows, const mgp_txt_gz* job) {
    using namespace txtgz;
    const int64_t n = job->n_cells;
    if (n < 0 || (n > 0 && (!job->cells || !job->names || !job->name_off || !job->member_bytes)))
        return set_err(MGP_E_INVALID, "mgp_txt_gz: bad arguments");
    st.n = n;
    st.total = 0;
    if (n == 0) return MGP_OK;
    if (n > (int64_t)1 << 26) return set_err(MGP_E_INVALID, "mgp_txt_gz: too many cells for one call");
    for (int64_t k = 0; k < n; ++k) {
        if (job->cells[k] < 0 || job->cells[k] >= n_rows) return set_err(MGP_E_INVALID, "mgp_txt_gz: cell out of range");
        const int64_t bl = job->name_off[k + 1] - job->name_off[k];
        if (bl < 0 || bl > 4096 || job->name_off[k] < 0)
            return set_err(MGP_E_INVALID, "mgp_txt_gz: barcode names of 0..4096 bytes");
    }
    const int64_t nm = kFiles * n;
    const size_t nbytes = (size_t)job->name_off[n];
    MGP_TRY(st.cells.ensure((size_t)n * 4));
    MGP_TRY(st.names.ensure(nbytes + 1));
    MGP_TRY(st.name_off.ensure((size_t)(n + 1) * 8));
    MGP_TRY(st.sizes.ensure((size_t)nm * 8));
    MGP_TRY(st.nlines.ensure((size_t)nm * 8));
    MGP_TRY(st.offs.ensure((size_t)3 * (nm + 1) * 8));
    MGP_TRY(st.member_bytes.ensure((size_t)nm * 4));
    MGP_TRY(st.dst_off.ensure((size_t)nm * 8));
    if (!st.shift_ready) {
        std::vector<uint32_t> M(txtgz::kShiftPow * 32);
        crc_shift_matrices(M.data());
        MGP_TRY(st.crc_shift.ensure(M.size() * 4));
        HIP_TRY(hipMemcpy(st.crc_shift.p, M.data(), M.size() * 4, hipMemcpyHostToDevice));
        st.shift_ready = true;
    }
    HIP_TRY(hipMemcpyAsync(st.cells.p, job->cells, (size_t)n * 4, hipMemcpyHostToDevice, s));
    if (nbytes) HIP_TRY(hipMemcpyAsync(st.names.p, job->names, nbytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(st.name_off.p, job->name_off, (size_t)(n + 1) * 8, hipMemcpyHostToDevice, s));
    Job jb{rows, n, st.cells.as<int32_t>(), st.names.as<char>(), st.name_off.as<int64_t>()};
    if (txt_sizes(jb, st.sizes.as<uint64_t>(), st.nlines.as<uint64_t>(), s) != 0)
        return set_err(MGP_E_HIP, "mgp_txt_gz: size kernel launch failed");
    std::vector<uint64_t> sz((size_t)nm), nl((size_t)nm), offs((size_t)3 * (nm + 1));
    HIP_TRY(hipMemcpyAsync(sz.data(), st.sizes.p, (size_t)nm * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(nl.data(), st.nlines.p, (size_t)nm * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    uint64_t* to = offs.data();
    uint64_t* lo = to + nm + 1;
    uint64_t* oo = lo + nm + 1;
    to[0] = lo[0] = oo[0] = 0;
    for (int64_t m = 0; m < nm; ++m) {
        to[m + 1] = to[m] + ((sz[(size_t)m] + 15) & ~uint64_t(15));  // (aligned: the parse loads 16 bytes)
        lo[m + 1] = lo[m] + nl[(size_t)m];
        oo[m + 1] = oo[m] + out_bound(sz[(size_t)m]);
        if (job->text_bytes) job->text_bytes[m] = (int64_t)sz[(size_t)m];
    }
    MGP_TRY(st.text.ensure(to[nm] + 256));  // (slack: a parse block reads up to 31 positions past a text)
    MGP_TRY(st.tok.ensure(4 * to[nm] + 1024));
    MGP_TRY(st.lines.ensure(12 * lo[nm] + 64));
    MGP_TRY(st.out.ensure(oo[nm] + 64));
    HIP_TRY(hipMemcpyAsync(st.offs.p, offs.data(), offs.size() * 8, hipMemcpyHostToDevice, s));
    Scratch sc{};
    sc.text_off = st.offs.as<uint64_t>();
    sc.text_n = st.sizes.as<uint64_t>();
    sc.line_off = sc.text_off + nm + 1;
    sc.out_off = sc.line_off + nm + 1;
    sc.text = st.text.as<uint8_t>();
    sc.tok = st.tok.as<uint32_t>();
    sc.lines = st.lines.as<uint32_t>();
    sc.out = st.out.as<uint32_t>();
    sc.member_bytes = st.member_bytes.as<uint32_t>();
    sc.crc_shift = st.crc_shift.as<uint32_t>();
    MGP_TRY(st.seg.ensure((size_t)nm * 257 * 4));
    MGP_TRY(st.crc.ensure((size_t)nm * 4));
    sc.seg = st.seg.as<uint32_t>();
    sc.crc = st.crc.as<uint32_t>();
    sc.prof = nullptr;
    const bool prof = std::getenv("MGP_TXT_PROF") != nullptr;
    if (prof) {
        MGP_TRY(st.prof.ensure((size_t)nm * 64));
        HIP_TRY(hipMemsetAsync(st.prof.p, 0, (size_t)nm * 64, s));
        sc.prof = st.prof.as<uint64_t>();
    }
    if (txt_deflate(jb, sc, s) != 0) return set_err(MGP_E_HIP, "mgp_txt_gz: deflate kernel launch failed");
    if (prof) {  // per-phase means over the members that have text (us), to stderr
        std::vector<uint64_t> pr((size_t)nm * 8);
        HIP_TRY(hipMemcpyAsync(pr.data(), st.prof.p, pr.size() * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        // stamps: 0 format start, 1 format end, 2 match end, 3 parse end, 4 code end; each
        // kernel's span over all members (first start to last end) and the mean per member
        double mean[3] = {0, 0, 0};
        uint64_t lo[3] = {UINT64_MAX, UINT64_MAX, UINT64_MAX}, hi[3] = {0, 0, 0};
        int64_t cnt = 0;
        for (int64_t m = 0; m < nm; ++m) {
            const uint64_t* q = pr.data() + m * 8;
            if (!q[4]) continue;
            ++cnt;
            mean[0] += (double)(q[1] - q[0]) * 0.01;
            lo[0] = std::min(lo[0], q[0]);
            hi[0] = std::max(hi[0], q[1]);
            hi[1] = std::max(hi[1], q[2]);
            hi[2] = std::max(hi[2], q[4]);
            mean[2] += (double)(q[4] - q[3]) * 0.01;
        }
        // format phases per member: 0 start, 5 sizes + scan, 6 text written, 7 own CRC, 1 end
        double fp[4] = {0, 0, 0, 0};
        for (int64_t m = 0; m < nm; ++m) {
            const uint64_t* q = pr.data() + m * 8;
            if (!q[4]) continue;
            fp[0] += (double)(q[5] - q[0]) * 0.01;
            fp[1] += (double)(q[6] - q[5]) * 0.01;
            fp[2] += (double)(q[7] - q[6]) * 0.01;
            fp[3] += (double)(q[1] - q[7]) * 0.01;
        }
        std::fprintf(stderr, "[mgp_txt_gz] %lld members: format %.1f ms (%.1f us per member: sizes %.1f, text %.1f, "
                     "crc %.1f, combine %.1f), match %.1f ms, code %.1f ms (tail %.1f us per member)\n", (long long)cnt,
                     (hi[0] - lo[0]) * 1e-5, mean[0] / cnt, fp[0] / cnt, fp[1] / cnt, fp[2] / cnt, fp[3] / cnt,
                     (hi[1] - hi[0]) * 1e-5, (hi[2] - hi[1]) * 1e-5, mean[2] / cnt);
    }
    std::vector<uint32_t> mb((size_t)nm);
    HIP_TRY(hipMemcpyAsync(mb.data(), st.member_bytes.p, (size_t)nm * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<uint64_t> dst((size_t)nm);
    uint64_t tot = 0;
    for (int64_t m = 0; m < nm; ++m) {
        dst[(size_t)m] = tot;
        tot += mb[(size_t)m];
        job->member_bytes[m] = mb[(size_t)m];
    }
    MGP_TRY(st.packed.ensure(tot + 64));
    HIP_TRY(hipMemcpyAsync(st.dst_off.p, dst.data(), (size_t)nm * 8, hipMemcpyHostToDevice, s));
    if (txt_pack(sc, nm, st.dst_off.as<uint64_t>(), st.packed.as<uint8_t>(), s) != 0)
        return set_err(MGP_E_HIP, "mgp_txt_gz: pack kernel launch failed");
    HIP_TRY(hipStreamSynchronize(s));
    st.total = tot;
    return MGP_OK;
}

int mgp_txt_gz_run(mgp_ctx* ctx, mgp_txt_gz* job, int64_t* total_bytes) {
    if (!ctx || !job) return set_err(MGP_E_INVALID, "null ctx/job");
    MGP_TRY(mgp_sync(ctx));
    HIP_TRY(hipSetDevice(ctx->dev));
    const Geom& g = ctx->g;
    if (!ctx->ran) return set_err(MGP_E_STATE, "mgp_txt_gz: no run to write (mgp_run first)");
    txtgz::Rows rows{reinterpret_cast<const uint4*>(ctx->counts16.p), ctx->depth16.as<uint16_t>(),
                     ctx->wide.as<uint8_t>(), ctx->counts.as<uint32_t>(), ctx->depth.as<uint32_t>(), g.L, g.W, g.nwin};
    MGP_TRY(txt_run(ctx->txt, ctx->s_comp, rows, g.nc, job));
    if (total_bytes) *total_bytes = (int64_t)ctx->txt.total;
    return MGP_OK;
}

int mgp_txt_gz_fetch(mgp_ctx* ctx, uint8_t* dst, int64_t cap) {
    if (!ctx || (!dst && ctx->txt.total)) return set_err(MGP_E_INVALID, "null ctx/dst");
    if (cap < (int64_t)ctx->txt.total) return set_err(MGP_E_INVALID, "mgp_txt_gz_fetch: destination too small");
    HIP_TRY(hipSetDevice(ctx->dev));
    if (ctx->txt.total) HIP_TRY(hipMemcpy(dst, ctx->txt.packed.p, ctx->txt.total, hipMemcpyDeviceToHost));
    return MGP_OK;
}

// ---------------------------------------------------------------------------
// mgp_h5_tiles: the HDF5 count datasets' chunks deflated on the device
// (IncrementalHDF5Writer, writers.py:60-131: 11 u16 planes, gzip-4 chunks of 1000 x 100)
// ---------------------------------------------------------------------------
int mgp_h5_tiles_run(mgp_ctx* ctx, mgp_h5_tiles* job, int64_t* total_bytes) {
    using namespace txtgz;
    if (!ctx || !job) return set_err(MGP_E_INVALID, "null ctx/job");
    MGP_TRY(mgp_sync(ctx));
    HIP_TRY(hipSetDevice(ctx->dev));
    if (!ctx->ran) return set_err(MGP_E_STATE, "mgp_h5_tiles: no run to write (mgp_run first)");
    const Geom& g = ctx->g;
    H5State& st = ctx->h5;
    st.total = 0;
    const int64_t nco = job->n_cols;
    const int crow = job->chunk_rows, ccol = job->chunk_cols;
    if (nco < 0 || crow <= 0 || ccol <= 0 || (int64_t)crow * ccol > (1 << 22) || !job->chunk_bytes ||
        (nco > 0 && !job->cell_of_col))
        return set_err(MGP_E_INVALID, "mgp_h5_tiles: bad arguments");
    const int64_t ncc_all = (nco + ccol - 1) / ccol;
    const int lo = job->col_chunk_lo, hi = job->col_chunk_hi;
    if (lo < 0 || hi < lo || hi > ncc_all) return set_err(MGP_E_INVALID, "mgp_h5_tiles: column chunks out of range");
    const int nrc = (g.L + crow - 1) / crow, ncc = hi - lo;
    const int64_t nch = (int64_t)kPlanes * nrc * ncc;
    if (nch == 0) {
        if (total_bytes) *total_bytes = 0;
        return MGP_OK;
    }
    if (nch > (int64_t)1 << 20) return set_err(MGP_E_INVALID, "mgp_h5_tiles: too many chunks for one call");
    for (int64_t j = 0; j < nco; ++j)
        if (job->cell_of_col[j] < -1 || job->cell_of_col[j] >= g.nc)
            return set_err(MGP_E_INVALID, "mgp_h5_tiles: cell of a column out of range");
    hipStream_t s = ctx->s_comp;
    const uint64_t chunk_raw = (uint64_t)crow * ccol * 2, stride = out_bound(chunk_raw);
    const uint64_t raw_stride = (chunk_raw + 15) & ~uint64_t(15);
    MGP_TRY(st.coc.ensure((size_t)std::max<int64_t>(nco, 1) * 4));
    MGP_TRY(st.raw.ensure((size_t)(nch * raw_stride) + 64));
    MGP_TRY(st.tok.ensure((size_t)(nch * h5_tok_words(chunk_raw)) * 4 + 64));
    MGP_TRY(st.out.ensure((size_t)(nch * stride) + 64));
    MGP_TRY(st.out_off.ensure((size_t)nch * 8));
    MGP_TRY(st.chunk_bytes.ensure((size_t)nch * 4));
    MGP_TRY(st.dst_off.ensure((size_t)nch * 8));
    MGP_TRY(st.sums.ensure((size_t)3 * g.L * 8));
    HIP_TRY(hipMemsetAsync(st.sums.p, 0, (size_t)3 * g.L * 8, s));
    std::vector<uint64_t> oo((size_t)nch);
    for (int64_t k = 0; k < nch; ++k) oo[(size_t)k] = (uint64_t)k * stride;
    if (nco) HIP_TRY(hipMemcpyAsync(st.coc.p, job->cell_of_col, (size_t)nco * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(st.out_off.p, oo.data(), (size_t)nch * 8, hipMemcpyHostToDevice, s));
    H5Job jb{ctx->counts16.as<uint4>(), ctx->tn5_16.as<uint32_t>(), ctx->depth16.as<uint16_t>(), g.L,
             st.coc.as<int32_t>(), nco, crow, ccol, nrc, lo, ncc, st.sums.as<unsigned long long>()};
    H5Scratch sc{st.raw.as<uint8_t>(), st.tok.as<uint32_t>(), st.out.as<uint32_t>(), st.out_off.as<uint64_t>(),
                 st.chunk_bytes.as<uint32_t>(), chunk_raw, stride, raw_stride, h5_tok_words(chunk_raw), nullptr};
    const bool prof = std::getenv("MGP_H5_PROF") != nullptr;
    if (prof) {
        MGP_TRY(st.prof.ensure((size_t)nch * 64));
        HIP_TRY(hipMemsetAsync(st.prof.p, 0, (size_t)nch * 64, s));
        sc.prof = st.prof.as<uint64_t>();
    }
    if (h5_deflate(jb, sc, s) != 0) return set_err(MGP_E_HIP, "mgp_h5_tiles: deflate kernel launch failed");
    if (prof) {  // per-phase means over the chunks (us) and the code kernel's span, to stderr
        // stamps: 0 start, 1 parse, 2 adler, 3 end; 4 lit/dist lengths, 5 header, 6 sizes (deflate_block)
        std::vector<uint64_t> pr((size_t)nch * 8);
        HIP_TRY(hipMemcpyAsync(pr.data(), st.prof.p, pr.size() * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        const int ord[7] = {0, 1, 2, 4, 5, 6, 3};  // phases in time order
        double m[6] = {0, 0, 0, 0, 0, 0};
        uint64_t a = UINT64_MAX, b = 0;
        for (int64_t k = 0; k < nch; ++k) {
            const uint64_t* q = pr.data() + k * 8;
            for (int i = 0; i < 6; ++i) m[i] += (double)(q[ord[i + 1]] - q[ord[i]]) * 0.01;
            a = std::min(a, q[0]);
            b = std::max(b, q[3]);
        }
        std::fprintf(stderr, "[mgp_h5_tiles] %lld chunks: parse %.1f us, adler %.1f, huffman %.1f, header %.1f, "
                     "sizes %.1f, encode %.1f us per chunk; span %.2f ms\n", (long long)nch, m[0] / nch, m[1] / nch,
                     m[2] / nch, m[3] / nch, m[4] / nch, m[5] / nch, (b - a) * 1e-5);
    }
    std::vector<uint32_t> cb((size_t)nch);
    HIP_TRY(hipMemcpyAsync(cb.data(), st.chunk_bytes.p, (size_t)nch * 4, hipMemcpyDeviceToHost, s));
    if (job->col_sums)
        HIP_TRY(hipMemcpyAsync(job->col_sums, st.sums.p, (size_t)3 * g.L * 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<uint64_t> dst((size_t)nch);
    uint64_t tot = 0;
    for (int64_t k = 0; k < nch; ++k) {
        dst[(size_t)k] = tot;
        tot += cb[(size_t)k];
        job->chunk_bytes[k] = cb[(size_t)k];
    }
    MGP_TRY(st.packed.ensure(tot + 64));
    HIP_TRY(hipMemcpyAsync(st.dst_off.p, dst.data(), (size_t)nch * 8, hipMemcpyHostToDevice, s));
    if (h5_pack(sc, nch, st.dst_off.as<uint64_t>(), st.packed.as<uint8_t>(), s) != 0)
        return set_err(MGP_E_HIP, "mgp_h5_tiles: pack kernel launch failed");
    HIP_TRY(hipStreamSynchronize(s));
    st.total = tot;
    if (total_bytes) *total_bytes = (int64_t)tot;
    return MGP_OK;
}

int mgp_h5_tiles_fetch(mgp_ctx* ctx, uint8_t* dst, int64_t cap) {
    if (!ctx || (!dst && ctx->h5.total)) return set_err(MGP_E_INVALID, "null ctx/dst");
    if (cap < (int64_t)ctx->h5.total) return set_err(MGP_E_INVALID, "mgp_h5_tiles_fetch: destination too small");
    HIP_TRY(hipSetDevice(ctx->dev));
    if (ctx->h5.total) HIP_TRY(hipMemcpy(dst, ctx->h5.packed.p, ctx->h5.total, hipMemcpyDeviceToHost));
    return MGP_OK;
}

int mgp_txt_gz_rows(int device, const uint32_t* counts, const uint32_t* depth, int32_t n_rows, int32_t mito_len,
                    mgp_txt_gz* job, uint8_t* dst, int64_t cap, int64_t* total_bytes) {
    if (!job || n_rows < 0 || mito_len <= 0 || (n_rows > 0 && (!counts || !depth)))
        return set_err(MGP_E_INVALID, "mgp_txt_gz_rows: bad arguments");
    HIP_TRY(hipSetDevice(device));
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int rc = MGP_OK;
    {
        TxtState st;
        const size_t npos = (size_t)n_rows * (size_t)mito_len;
        rc = st.rows_c.ensure(npos * 32 + 64);
        if (rc == MGP_OK) rc = st.rows_d.ensure(npos * 4 + 64);
        if (rc == MGP_OK && npos) {
            if (hipMemcpy(st.rows_c.p, counts, npos * 32, hipMemcpyHostToDevice) != hipSuccess ||
                hipMemcpy(st.rows_d.p, depth, npos * 4, hipMemcpyHostToDevice) != hipSuccess)
                rc = set_err(MGP_E_HIP, "mgp_txt_gz_rows: upload failed");
        }
        txtgz::Rows rows{nullptr, nullptr, nullptr, st.rows_c.as<uint32_t>(), st.rows_d.as<uint32_t>(), mito_len,
                         mito_len, 1};
        if (rc == MGP_OK) rc = txt_run(st, s, rows, n_rows, job);
        if (rc == MGP_OK && total_bytes) *total_bytes = (int64_t)st.total;
        if (rc == MGP_OK && (int64_t)st.total > cap) rc = set_err(MGP_E_INVALID, "mgp_txt_gz_rows: destination too small");
        if (rc == MGP_OK && st.total && hipMemcpy(dst, st.packed.p, st.total, hipMemcpyDeviceToHost) != hipSuccess)
            rc = set_err(MGP_E_HIP, "mgp_txt_gz_rows: download failed");
    }
    (void)hipStreamDestroy(s);
    return rc;
}

}  // extern "C"
