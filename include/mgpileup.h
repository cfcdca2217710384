/*
 * mgpileup.h — C-ABI of the MI355X per-barcode chrM pileup engine (libmgpileup.so).
 *
 * This is the drop-in boundary for mgatk2's `src/processing` hot path. The
 * reference is pure Python; there is no FFI in it, so every entry point below
 * names the reference interface it replaces (paths relative to the reference
 * repo root, file:line):
 *
 *   mgp_open / mgp_close      replace constructing `PileupGenerator(config)` and
 *                             `CellProcessor(config, output_dir)`
 *                             (src/processing/pileup.py:13, processors.py:59) with a
 *                             device context that owns all HBM state.
 *   mgp_push_batch            replaces the per-record append into
 *                             `reads_by_barcode[barcode]` inside
 *                             `BAMReader.collect_reads_by_barcode`
 *                             (src/processing/readers.py:85-165): the host hands over
 *                             the chrM records of a coordinate-sorted BAM as SoA
 *                             arrays + packed per-read payload records.
 *   mgp_run                   replaces the filter+dedup block (readers.py:95-150),
 *                             `process_cells_progressive` -> `process_barcode_worker`
 *                             -> `generate_pileup` + `filter_strand_bias`
 *                             (processors.py:20-55,87-144; pileup.py:18-154) and the
 *                             per-cell statistics / reference-allele tallies of the
 *                             writers (writers.py:187-229,340-349,437-458).
 *   mgp_fetch                 copies the results (the arrays the writers consume)
 *                             back into caller-owned host buffers.
 *   mgp_last_error            replaces the exception taxonomy at the boundary
 *                             (src/core/exceptions.py); the Python wrapper maps
 *                             negative return codes to those exception classes.
 *   mgp_comm_*                the one cross-GPU exchange: an RCCL all-reduce of the
 *                             reference-allele tallies (writers.py:221-222,340-349)
 *                             when cells are sharded over GPUs.
 *   mgp_synth_generate        device-side synthetic workload generator (bench only;
 *                             the host mirror is mgatk2_amd/synth.py, bit-identical).
 *
 * All pointers are plain host pointers; no C++ or torch types cross the ABI.
 * A context is not thread-safe: drive it from one host thread. Contexts on
 * different devices may run concurrently.
 */
#ifndef MGPILEUP_H
#define MGPILEUP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGP_ABI_VERSION 7  /* 2: fixed seq/CIGAR offsets for reads <= 64 bases;
                              3: synth cell shards, cell-range and 16-bit fetches, streaming runs;
                              4: batches without rec_off / span columns and the rows target (the
                                 round-3 "v3.1" entry points), pushed records checked against
                                 their batch's payload (MGP_E_INVALID), mgp_copy_wait, batches
                                 without a start column,
                                 mgp_synth_params.n_rec_off, rows targets with min_reads > 1;
                              5: mgp_set_cell_range (one device's cells of whole batches),
                                 mgp_push_batch16 (16-bit barcode / |tlen| columns), dense
                                 64-byte batches paired on the device;
                              6: mgp_txt_gz_* (the txt count files formatted and deflated on the
                                 device);
                              7: mgp_set_rows_target (an 8-bit rows target beside the 16-bit one),
                                 mgp_h5_tiles_* (the HDF5 chunks deflated on the device) */

/* ---- return codes (0 = success) ------------------------------------------ */
#define MGP_OK               0
#define MGP_E_INVALID      (-1)  /* invalid argument                           -> InvalidInputError */
#define MGP_E_HIP          (-2)  /* HIP runtime error                          -> ProcessingError   */
#define MGP_E_OOM          (-3)  /* device allocation failed                   -> ProcessingError   */
#define MGP_E_UNSORTED     (-4)  /* records not in coordinate order            -> BAMFormatError    */
#define MGP_E_BADREAD      (-5)  /* kept read without SEQ/QUAL (readers.py:157-158 raises) -> BAMReadError */
#define MGP_E_SPAN         (-6)  /* a read's reference reach exceeds its declared span   -> InvalidInputError */
#define MGP_E_STATE        (-7)  /* call out of order (e.g. fetch before run)  -> ProcessingError   */
#define MGP_E_COMM         (-8)  /* RCCL failure                               -> ProcessingError   */

/* ---- dedup modes (src/cli/utils.py:164-169, readers.py:118-150) ---------- */
#define MGP_DEDUP_NONE        0  /* "none"                           */
#define MGP_DEDUP_START       1  /* "alignment_start":  (start, strand)        */
#define MGP_DEDUP_START_FRAG  2  /* "alignment_and_fragment_length": (start, strand, |tlen|) */

/* ---- per-read flag bits carried in mgp_batch.flag ------------------------ */
/* The low 12 bits are the raw BAM FLAG word. Bit 12 is set by the host when
 * the record has no SEQ or no QUAL (pysam would return None and the reference
 * raises BAMReadError when such a read is kept: readers.py:157-158,167-168). */
#define MGP_FLAG_PAIRED        0x0001u
#define MGP_FLAG_UNMAPPED      0x0004u
#define MGP_FLAG_REVERSE       0x0010u
#define MGP_FLAG_SECONDARY     0x0100u
#define MGP_FLAG_SUPPLEMENTARY 0x0800u
#define MGP_FLAG_NOSEQQUAL     0x1000u
#define MGP_FLAG_PACKED        0x2000u  /* payload record i uses the packed 64-byte layout (below) */
#define MGP_FLAG_PACK32        0x4000u  /* payload record i uses the 32-byte layout (below) */

/* mgp_config.flags */
#define MGP_CFG_KEEP_TN5       0x1  /* keep Tn5 counts at positions of depth 0 (the unfiltered
                                       generate_pileup() view, pileup.py:100-124); off = the
                                       strand-filtered result the writers consume (pileup.py:151-152) */
#define MGP_CFG_STREAM         0x2  /* streaming runs: each mgp_push_batch queues, behind its own
                                       copies, the hot path of the position windows whose reads have
                                       all arrived (coordinate order), so the copies of later batches
                                       overlap the compute of earlier ones; mgp_run does the rest.
                                       Set reserve_reads to the run's read count. Results are those of
                                       a resident run (reads a segment cannot serve rerun it resident). */

/* Engine configuration: the POD restatement of PipelineConfig
 * (src/core/config.py:77-114) restricted to what the hot path reads. */
typedef struct mgp_config {
    int32_t min_baseq;          /* QualityThresholds.min_baseq          (config.py:11) */
    int32_t min_mapq;           /* QualityThresholds.min_mapq           (config.py:12) */
    int32_t min_dist_from_end;  /* QualityThresholds.min_distance_from_end; the reference
                                   always uses 5 (pipeline.py:239-254 never passes it) */
    int32_t dedup_mode;         /* MGP_DEDUP_*                                          */
    double  max_strand_bias;    /* QualityThresholds.max_strand_bias    (config.py:13) */
    int32_t min_reads;          /* PipelineConfig.min_reads_per_cell    (processors.py:22) */
    int32_t n_cells;            /* whitelist length = HDF5 column count (writers.py:42) */
    int32_t mito_len;           /* PipelineConfig.mito_length, 16569    (config.py:95)  */
    int32_t flags;              /* MGP_CFG_* bits                                       */
    int64_t reserve_reads;      /* capacity hint for resident reads (grows on demand)   */
    int64_t reserve_payload;    /* capacity hint for resident payload bytes             */
} mgp_config;

/* One batch of chrM records in BAM order (host pointers; pinned memory from
 * mgp_host_alloc gives asynchronous H2D). Records of consecutive batches must
 * continue the coordinate order.
 *
 * Payload record i lives at payload + rec_off[i] (16-byte aligned):
 *   int32  start      0-based reference_start
 *   uint32 l_seq      len(query_sequence), soft clips included
 *   uint16 n_cigar
 *   uint16 flag       same word as flag[i]
 *   uint32 cigar_off  byte offset of cigar[] from the record start (= mgp_cigar_offset(l_seq))
 *   uint8  qual[l_seq]              raw Phred bytes (as BAM stores them), at +16
 *   uint8  seq[(l_seq + 1) / 2]     BAM 4-bit codes, high nibble first, at +mgp_seq_offset(l_seq)
 *   uint32 cigar[n_cigar]           BAM encoding (len << 4 | op), at +cigar_off
 * qual gets at least 64 bytes and seq at least 32, so for reads of <= 64 bases
 * every field has a fixed place: qual +16, seq +80, cigar +112, and a record
 * with <= 4 CIGAR operations is exactly one 128-byte line that a kernel loads
 * with 8 independent 16-byte loads and indexes statically. Record size =
 * round_up(cigar_off + 4 * n_cigar, 16). Records are gathered in random order,
 * so producers should place them at 128-byte aligned offsets; any 16-byte
 * aligned placement is accepted. Kernels may read up to 128 bytes from a
 * record start: keep >= 128 bytes after the last record (mgp_push_batch pads).
 *
 * Packed record (flag[i] has MGP_FLAG_PACKED): 64 bytes, everything the pileup
 * reads of a short read in half a cache line (the pileup gathers one record per
 * read in random order, so its bytes per read set the gather traffic):
 *   int32  start
 *   uint8  l_seq                    1 .. MGP_PACK_MAX_LEN
 *   uint8  n_cigar | reverse << 7   n_cigar <= 4; reverse = flag & MGP_FLAG_REVERSE
 *   uint16 cigar[4]                 len << 4 | op (len < 4096), unused entries 0
 *   uint8  base[l_seq] at +14       qual << 2 | b for the codes A, C, G, T (b = 0..3);
 *                                   0xFF for any other code (pileup.py:83-86 never counts it)
 * A read may be packed iff it has SEQ and QUAL, l_seq <= 50, every qual <= 62,
 * n_cigar <= 4 with every length < 4096 and at most 2 aligned (M, =, X)
 * operations, and -2^28 <= start < 2^28 (mgp_pack_record). The layout keeps
 * every bit the pileup uses; it drops the code and quality of non-ACGT bases,
 * so producers that must reproduce query_sequence (the SimpleRead API) write
 * the full layout. Packed records are placed at 64-byte aligned offsets.
 */
#define MGP_PACK_MAX_LEN 50
#define MGP_PACK_BYTES   64
#define MGP_PACK32_BYTES 32
#if defined(__HIPCC__)
#define MGP_HD __host__ __device__
#else
#define MGP_HD
#endif
static inline MGP_HD uint32_t mgp_seq_offset(uint32_t l_seq) {
    const uint32_t q = (l_seq + 3u) & ~3u;
    return 16u + (q > 64u ? q : 64u);
}
static inline MGP_HD uint32_t mgp_cigar_offset(uint32_t l_seq) {
    const uint32_t b = ((l_seq + 1u) / 2u + 3u) & ~3u;
    return mgp_seq_offset(l_seq) + (b > 32u ? b : 32u);
}

/* Bytes of the record at rec (flag = its flag word): 64 for a packed record,
 * cigar_off + 4 * n_cigar for a full one (before any alignment padding). */
static inline MGP_HD uint32_t mgp_record_bytes(const uint8_t *rec, uint16_t flag) {
    uint32_t l_seq, n_cigar;
    if (flag & MGP_FLAG_PACK32) return MGP_PACK32_BYTES;
    if (flag & MGP_FLAG_PACKED) return MGP_PACK_BYTES;
    l_seq = (uint32_t)rec[4] | ((uint32_t)rec[5] << 8) | ((uint32_t)rec[6] << 16) | ((uint32_t)rec[7] << 24);
    n_cigar = (uint32_t)rec[8] | ((uint32_t)rec[9] << 8);
    return mgp_cigar_offset(l_seq) + 4u * n_cigar;
}

/* Expand a packed record into the full layout in full[0..128) (a non-ACGT base,
 * byte >= 252, becomes code 15 = N with quality 0; the header flag word holds
 * only MGP_FLAG_REVERSE). */
static inline MGP_HD void mgp_unpack_record(const uint8_t *p, uint8_t *full) {
    uint32_t k;
    const uint32_t lseq = p[4] <= MGP_PACK_MAX_LEN ? p[4] : MGP_PACK_MAX_LEN;
    const uint32_t nc = (p[5] & 0x7Fu) <= 4u ? (p[5] & 0x7Fu) : 4u;
    const uint32_t coff = mgp_cigar_offset(lseq), soff = mgp_seq_offset(lseq);
    for (k = 0; k < 128u; ++k) full[k] = 0;
    for (k = 0; k < 4u; ++k) full[k] = p[k];
    full[4] = (uint8_t)lseq;
    full[8] = (uint8_t)nc;
    full[10] = (uint8_t)((p[5] & 0x80u) ? MGP_FLAG_REVERSE : 0u);
    full[12] = (uint8_t)coff;
    for (k = 0; k < nc; ++k) {
        full[coff + 4 * k] = p[6 + 2 * k];
        full[coff + 4 * k + 1] = p[7 + 2 * k];
    }
    for (k = 0; k < lseq; ++k) {
        const uint8_t v = p[14 + k];
        const uint8_t code = v >= 252u ? (uint8_t)15 : (uint8_t)(1u << (v & 3u));
        full[16 + k] = v >= 252u ? (uint8_t)0 : (uint8_t)(v >> 2);
        full[soff + (k >> 1)] |= (k & 1u) ? code : (uint8_t)(code << 4);
    }
}

/* Write the packed record of one read into out[0..64) and return 1, or return 0
 * (out untouched) when the read does not fit the packed layout. seq holds BAM
 * 4-bit codes, high nibble first; qual raw Phred bytes; cigar BAM words. */
static inline MGP_HD int mgp_pack_record(int32_t start, uint32_t l_seq, uint16_t flag, uint32_t n_cigar,
                                         const uint32_t *cigar, const uint8_t *seq, const uint8_t *qual,
                                         uint8_t *out) {
    uint32_t k, blocks = 0;
    if ((flag & MGP_FLAG_NOSEQQUAL) || l_seq == 0u || l_seq > MGP_PACK_MAX_LEN || n_cigar > 4u) return 0;
    if (start < -(1 << 28) || start >= (1 << 28)) return 0;
    for (k = 0; k < n_cigar; ++k) {
        const uint32_t op = cigar[k] & 15u;
        if ((cigar[k] >> 4) >= 4096u) return 0;
        blocks += (op == 0u || op == 7u || op == 8u);
    }
    if (blocks > 2u) return 0;
    for (k = 0; k < l_seq; ++k)
        if (qual[k] > 62u) return 0;
    for (k = 0; k < 4u; ++k) out[k] = (uint8_t)((uint32_t)start >> (8u * k));
    out[4] = (uint8_t)l_seq;
    out[5] = (uint8_t)(n_cigar | ((flag & MGP_FLAG_REVERSE) ? 0x80u : 0u));
    for (k = 0; k < 4u; ++k) {
        const uint32_t c = k < n_cigar ? cigar[k] : 0u;
        out[6 + 2 * k] = (uint8_t)c;
        out[7 + 2 * k] = (uint8_t)(c >> 8);
    }
    for (k = 0; k < MGP_PACK_MAX_LEN; ++k) {
        uint8_t v = 0xFF;  /* past l_seq: never counted */
        if (k < l_seq) {
            const uint32_t code = (k & 1u) ? (seq[k >> 1] & 15u) : (uint32_t)(seq[k >> 1] >> 4);
            const int b = code == 1u ? 0 : code == 2u ? 1 : code == 4u ? 2 : code == 8u ? 3 : -1;
            v = b < 0 ? (uint8_t)0xFF : (uint8_t)((qual[k] << 2) | (uint32_t)b);
        }
        out[14 + k] = v;
    }
    return 1;
}

/* 32-byte record (flag[i] has MGP_FLAG_PACK32): what the pileup reads of a short
 * read under ONE (min_baseq, min_dist_from_end) pair, four records per 128-byte
 * line (the pileup's gathers cost one line request each, whatever the record size):
 *   uint16 start                    0 <= start < 65536
 *   uint8  l_seq                    1 .. MGP_PACK_MAX_LEN
 *   uint8  n_cigar | min_dist << 3 | reverse << 7   n_cigar <= 4, min_dist <= 15
 *   uint16 cigar[4]                 len << 4 | op (len < 4096), unused entries 0
 *   3-bit codes                     code k (k < 50) at bit 96 + 3k of the record:
 *                                   0..3 = the base A, C, G, T, counted; 4 = not counted
 *   int8   min_baseq at byte 31     the threshold the codes were made for
 * Query position k is counted (pileup.py:55-95) iff it lies in the query range of
 * an aligned (M, =, X) operation as the reference walks the CIGAR (an insertion
 * does not advance the query position: quirk Q1), min_dist <= k < l_seq - min_dist
 * (all k when min_dist is 0), int8(qual[k]) >= min_baseq and the base is A, C, G
 * or T; the reference-range clamp and the pileup window are applied by the engine.
 * A read may be packed so iff it has SEQ and QUAL, 1 <= l_seq <= 50, n_cigar <= 4
 * with every length < 4096 and at most 2 aligned operations, 0 <= start < 65536,
 * -128 <= min_baseq <= 127 and 0 <= min_dist <= 15 (a negative min_dist_from_end
 * acts as 0). The engine refuses a run whose thresholds are not the records'
 * (MGP_E_INVALID). Records sit at 32-byte multiples. */
static inline MGP_HD int mgp_pack32_record(int32_t start, uint32_t l_seq, uint16_t flag, uint32_t n_cigar,
                                           const uint32_t *cigar, const uint8_t *seq, const uint8_t *qual,
                                           int32_t min_baseq, int32_t min_dist, uint8_t *out) {
    uint32_t k, blocks = 0, q = 0;
    uint64_t inblk = 0;  /* query positions inside an aligned operation's range */
    int32_t md = min_dist > 0 ? min_dist : 0;
    if ((flag & MGP_FLAG_NOSEQQUAL) || l_seq == 0u || l_seq > MGP_PACK_MAX_LEN || n_cigar > 4u) return 0;
    if (start < 0 || start >= 65536 || min_baseq < -128 || min_baseq > 127 || md > 15) return 0;
    for (k = 0; k < n_cigar; ++k) {
        const uint32_t op = cigar[k] & 15u, len = cigar[k] >> 4;
        if (len >= 4096u) return 0;
        if (op == 0u || op == 7u || op == 8u) {
            uint32_t j;
            ++blocks;
            for (j = q; j < q + len && j < l_seq; ++j) inblk |= 1ull << j;
        }
        if (op == 0u || op == 7u || op == 8u || op == 4u) q += len;
    }
    if (blocks > 2u) return 0;
    for (k = 0; k < 32u; ++k) out[k] = 0;
    out[0] = (uint8_t)start;
    out[1] = (uint8_t)((uint32_t)start >> 8);
    out[2] = (uint8_t)l_seq;
    out[3] = (uint8_t)(n_cigar | ((uint32_t)md << 3) | ((flag & MGP_FLAG_REVERSE) ? 0x80u : 0u));
    for (k = 0; k < n_cigar; ++k) {
        out[4 + 2 * k] = (uint8_t)cigar[k];
        out[5 + 2 * k] = (uint8_t)(cigar[k] >> 8);
    }
    for (k = 0; k < MGP_PACK_MAX_LEN; ++k) {
        uint32_t v = 4u;
        if (k < l_seq && ((inblk >> k) & 1u) && (int32_t)k >= md && (int32_t)k < (int32_t)l_seq - md &&
            (int32_t)(int8_t)qual[k] >= min_baseq) {
            const uint32_t code = (k & 1u) ? (seq[k >> 1] & 15u) : (uint32_t)(seq[k >> 1] >> 4);
            v = code == 1u ? 0u : code == 2u ? 1u : code == 4u ? 2u : code == 8u ? 3u : 4u;
        }
        {
            const uint32_t bit = 96u + 3u * k;
            out[bit >> 3] |= (uint8_t)(v << (bit & 7u));
            if ((bit & 7u) > 5u) out[(bit >> 3) + 1] |= (uint8_t)(v >> (8u - (bit & 7u)));
        }
    }
    out[31] = (uint8_t)(int8_t)min_baseq;
    return 1;
}

/* Expand a 32-byte record into the full layout in full[0..128): a counted base
 * becomes its code with quality 127, any other N with quality 0 (the same pileup
 * under the record's thresholds). */
static inline MGP_HD void mgp_unpack32_record(const uint8_t *p, uint8_t *full) {
    uint32_t k;
    const uint32_t lseq = p[2] <= MGP_PACK_MAX_LEN ? p[2] : MGP_PACK_MAX_LEN;
    const uint32_t nc = (p[3] & 7u) <= 4u ? (p[3] & 7u) : 4u;
    const uint32_t coff = mgp_cigar_offset(lseq), soff = mgp_seq_offset(lseq);
    for (k = 0; k < 128u; ++k) full[k] = 0;
    full[0] = p[0];
    full[1] = p[1];
    full[4] = (uint8_t)lseq;
    full[8] = (uint8_t)nc;
    full[10] = (uint8_t)((p[3] & 0x80u) ? MGP_FLAG_REVERSE : 0u);
    full[12] = (uint8_t)coff;
    for (k = 0; k < nc; ++k) {
        full[coff + 4 * k] = p[4 + 2 * k];
        full[coff + 4 * k + 1] = p[5 + 2 * k];
    }
    for (k = 0; k < lseq; ++k) {
        const uint32_t bit = 96u + 3u * k;
        const uint32_t w = (uint32_t)p[bit >> 3] | ((uint32_t)p[(bit >> 3) + 1] << 8);
        const uint32_t v = (w >> (bit & 7u)) & 7u;
        const uint8_t code = v < 4u ? (uint8_t)(1u << v) : (uint8_t)15;
        full[16 + k] = v < 4u ? (uint8_t)127 : (uint8_t)0;
        full[soff + (k >> 1)] |= (k & 1u) ? code : (uint8_t)(code << 4);
    }
}

typedef struct mgp_batch {
    int64_t         n_reads;
    const int32_t  *start;      /* reference_start; NULL: taken from each record on the device
                                   (every layout holds it; ABI 4)                        */
    const int32_t  *bc;         /* whitelist index of the CB tag, -1 if absent or not whitelisted */
    const int32_t  *tlen;       /* signed template_length                           */
    const uint16_t *flag;       /* BAM flag | MGP_FLAG_NOSEQQUAL                    */
    const uint8_t  *mapq;       /* mapping_quality                                  */
    const uint32_t *span;       /* max(reference span of the CIGAR, l_seq); NULL: taken
                                   from the records' CIGARs on the device (ABI v3.1)     */
    const uint64_t *rec_off;    /* byte offset of record i inside `payload`; NULL: dense
                                   records in BAM order, record i at i x payload_bytes /
                                   n_reads (a multiple of 16; ABI v3.1)                  */
    const uint8_t  *payload;
    int64_t         payload_bytes;
} mgp_batch;

/* A batch with 16-bit barcode and |tlen| columns (ABI 5): for contexts of at most 65535
 * cells whose reads all have |template_length| < 65536 (the engine keys duplicates on
 * abs(tlen) only, readers.py:128-131, so the sign is not needed). The records are dense
 * in BAM order (record i at i x payload_bytes / n_reads; start and span taken from the
 * records, as for an mgp_batch without those columns). 7 bytes of columns per read
 * instead of 11 cross the host link. */
typedef struct mgp_batch16 {
    int64_t         n_reads;
    const uint16_t *bc;         /* whitelist index of the CB tag; 0xFFFF if absent or not whitelisted */
    const uint16_t *abs_tlen;   /* |template_length|                                 */
    const uint16_t *flag;       /* BAM flag | MGP_FLAG_NOSEQQUAL                    */
    const uint8_t  *mapq;       /* mapping_quality                                  */
    const uint8_t  *payload;    /* dense records in BAM order                       */
    int64_t         payload_bytes;
} mgp_batch16;

/* Run-level statistics (readers.py:193-199). */
typedef struct mgp_stats {
    int64_t total_reads;                   /* every record fed (readers.py:93)               */
    int64_t filtered_reads;                /* reads kept after filters + dedup (readers.py:165) */
    int64_t n_barcodes;                    /* cells with >= 1 kept read (readers.py:196)      */
    int64_t duplicate_reads_with_length;   /* (start,strand,|tlen|) duplicates (readers.py:141-142) */
    int64_t duplicate_reads_position_only; /* (start,strand) duplicates (readers.py:143-144) */
    int64_t cells_passed;                  /* cells that produce a result (processors.py:22,30-31) */
    int32_t max_span;                      /* max declared span over valid reads             */
    int32_t error_bits;                    /* internal: nonzero => a check failed            */
} mgp_stats;

/* Results; every pointer is caller-owned host memory or NULL (= skip).
 * Per-position arrays are cell-major: [n_cells][mito_len][k]. Counts are the
 * strand-filtered per-position values the writers emit (pileup.py:128-154):
 * a cell that does not pass (processors.py:22,30-31) is all zero. */
typedef struct mgp_result {
    uint32_t *counts;      /* [n_cells][mito_len][8]: A_fwd,A_rev,C_fwd,C_rev,G_fwd,G_rev,T_fwd,T_rev */
    uint32_t *tn5;         /* [n_cells][mito_len][2]: tn5_cuts_fwd, tn5_cuts_rev (0 where depth==0) */
    uint32_t *depth;       /* [n_cells][mito_len]   filtered depth (pileup.py:150)  */
    uint32_t *n_reads;     /* [n_cells] kept reads (after dedup, before MAPQ)       */
    uint8_t  *any_paired;  /* [n_cells] any kept read is_paired (processors.py:34)  */
    uint8_t  *passed;      /* [n_cells] cell produced a result                      */
    uint32_t *covered;     /* [n_cells] positions with filtered depth > 0           */
    uint64_t *depth_sum;   /* [n_cells] sum of filtered depth                       */
    uint32_t *depth_max;   /* [n_cells] max filtered depth                          */
    uint32_t *median_lo;   /* [n_cells] lower middle of sorted covered depths       */
    uint32_t *median_hi;   /* [n_cells] upper middle (equal to lo when covered is odd) */
    uint32_t *first_read;  /* [n_cells] BAM index of the first kept read (dict order), UINT32_MAX if none */
    uint64_t *ref_tally;   /* [mito_len][4] sum over passing cells of A,C,G,T totals (all ranks after comm) */
    mgp_stats *stats;
} mgp_result;

/* Parameters of the device-side synthetic generator. */
typedef struct mgp_synth_params {
    uint64_t seed;
    int64_t  n_reads;
    int32_t  read_len;          /* 50 */
    int32_t  n_cells;           /* must equal the context's n_cells */
    const uint32_t *cell_cdf;   /* host array [n_cells]: cumulative thresholds in [0, 2^32) */
    const uint8_t  *ref_codes;  /* host array [mito_len]: reference bases as BAM 4-bit codes */
    int32_t  rec_align;         /* record placement: offsets are multiples of this (16..4096, pow2) */
    int32_t  pack;              /* 1: reads that fit get the packed 64-byte layout (MGP_FLAG_PACKED);
                                   2: the 32-byte layout (MGP_FLAG_PACK32) for pack_min_baseq */
    /* optional placement (host arrays, NULL = dense in BAM order at rec_align):
     * record i is written at rec_off[i] of a payload_bytes payload, e.g. the
     * producer placement of mgp_place_records (include/mgpileup_host.h) */
    const uint64_t *rec_off;
    int64_t  payload_bytes;
    /* optional cell shard of the global read set (cell_hi > cell_lo; the context's
     * n_cells must be cell_hi - cell_lo): only the reads of cells [cell_lo, cell_hi)
     * are kept, their barcode rebased to cell_lo, in BAM order; of the reads without
     * a whitelisted barcode those with read index % shard_world == shard_rank are
     * kept (shard_world = 0: none). rec_off, when given, places the kept reads
     * (index in the shard). One seed, one global set: the shards of ranks 0..N-1
     * over a partition of the cells are exactly the global set split by cell
     * (processors.py:112-144's per-cell parallelism, one GPU per cell range). */
    int32_t  cell_lo, cell_hi;
    int32_t  shard_rank, shard_world;
    int32_t  pack_min_baseq;    /* pack == 2: the min_baseq the 32-byte records are made for */
    int32_t  pack_min_dist;     /* pack == 2: the min_dist_from_end they are made for (0..15) */
    int64_t  n_rec_off;         /* entries of rec_off: must equal the reads generated (all n_reads,
                                   or a shard's kept reads), else MGP_E_INVALID */
} mgp_synth_params;

/* The pileup's 16-bit result rows, as the run leaves them in HBM (half the bytes of
 * the u32 arrays of mgp_result). Exact wherever the cell's window is not `wide`
 * (a cell window of more than 65535 reads: its 16-bit values saturate at 65535,
 * the HDF5 form of writers.py:205-218; mgp_fetch_cells gives the exact values). */
typedef struct mgp_rows16 {
    uint16_t *counts;   /* [cells][mito_len][8]: A_fwd, A_rev, ... T_rev */
    uint16_t *tn5;      /* [cells][mito_len][2]                          */
    uint16_t *depth;    /* [cells][mito_len]                             */
    uint8_t  *wide;     /* [cells][n_windows] (mgp_windows)              */
} mgp_rows16;

typedef struct mgp_ctx mgp_ctx;

int         mgp_abi_version(void);
const char *mgp_last_error(void);  /* message of the last failing call on this thread; the
                                     * wrapper raises the matching src/core/exceptions.py class */
int         mgp_device_count(int *out);

/* Replaces the per-run setup of CellProcessor(config, output_dir)
 * (src/processing/processors.py:59-61) + PipelineConfig (src/core/config.py:77-114). */
int  mgp_open(const mgp_config *cfg, int hip_device, mgp_ctx **out);
void mgp_close(mgp_ctx *ctx);

/* Pinned host memory helpers (hipHostMalloc / hipHostFree). */
int  mgp_host_alloc(int64_t bytes, void **out);
int  mgp_host_free(void *p);

/* Append a batch to the device-resident read set (async H2D on the copy stream).
 * Every record must lie inside the batch's payload (its offset, header and, for the
 * full layout, its CIGAR words); a batch that breaks this is checked on the device
 * and the next run fails with MGP_E_INVALID without reading any record (ABI 4).
 * Replaces the accumulation of reads_by_barcode in
 * BAMReader.collect_reads_by_barcode (src/processing/readers.py:85-165): the
 * batch is every fetch(mito_chr) record in BAM order, unfiltered. */
int  mgp_push_batch(mgp_ctx *ctx, const mgp_batch *batch);
/* Drop resident reads (keeps allocations). */
int  mgp_reset(mgp_ctx *ctx);
/* Number of resident reads / payload bytes. */
int  mgp_resident(mgp_ctx *ctx, int64_t *n_reads, int64_t *payload_bytes);

/* Run the whole hot path over the resident reads (async on the compute stream,
 * with one host wait for the input check's flag bits while the scan runs):
 * the input check (coordinate order as pysam's fetch yields it, readers.py:87-92;
 * declared spans; record placement), the record filters and dedup of
 * readers.py:95-150, process_barcode_worker
 * (processors.py:20-55) = generate_pileup + filter_strand_bias
 * (pileup.py:18-154) for every cell, the per-cell statistics of
 * processors.py:33-51 / writers.py:187-197 and the reference-allele tallies of
 * writers.py:221-222,340-349. */
int  mgp_run(mgp_ctx *ctx);
/* Wait for the last run; returns the run's check status (MGP_E_UNSORTED, ...).
 * A run whose speculative compact grouping did not fit the resident reads is
 * run again here on the fallback path before the status is returned. */
int  mgp_sync(mgp_ctx *ctx);
/* D2H the results of the last run into caller buffers (implies mgp_sync):
 * the dense form of the per-cell result dicts (processors.py:41-51) and of the
 * stats dict (readers.py:193-199). */
int  mgp_fetch(mgp_ctx *ctx, mgp_result *out);
/* mgp_fetch for cells [lo, hi) only: every per-cell and per-position array holds
 * hi - lo cells (cell lo first); ref_tally and stats are the run's. */
int  mgp_fetch_cells(mgp_ctx *ctx, int32_t lo, int32_t hi, mgp_result *out);
/* The 16-bit result rows of cells [lo, hi) (implies mgp_sync); NULL members are skipped. */
int  mgp_fetch_rows16(mgp_ctx *ctx, int32_t lo, int32_t hi, mgp_rows16 *out);

/* The txt count files on the device (ABI 6). Replaces IncrementalTextWriter.write_cell
 * and finalize's gzip at compresslevel 9 (src/file_io/writers.py:430-486): for each
 * listed cell, in order, its lines
 *   output.coverage.txt  "pos,barcode,depth"    (depth > 0)
 *   output.{A,C,G,T}.txt "pos,barcode,fwd,rev"  (depth > 0 and fwd + rev > 0)
 * (1-based pos, unbounded integers) are formatted from the run's count rows in HBM and
 * deflated there into one gzip member per (file, cell); a member is 0 bytes when the
 * cell has no line in that file. Each output file is its members concatenated in cell
 * order: gzip readers decompress it to exactly the reference's text. */
typedef struct mgp_txt_gz {
    int64_t        n_cells;      /* cells to write                                         */
    const int32_t *cells;        /* host: the context's cell index of each, in output order */
    const char    *names;        /* host: their barcodes, concatenated (no separators)     */
    const int64_t *name_off;     /* host: n_cells + 1 offsets into names (each 0..4096 bytes) */
    int64_t       *member_bytes; /* host out: [5][n_cells] member sizes, files coverage, A, C, G, T */
    int64_t       *text_bytes;   /* host out (may be NULL): [5][n_cells] decompressed sizes */
} mgp_txt_gz;
/* Format and deflate the members of `job` (implies mgp_sync; after mgp_run). *total_bytes
 * = the sum of member_bytes; the members stay on the device, file-major (all coverage
 * members in cell order, then A, C, G, T), until mgp_txt_gz_fetch or the next call. */
int  mgp_txt_gz_run(mgp_ctx *ctx, mgp_txt_gz *job, int64_t *total_bytes);
/* The last mgp_txt_gz_run's members (total_bytes of them) into dst (cap >= total). */
int  mgp_txt_gz_fetch(mgp_ctx *ctx, uint8_t *dst, int64_t cap);
/* The same from caller-supplied u32 rows (counts [n_rows][mito_len][8], depth
 * [n_rows][mito_len]) on `device`, no engine context: the members into dst (cap bytes;
 * MGP_E_INVALID with *total_bytes set when it is too small). */
int  mgp_txt_gz_rows(int device, const uint32_t *counts, const uint32_t *depth, int32_t n_rows, int32_t mito_len,
                     mgp_txt_gz *job, uint8_t *dst, int64_t cap, int64_t *total_bytes);
/* ABI v3.1: the 16-bit rows of every cell go to `rows` (pinned host arrays for all
 * cells from mgp_host_alloc, written by the device through their mapping) as the
 * windows complete: each streaming segment writes its windows' rows on a
 * device-to-host stream behind its pileup, while the copies of
 * later batches still run the other way; the wide flags follow the run, and mgp_sync
 * waits for all of it. The caller then needs no mgp_fetch_rows16. With min_reads > 1 the
 * gate (processors.py:22) also zeroes the target rows of the cells it drops, after the
 * last segment's rows have landed (ABI 4). A target may also be set during a
 * streaming run (not replaced): the rows of the windows piled so far are copied at
 * once, the later ones as they complete, so the caller can allocate it while the
 * first batches go in (ABI 4). NULL stops it (not during a streaming run). Replaces the
 * reference's per-cell write_cell after each worker (processors.py:112-144): results
 * leave the device while ingest continues. */
int  mgp_set_rows16_target(mgp_ctx *ctx, const mgp_rows16 *rows);
/* The 8-bit form of the same rows (ABI 7): a (cell, window) whose every count, tn5 cut
 * and depth is at most 255 (the pileup's flush knows it when it writes the window) has
 * its rows written here, one byte per value, and `narrow` set; the others go to the
 * 16-bit target as before (narrow 0). Exact values: the 16-bit target where narrow is 0
 * and wide is 0, these bytes where narrow is 1, mgp_fetch_cells where wide is 1. Half
 * the bytes leave the device for a cell of depth below 256 (the rows cross the host
 * link while later batches still come the other way). */
typedef struct mgp_rows8 {
    uint8_t *counts;    /* [cells][mito_len][8] (pinned, mgp_host_alloc) */
    uint8_t *tn5;       /* [cells][mito_len][2]                          */
    uint8_t *depth;     /* [cells][mito_len]                             */
    uint8_t *narrow;    /* [cells][n_windows]: 1 = this window's rows are here */
} mgp_rows8;
/* mgp_set_rows16_target(ctx, rows16) with the 8-bit target rows8 beside it (NULL: the
 * 16-bit target alone); rows16 NULL stops both. */
int  mgp_set_rows_target(mgp_ctx *ctx, const mgp_rows16 *rows16, const mgp_rows8 *rows8);
/* The HDF5 count datasets' chunks deflated on the device (ABI 7). Replaces the gzip-4
 * filter pipeline of IncrementalHDF5Writer's 11 datasets (src/file_io/writers.py:60-131:
 * A_fwd, A_rev, C_fwd, C_rev, G_fwd, G_rev, T_fwd, T_rev, tn5_cuts_fwd, tn5_cuts_rev in
 * counts.h5 and coverage in metadata.h5, u16 [mito_len][n_cols], chunks of
 * chunk_rows x chunk_cols): plane values min(v, 65535) of the last run's cells, column j
 * holding cell cell_of_col[j] (-1: zeros), edge chunks padded with 0, each chunk one
 * zlib stream (the H5Z_DEFLATE form; runs and dynamic Huffman codes, about zlib level
 * 4's size). One call covers the column chunks [col_chunk_lo, col_chunk_hi); its streams
 * stay on the device, plane-major, then row chunk, then column chunk, until
 * mgp_h5_tiles_fetch or the next call. The caller writes them with H5Dwrite_chunk. */
typedef struct mgp_h5_tiles {
    int64_t        n_cols;          /* columns of the datasets                           */
    const int32_t *cell_of_col;     /* host: the context's cell of each column, -1: none */
    int32_t        chunk_rows, chunk_cols;
    int32_t        col_chunk_lo, col_chunk_hi;
    int64_t       *chunk_bytes;     /* host out: [11][row chunks][hi - lo] stream sizes  */
    int64_t       *col_sums;        /* host out (may be NULL): [3][mito_len] per-position sums over
                                       this call's columns of coverage, tn5 fwd, tn5 rev (the
                                       QC report's, writers.py / report.py)               */
} mgp_h5_tiles;
int  mgp_h5_tiles_run(mgp_ctx *ctx, mgp_h5_tiles *job, int64_t *total_bytes);
int  mgp_h5_tiles_fetch(mgp_ctx *ctx, uint8_t *dst, int64_t cap);
/* Position windows of the pileup (the `wide` flags' second dimension). */
int  mgp_windows(mgp_ctx *ctx, int32_t *n_windows, int32_t *window_width);
/* Wait until the H2D copies of every batch pushed so far have completed: the caller may
 * then reuse those host buffers (until then a pushed batch's arrays must stay untouched).
 * A producer that decodes into a ring of pinned buffers calls it before refilling one. */
int  mgp_copy_wait(mgp_ctx *ctx);
/* The context's cells are whitelist indices [cell_lo, cell_hi) of the pushed batches
 * (n_cells = cell_hi - cell_lo): every pushed read's barcode index is rebased on the
 * device behind its copy (bc - cell_lo inside the range, -1 = not this context's
 * cells outside it), so the devices of a multi-GPU run can all take the same whole
 * batches and nothing routes reads on the host. Reads outside the range count only
 * toward total_reads, like reads without a whitelisted barcode; first_read then
 * indexes the whole pushed stream. Set it before the first push of a run (it stays for
 * the context's later runs). Without it a barcode index >= n_cells is an error
 * (MGP_E_INVALID). Replaces the reference's split of the barcodes
 * over its worker pool (processors.py:112-144) with a split by device. */
int  mgp_set_cell_range(mgp_ctx *ctx, int32_t cell_lo, int32_t cell_hi);
/* Append a batch with 16-bit barcode and |tlen| columns (mgp_batch16; the device widens
 * them behind the copy). Same semantics and errors as mgp_push_batch for a batch without
 * rec_off, start and span columns; MGP_E_INVALID when n_cells > 65535, or with a cell
 * range (mgp_set_cell_range: the columns then hold whole-whitelist indices) when
 * cell_hi > 65535 (index 0xFFFF is the no-barcode sentinel). Replaces the
 * reference's per-read SimpleRead fields (readers.py:153-163) at the host link. */
int  mgp_push_batch16(mgp_ctx *ctx, const mgp_batch16 *batch);
/* Streaming on (1) or off (0) for the next pushes (initially MGP_CFG_STREAM). */
int  mgp_set_streaming(mgp_ctx *ctx, int on);
/* Streaming: segments queued by pushes so far (all runs), and whether the last run
 * finished a streamed run (0: it ran resident). */
int  mgp_stream_info(mgp_ctx *ctx, int64_t *segments, int32_t *last_streamed);
/* Convenience: mgp_run + mgp_fetch. */
int  mgp_finish(mgp_ctx *ctx, mgp_result *out);

/* Per-stage device times (ms), averaged over the last `last_runs` runs (<= 64),
 * measured with HIP events recorded on the compute stream around each stage.
 * names: comma-separated stage names written into `names`. */
int  mgp_kernel_times(mgp_ctx *ctx, int last_runs, float *ms, int max_n, int *n_out, char *names, int names_len);
/* Which stages the next runs bracket with HIP events: all (1, the default) or the
 * pileup's only (0). Every event is a marker between two kernels of the compute
 * stream, so a run timed for its wall clock records only the pileup's;
 * mgp_kernel_times averages each stage over the runs that recorded it. */
int  mgp_set_stage_timing(mgp_ctx *ctx, int all_stages);

/* RCCL: rank 0 creates the unique id (128 bytes), every rank joins. After init,
 * mgp_run all-reduces ref_tally over the communicator (no reference
 * counterpart: the reference sums position_base_counts in one process,
 * writers.py:221-222). */
int  mgp_comm_unique_id(uint8_t *out128);
int  mgp_comm_init(mgp_ctx *ctx, const uint8_t *uid128, int nranks, int rank);

/* Fill the resident read set with the synthetic workload (replaces it). */
int  mgp_synth_generate(mgp_ctx *ctx, const mgp_synth_params *p);
/* Copy resident inputs back to host (used by tests to check the device
 * generator against the host mirror). Any pointer may be NULL. */
int  mgp_download_inputs(mgp_ctx *ctx, int32_t *start, int32_t *bc, int32_t *tlen,
                         uint16_t *flag, uint8_t *mapq, uint32_t *span,
                         uint64_t *rec_off, uint8_t *payload);

#ifdef __cplusplus
}
#endif
#endif /* MGPILEUP_H */
