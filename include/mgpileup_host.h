/*
 * mgpileup_host.h — host-side C-ABI of libmgphost.so (no GPU needed).
 *
 * BAM ingest for the engine: replaces what pysam does under
 * `BAMReader.collect_reads_by_barcode` (src/processing/readers.py:85-165):
 * BGZF inflate (multithreaded), `.bai` seek to the chrM records
 * (`bam.fetch(mito_chr)`, readers.py:87-88), record decode, CB-tag whitelist
 * lookup (readers.py:104-111), and packing into the engine's SoA batch +
 * payload records (include/mgpileup.h). Also the two reader-side checks
 * (readers.py:35-61) and the barcode auto-extraction pass
 * (src/file_io/barcode_extraction.py:12-46).
 *
 * pysam semantics kept: query_sequence includes soft clips and is None when
 * l_seq == 0; query_qualities is None when l_seq == 0 or qual[0] == 0xFF (both
 * mapped to MGP_FLAG_NOSEQQUAL); cigartuples from the BAM CIGAR (or the CG tag
 * for > 65535 operations); template_length is the signed TLEN.
 */
#ifndef MGPILEUP_HOST_H
#define MGPILEUP_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mgp_bam mgp_bam;

/* Decoded reads of one reference, in BAM order, as an engine batch. The arrays
 * are owned by the library until mgp_bam_free_batch. */
typedef struct mgp_bam_batch {
    int64_t   n_reads;
    int32_t  *start;
    int32_t  *bc;
    int32_t  *tlen;
    uint16_t *flag;
    uint8_t  *mapq;
    uint32_t *span;
    uint64_t *rec_off;
    uint8_t  *payload;
    int64_t   payload_bytes;
    int64_t   n_with_tag;      /* records carrying the barcode tag (any type) */
    int64_t   first_tag_index; /* index of the first record with the tag, -1 if none */
} mgp_bam_batch;

const char *mgp_host_last_error(void);

/* Open a BAM (BGZF) file and parse its header; uses `<path>.bai` when present. */
int  mgp_bam_open(const char *path, int n_threads, mgp_bam **out);
void mgp_bam_close(mgp_bam *bam);
int  mgp_bam_n_refs(mgp_bam *bam);
const char *mgp_bam_ref_name(mgp_bam *bam, int tid);
int64_t mgp_bam_ref_len(mgp_bam *bam, int tid);
int  mgp_bam_has_index(mgp_bam *bam);

/* Barcode whitelist: CB value -> index in `barcodes` (last duplicate wins, as
 * the reference's dict); `tag` is the 2-character tag name (e.g. "CB"). */
int  mgp_bam_set_barcodes(mgp_bam *bam, const char *tag, const char *const *barcodes, int n);

/* Bulk calling (readers.py:74,97-99): every record is assigned to `cell`
 * whatever its tag; -1 switches back to whitelist lookup. Reset by
 * mgp_bam_set_barcodes. */
int  mgp_bam_set_bulk(mgp_bam *bam, int32_t cell);

/* pack != 0: records that fit the packed 64-byte layout (include/mgpileup.h,
 * MGP_FLAG_PACKED) are written in it; the pileup reads half the bytes per read.
 * Packing drops the code and quality of non-ACGT bases, so callers that rebuild
 * query_sequence/query_qualities (the SimpleRead API) leave it off (default). */
int  mgp_bam_set_pack(mgp_bam *bam, int pack);
/* 32-byte records (MGP_FLAG_PACK32, include/mgpileup.h) for reads that fit, made for
 * the run's min_baseq (in [-128, 127]) and min_dist_from_end (<= 15); the others get
 * the packed 64-byte or the full layout. Turns packing on. The engine refuses them
 * under other thresholds. */
int  mgp_bam_set_pack32(mgp_bam *bam, int on, int min_baseq, int min_dist);

/* Payload placement of mgp_bam_read_ref (MGP_PLACE_DENSE default, or
 * MGP_PLACE_PAIRED: see mgp_place_records below). */
int  mgp_bam_set_placement(mgp_bam *bam, int mode);

/* Decode every record of reference `tid` (fetch(contig) order) into `out`.
 * Records are placed at multiples of `rec_align` bytes (16..4096, power of 2). */
int  mgp_bam_read_ref(mgp_bam *bam, int tid, int rec_align, mgp_bam_batch *out);
void mgp_bam_free_batch(mgp_bam_batch *b);

/* Records of reference `tid` per the index's metadata pseudo-bin (mapped + placed
 * unmapped, as `samtools idxstats` counts them): the engine's reserve for a streamed
 * run. -1 without an index or without the pseudo-bin. */
int64_t mgp_bam_ref_records(mgp_bam *bam, int tid);

/* Streaming decode of reference `tid` in batches: the one pass of
 * readers.py:84-93 (`for read in bam.fetch(mito_chr)`), handed out as the engine's
 * batches while later BGZF blocks are still being read, so the decode overlaps the
 * device's copies and compute. The settings of `bam` at open (barcodes, bulk, packing,
 * placement) apply; `bam` must outlive the stream. */
typedef struct mgp_bam_stream mgp_bam_stream;
int mgp_bam_stream_open(mgp_bam *bam, int tid, int rec_align, mgp_bam_stream **out);
/* Decode the next records into the caller's arrays (`into`'s start, bc, tlen, flag,
 * mapq, span and rec_off hold cap_reads entries, payload cap_payload bytes; e.g.
 * pinned memory from mgp_host_alloc): as many records as fit both, in BAM order, with
 * the batch's own payload placement (offsets from 0; paired lines never span
 * batches: cap_payload needs 64 KiB + 256 bytes per whitelisted cell of slack).
 * Sets into->n_reads and payload_bytes (256 zeroed bytes follow the payload when
 * they fit); n_with_tag / first_tag_index count over the stream so far. Returns the
 * records decoded, 0 at the end of the reference, -1 on error. */
int64_t mgp_bam_stream_next(mgp_bam_stream *s, int64_t cap_reads, int64_t cap_payload, mgp_bam_batch *into);
void mgp_bam_stream_close(mgp_bam_stream *s);

/* Tag presence check of BAMReader._validate_bam_file (readers.py:53-59): index of
 * the first of the first `max_records` records of `tid` that carries `tag`, -1
 * if none does, -2 on error. `*n_checked` = records examined. */
int64_t mgp_bam_find_tag(mgp_bam *bam, int tid, const char *tag, int64_t max_records, int64_t *n_checked);

/* Barcode auto-extraction pass (barcode_extraction.py:12-46): counts of the
 * tag's string value over records of `tid` that are neither unmapped nor
 * duplicates. Returns the number of distinct values; `*blob` receives
 * "value\0count\n"-free packed entries: for each value, a NUL-terminated string
 * followed by an int64 count (8 bytes, little endian). Free with mgp_host_buf_free. */
int64_t mgp_bam_count_tag(mgp_bam *bam, int tid, const char *tag, uint8_t **blob, int64_t *blob_bytes);
void mgp_host_buf_free(void *p);

/* txt output at scale (IncrementalTextWriter, src/file_io/writers.py:430-510):
 * appends (append != 0) or writes `<prefix>.{coverage,A,C,G,T}.txt.gz` for the
 * cells `cells[0..n_write)` in that order, named `names[k]`, from the engine's
 * cell-major `counts` [*][mito_len][8] and `depth` [*][mito_len] (mgp_result).
 * Lines "pos,bc,depth" / "pos,bc,fwd,rev" (1-based pos) for depth > 0 (and
 * fwd+rev > 0). Each group of cells is one gzip member at `level`, deflated on
 * `n_threads` threads (0 = all cores). */
int mgp_txt_write_cells(const char *prefix, const uint32_t *counts, const uint32_t *depth, int64_t mito_len,
                        const int64_t *cells, int64_t n_write, const char *const *names, int level,
                        int n_threads, int append);
/* The same from the engine's exact 16-bit rows (mgp_fetch_rows16 when no window is
 * wide): half the bytes of the u32 form between device and host. */
int mgp_txt_write_cells16(const char *prefix, const uint16_t *counts, const uint16_t *depth, int64_t mito_len,
                          const int64_t *cells, int64_t n_write, const char *const *names, int level,
                          int n_threads, int append);

/* Write an engine batch as a coordinate-sorted BAM (test and benchmark inputs; the
 * inverse of mgp_bam_read_ref). References `ref_names`/`ref_lens`; every record goes
 * to reference `tid`. Record i carries `tag`:Z:barcodes[bc[i]] when bc[i] >= 0;
 * records with bc < 0 alternate between `unlisted` (if not NULL) and no tag.
 * BGZF blocks are deflated at `level` on `n_threads` threads; `write_index` also
 * writes `<path>.bai`. */
int mgp_bam_write(const char *path, const char *const *ref_names, const int64_t *ref_lens, int n_ref, int tid,
                  const mgp_bam_batch *batch, const char *const *barcodes, int n_barcodes, const char *tag,
                  const char *unlisted, int level, int n_threads, int write_index);

/* HDF5 output at scale (IncrementalHDF5Writer, src/file_io/writers.py:60-406):
 * deflates every (crow x ccol) chunk of a row-major `rows x cols` array of
 * `elem_size`-byte elements, in the form of the HDF5 deflate filter (zlib
 * stream of the full chunk, edge chunks padded with 0), on `n_threads`
 * threads. Chunks are numbered row-major over the chunk grid; chunk t occupies
 * blob[offsets[t], offsets[t+1]) (`offsets` has n_chunks + 1 entries).
 * Returns the number of chunks, -1 on error. Free `*blob` with mgp_host_buf_free. */
int64_t mgp_deflate_tiles(const void *data, int64_t rows, int64_t cols, int32_t elem_size, int64_t crow,
                          int64_t ccol, int level, int n_threads, uint8_t **blob, int64_t *offsets);

/* The HDF5 planes straight from the engine's cell-major rows (IncrementalHDF5Writer,
 * writers.py:200-218): plane e is plane[p][j] = min(rows[cell_of_col[j]][p][elems[e]],
 * 65535) (0 where cell_of_col[j] < 0) as a row-major [L][n_cols] u16 array; `rows` is
 * [n_rows][L][row_elems] of elem_size 2 (the exact 16-bit rows) or 4 (u32). Each plane
 * is cut into (crow x ccol) chunks and deflated as mgp_deflate_tiles does, all planes of
 * a chunk from one read of the cells' rows, on n_threads threads. Chunk t of plane e
 * is blob[offsets[e * n_chunks + t], offsets[e * n_chunks + t + 1]) (`offsets` has
 * n_planes * n_chunks + 1 entries). Returns n_chunks per plane, -1 on error. */
int64_t mgp_h5_plane_tiles(const void *rows, int32_t elem_size, int64_t row_elems, int64_t n_rows, int64_t L,
                           const int64_t *cell_of_col, int64_t n_cols, const int32_t *elems, int32_t n_planes,
                           int64_t crow, int64_t ccol, int level, int n_threads, uint8_t **blob, int64_t *offsets);

/* Payload placement for producers: rec_off[i] for records of rec_bytes[i]
 * bytes, in BAM order. MGP_PLACE_DENSE: consecutive, each rounded up to
 * rec_align. MGP_PLACE_PAIRED: two consecutive packed (64-byte) records of one
 * cell share a 128-byte line, four consecutive 32-byte (MGP_FLAG_PACK32) records
 * of one cell likewise (one streaming pass, lines opened in BAM order;
 * reads the engine's filters drop pair among themselves; full records take
 * 128-byte aligned slots of their own), so one line request of the pileup's
 * gather serves two reads of the cell it piles. With the start and tlen columns
 * (either may be NULL: no such rule), a read that repeats the start, strand and
 * |tlen| of an earlier read of its cell (a duplicate whenever dedup is on,
 * readers.py:118-150) is placed with the dropped reads. Returns the payload
 * bytes, -1 on error. Replaces no reference code (pysam hands out Python
 * objects). */
#define MGP_PLACE_DENSE  0
#define MGP_PLACE_PAIRED 1
int64_t mgp_place_records(int64_t n, const int32_t *bc, const uint16_t *flag, const int32_t *start,
                          const int32_t *tlen, const uint32_t *rec_bytes, int32_t n_cells, int32_t mode,
                          int32_t rec_align, uint64_t *rec_off);

/* Cell sharding: gather the payload records idx[0..m) of a
 * batch into a new payload for one device. mgp_gather_offsets reads each
 * record's size from its header (mgp_record_bytes; any source placement),
 * rebases the cell ids to [cell_lo, cell_lo + n_cells) (-1 outside), places the
 * subset with mgp_place_records(mode, rec_align; start/tlen as given, may be
 * NULL) and returns the new payload
 * bytes (-1 on error). mgp_gather_records copies the records there on
 * n_threads threads; `out` must be zero-filled by the caller (gaps stay as they
 * are). Replaces no reference code: the reference runs on one process. */
int64_t mgp_gather_offsets(const uint8_t *payload, const uint64_t *rec_off, const uint16_t *flag, const int32_t *bc,
                           const int32_t *start, const int32_t *tlen, int64_t n_total, int64_t payload_bytes,
                           const int64_t *idx, int64_t m, int32_t cell_lo, int32_t n_cells, int32_t mode,
                           int32_t rec_align, uint64_t *out_off);
int mgp_gather_records(const uint8_t *payload, const uint64_t *rec_off, const uint16_t *flag, int64_t n_total,
                       int64_t payload_bytes, const int64_t *idx, int64_t m, const uint64_t *out_off,
                       int64_t out_bytes, uint8_t *out, int n_threads);
/* The reads of each cell range [bounds[d], bounds[d + 1]) (d < nd; bounds not
 * decreasing): their indices, range by range and in batch order inside a range,
 * into idx (room for n), their numbers into counts[nd]; returns the total (-1 on
 * bad arguments). One pass for all the devices of a multi-device stream. */
int64_t mgp_split_by_range(const int32_t *bc, int64_t n, const int64_t *bounds, int32_t nd, int64_t *counts,
                           int64_t *idx);

/* The 16-bit columns of a decoded batch (mgp_batch16, include/mgpileup.h): bc16 =
 * bc (0xFFFF for < 0), tlen16 = |tlen|. Returns bit 0 set when the records are dense
 * at one stride (payload_bytes = n x stride, stride a multiple of 16, and every
 * rec_off[i] = stride x i when rec_off is given: the batch may go without rec_off),
 * bit 1 set when every key fits (barcode index and |tlen| below 0xFFFF, n_cells <=
 * 0xFFFF); both (3): the batch may go as an mgp_batch16 with bc16 / tlen16. -1 on bad
 * arguments. Replaces nothing in the reference: the
 * per-read fields of readers.py:153-163, in the form the host link carries. */
int mgp_batch_columns16(int64_t n, const int32_t *bc, const int32_t *tlen, const uint64_t *rec_off,
                        int64_t payload_bytes, int32_t n_cells, uint16_t *bc16, uint16_t *tlen16, int n_threads);

/* One device's batch of a routed stream (mgp_route_batch): caller-owned arrays of
 * cap_reads entries and cap_payload bytes; the router fills n_reads, payload_bytes
 * (plus 256 zeroed bytes after it) and narrow: 1 = bc16 / tlen16 (local cell index,
 * |tlen|) with the records dense at one stride (mgp_push_batch16), 0 = bc32 / tlen32 /
 * rec_off (mgp_push_batch). flag, mapq and payload in both forms. */
typedef struct mgp_route_part {
    int64_t   cap_reads, cap_payload;
    uint16_t *bc16, *tlen16;
    int32_t  *bc32, *tlen32;
    uint16_t *flag;
    uint8_t  *mapq;
    uint64_t *rec_off;
    uint8_t  *payload;
    int64_t   n_reads, payload_bytes;   /* out */
    int32_t   narrow, pad;              /* out */
} mgp_route_part;

/* The multi-device stream's router (the reference's split of the
 * barcodes over its pool, processors.py:112-144, becomes a split over devices): every
 * read of the batch (records at rec_off[i], or dense at payload_bytes / n x i when
 * rec_off is NULL) whose barcode index lies in [bounds[d], bounds[d + 1]) and whose flag
 * passes readers.py:96 (not unmapped / secondary / supplementary) goes to parts[d], in
 * batch order, its index rebased to bounds[d]; the other reads go nowhere (they count
 * only toward total_reads). first_seen (may be NULL; bounds[n_parts] - bounds[0]
 * entries, 0xFFFFFFFF = not yet): lowered to first_index + i for each routed read i, so
 * over a stream it ends as each cell's first read in BAM order (reads_by_barcode's
 * insertion order, readers.py:104-163). Returns 0, 1 when a part's arrays are too small
 * (nothing written: route fewer reads at once), -1 on bad arguments or a record outside
 * the payload. */
int mgp_route_batch(int64_t n, const int32_t *bc, const int32_t *tlen, const uint16_t *flag, const uint8_t *mapq,
                    const uint64_t *rec_off, const uint8_t *payload, int64_t payload_bytes, int32_t n_parts,
                    const int32_t *bounds, int64_t first_index, uint32_t *first_seen, mgp_route_part *parts,
                    int n_threads);

/* 32-byte records (MGP_FLAG_PACK32, include/mgpileup.h) from a batch's full-layout
 * records, for one run's (min_baseq, min_dist_from_end): out32[i] (32 bytes, dense
 * in batch order) and out_flag[i] = flag[i] | MGP_FLAG_PACK32 for every full record
 * with SEQ and QUAL that fits the layout; the others get a zeroed slot and their own
 * flag word (the caller keeps their records). The same mgp_pack32_record the BAM
 * decoder calls per decoded record: the per-base filter of pileup.py:67-88 moved to
 * the producer. Returns the number of records packed, -1 on error (a record outside
 * the payload). */
int64_t mgp_repack32(int64_t n, const uint8_t *payload, int64_t payload_bytes, const uint64_t *rec_off,
                     const uint16_t *flag, int32_t min_baseq, int32_t min_dist, uint8_t *out32,
                     uint16_t *out_flag, int n_threads);

#ifdef __cplusplus
}
#endif
#endif /* MGPILEUP_HOST_H */
