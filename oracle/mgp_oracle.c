/*
 * mgp_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of the reference
 * mgatk2 hot path, used as the parity checker for the HIP engine and as the
 * `cpu_baseline` leg of bench.py ("port"). Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline may load it. The product path never does.
 *
 * It consumes exactly the engine's input (mgp_batch SoA + payload records, see
 * include/mgpileup.h) and produces exactly the engine's output (mgp_result), but
 * computes them the way the reference does, in the reference's order:
 *
 *   oracle_run  step 1  BAMReader.collect_reads_by_barcode (readers.py:85-165):
 *                       one pass in BAM order; skip unmapped/secondary/supplementary
 *                       (:96-97) and reads without a whitelisted CB (:104-111);
 *                       two per-barcode "seen" sets (:118-150), both always updated,
 *                       both duplicate counters always incremented, the read dropped
 *                       by the selected mode; kept reads appended per barcode in
 *                       first-seen barcode order (defaultdict insertion order).
 *               step 2  process_barcode_worker (processors.py:20-55) per barcode:
 *                       min-reads gate (:22), generate_pileup (pileup.py:18-126),
 *                       filter_strand_bias (pileup.py:128-154), depth stats.
 *               step 3  writer-side statistics: median (np.median, writers.py:190),
 *                       reference-allele tallies over written cells
 *                       (writers.py:220-222 / 457-458).
 *
 * Pinned against the reference itself: tests/golden/ holds vectors produced by
 * running the reference (imported from /root/reference with stub pysam/h5py, see
 * tests/golden/make_golden.py) on the same inputs; tests/test_oracle_golden.py
 * checks this file against them bit for bit.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mgpileup.h"

#define ORC_OK 0
#define ORC_E_INVALID (-1)
#define ORC_E_OOM (-3)
#define ORC_E_BADREAD (-5)

/* ---- open-addressing hash set of (bc, start, strand[, |tlen|]) keys -------- */
typedef struct {
    int32_t bc, start;
    uint32_t tl;     /* |tlen| or 0xFFFFFFFF for the position-only set */
    uint32_t strand; /* 0/1, 2 = empty slot */
} key_t;

typedef struct {
    key_t *slot;
    uint64_t mask, used;
} kset_t;

static uint64_t khash(const key_t *k) {
    uint64_t z = (uint64_t)(uint32_t)k->bc * 0x9E3779B97F4A7C15ull ^ (uint64_t)(uint32_t)k->start * 0xC2B2AE3D27D4EB4Full ^
                 (uint64_t)k->tl * 0x165667B19E3779F9ull ^ (uint64_t)k->strand * 0x27D4EB2F165667C5ull;
    z ^= z >> 31;
    z *= 0xbf58476d1ce4e5b9ull;
    z ^= z >> 29;
    return z;
}

static int kset_init(kset_t *s, uint64_t expect) {
    uint64_t cap = 1024;
    while (cap < expect * 2) cap <<= 1;
    s->slot = (key_t *)malloc(cap * sizeof(key_t));
    if (!s->slot) return ORC_E_OOM;
    for (uint64_t i = 0; i < cap; ++i) s->slot[i].strand = 2;
    s->mask = cap - 1;
    s->used = 0;
    return ORC_OK;
}

static int kset_grow(kset_t *s) {
    kset_t n;
    if (kset_init(&n, (s->mask + 1)) != ORC_OK) return ORC_E_OOM;
    for (uint64_t i = 0; i <= s->mask; ++i) {
        if (s->slot[i].strand == 2) continue;
        uint64_t h = khash(&s->slot[i]) & n.mask;
        while (n.slot[h].strand != 2) h = (h + 1) & n.mask;
        n.slot[h] = s->slot[i];
        n.used++;
    }
    free(s->slot);
    *s = n;
    return ORC_OK;
}

/* returns 1 if the key was present; inserts it in any case (set.add). */
static int kset_test_add(kset_t *s, const key_t *k, int *err) {
    if ((s->used + 1) * 2 > s->mask + 1) {
        if (kset_grow(s) != ORC_OK) {
            *err = ORC_E_OOM;
            return 0;
        }
    }
    uint64_t h = khash(k) & s->mask;
    for (;;) {
        key_t *e = &s->slot[h];
        if (e->strand == 2) {
            *e = *k;
            s->used++;
            return 0;
        }
        if (e->bc == k->bc && e->start == k->start && e->tl == k->tl && e->strand == k->strand) return 1;
        h = (h + 1) & s->mask;
    }
}

/* ---- packed record -> the full layout (include/mgpileup.h) -------------------
 * A non-ACGT base (0xFF; any byte >= 252) becomes code 15 (N) with quality 0:
 * pileup.py:83-86 never counts it, whatever its quality. */
static void unpack_packed(const uint8_t *p, uint8_t *full) {
    int32_t start;
    uint32_t k;
    memcpy(&start, p, 4);
    const uint32_t lseq = p[4] <= MGP_PACK_MAX_LEN ? p[4] : MGP_PACK_MAX_LEN;
    const uint16_t ncig = (uint16_t)(p[5] & 0x7Fu) <= 4 ? (uint16_t)(p[5] & 0x7Fu) : 4;
    const uint16_t flag = (p[5] & 0x80u) ? (uint16_t)MGP_FLAG_REVERSE : 0;
    const uint32_t coff = mgp_cigar_offset(lseq), soff = mgp_seq_offset(lseq);
    memset(full, 0, 128);
    memcpy(full, &start, 4);
    memcpy(full + 4, &lseq, 4);
    memcpy(full + 8, &ncig, 2);
    memcpy(full + 10, &flag, 2);
    memcpy(full + 12, &coff, 4);
    for (k = 0; k < ncig; ++k) {
        const uint32_t c = (uint32_t)p[6 + 2 * k] | ((uint32_t)p[7 + 2 * k] << 8);
        memcpy(full + coff + 4 * k, &c, 4);
    }
    for (k = 0; k < lseq; ++k) {
        const uint8_t v = p[14 + k];
        const int never = v >= 252; /* 0xFF; quality 63 does not exist in the layout */
        const uint8_t code = never ? 15 : (uint8_t)(1u << (v & 3u));
        full[16 + k] = never ? 0 : (uint8_t)(v >> 2);
        full[soff + (k >> 1)] |= (k & 1) ? code : (uint8_t)(code << 4);
    }
}

/* ---- one read's pileup (pileup.py:32-95) ------------------------------------ */
static void pile_read(const uint8_t *rec, const mgp_config *cfg, uint32_t *bc8, uint32_t *tn5) {
    int32_t start;
    uint32_t lseq, coff;
    uint16_t ncig, flag;
    memcpy(&start, rec, 4);
    memcpy(&lseq, rec + 4, 4);
    memcpy(&ncig, rec + 8, 2);
    memcpy(&flag, rec + 10, 2);
    memcpy(&coff, rec + 12, 4);
    const uint8_t *qual = rec + 16;
    const uint8_t *seq = rec + mgp_seq_offset(lseq);
    const uint8_t *cig = rec + coff;
    const int64_t L = cfg->mito_len;
    const int is_reverse = (flag & MGP_FLAG_REVERSE) != 0;
    const int strand_idx = is_reverse ? 1 : 0;
    const int64_t read_length = lseq;

    /* pileup.py:43-50 */
    if (is_reverse) {
        int64_t sp = (int64_t)start + read_length - 1;
        if (sp >= 0 && sp < L) tn5[sp * 2 + 1]++;
    } else {
        int64_t sp = start;
        if (sp >= 0 && sp < L) tn5[sp * 2 + 0]++;
    }

    int64_t ref_pos = start, query_pos = 0;
    for (uint32_t o = 0; o < ncig; ++o) {
        uint32_t c;
        memcpy(&c, cig + 4 * o, 4);
        const uint32_t op = c & 15u;
        const int64_t length = c >> 4;
        if (op == 0 || op == 7 || op == 8) {
            int64_t start_refpos = ref_pos > 0 ? ref_pos : 0;
            int64_t end_refpos = ref_pos + length < L ? ref_pos + length : L;
            if (start_refpos >= end_refpos) {
                query_pos += length;
                ref_pos += length;
                continue;
            }
            int64_t offset = start_refpos - ref_pos;
            int64_t vq0, vq1;
            if (cfg->min_dist_from_end > 0) {
                vq0 = cfg->min_dist_from_end;
                vq1 = read_length - cfg->min_dist_from_end;
            } else {
                vq0 = 0;
                vq1 = read_length;
            }
            for (int64_t i = 0; i < end_refpos - start_refpos; ++i) {
                int64_t cq = query_pos + offset + i;
                if (!(vq0 <= cq && cq < vq1)) continue;
                if (cq >= read_length) continue; /* Python would raise; unreachable while min_dist > 0 */
                if ((int)(int8_t)qual[cq] < cfg->min_baseq) continue; /* np.int8 cast, readers.py:158 */
                const uint8_t sb = seq[cq >> 1];
                const uint32_t code = (cq & 1) ? (sb & 15u) : (sb >> 4);
                int bi;
                switch (code) { /* chr(b).upper() in ACGT */
                    case 1: bi = 0; break;
                    case 2: bi = 1; break;
                    case 4: bi = 2; break;
                    case 8: bi = 3; break;
                    default: bi = -1;
                }
                if (bi < 0) continue;
                bc8[(start_refpos + i) * 8 + bi * 2 + strand_idx]++;
            }
            query_pos += length;
            ref_pos += length;
        } else if (op == 2 || op == 3) {
            ref_pos += length;
        } else if (op == 4) {
            query_pos += length;
        }
        /* op 1 (I), 5 (H), 6 (P): no branch in pileup.py:55-95 */
    }
}

static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return x < y ? -1 : x > y;
}

/* Full restatement. `order_out` (optional, [n_cells]) receives the barcode
 * indices in first-seen order, -1 padded; returns the number of such barcodes
 * through *n_order. */
int oracle_run(const mgp_config *cfg, const mgp_batch *b, mgp_result *out, int32_t *order_out, int32_t *n_order) {
    if (!cfg || !b || !out) return ORC_E_INVALID;
    const int64_t n = b->n_reads;
    const int nc = cfg->n_cells;
    const int64_t L = cfg->mito_len;
    int err = ORC_OK;

    /* step 1: reader + dedup (readers.py:85-165) */
    int64_t *cnt = (int64_t *)calloc((size_t)nc + 1, sizeof(int64_t));
    int32_t *order = (int32_t *)malloc(((size_t)nc + 1) * sizeof(int32_t));
    uint8_t *keep = (uint8_t *)calloc((size_t)n + 1, 1);
    if (!cnt || !order || !keep) return ORC_E_OOM;
    int32_t n_seen = 0;
    kset_t with_len, pos_only;
    const int skip = cfg->dedup_mode == MGP_DEDUP_NONE;
    const int use_fragment_length = cfg->dedup_mode == MGP_DEDUP_START_FRAG;
    if (!skip) {
        if (kset_init(&with_len, (uint64_t)(n / 2 + 16)) || kset_init(&pos_only, (uint64_t)(n / 2 + 16))) return ORC_E_OOM;
    }
    int64_t filtered = 0, dup_len = 0, dup_pos = 0;
    for (int64_t i = 0; i < n; ++i) {
        const uint16_t f = b->flag[i];
        if (f & (MGP_FLAG_UNMAPPED | MGP_FLAG_SECONDARY | MGP_FLAG_SUPPLEMENTARY)) continue;
        const int32_t bc = b->bc[i];
        if (bc < 0 || bc >= nc) continue;
        if (!skip) {
            key_t kl, kp;
            const int64_t t = b->tlen[i];
            kl.bc = kp.bc = bc;
            kl.start = kp.start = b->start[i];
            kl.strand = kp.strand = (f & MGP_FLAG_REVERSE) ? 1u : 0u;
            kl.tl = (uint32_t)(t < 0 ? -t : t);
            kp.tl = 0xFFFFFFFFu;
            const int is_fragment_length_dup = kset_test_add(&with_len, &kl, &err);
            const int is_position_only_dup = kset_test_add(&pos_only, &kp, &err);
            if (err) return err;
            if (is_fragment_length_dup) dup_len++;
            if (is_position_only_dup) dup_pos++;
            if (use_fragment_length && is_fragment_length_dup) continue;
            if (!use_fragment_length && is_position_only_dup) continue;
        }
        /* SimpleRead(...) conversion: query_sequence.encode / np.array(query_qualities) */
        if (f & MGP_FLAG_NOSEQQUAL) {
            err = ORC_E_BADREAD;
            break;
        }
        if (cnt[bc] == 0) order[n_seen++] = bc;
        cnt[bc]++;
        keep[i] = 1;
        filtered++;
    }
    if (!skip) {
        free(with_len.slot);
        free(pos_only.slot);
    }
    if (err) {
        free(cnt);
        free(order);
        free(keep);
        return err;
    }

    /* 32-byte records stand for one (min_baseq, min_dist) pair (bytes 31 and 3,
     * include/mgpileup.h): a run under another pair is refused, as the engine does */
    for (int64_t i = 0; i < n; ++i)
        if (b->flag[i] & MGP_FLAG_PACK32) {
            const uint8_t *r = b->payload + b->rec_off[i];
            const int32_t md = cfg->min_dist_from_end > 0 ? cfg->min_dist_from_end : 0;
            if ((int32_t)(int8_t)r[31] != cfg->min_baseq || (int32_t)((r[3] >> 3) & 15u) != md) {
                err = ORC_E_BADREAD;
                break;
            }
        }
    if (err) {
        free(cnt);
        free(order);
        free(keep);
        return err;
    }

    /* per-barcode read lists in BAM order (reads_by_barcode[barcode].append) */
    int64_t *off = (int64_t *)malloc(((size_t)nc + 1) * sizeof(int64_t));
    int64_t *lst = (int64_t *)malloc(((size_t)filtered + 1) * sizeof(int64_t));
    int64_t *fill = (int64_t *)calloc((size_t)nc + 1, sizeof(int64_t));
    if (!off || !lst || !fill) return ORC_E_OOM;
    off[0] = 0;
    for (int c = 0; c < nc; ++c) off[c + 1] = off[c] + cnt[c];
    for (int64_t i = 0; i < n; ++i)
        if (keep[i]) {
            const int32_t bc = b->bc[i];
            lst[off[bc] + fill[bc]++] = i;
        }

    /* zero outputs */
    if (out->counts) memset(out->counts, 0, (size_t)nc * L * 32);
    if (out->tn5) memset(out->tn5, 0, (size_t)nc * L * 8);
    if (out->depth) memset(out->depth, 0, (size_t)nc * L * 4);
    if (out->ref_tally) memset(out->ref_tally, 0, (size_t)L * 32);
    for (int c = 0; c < nc; ++c) {
        if (out->n_reads) out->n_reads[c] = (uint32_t)cnt[c];
        if (out->any_paired) out->any_paired[c] = 0;
        if (out->passed) out->passed[c] = 0;
        if (out->covered) out->covered[c] = 0;
        if (out->depth_sum) out->depth_sum[c] = 0;
        if (out->depth_max) out->depth_max[c] = 0;
        if (out->median_lo) out->median_lo[c] = 0;
        if (out->median_hi) out->median_hi[c] = 0;
        if (out->first_read) out->first_read[c] = cnt[c] ? (uint32_t)lst[off[c]] : 0xFFFFFFFFu;
    }

    /* step 2: per cell, in dict (first-seen) order (processors.py:63-85) */
    uint32_t *bc8 = (uint32_t *)malloc((size_t)L * 8 * sizeof(uint32_t));
    uint32_t *tn5 = (uint32_t *)malloc((size_t)L * 2 * sizeof(uint32_t));
    uint32_t *dep = (uint32_t *)malloc((size_t)L * sizeof(uint32_t));
    if (!bc8 || !tn5 || !dep) return ORC_E_OOM;
    int64_t cells_passed = 0;
    const int64_t min_reads = cfg->min_reads;
    for (int32_t oi = 0; oi < n_seen; ++oi) {
        const int c = order[oi];
        const int64_t nr = cnt[c];
        int paired = 0;
        for (int64_t k = 0; k < nr; ++k)
            if (b->flag[lst[off[c] + k]] & MGP_FLAG_PAIRED) paired = 1;
        if (out->any_paired) out->any_paired[c] = (uint8_t)paired;
        if (nr == 0 || nr < min_reads) continue; /* processors.py:22 */
        memset(bc8, 0, (size_t)L * 8 * sizeof(uint32_t));
        memset(tn5, 0, (size_t)L * 2 * sizeof(uint32_t));
        for (int64_t k = 0; k < nr; ++k) {
            const int64_t i = lst[off[c] + k];
            if ((int)b->mapq[i] < cfg->min_mapq) continue; /* pileup.py:33 */
            if (b->flag[i] & MGP_FLAG_PACK32) {
                /* 32-byte record: its codes stand for base + quality + block +
                 * end distance (include/mgpileup.h, made for the run's thresholds) */
                uint8_t full[128];
                mgp_unpack32_record(b->payload + b->rec_off[i], full);
                pile_read(full, cfg, bc8, tn5);
            } else if (b->flag[i] & MGP_FLAG_PACKED) {
                uint8_t full[128];
                unpack_packed(b->payload + b->rec_off[i], full);
                pile_read(full, cfg, bc8, tn5);
            } else {
                pile_read(b->payload + b->rec_off[i], cfg, bc8, tn5);
            }
        }
        /* dict of positions with depth > 0 or a tn5 cut (pileup.py:100-124),
         * then filter_strand_bias (pileup.py:128-154) */
        int64_t covered = 0;
        uint64_t dsum = 0;
        uint32_t dmax = 0;
        for (int64_t p = 0; p < L; ++p) {
            uint32_t *v = bc8 + p * 8;
            uint32_t depth0 = 0;
            for (int x = 0; x < 8; ++x) depth0 += v[x];
            dep[p] = 0;
            if (depth0 == 0 && tn5[p * 2] + tn5[p * 2 + 1] == 0) continue;
            uint32_t d = 0;
            for (int bi = 0; bi < 4; ++bi) {
                const uint32_t fwd = v[2 * bi], rev = v[2 * bi + 1], total = fwd + rev;
                if (total > 0) {
                    const double bias = (double)(fwd > rev ? fwd : rev) / (double)total;
                    if (bias > cfg->max_strand_bias) {
                        v[2 * bi] = 0;
                        v[2 * bi + 1] = 0;
                    }
                }
                d += v[2 * bi] + v[2 * bi + 1];
            }
            if (d == 0) continue; /* pileup.py:152 */
            dep[p] = d;
            covered++;
            dsum += d;
            if (d > dmax) dmax = d;
        }
        if (covered == 0) continue; /* processors.py:30-31 -> None */
        cells_passed++;
        if (out->passed) out->passed[c] = 1;
        if (out->covered) out->covered[c] = (uint32_t)covered;
        if (out->depth_sum) out->depth_sum[c] = dsum;
        if (out->depth_max) out->depth_max[c] = dmax;
        for (int64_t p = 0; p < L; ++p) {
            if (!dep[p]) continue;
            const size_t P = (size_t)c * L + p;
            if (out->counts) memcpy(out->counts + P * 8, bc8 + p * 8, 32);
            if (out->tn5) memcpy(out->tn5 + P * 2, tn5 + p * 2, 8);
            if (out->depth) out->depth[P] = dep[p];
            if (out->ref_tally)
                for (int bi = 0; bi < 4; ++bi) out->ref_tally[p * 4 + bi] += bc8[p * 8 + 2 * bi] + bc8[p * 8 + 2 * bi + 1];
        }
        /* step 3: np.median of the kept depths (writers.py:190) */
        if (out->median_lo || out->median_hi) {
            uint32_t *dd = (uint32_t *)malloc((size_t)covered * sizeof(uint32_t));
            if (!dd) return ORC_E_OOM;
            int64_t m = 0;
            for (int64_t p = 0; p < L; ++p)
                if (dep[p]) dd[m++] = dep[p];
            qsort(dd, (size_t)m, sizeof(uint32_t), cmp_u32);
            if (out->median_lo) out->median_lo[c] = dd[(m - 1) / 2];
            if (out->median_hi) out->median_hi[c] = dd[m / 2];
            free(dd);
        }
    }
    if (out->stats) {
        mgp_stats *s = out->stats;
        memset(s, 0, sizeof(*s));
        s->total_reads = n;
        s->filtered_reads = filtered;
        s->n_barcodes = n_seen;
        s->duplicate_reads_with_length = dup_len;
        s->duplicate_reads_position_only = dup_pos;
        s->cells_passed = cells_passed;
    }
    if (order_out)
        for (int32_t k = 0; k < nc; ++k) order_out[k] = k < n_seen ? order[k] : -1;
    if (n_order) *n_order = n_seen;
    free(bc8);
    free(tn5);
    free(dep);
    free(cnt);
    free(order);
    free(keep);
    free(off);
    free(lst);
    free(fill);
    return ORC_OK;
}
