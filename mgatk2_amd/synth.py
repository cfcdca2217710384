"""Synthetic chrM workload and the SoA/record packer.

The engine's input is the chrM records of a coordinate-sorted BAM, as SoA key
arrays plus one packed payload record per read (layout in include/mgpileup.h).
This module builds that input two ways:

* :func:`synth_reads` — the seeded synthetic workload. It is counter-based:
  every field is a pure function of ``(seed, read index, field id)`` through
  :func:`shash`, so the device generator in ``csrc/mgp_synth.hip`` (used by
  bench.py to create 200M-read inputs directly in HBM) produces the same bytes;
  ``tests/test_gpu_parity.py`` checks that equality.
* :func:`pack_reads` — packs arbitrary read records (dicts with pysam-like
  fields) for hand-written known-answer cases.

Reads are L=50 by default; starts are stratified-uniform over
``[0, mito_len - L]`` and therefore sorted; ~15% full duplicates and ~3%
position-only duplicates of the previous read; lognormal reads/cell; 3%
non-whitelisted and 1% untagged barcodes; 0.5% secondary, 0.5% supplementary,
0.2% unmapped; 5% MAPQ 0; CIGAR 90% ``50M`` / 5% ``kS(50-k)M`` / 3% with an
insertion / 2% with a deletion; Q37 for 80% of bases; 1% substitutions, 0.1% N.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

MITO_LEN = 16569

# splitmix64 constants (csrc/mgp_kernels.h)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_C_SEED = 0x9E3779B97F4A7C15
_C_I = np.uint64(0xD1B54A32D192ED03)
_C_K = 0x8CB92BA72F3D8DD7
_MASK64 = (1 << 64) - 1

# thresholds on a 24-bit uniform (csrc/mgp_synth.hip)
DUP_FULL = 2516582
DUP_PART = 3019898
CAT_NOCB = 671088
CAT_SEC = 754974
CAT_SUPP = 838860
CAT_UNMAP = 872415
MAPQ0 = 838860
CIG_M = 15099494
CIG_S = 15938355
CIG_I = 16441671
QUAL37 = 13421772
BASE_N = 16777
BASE_SUB = 184549

FLAG_PAIRED = 0x1
FLAG_UNMAPPED = 0x4
FLAG_REVERSE = 0x10
FLAG_SECONDARY = 0x100
FLAG_SUPPLEMENTARY = 0x800
FLAG_NOSEQQUAL = 0x1000
FLAG_PACKED = 0x2000  # the record uses the packed 64-byte layout (include/mgpileup.h)
FLAG_PACK32 = 0x4000  # the record uses the 32-byte layout (include/mgpileup.h)
PACK_MAX_LEN = 50
PACK_BYTES = 64
PACK32_BYTES = 32

CODES = np.array([1, 2, 4, 8], dtype=np.uint8)  # BAM 4-bit A, C, G, T
SEQ_NT16 = "=ACMGRSVTWYHKDBN"
_NT16_IDX = {ch: i for i, ch in enumerate(SEQ_NT16)}


def _mix64(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def shash(seed: int, i, k) -> np.ndarray:
    """Counter-based hash ``mix64(seed*C1 + i*C2 + k*C3)`` (mod 2^64), vectorised."""
    i = np.asarray(i, dtype=np.uint64)
    k = np.asarray(k, dtype=np.uint64)
    base = np.uint64((seed * _C_SEED) & _MASK64)
    with np.errstate(over="ignore"):
        z = base + i * _C_I + k * np.uint64(_C_K)
        return _mix64(z)


def _u24(h: np.ndarray) -> np.ndarray:
    return (h >> np.uint64(40)).astype(np.int64)


def ref_codes(seed: int, mito_len: int = MITO_LEN) -> np.ndarray:
    """Synthetic chrM reference as BAM 4-bit codes (uniform ACGT)."""
    h = shash(seed ^ 0x5EED, np.arange(mito_len, dtype=np.uint64), 0)
    return CODES[(h & np.uint64(3)).astype(np.int64)]


def cell_cdf(seed: int, n_cells: int, sigma: float = 0.5) -> np.ndarray:
    """Lognormal(sigma) reads-per-cell weights as cumulative u32 thresholds."""
    if n_cells <= 0:
        return np.zeros(0, dtype=np.uint32)
    c = np.arange(n_cells, dtype=np.uint64)
    h1 = shash(seed ^ 0xCE11, c, 0)
    h2 = shash(seed ^ 0xCE11, c, 1)
    u1 = ((h1 >> np.uint64(11)).astype(np.float64) + 1.0) / 2.0**53
    u2 = (h2 >> np.uint64(11)).astype(np.float64) / 2.0**53
    z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    w = np.exp(sigma * z)
    cdf = np.cumsum(w) / w.sum()
    t = np.floor(cdf * 2.0**32).astype(np.uint64)
    t = np.minimum(t, np.uint64(0xFFFFFFFF))
    t[-1] = np.uint64(0xFFFFFFFF)
    return t.astype(np.uint32)


def barcode_names(n_cells: int, seed: int = 0) -> list[str]:
    """Deterministic whitelisted 16-mer + '-1' barcodes."""
    h = shash(seed ^ 0xBA5E, np.arange(n_cells, dtype=np.uint64), 0)
    out = []
    for v in h.tolist():
        s = "".join("ACGT"[(v >> (2 * k)) & 3] for k in range(16))
        out.append(s + "-1")
    # collisions are astronomically unlikely; make them impossible
    seen: dict[str, int] = {}
    for i, s in enumerate(out):
        if s in seen:
            out[i] = s[:-2] + f"-{i + 2}"
        seen[out[i]] = i
    return out


@dataclass
class ReadSoA:
    """Engine input: SoA key arrays + packed payload records (BAM order)."""

    start: np.ndarray
    bc: np.ndarray
    tlen: np.ndarray
    flag: np.ndarray
    mapq: np.ndarray
    span: np.ndarray
    rec_off: np.ndarray
    payload: np.ndarray
    extra: dict = field(default_factory=dict)
    _bam_order: bool | None = field(default=None, repr=False, compare=False)

    @property
    def n(self) -> int:
        return int((self.start if self.start is not None else self.bc).shape[0])

    @property
    def in_bam_order(self) -> bool:
        """Whether the payload records follow the reads' order (computed once: slicing a
        large batch into chunks must not rescan rec_off per chunk)."""
        if self._bam_order is None:
            ro = self.rec_off.astype(np.int64)
            self._bam_order = not (self.n > 1 and bool(np.any(np.diff(ro) < 0)))
        return self._bam_order

    def slice(self, lo: int, hi: int) -> ReadSoA:
        """Reads [lo, hi) as a standalone batch (payload re-based). A payload whose
        records are not in BAM order (paired placement) is gathered and re-placed."""
        if hi <= lo:
            return empty_soa()
        if not self.in_bam_order:
            from .shard import shard_soa

            sub = ReadSoA(self.start[lo:hi], self.bc[lo:hi], self.tlen[lo:hi], self.flag[lo:hi], self.mapq[lo:hi],
                          self.span[lo:hi], self.rec_off[lo:hi], self.payload)
            nc = int(self.bc.max()) + 1
            return shard_soa(sub, 0, nc, paired=True, keep_all=True)[0]
        p0 = int(self.rec_off[lo])
        p1 = int(self.rec_off[hi]) if hi < self.n else int(self.payload.shape[0])
        return ReadSoA(
            self.start[lo:hi].copy(),
            self.bc[lo:hi].copy(),
            self.tlen[lo:hi].copy(),
            self.flag[lo:hi].copy(),
            self.mapq[lo:hi].copy(),
            self.span[lo:hi].copy(),
            (self.rec_off[lo:hi] - np.uint64(p0)).astype(np.uint64),
            self.payload[p0:p1].copy(),
        )


def relocate(soa: ReadSoA, paired: bool = False, rec_align: int = 64, n_cells: int | None = None) -> ReadSoA:
    """The same reads with their payload records moved to the producer placement
    (mgp_place_records): dense in BAM order at `rec_align`, or paired (two
    consecutive packed records of a cell per 128-byte line). Record bytes are
    unchanged; only rec_off and the payload's arrangement differ."""
    from .shard import shard_soa

    nc = int(soa.bc.max()) + 1 if n_cells is None and soa.n else int(n_cells or 0)
    out, idx = shard_soa(soa, 0, nc, rec_align=rec_align, paired=paired, keep_all=True)
    out.extra.update(soa.extra)
    return out


def empty_soa() -> ReadSoA:
    return ReadSoA(
        np.zeros(0, np.int32),
        np.zeros(0, np.int32),
        np.zeros(0, np.int32),
        np.zeros(0, np.uint16),
        np.zeros(0, np.uint8),
        np.zeros(0, np.uint32),
        np.zeros(0, np.uint64),
        np.zeros(0, np.uint8),
    )


def concat_soa(parts: list[ReadSoA]) -> ReadSoA:
    parts = [p for p in parts if p.n]
    if not parts:
        return empty_soa()
    offs = []
    pay = []
    base = 0
    for p in parts:
        base = (base + 255) & ~255
        offs.append(p.rec_off + np.uint64(base))  # records keep their alignment
        pad = base - sum(x.shape[0] for x in pay)
        if pad:
            pay.append(np.zeros(pad, np.uint8))
        pay.append(p.payload)
        base += p.payload.shape[0]
    return ReadSoA(
        np.concatenate([p.start for p in parts]),
        np.concatenate([p.bc for p in parts]),
        np.concatenate([p.tlen for p in parts]),
        np.concatenate([p.flag for p in parts]),
        np.concatenate([p.mapq for p in parts]),
        np.concatenate([p.span for p in parts]),
        np.concatenate(offs).astype(np.uint64),
        np.concatenate(pay),
    )


def seq_offset(lseq):
    """Byte offset of the packed sequence inside a record (include/mgpileup.h):
    qual[] at +16 gets at least 64 bytes, so reads of <= 64 bases have seq at +80."""
    lseq = np.asarray(lseq, np.int64)
    return 16 + np.maximum(64, (lseq + 3) & ~3)


def cigar_offset(lseq):
    """Byte offset of the CIGAR inside a record (include/mgpileup.h): seq[] gets at
    least 32 bytes, so reads of <= 64 bases have their CIGAR at +112 and a record
    with <= 4 CIGAR operations is exactly one 128-byte line."""
    lseq = np.asarray(lseq, np.int64)
    return seq_offset(lseq) + np.maximum(32, ((lseq + 1) // 2 + 3) & ~3)


REC_ALIGN = 64  # records are gathered at random: a packed record is one 64-byte half line


def packable_mask(start, flag, lseq, ncig, cig, qual) -> np.ndarray:
    """Which reads fit the packed layout (mgp_pack_record in include/mgpileup.h).
    cig: [m, k] BAM words (entries past ncig ignored); qual: [m, lseq] bytes."""
    start = np.asarray(start, np.int64)
    lseq = np.asarray(lseq, np.int64)
    ncig = np.asarray(ncig, np.int64)
    ok = ((np.asarray(flag) & FLAG_NOSEQQUAL) == 0) & (lseq >= 1) & (lseq <= PACK_MAX_LEN) & (ncig <= 4)
    ok &= (start >= -(1 << 28)) & (start < (1 << 28))
    cig = np.asarray(cig, np.int64).reshape(start.shape[0], -1)
    used = np.arange(cig.shape[1])[None, :] < ncig[:, None]
    op = cig & 15
    ok &= ~np.any(used & ((cig >> 4) >= 4096), axis=1)
    ok &= np.sum(used & ((op == 0) | (op == 7) | (op == 8)), axis=1) <= 2
    ok &= np.all(np.asarray(qual) <= 62, axis=1) if np.asarray(qual).size else True
    return ok


def pack_bytes(start, lseq, reverse, ncig, cig, qual, code) -> np.ndarray:
    """Packed records [m, 64] (include/mgpileup.h): header, CIGAR as u16, one
    byte per base (qual << 2 | b for A, C, G, T; 0xFF otherwise and past l_seq)."""
    m = np.asarray(start).shape[0]
    out = np.full((m, PACK_BYTES), 0xFF, np.uint8)
    out[:, 0:4] = np.asarray(start, "<i4").reshape(m, 1).view(np.uint8)
    out[:, 4] = np.asarray(lseq, np.uint8)
    out[:, 5] = (np.asarray(ncig, np.uint8) | np.where(np.asarray(reverse), 0x80, 0)).astype(np.uint8)
    c16 = np.zeros((m, 4), "<u2")
    cig = np.asarray(cig, np.int64).reshape(m, -1)
    for k in range(min(4, cig.shape[1])):
        c16[:, k] = np.where(np.asarray(ncig) > k, cig[:, k], 0).astype("<u2")
    out[:, 6:14] = c16.view(np.uint8).reshape(m, 8)
    code = np.asarray(code, np.int64)
    qual = np.asarray(qual, np.int64)
    n = code.shape[1]
    b = np.select([code == 1, code == 2, code == 4, code == 8], [0, 1, 2, 3], -1)
    v = np.where(b >= 0, (qual << 2) | np.maximum(b, 0), 0xFF)
    v = np.where(np.arange(n)[None, :] < np.asarray(lseq, np.int64).reshape(m, 1), v, 0xFF)
    out[:, 14 : 14 + n] = v.astype(np.uint8)
    return out


def pack32_mask(start, flag, lseq, ncig, cig, min_baseq: int, min_dist: int = 5) -> np.ndarray:
    """Which reads fit the 32-byte layout for these thresholds (mgp_pack32_record)."""
    start = np.asarray(start, np.int64)
    lseq = np.asarray(lseq, np.int64)
    ncig = np.asarray(ncig, np.int64)
    ok = ((np.asarray(flag) & FLAG_NOSEQQUAL) == 0) & (lseq >= 1) & (lseq <= PACK_MAX_LEN) & (ncig <= 4)
    ok &= (start >= 0) & (start < 65536) & (-128 <= int(min_baseq) <= 127) & (int(min_dist) <= 15)
    cig = np.asarray(cig, np.int64).reshape(start.shape[0], -1)
    used = np.arange(cig.shape[1])[None, :] < ncig[:, None]
    op = cig & 15
    ok &= ~np.any(used & ((cig >> 4) >= 4096), axis=1)
    ok &= np.sum(used & ((op == 0) | (op == 7) | (op == 8)), axis=1) <= 2
    return ok


def _counted_positions(lseq, ncig, cig, n: int, min_dist: int) -> np.ndarray:
    """[m, n] bool: query position k lies in an aligned operation's query range as the
    reference walks the CIGAR (pileup.py:55-95: an insertion does not advance the
    query position, quirk Q1) and min_dist <= k < l_seq - min_dist."""
    lseq = np.asarray(lseq, np.int64).reshape(-1)
    m = lseq.shape[0]
    cig = np.asarray(cig, np.int64).reshape(m, -1)
    ncig = np.asarray(ncig, np.int64).reshape(m)
    k = np.arange(n)[None, :]
    inblk = np.zeros((m, n), bool)
    q = np.zeros(m, np.int64)
    for j in range(cig.shape[1]):
        live = ncig > j
        op, ln = cig[:, j] & 15, cig[:, j] >> 4
        aligned = live & ((op == 0) | (op == 7) | (op == 8))
        inblk |= aligned[:, None] & (k >= q[:, None]) & (k < (q + ln)[:, None])
        q = q + np.where(live & (aligned | (op == 4)), ln, 0)
    md = max(int(min_dist), 0)
    return inblk & (k < lseq[:, None]) & (k >= md) & (k < (lseq - md)[:, None])


def pack32_bytes(start, lseq, reverse, ncig, cig, qual, code, min_baseq: int, min_dist: int = 5) -> np.ndarray:
    """32-byte records [m, 32] (include/mgpileup.h): u16 start, l_seq, n_cigar |
    min_dist << 3 | reverse << 7, CIGAR as u16, then a 3-bit code per position at
    bit 96 + 3k (0..3 = the counted base A, C, G, T; 4 = not counted), min_baseq in
    byte 31."""
    m = np.asarray(start).shape[0]
    md = max(int(min_dist), 0)
    out = np.zeros((m, PACK32_BYTES), np.uint8)
    out[:, 0:2] = np.asarray(start, "<u2").reshape(m, 1).view(np.uint8)
    out[:, 2] = np.asarray(lseq, np.uint8)
    out[:, 3] = (np.asarray(ncig, np.uint8) | (md << 3) | np.where(np.asarray(reverse), 0x80, 0)).astype(np.uint8)
    c16 = np.zeros((m, 4), "<u2")
    cig = np.asarray(cig, np.int64).reshape(m, -1)
    for k in range(min(4, cig.shape[1])):
        c16[:, k] = np.where(np.asarray(ncig) > k, cig[:, k], 0).astype("<u2")
    out[:, 4:12] = c16.view(np.uint8).reshape(m, 8)
    code = np.asarray(code, np.int64)
    qual = np.asarray(qual, np.int64)
    n = code.shape[1]
    b = np.select([code == 1, code == 2, code == 4, code == 8], [0, 1, 2, 3], -1)
    q8 = np.where(qual >= 128, qual - 256, qual)  # int8(qual): >= 128 wraps (pileup.py Q5)
    cnt = _counted_positions(lseq, ncig, cig, n, md) & (b >= 0) & (q8 >= int(min_baseq))
    v = np.full((m, PACK_MAX_LEN), 4, np.uint64)
    v[:, :n] = np.where(cnt, np.maximum(b, 0), 4).astype(np.uint64)
    bits = np.zeros((m, 4), np.uint64)  # bits 96..351 of the record, as 4 little-endian u64 words
    for k in range(PACK_MAX_LEN):
        pos = 3 * k
        bits[:, pos >> 6] |= v[:, k] << np.uint64(pos & 63)
        if (pos & 63) > 61:
            bits[:, (pos >> 6) + 1] |= v[:, k] >> np.uint64(64 - (pos & 63))
    out[:, 12:31] = bits.view(np.uint8).reshape(m, 32)[:, :19]
    out[:, 31] = np.uint8(int(min_baseq) & 0xFF)
    return out


def rec_size(ncig, lseq, align: int = 16):
    """Bytes a record occupies when records are placed at multiples of `align`."""
    return (cigar_offset(lseq) + 4 * np.asarray(ncig, np.int64) + align - 1) & ~(align - 1)


def _synth_chunk(seed, i0, i1, n, read_len, n_cells, mito_len, cdf, ref):
    """Fields of reads [i0, i1) (needs the ancestors, which hash from the index)."""
    rl = read_len
    # ancestors: walk back to the last ORIG (A) / last non-FULL (B) read
    lo = max(0, i0 - 64)
    while True:
        idx = np.arange(lo, i1, dtype=np.uint64)
        t = _u24(shash(seed, idx, 1))
        typ = np.where(t < DUP_FULL, 1, np.where(t < DUP_PART, 2, 0))
        if lo == 0:
            typ[0] = 0
        # need an ORIG at or before i0 inside the window (or lo == 0)
        first_orig = np.flatnonzero(typ[: i0 - lo + 1] == 0)
        first_nf = np.flatnonzero(typ[: i0 - lo + 1] != 1)
        if lo == 0 or (first_orig.size and first_nf.size):
            break
        lo = max(0, lo - 4096)
    ar = np.arange(lo, i1, dtype=np.int64)
    A = np.maximum.accumulate(np.where(typ == 0, ar, -1))
    B = np.maximum.accumulate(np.where(typ != 1, ar, -1))
    A = A[i0 - lo :].astype(np.uint64)
    B = B[i0 - lo :].astype(np.uint64)
    i = np.arange(i0, i1, dtype=np.uint64)
    m = i.shape[0]

    spanpos = np.uint64(mito_len - rl + 1)
    u = shash(seed, A, 2) >> np.uint64(40)
    with np.errstate(over="ignore"):
        s0 = ((A * spanpos + ((u * spanpos) >> np.uint64(24))) // np.uint64(n)).astype(np.int32)
    if n_cells > 0:
        hc = (shash(seed, A, 3) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        cell = np.searchsorted(cdf, hc, side="right").astype(np.int32)
        cell = np.minimum(cell, n_cells - 1)
    else:
        cell = np.full(m, -1, np.int32)
    strand = (shash(seed, A, 4) >> np.uint64(63)).astype(np.int32)
    tabs = (60 + (shash(seed, B, 5) % np.uint64(541))).astype(np.int32)

    cat = _u24(shash(seed, i, 6))
    bc = np.where(cat < CAT_NOCB, -1, cell).astype(np.int32)
    flag = (FLAG_PAIRED | np.where(strand == 1, FLAG_REVERSE, 0)).astype(np.int64)
    flag |= np.where((cat >= CAT_NOCB) & (cat < CAT_SEC), FLAG_SECONDARY, 0)
    flag |= np.where((cat >= CAT_SEC) & (cat < CAT_SUPP), FLAG_SUPPLEMENTARY, 0)
    flag |= np.where((cat >= CAT_SUPP) & (cat < CAT_UNMAP), FLAG_UNMAPPED, 0)
    flag = flag.astype(np.uint16)
    mapq = np.where(_u24(shash(seed, i, 7)) < MAPQ0, 0, 60).astype(np.uint8)

    x = _u24(shash(seed, i, 8))
    p = shash(seed, i, 9)
    cls = np.where(x < CIG_M, 0, np.where(x < CIG_S, 1, np.where(x < CIG_I, 2, 3)))
    a = np.zeros(m, np.int64)
    b = np.zeros(m, np.int64)
    s_mask = cls == 1
    a[s_mask] = 1 + (p[s_mask] % np.uint64(10)).astype(np.int64)
    id_mask = cls >= 2
    a[id_mask] = 10 + (p[id_mask] % np.uint64(31)).astype(np.int64)
    b[id_mask] = 1 + ((p[id_mask] >> np.uint64(16)) % np.uint64(3)).astype(np.int64)
    ncig = np.choose(cls, [1, 2, 3, 3]).astype(np.int64)
    span = np.where(cls == 3, rl + b, rl).astype(np.uint32)

    cig = np.zeros((m, 3), np.uint32)
    M = cls == 0
    cig[M, 0] = (rl << 4) | 0
    cig[s_mask, 0] = (a[s_mask] << 4) | 4
    cig[s_mask, 1] = ((rl - a[s_mask]) << 4) | 0
    Im = cls == 2
    cig[Im, 0] = (a[Im] << 4) | 0
    cig[Im, 1] = (b[Im] << 4) | 1
    cig[Im, 2] = ((rl - a[Im] - b[Im]) << 4) | 0
    Dm = cls == 3
    cig[Dm, 0] = (a[Dm] << 4) | 0
    cig[Dm, 1] = (b[Dm] << 4) | 2
    cig[Dm, 2] = ((rl - a[Dm]) << 4) | 0

    q = np.arange(rl, dtype=np.uint64)
    hq = shash(seed, i[:, None], np.uint64(1000) + q[None, :])
    qual = np.where(_u24(hq) < QUAL37, 37, 2 + (hq % np.uint64(35)).astype(np.int64)).astype(np.uint8)
    del hq
    qi = q.astype(np.int64)[None, :]
    ac, bcol = a[:, None], b[:, None]
    d = np.broadcast_to(qi, (m, rl)).copy()
    rnd = np.zeros((m, rl), bool)
    c1 = (cls == 1)[:, None]
    rnd |= c1 & (qi < ac)
    d = np.where(c1, qi - ac, d)
    c2 = (cls == 2)[:, None]
    rnd |= c2 & (qi >= ac) & (qi < ac + bcol)
    d = np.where(c2 & (qi >= ac + bcol), qi - bcol, d)
    c3 = (cls == 3)[:, None]
    d = np.where(c3 & (qi >= ac), qi + bcol, d)
    hs = shash(seed, i[:, None], np.uint64(100000) + q[None, :])
    mm = _u24(hs)
    rpos = (s0.astype(np.int64)[:, None] + np.where(rnd, 0, d)) % mito_len
    rc = ref[rpos]
    rc_idx = np.searchsorted(CODES, rc)  # 1,2,4,8 -> 0..3
    sub = CODES[(rc_idx + 1 + ((hs & np.uint64(255)) % np.uint64(3)).astype(np.int64)) & 3]
    code = np.where(mm < BASE_N, 15, np.where(mm < BASE_SUB, sub, rc)).astype(np.uint8)
    code = np.where(rnd, CODES[(hs & np.uint64(3)).astype(np.int64)], code).astype(np.uint8)
    del hs, mm, rpos, rc, sub, d, rnd

    return dict(
        start=s0, bc=bc, tlen=np.where(strand == 1, -tabs, tabs).astype(np.int32), flag=flag, mapq=mapq,
        span=span, ncig=ncig, cig=cig, qual=qual, code=code,
    )


def _pack_fixed(start, flag, ncig, cig, qual, code, rl, align=REC_ALIGN, pack=True, pack32=None, pack32_dist=5):
    """Pack records for reads of one read length (vectorised). Returns (rec_off,
    payload, flag): reads that fit get the packed layout and MGP_FLAG_PACKED;
    with pack32 (a min_baseq), reads that fit the 32-byte layout get it first
    (MGP_FLAG_PACK32, 32-byte records at multiples of min(align, 32))."""
    m = start.shape[0]
    p32 = (pack32_mask(start, flag, np.full(m, rl), ncig, cig, pack32, pack32_dist) if pack32 is not None
           else np.zeros(m, bool))
    pk = packable_mask(start, flag, np.full(m, rl), ncig, cig, qual) & ~p32 if pack else np.zeros(m, bool)
    flag = (flag | np.where(pk, FLAG_PACKED, 0) | np.where(p32, FLAG_PACK32, 0)).astype(np.uint16)
    a32 = min(align, PACK32_BYTES)
    sizes = np.where(pk, (PACK_BYTES + align - 1) & ~(align - 1), rec_size(ncig, np.full(m, rl), align))
    sizes = np.where(p32, (PACK32_BYTES + a32 - 1) & ~(a32 - 1), sizes)
    roff = np.zeros(m, np.uint64)
    if m:
        roff[1:] = np.cumsum(sizes[:-1]).astype(np.uint64)
    total = int(sizes.sum())
    pay = np.zeros(total, np.uint8)
    ro = roff.astype(np.int64)
    if p32.any():
        pr = pack32_bytes(start[p32], np.full(int(p32.sum()), rl), (flag[p32] & FLAG_REVERSE) != 0, ncig[p32],
                          cig[p32], qual[p32], code[p32], pack32, pack32_dist)
        pay[ro[p32, None] + np.arange(PACK32_BYTES)[None, :]] = pr
    if pk.any():
        pr = pack_bytes(start[pk], np.full(int(pk.sum()), rl), (flag[pk] & FLAG_REVERSE) != 0, ncig[pk], cig[pk],
                        qual[pk], code[pk])
        pay[ro[pk, None] + np.arange(PACK_BYTES)[None, :]] = pr
    fu = ~pk & ~p32
    mf = int(fu.sum())
    if mf == 0:
        return roff, pay, flag
    ro = ro[fu]
    coff = int(cigar_offset(rl))
    hdr = np.zeros(mf, dtype=[("start", "<i4"), ("lseq", "<u4"), ("ncig", "<u2"), ("flag", "<u2"), ("coff", "<u4")])
    hdr["start"] = start[fu]
    hdr["lseq"] = rl
    hdr["ncig"] = ncig[fu]
    hdr["flag"] = flag[fu]
    hdr["coff"] = coff
    hb = hdr.view(np.uint8).reshape(mf, 16)
    pay[ro[:, None] + np.arange(16)[None, :]] = hb
    pay[(ro + 16)[:, None] + np.arange(rl)[None, :]] = qual[fu]
    nb = (rl + 1) // 2
    c = code[fu]
    if rl & 1:
        c = np.concatenate([c, np.zeros((mf, 1), np.uint8)], axis=1)
    packed = ((c[:, 0::2] << 4) | c[:, 1::2]).astype(np.uint8)
    pay[(ro + int(seq_offset(rl)))[:, None] + np.arange(nb)[None, :]] = packed
    cf, nf = cig[fu], ncig[fu]
    cb = cf.astype("<u4").view(np.uint8).reshape(mf, -1)
    for k in range(cf.shape[1]):
        sel = nf > k
        pay[(ro[sel, None] + coff + 4 * k + np.arange(4)[None, :])] = cb[sel, 4 * k : 4 * k + 4]
    return roff, pay, flag


def synth_reads(
    seed: int, n_reads: int, n_cells: int, read_len: int = 50, mito_len: int = MITO_LEN, chunk: int = 262144,
    rec_align: int = REC_ALIGN, pack: bool = True, pack32: int | None = None, pack32_dist: int = 5,
) -> ReadSoA:
    """Host mirror of the device generator (bit-identical). pack: reads that fit
    get the packed 64-byte record layout (all of them at read_len <= 50); pack32
    (a min_baseq): the 32-byte layout made for that threshold instead."""
    if read_len < 48:
        raise ValueError("read_len must be >= 48")
    cdf = cell_cdf(seed, n_cells)
    ref = ref_codes(seed, mito_len)
    parts = []
    for i0 in range(0, n_reads, chunk):
        i1 = min(n_reads, i0 + chunk)
        f = _synth_chunk(seed, i0, i1, n_reads, read_len, n_cells, mito_len, cdf, ref)
        roff, pay, flag = _pack_fixed(f["start"], f["flag"], f["ncig"], f["cig"], f["qual"], f["code"], read_len,
                                      rec_align, pack, pack32, pack32_dist)
        parts.append(ReadSoA(f["start"], f["bc"], f["tlen"], flag, f["mapq"], f["span"], roff, pay))
    soa = _concat_dense(parts)
    soa.extra.update(cdf=cdf, ref=ref, seed=seed, read_len=read_len)
    return soa


def _concat_dense(parts: list[ReadSoA]) -> ReadSoA:
    """Concatenate without padding between parts (the device layout)."""
    if not parts:
        return empty_soa()
    offs, base = [], 0
    for p in parts:
        offs.append(p.rec_off + np.uint64(base))
        base += p.payload.shape[0]
    return ReadSoA(
        np.concatenate([p.start for p in parts]),
        np.concatenate([p.bc for p in parts]),
        np.concatenate([p.tlen for p in parts]),
        np.concatenate([p.flag for p in parts]),
        np.concatenate([p.mapq for p in parts]),
        np.concatenate([p.span for p in parts]),
        np.concatenate(offs).astype(np.uint64),
        np.concatenate([p.payload for p in parts]),
    )


# ---------------------------------------------------------------------------
# generic packer (pysam-like records)
# ---------------------------------------------------------------------------
def cigar_ref_span(cigar) -> int:
    return sum(length for op, length in cigar if op in (0, 2, 3, 7, 8))


def pack_reads(reads: list[dict], rec_align: int = REC_ALIGN, pack: bool = True,
               pack32: int | None = None, pack32_dist: int = 5) -> ReadSoA:
    """Pack pysam-like read dicts into the engine input. pack: reads that fit get
    the packed 64-byte layout (include/mgpileup.h), which keeps what the pileup
    reads but not the code and quality of non-ACGT bases; pack32 (a min_baseq):
    reads that fit get the 32-byte layout made for that threshold first.

    Keys: ``reference_start``, ``flag`` (BAM flag), ``mapping_quality``,
    ``cigartuples`` (list of (op, len) or None), ``query_sequence`` (str or
    None), ``query_qualities`` (list of ints or None), ``template_length``,
    ``bc`` (whitelist index or -1).
    """
    n = len(reads)
    start = np.zeros(n, np.int32)
    bc = np.zeros(n, np.int32)
    tlen = np.zeros(n, np.int32)
    flag = np.zeros(n, np.uint16)
    mapq = np.zeros(n, np.uint8)
    span = np.zeros(n, np.uint32)
    roff = np.zeros(n, np.uint64)
    chunks = []
    off = 0
    for i, r in enumerate(reads):
        seq = r.get("query_sequence")
        qual = r.get("query_qualities")
        cig = r.get("cigartuples") or []
        lseq = len(seq) if seq is not None else 0
        f = int(r.get("flag", 0))
        if seq is None or qual is None:
            f |= FLAG_NOSEQQUAL
        start[i] = r["reference_start"]
        bc[i] = r.get("bc", -1)
        tlen[i] = r.get("template_length", 0)
        flag[i] = f
        mapq[i] = r.get("mapping_quality", 60)
        span[i] = max(cigar_ref_span(cig), lseq)
        roff[i] = off
        if (pack or pack32 is not None) and seq is not None and qual is not None and lseq:
            cw = np.array([[(ln << 4) | op for op, ln in cig] or [0]], np.int64)
            qa = (np.asarray(qual, dtype=np.int64) & 0xFF).reshape(1, -1)
            if pack32 is not None and pack32_mask([start[i]], [f], [lseq], [len(cig)], cw, pack32, pack32_dist)[0]:
                codes = np.array([[_NT16_IDX[ch] for ch in seq.upper()]], np.int64)
                f |= FLAG_PACK32
                flag[i] = f
                a32 = min(rec_align, PACK32_BYTES)
                size = (PACK32_BYTES + a32 - 1) & ~(a32 - 1)
                rec = np.zeros(size, np.uint8)
                rec[:PACK32_BYTES] = pack32_bytes([start[i]], [lseq], [(f & FLAG_REVERSE) != 0], [len(cig)], cw, qa,
                                                  codes, pack32, pack32_dist)[0]
                chunks.append(rec)
                off += size
                continue
            if pack and packable_mask([start[i]], [f], [lseq], [len(cig)], cw, qa)[0]:
                codes = np.array([[_NT16_IDX[ch] for ch in seq.upper()]], np.int64)
                f |= FLAG_PACKED
                flag[i] = f
                size = (PACK_BYTES + rec_align - 1) & ~(rec_align - 1)
                rec = np.zeros(size, np.uint8)
                rec[:PACK_BYTES] = pack_bytes([start[i]], [lseq], [(f & FLAG_REVERSE) != 0], [len(cig)], cw, qa,
                                              codes)[0]
                chunks.append(rec)
                off += size
                continue
        size = int(rec_size(len(cig), lseq, rec_align))
        coff = int(cigar_offset(lseq))
        rec = np.zeros(size, np.uint8)
        hdr = np.array([(start[i], lseq, len(cig), f, coff)],
                       dtype=[("s", "<i4"), ("l", "<u4"), ("n", "<u2"), ("f", "<u2"), ("c", "<u4")])
        rec[:16] = hdr.view(np.uint8)
        if lseq:
            if qual is not None:
                rec[16 : 16 + lseq] = np.asarray(qual, dtype=np.int64) & 0xFF
            else:
                rec[16 : 16 + lseq] = 0xFF
            codes = [_NT16_IDX[ch] for ch in seq.upper()] if seq is not None else []
            if lseq & 1:
                codes.append(0)
            codes = np.array(codes, np.uint8)
            so = int(seq_offset(lseq))
            rec[so : so + (lseq + 1) // 2] = (codes[0::2] << 4) | codes[1::2]
        if cig:
            rec[coff : coff + 4 * len(cig)] = np.array([(ln << 4) | op for op, ln in cig], "<u4").view(np.uint8)
        chunks.append(rec)
        off += size
    payload = np.concatenate(chunks) if chunks else np.zeros(0, np.uint8)
    return ReadSoA(start, bc, tlen, flag, mapq, span, roff, payload)


def unpack_record(payload: np.ndarray, off: int, flag: int = 0) -> dict:
    """Decode one payload record (flag: the read's flag word, which tells the
    layout). A packed record gives ``N`` with quality 0 for its non-ACGT bases
    and no ``flag`` key beyond the reverse bit."""
    if int(flag) & FLAG_PACK32:
        r = payload[off : off + PACK32_BYTES]
        start = int(r[:2].view("<u2")[0])
        lseq = int(r[2])
        ncig = int(r[3]) & 7
        cig = r[4:12].view("<u2").astype(np.int64).tolist()[:ncig]
        w = int.from_bytes(bytes(r[12:31]), "little")
        v = [(w >> (3 * k)) & 7 for k in range(lseq)]
        seq = "".join("ACGT"[x] if x < 4 else "N" for x in v)
        return dict(
            reference_start=start, flag=FLAG_REVERSE if r[3] & 0x80 else 0,
            cigartuples=[(c & 15, c >> 4) for c in cig], query_sequence=seq,
            query_qualities=[127 if x < 4 else 0 for x in v], min_baseq=int(r[31].astype(np.int8)),
            min_dist=(int(r[3]) >> 3) & 15,
        )
    if int(flag) & FLAG_PACKED:
        r = payload[off : off + PACK_BYTES]
        start = int(r[:4].view("<i4")[0])
        lseq = int(r[4])
        ncig = int(r[5]) & 0x7F
        cig = r[6:14].view("<u2").astype(np.int64).tolist()[:ncig]
        b = r[14 : 14 + lseq].astype(np.int64)
        never = b >= 252  # 0xFF: a non-ACGT base
        seq = "".join("N" if nv else "ACGT"[x & 3] for x, nv in zip(b.tolist(), never.tolist()))
        qual = np.where(never, 0, b >> 2).tolist()
        return dict(
            reference_start=start, flag=FLAG_REVERSE if r[5] & 0x80 else 0,
            cigartuples=[(c & 15, c >> 4) for c in cig], query_sequence=seq, query_qualities=qual,
        )
    hdr = payload[off : off + 16].view(np.uint8)
    start = int(hdr[:4].view("<i4")[0])
    lseq = int(hdr[4:8].view("<u4")[0])
    ncig = int(hdr[8:10].view("<u2")[0])
    flag = int(hdr[10:12].view("<u2")[0])
    coff = int(hdr[12:16].view("<u4")[0])
    cig = payload[off + coff : off + coff + 4 * ncig].view("<u4").tolist() if ncig else []
    qual = payload[off + 16 : off + 16 + lseq].tolist()
    so = off + int(seq_offset(lseq))
    sb = payload[so : so + (lseq + 1) // 2]
    codes = np.stack([sb >> 4, sb & 15], axis=1).reshape(-1)[:lseq]
    seq = "".join(SEQ_NT16[c] for c in codes.tolist())
    return dict(
        reference_start=start, flag=flag, cigartuples=[(c & 15, c >> 4) for c in cig],
        query_sequence=seq, query_qualities=qual,
    )
