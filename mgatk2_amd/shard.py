"""Cell sharding over GPUs.

Cells are independent: dedup keys, pileup, strand filter and per-cell stats
are all per barcode (readers.py:75-76, processors.py:20-55). A read set is
split into contiguous whitelist ranges balanced by read count. Each shard keeps
its reads in BAM order, with cell ids rebased to the range. Shards run on
separate devices, and the per-shard results are concatenated along the cell
axis. The reference-allele tallies are summed, on the host or with the RCCL
all-reduce inside ``mgp_run`` when ranks are processes.

Reads with no whitelisted barcode (bc = -1) belong to no shard. They count only
toward ``total_reads``, which the merge restores from the input size.
"""

from __future__ import annotations

import numpy as np

from .engine import EngineResult
from .synth import ReadSoA


def partition_cells(reads_per_cell: np.ndarray, n_shards: int) -> np.ndarray:
    """Boundaries b[0]=0 <= ... <= b[n]=n_cells of contiguous cell ranges with
    about equal read totals (each range gets the cells whose cumulative count
    midpoint falls in its share)."""
    w = np.asarray(reads_per_cell, dtype=np.float64)
    n_cells = w.size
    if n_shards <= 1 or n_cells == 0:
        return np.array([0, n_cells], np.int64)
    total = w.sum()
    if total <= 0:
        return np.linspace(0, n_cells, n_shards + 1).round().astype(np.int64)
    mid = np.cumsum(w) - w / 2
    owner = np.minimum((mid / total * n_shards).astype(np.int64), n_shards - 1)
    b = np.searchsorted(owner, np.arange(n_shards + 1), side="left").astype(np.int64)
    b[-1] = n_cells
    return b


def reads_per_cell(soa: ReadSoA, n_cells: int) -> np.ndarray:
    bc = soa.bc[soa.bc >= 0]
    return np.bincount(bc, minlength=n_cells)[:n_cells]


def split_by_range(bc: np.ndarray, bounds) -> list[np.ndarray]:
    """The read indices of each cell range [bounds[d], bounds[d + 1]) in batch order
    (libmgphost `mgp_split_by_range`: one pass over the batch for all ranges)."""
    from .bam import host_library

    lib = host_library()
    b = np.ascontiguousarray(bounds, np.int64)
    nd = b.size - 1
    bc = np.ascontiguousarray(bc, np.int32)
    counts = np.zeros(max(nd, 1), np.int64)
    idx = np.empty(max(bc.size, 1), np.int64)
    tot = lib.mgp_split_by_range(bc.ctypes.data, bc.size, b.ctypes.data, nd, counts.ctypes.data, idx.ctypes.data)
    if tot < 0:
        raise ValueError((lib.mgp_host_last_error() or b"").decode())
    cuts = np.concatenate([[0], np.cumsum(counts[:nd])])
    return [idx[cuts[d]:cuts[d + 1]] for d in range(nd)]


def shard_soa(soa: ReadSoA, lo: int, hi: int, rec_align: int = 64, paired: bool = True,
              keep_all: bool = False, idx: np.ndarray | None = None) -> tuple[ReadSoA, np.ndarray]:
    """Reads of cells [lo, hi) in BAM order, cell ids rebased to lo, payload
    records gathered into a new payload (native, multithreaded: libmgphost.so
    `mgp_gather_offsets` / `mgp_gather_records`), placed by the producer
    placement (two consecutive packed records of a cell per 128-byte line when
    `paired`, else dense at `rec_align`). keep_all: every read (lo must be 0;
    reads outside the range keep their bc). Returns (batch, original read
    indices). idx: the range's read indices when the caller has them already."""
    from .bam import PLACE_DENSE, PLACE_PAIRED, host_library, host_threads

    if keep_all:
        if lo != 0:
            raise ValueError("keep_all needs lo == 0")
        idx = np.arange(soa.n, dtype=np.int64)
    elif idx is None:
        idx = np.flatnonzero((soa.bc >= lo) & (soa.bc < hi)).astype(np.int64)
    else:  # the range's reads, given (split_by_range)
        idx = np.ascontiguousarray(idx, np.int64)
    lib = host_library()
    roff = np.ascontiguousarray(soa.rec_off, dtype=np.uint64)
    flag = np.ascontiguousarray(soa.flag, dtype=np.uint16)
    bc = np.ascontiguousarray(soa.bc, dtype=np.int32)
    start = np.ascontiguousarray(soa.start, dtype=np.int32)
    tlen = np.ascontiguousarray(soa.tlen, dtype=np.int32)
    pay = np.ascontiguousarray(soa.payload)
    new_off = np.zeros(max(idx.size, 1), np.uint64)
    total = lib.mgp_gather_offsets(pay.ctypes.data, roff.ctypes.data, flag.ctypes.data, bc.ctypes.data,
                                   start.ctypes.data, tlen.ctypes.data, soa.n,
                                   pay.shape[0], idx.ctypes.data, idx.size, int(lo), int(hi - lo),
                                   PLACE_PAIRED if paired else PLACE_DENSE, rec_align, new_off.ctypes.data)
    if total < 0:
        raise ValueError((lib.mgp_host_last_error() or b"").decode())
    payload = np.zeros(total, np.uint8)
    if idx.size and lib.mgp_gather_records(pay.ctypes.data, roff.ctypes.data, flag.ctypes.data, soa.n, pay.shape[0],
                                           idx.ctypes.data, idx.size, new_off.ctypes.data, total,
                                           payload.ctypes.data, host_threads()) != 0:
        raise ValueError((lib.mgp_host_last_error() or b"").decode())
    out = ReadSoA(
        soa.start[idx].copy(), (soa.bc[idx] - lo).astype(np.int32) if lo else soa.bc[idx].astype(np.int32),
        soa.tlen[idx].copy(), soa.flag[idx].copy(),
        soa.mapq[idx].copy(), soa.span[idx].copy(), new_off[: idx.size].copy(), payload,
    )
    return out, idx


_STAT_SUM = ("filtered_reads", "n_barcodes", "duplicate_reads_with_length", "duplicate_reads_position_only",
             "cells_passed")


def merge_results(parts: list[tuple[EngineResult, int, int, np.ndarray]], n_cells: int, total_reads: int,
                  tally_reduced: bool = False) -> EngineResult:
    """Concatenate shard results [(res, lo, hi, orig_index)] along cells.

    ``first_read`` is mapped back to BAM indices of the whole read set. The
    tallies are summed, unless they were already all-reduced over the shards
    (``tally_reduced``), in which case the shards agree and one is kept."""
    parts = sorted(parts, key=lambda p: p[1])
    cov = [lo for _, lo, _, _ in parts] + [n_cells]
    if cov[0] != 0 or any(parts[i][2] != cov[i + 1] for i in range(len(parts))):
        raise ValueError("shards must tile [0, n_cells) contiguously")
    r0 = parts[0][0]
    dense = r0.counts is not None
    L = r0.ref_tally.shape[0]
    out = EngineResult.alloc(n_cells, L, dense=dense)
    for res, lo, hi, idx in parts:
        for k in ("counts", "tn5", "depth"):
            if dense:
                getattr(out, k)[lo:hi] = getattr(res, k)
        for k in ("n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max", "median_lo",
                  "median_hi"):
            getattr(out, k)[lo:hi] = getattr(res, k)
        fr = res.first_read.astype(np.int64)
        has = res.n_reads > 0
        mapped = np.full(hi - lo, np.iinfo(np.uint32).max, np.int64)
        mapped[has] = idx[fr[has]]
        out.first_read[lo:hi] = mapped.astype(np.uint32)
        if not tally_reduced:
            out.ref_tally += res.ref_tally
    if tally_reduced:
        out.ref_tally[:] = r0.ref_tally
    st = {k: sum(int(p[0].stats.get(k, 0)) for p in parts) for k in _STAT_SUM}
    st["total_reads"] = int(total_reads)
    st["max_span"] = max(int(p[0].stats.get("max_span", 0)) for p in parts)
    st["error_bits"] = 0
    out.stats = st
    return out
