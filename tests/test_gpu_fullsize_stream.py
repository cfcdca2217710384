"""GPU, full size: the bench's headline path exactly as bench.py streams it, and the
C5 configuration streamed and split by cell.

* C4 (200M reads x 10k cells, `run` parameters) through bench.StreamSet, the code the
  bench's timed step runs: dense 64-byte quality-carrying records in pinned host
  batches of 16M reads, 16-bit barcode / |tlen| columns (mgp_push_batch16), on-device
  pairing, streamed segments, and the count rows written into pinned host memory as
  windows complete (mgp_set_rows_target: 8-bit rows for the (cell, window) pairs whose
  values all fit a byte, 16-bit rows for the others). Checked from the host rows the
  step delivered: the per-cell invariants over every cell, the run statistics and
  tallies, a second step byte-identical, and 8 x 8 whole cells bit-exact against the
  oracle on the quality-carrying full records of exactly their reads.
* C5 (1B reads x 100k cells) streamed the same way at its best batch size (80M reads,
  profiles/r05/bench_c5_r5j.log), with the same checks.
* C5 split into 8 read-balanced cell shards (bench.cell_bounds), each streamed as
  bench.py's rank r streams its shard at N = 8, as sequential contexts on one GPU:
  every shard's host rows and per-cell statistics equal the global run's cells bit
  for bit; tallies and read counts add up (processors.py:112-144).

Reference: pileup.py:18-154 (the counts), processors.py:20-55 (per-cell stats).
"""

from __future__ import annotations

import numpy as np
import pytest

from test_gpu_parity import FULL_KEYS, _oracle_cells_from_quality_records, _rows16_invariants

pytestmark = pytest.mark.gpu

RUN = dict(min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1)
PER_CELL = ("n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max", "median_lo", "median_hi")


def _delivered(ss, res, lo, hi) -> dict:
    """Cells [lo, hi) as the step left them in host memory (copies)."""
    d = {k: v.copy() for k, v in ss.cells(lo, hi).items()}
    for k in PER_CELL:
        d[k] = getattr(res, k)[lo:hi].copy()
    return d


def _streamed_full_size(engine_lib, oracle_lib, n, nc, seed, batch, ranges, chunk):
    import bench
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import cell_cdf, ref_codes

    cfg = EngineConfig(n_cells=nc, **RUN)
    cdf, ref = cell_cdf(seed, nc), ref_codes(seed)
    with Engine(cfg) as eng:
        eng.synth(seed, n, cdf, ref, read_len=50, rec_align=64, pack=True)  # the bench's stream leg inputs
        ss = bench.StreamSet(eng, cfg, "packed", columns16=True)
        # 16-bit columns (mgp_push_batch16) whenever the cells allow them (C5's 100k cells do not)
        assert ss.narrow == (nc <= 0xFFFF)
        assert ss.rows_target, "pinned rows target expected"
        bs = ss.auto_batch("auto") if batch == "auto" else batch
        batches = ss.batches(bs)
        seg0 = eng.stream_info()[0]
        res = ss.step(batches, True)
        segs, streamed = eng.stream_info()
        assert streamed and segs - seg0 >= 4, (segs - seg0, streamed)
        assert not ss.rows.wide.any() and not ss.exact
        assert ss.rows8 is not None and ss.rows8.narrow.any()  # (the bench's default: 8-bit rows beside)
        st = res.stats
        assert st["total_reads"] == n and st["error_bits"] == 0
        tally = np.zeros_like(res.ref_tally)
        for lo in range(0, nc, chunk):
            hi = min(nc, lo + chunk)
            tally += _rows16_invariants(ss.rows16(lo, hi), res, lo, hi)
        np.testing.assert_array_equal(res.ref_tally, tally)
        ok = res.passed.astype(bool)
        assert st["filtered_reads"] == int(res.n_reads.sum())
        assert st["n_barcodes"] == int((res.n_reads > 0).sum())
        assert st["cells_passed"] == int(ok.sum())
        assert st["duplicate_reads_with_length"] <= st["duplicate_reads_position_only"]
        got = {r: _delivered(ss, res, *r) for r in ranges}
        # a second step over the same pinned batches: the same bytes in host memory
        first = ss.rows16(0, chunk)
        again = ss.step(batches, True)
        second = ss.rows16(0, chunk)
        for k in ("counts", "tn5", "depth", "wide"):
            np.testing.assert_array_equal(getattr(second, k), getattr(first, k), err_msg=f"second step {k}")
        for k in ("n_reads", "covered", "depth_sum", "median_lo", "median_hi", "ref_tally"):
            np.testing.assert_array_equal(getattr(res, k), getattr(again, k), err_msg=f"second step {k}")
        del first, second
    for (lo, hi), g in got.items():
        exp = _oracle_cells_from_quality_records(oracle_lib, cfg, seed, n, cdf, ref, lo, hi)
        for k in FULL_KEYS:
            np.testing.assert_array_equal(g[k], getattr(exp, k), err_msg=f"streamed cells {lo}-{hi} {k}")
    return res


@pytest.mark.timeout(900)
def test_c4_streamed_headline_path_full_size(engine_lib, oracle_lib):
    """C4 exactly as the bench's timed step streams it (see the module docstring)."""
    nc = 10_000
    # 8 ranges of 8 whole cells (64 cells, spread over the cell range) against the oracle
    ranges = tuple((lo, lo + 8) for lo in (0, 1250, 2500, 3750, 5000, 6250, 7500, nc - 8))
    _streamed_full_size(engine_lib, oracle_lib, 200_000_000, nc, 20251015 + 4, "auto", ranges, 2500)


@pytest.mark.timeout(1200)
def test_c5_streamed_full_size(engine_lib, oracle_lib):
    """C5 streamed at its best batch size (80M reads, 13 batches)."""
    nc = 100_000
    _streamed_full_size(engine_lib, oracle_lib, 1_000_000_000, nc, 20251015 + 5, 80_000_000,
                        ((0, 8), (49_996, 50_012), (nc - 8, nc)), 5000)


@pytest.mark.timeout(1200)
def test_c5_eight_streamed_cell_shards_equal_the_global_run(engine_lib):
    """C5 in its 8-GPU form: the read-balanced contiguous cell ranges of
    bench.cell_bounds(cdf, 8); rank r's reads generated as that cell shard of the
    global set (its cells' reads plus a share of the reads without a whitelisted
    barcode) and streamed as bench.py's stream leg does on rank r; run here as 8
    sequential contexts on one device. Each shard's pinned host rows and per-cell
    statistics equal the global (resident) run's cells bit for bit, and the tallies and
    run statistics add up."""
    import bench
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import cell_cdf, ref_codes

    n, nc, seed, world = 1_000_000_000, 100_000, 20251015 + 5, 8
    cfg = EngineConfig(n_cells=nc, **RUN)
    cdf, ref = cell_cdf(seed, nc), ref_codes(seed)
    b = bench.cell_bounds(cdf, world)
    assert b[0] == 0 and b[-1] == nc and np.all(np.diff(b) > 0)
    with Engine(cfg) as eng:
        eng.synth(seed, n, cdf, ref, read_len=50, rec_align=64, pack=True)
        eng.run()
        whole = eng.fetch(dense=False)
        rows = [eng.fetch_rows16(int(b[r]), int(b[r + 1])) for r in range(world)]
    assert whole.stats["error_bits"] == 0
    tally = np.zeros_like(whole.ref_tally)
    sums = dict.fromkeys(("total_reads", "filtered_reads", "duplicate_reads_with_length",
                          "duplicate_reads_position_only", "cells_passed", "n_barcodes"), 0)
    for r in range(world):
        lo, hi = int(b[r]), int(b[r + 1])
        scfg = EngineConfig(**{**cfg.__dict__, "n_cells": hi - lo})
        with Engine(scfg) as e2:
            e2.synth(seed, n, cdf, ref, read_len=50, rec_align=64, pack=True, cells=(lo, hi), shard=(r, world))
            ss = bench.StreamSet(e2, scfg, "packed", columns16=True)
            part = ss.step(ss.batches(ss.auto_batch("auto")), True)
            assert e2.stream_info()[1], f"rank {r}: not streamed"
            assert part.stats["error_bits"] == 0
            got = ss.rows16(0, hi - lo)
            for k in ("counts", "tn5", "depth", "wide"):
                np.testing.assert_array_equal(getattr(got, k), getattr(rows[r], k), err_msg=f"rank {r} rows {k}")
            del got
            for k in PER_CELL:
                np.testing.assert_array_equal(getattr(part, k), getattr(whole, k)[lo:hi], err_msg=f"rank {r} {k}")
            tally += part.ref_tally
            for k in sums:
                sums[k] += part.stats[k]
            del ss
        rows[r] = None
    np.testing.assert_array_equal(tally, whole.ref_tally)
    for k, v in sums.items():
        assert v == whole.stats[k], k
