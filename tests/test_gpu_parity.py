"""GPU parity: the HIP engine (through the C-ABI) against the reference goldens and
the oracle, bit-exact. Every test here needs an MI355X."""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

from golden_io import CASES, Golden, check_result

pytestmark = pytest.mark.gpu

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))


def run_engine(engine_lib, cfg, soa, batches=1, dense=True):
    with engine_lib.Engine(cfg) as eng:
        if batches <= 1:
            eng.push(soa)
        else:
            cuts = np.linspace(0, soa.n, batches + 1).astype(int)
            for a, b in zip(cuts[:-1], cuts[1:]):
                eng.push(soa.slice(int(a), int(b)))
        eng.run()
        return eng.fetch(dense)


def assert_same(a, b, what=""):
    for k in ("counts", "tn5", "depth", "n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max",
              "median_lo", "median_hi", "ref_tally"):
        x, y = getattr(a, k), getattr(b, k)
        if x is None or y is None:
            continue
        np.testing.assert_array_equal(x, y, err_msg=f"{what}: {k}")
    np.testing.assert_array_equal(a.cell_order(), b.cell_order(), err_msg=f"{what}: order")
    for k in ("total_reads", "filtered_reads", "n_barcodes", "duplicate_reads_with_length",
              "duplicate_reads_position_only", "cells_passed"):
        assert a.stats[k] == b.stats[k], (what, k, a.stats[k], b.stats[k])


@pytest.mark.parametrize("case", CASES)
def test_engine_matches_reference_goldens(case, engine_lib):
    g = Golden(case)
    res = run_engine(engine_lib, g.config(), g.soa)
    check_result(res, g)


@pytest.mark.parametrize("case", ["synth_run", "kat_tenx"])
def test_engine_batched_push_equals_single(case, engine_lib):
    g = Golden(case)
    one = run_engine(engine_lib, g.config(), g.soa)
    many = run_engine(engine_lib, g.config(), g.soa, batches=5)
    assert_same(one, many, case)


CONFIGS = {
    "tenx": dict(min_baseq=0, min_mapq=0, dedup_mode="alignment_start", min_reads=0),
    "run": dict(min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1),
    "bias": dict(min_baseq=10, min_mapq=1, dedup_mode="none", min_reads=40, max_strand_bias=0.8),
}


_SYNTH_CACHE: dict = {}


def _synth(seed, n, nc):
    from mgatk2_amd.synth import synth_reads

    key = (seed, n, nc)
    if key not in _SYNTH_CACHE:
        _SYNTH_CACHE.clear()
        _SYNTH_CACHE[key] = synth_reads(seed, n, nc)
    return _SYNTH_CACHE[key]


@pytest.mark.parametrize("n_reads,n_cells", [(50_000, 7), (300_000, 200), (1_000_000, 500)])
@pytest.mark.parametrize("cfgname", sorted(CONFIGS))
def test_engine_matches_oracle_synth(engine_lib, oracle_lib, cfgname, n_reads, n_cells):
    from mgatk2_amd.engine import EngineConfig

    soa = _synth(1000 + n_reads + n_cells, n_reads, n_cells)
    cfg = EngineConfig(n_cells=n_cells, **CONFIGS[cfgname])
    res = run_engine(engine_lib, cfg, soa)
    exp, _ = oracle_lib.oracle_run(cfg, soa)
    assert_same(res, exp, f"{cfgname} {n_reads}x{n_cells}")


@pytest.mark.parametrize("n_reads,n_cells", [(300_000, 200), (1_000_000, 500)])
@pytest.mark.parametrize("cfgname", sorted(CONFIGS))
def test_pass_a_wide_form(engine_lib, oracle_lib, monkeypatch, cfgname, n_reads, n_cells):
    """Grouping pass A's 512-thread form, which the engine picks only for sets of
    several 4096-read steps per (bin, part) workgroup (C4, C5), forced on small sets
    (MGP_GA_WIDE_MIN=0): the same counts as the oracle."""
    from mgatk2_amd.engine import EngineConfig

    monkeypatch.setenv("MGP_GA_WIDE_MIN", "0")
    soa = _synth(1000 + n_reads + n_cells, n_reads, n_cells)
    cfg = EngineConfig(n_cells=n_cells, **CONFIGS[cfgname])
    res = run_engine(engine_lib, cfg, soa)
    exp, _ = oracle_lib.oracle_run(cfg, soa)
    assert_same(res, exp, f"wide pass A {cfgname} {n_reads}x{n_cells}")


def test_device_generator_equals_host_mirror(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    for n, nc, seed in [(1, 3, 5), (4097, 11, 6), (70_001, 33, 7)]:
        host = synth_reads(seed, n, nc)
        with engine_lib.Engine(EngineConfig(n_cells=nc)) as eng:
            eng.synth(seed, n, host.extra["cdf"], host.extra["ref"])
            dev = eng.download_inputs()
        for k in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off", "payload"):
            np.testing.assert_array_equal(getattr(dev, k), getattr(host, k), err_msg=f"{k} n={n}")


# ---------------------------------------------------------------------------
# record layouts (include/mgpileup.h): full 128-byte and packed 64-byte records
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("case", CASES)
def test_engine_matches_reference_goldens_packed(case, engine_lib, tmp_path):
    """The golden reads through the native BAM decoder with packing on."""
    from mgatk2_amd.bam import BamFile, soa_to_bam
    from mgatk2_amd.synth import FLAG_PACKED

    g = Golden(case)
    soa_to_bam(tmp_path / "x.bam", g.soa, g.whitelist)
    with BamFile(tmp_path / "x.bam") as bam:
        soa = bam.read_soa("chrM", g.whitelist, pack=True)
    assert (soa.flag & FLAG_PACKED).any()
    check_result(run_engine(engine_lib, g.config(), soa), g)


def _mixed_layout_synth(seed, n, nc, frac_full):
    """Synthetic reads where a random fraction keeps the full layout (one base
    quality raised to 63..70, which the packed layout cannot hold): waves pile
    packed and full records side by side."""
    from mgatk2_amd.synth import ReadSoA, _pack_fixed, _synth_chunk, cell_cdf, ref_codes

    cdf, ref = cell_cdf(seed, nc), ref_codes(seed)
    f = _synth_chunk(seed, 0, n, n, 50, nc, 16569, cdf, ref)
    rng = np.random.default_rng(seed)
    sel = rng.random(n) < frac_full
    pos = rng.integers(0, 50, n)
    f["qual"][sel, pos[sel]] = rng.integers(63, 71, int(sel.sum()))
    roff, pay, flag = _pack_fixed(f["start"], f["flag"], f["ncig"], f["cig"], f["qual"], f["code"], 50)
    return ReadSoA(f["start"], f["bc"], f["tlen"], flag, f["mapq"], f["span"], roff, pay)


@pytest.mark.parametrize("frac_full", [0.0, 0.05, 0.5, 1.0])
@pytest.mark.parametrize("cfgname", sorted(CONFIGS))
def test_mixed_record_layouts_match_oracle(engine_lib, oracle_lib, cfgname, frac_full):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import FLAG_PACKED

    soa = _mixed_layout_synth(77, 200_000, 60, frac_full)
    frac = float(np.mean((soa.flag & FLAG_PACKED) == 0))
    assert abs(frac - frac_full) < 0.01
    cfg = EngineConfig(n_cells=60, **CONFIGS[cfgname])
    res = run_engine(engine_lib, cfg, soa)
    exp, _ = oracle_lib.oracle_run(cfg, soa)
    assert_same(res, exp, f"{cfgname} full={frac_full}")


def test_packed_and_full_layouts_give_identical_results(engine_lib):
    """Quality thresholds around the packed range: 0, 37, 62, 63 and a negative one."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    pk = synth_reads(31, 300_000, 90, pack=True)
    fu = synth_reads(31, 300_000, 90, pack=False)
    for q in (-5, 0, 37, 62, 63):
        cfg = EngineConfig(n_cells=90, min_baseq=q, min_mapq=30, dedup_mode="alignment_and_fragment_length")
        assert_same(run_engine(engine_lib, cfg, pk), run_engine(engine_lib, cfg, fu), f"min_baseq {q}")


@pytest.mark.parametrize("cuts", [(0, 40_000, 100_000, 150_000), (0, 40_001, 100_003, 150_000)])
def test_dense_packed_payload_batches(engine_lib, oracle_lib, cuts):
    """A fully packed payload at a 64-byte stride lets grouping pass A compute
    the record offsets (the input check in k_bin_count). Batches whose payload bases
    keep the stride (first cut) stay dense; batches that break it (second cut:
    the 256-byte batch alignment moves the offsets) fall back to reading them.
    Both equal one push and the oracle."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import FLAG_PACKED

    soa = _synth(99, 150_000, 50)
    assert (soa.flag & FLAG_PACKED).all() and np.array_equal(soa.rec_off, np.arange(soa.n, dtype=np.uint64) * 64)
    cfg = EngineConfig(n_cells=50)
    one = run_engine(engine_lib, cfg, soa)
    with engine_lib.Engine(cfg) as eng:
        for a, b in zip(cuts[:-1], cuts[1:]):
            eng.push(soa.slice(a, b))
        eng.run()
        many = eng.fetch(True)
    assert_same(one, many, str(cuts))
    exp, _ = oracle_lib.oracle_run(cfg, soa)
    assert_same(one, exp, "oracle")


def test_packed_record_out_of_limits_raises(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import InvalidInputError
    from mgatk2_amd.synth import FLAG_PACKED, pack_reads

    soa = pack_reads([_read(100, [(0, 30)], "A" * 30, 0)])
    assert soa.flag[0] & FLAG_PACKED
    soa.payload[int(soa.rec_off[0]) + 4] = 60  # l_seq past the layout's 50
    with engine_lib.Engine(EngineConfig(n_cells=1, min_mapq=0)) as eng:
        eng.push(soa)
        eng.run()
        with pytest.raises(InvalidInputError):
            eng.sync()


def test_rerun_is_idempotent(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    soa = synth_reads(42, 200_000, 64)
    with engine_lib.Engine(EngineConfig(n_cells=64)) as eng:
        eng.push(soa)
        eng.run()
        a = eng.fetch()
        eng.run()
        eng.run()
        b = eng.fetch()
    assert_same(a, b, "rerun")


# ---------------------------------------------------------------------------
# edge cases
# ---------------------------------------------------------------------------
def _read(start, cigar, seq, bc, flag=0x1, mapq=60, tlen=100, qual=None):
    return dict(reference_start=start, cigartuples=cigar, query_sequence=seq,
                query_qualities=qual if qual is not None else [30] * len(seq), bc=bc, flag=flag,
                mapping_quality=mapq, template_length=tlen)


def _both(engine_lib, oracle_lib, reads, n_cells, **kw):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import pack_reads

    cfg = EngineConfig(n_cells=n_cells, **({"min_baseq": 0, "min_mapq": 0, "min_reads": 0} | kw))
    soa = pack_reads(reads)
    res = run_engine(engine_lib, cfg, soa)
    exp, _ = oracle_lib.oracle_run(cfg, soa)
    assert_same(res, exp, "edge")
    return res


def test_empty_input(engine_lib, oracle_lib):
    res = _both(engine_lib, oracle_lib, [], 5)
    assert res.stats["total_reads"] == 0 and res.passed.sum() == 0


def test_zero_cells(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import pack_reads

    soa = pack_reads([_read(10, [(0, 20)], "A" * 20, -1)])
    res = run_engine(engine_lib, EngineConfig(n_cells=0), soa)
    assert res.stats["total_reads"] == 1 and res.stats["filtered_reads"] == 0


def test_single_read_and_all_invalid(engine_lib, oracle_lib):
    _both(engine_lib, oracle_lib, [_read(100, [(0, 30)], "ACGT" * 7 + "AC", 0)], 1)
    _both(engine_lib, oracle_lib, [_read(100, [(0, 30)], "A" * 30, 0, flag=0x4),
                                   _read(101, [(0, 30)], "A" * 30, -1)], 3)


def test_long_span_reads(engine_lib, oracle_lib):
    """N/D ops with a reach far beyond one pileup window (16569/17 positions)."""
    reads = [
        _read(50, [(0, 10), (3, 9000), (0, 30)], "A" * 40, 0),
        _read(60, [(0, 10), (3, 16000), (0, 30)], "C" * 40, 0, flag=0x11),
        _read(3000, [(0, 20), (2, 5000), (0, 20)], "G" * 40, 1),
        _read(9000, [(0, 40)], "T" * 40, 1),
    ]
    _both(engine_lib, oracle_lib, reads, 2)


def test_pileup_crowded_start(engine_lib, oracle_lib):
    """Thousands of reads of one cell at one start: large dedup group."""
    rng = np.random.default_rng(3)
    reads = []
    for k in range(3000):
        t = int(rng.integers(60, 90))
        reads.append(_read(500, [(0, 30)], "ACGT" * 7 + "AC", int(k % 2), flag=0x11 if k % 3 == 0 else 0x1,
                           tlen=t))
    for mode in ("alignment_start", "alignment_and_fragment_length", "none"):
        _both(engine_lib, oracle_lib, reads, 2, dedup_mode=mode)


def test_unsorted_input_raises(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import BAMFormatError
    from mgatk2_amd.synth import pack_reads

    soa = pack_reads([_read(200, [(0, 30)], "A" * 30, 0), _read(100, [(0, 30)], "A" * 30, 0)])
    with engine_lib.Engine(EngineConfig(n_cells=1)) as eng:
        eng.push(soa)
        eng.run()
        with pytest.raises(BAMFormatError):
            eng.sync()


def test_badread_raises_like_reference(engine_lib):
    from make_golden import kat_reads

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import BAMReadError
    from mgatk2_amd.synth import pack_reads

    reads, nc = kat_reads()
    soa = pack_reads(reads)
    with engine_lib.Engine(EngineConfig(n_cells=nc, min_baseq=0, min_mapq=0, dedup_mode="none")) as eng:
        eng.push(soa)
        eng.run()
        with pytest.raises(BAMReadError):
            eng.sync()
    # with dedup on, the QUAL-less read is a duplicate: no error
    run_engine(engine_lib, EngineConfig(n_cells=nc, min_baseq=0, min_mapq=0, dedup_mode="alignment_start"), soa)


def test_overflow_bin_and_end_clamp(engine_lib, oracle_lib):
    reads = [
        _read(16500, [(0, 100)], "ACGT" * 25, 0),
        _read(16568, [(4, 5), (0, 30)], "T" * 35, 0, flag=0x11),
        _read(16569, [(0, 30)], "A" * 30, 0),
        _read(20000, [(0, 30)], "A" * 30, 1),
        _read(20000, [(0, 30)], "A" * 30, 1),
    ]
    _both(engine_lib, oracle_lib, reads, 2)


@pytest.mark.parametrize("narrow", ["0", "1"])
def test_deep_cell_median_fallback(engine_lib, oracle_lib, monkeypatch, narrow):
    """Depth >= 8192 at some positions: the median leaves the LDS histogram path.
    9000 reads of one cell start in one bin: with 8-bit start-bin counters
    (MGP_HIST_NARROW=1) they wrap, and the bin is counted again in 32 bits."""
    monkeypatch.setenv("MGP_HIST_NARROW", narrow)
    reads = [_read(1000, [(0, 30)], "ACGT" * 7 + "AC", 0, tlen=100 + k) for k in range(9000)]
    reads += [_read(2000 + 40 * k, [(0, 30)], "G" * 30, 0, tlen=77) for k in range(200)]
    reads += [_read(3000, [(0, 30)], "T" * 30, 1, tlen=100 + k) for k in range(50)]
    reads.sort(key=lambda r: r["reference_start"])
    res = _both(engine_lib, oracle_lib, reads, 2, dedup_mode="alignment_and_fragment_length")
    assert res.depth_max[0] >= 8192


@pytest.mark.parametrize("n_cells,slice_cells,xcd,narrow", [
    (45_000, None, "1", "0"), (45_000, None, "1", None), (5_000, 1024, "1", "0"), (3_001, 64, "1", "0"),
    (5_000, 1024, "0", "0"), (5_000, 1024, "1", "1"), (3_001, 64, "1", "1"), (3_001, None, "1", "1")])
def test_many_cells_sliced_histogram(engine_lib, oracle_lib, monkeypatch, n_cells, slice_cells, xcd, narrow):
    """More cells than one LDS histogram holds: the bins are counted in cell
    slices (45k cells with 32-bit counters: 2 slices; smaller slices forced with
    MGP_HIST_SLICE_CELLS: 5 and 47, the last one ragged), whose group totals must
    line up; the slices of a bin dealt to one XCD (default) or in slice-major
    order (MGP_HIST_XCD=0). narrow None: the engine's choice (45k cells: one slice
    of 8-bit counters); "1"/"0": 8-bit / 32-bit counters forced."""
    from mgatk2_amd.engine import EngineConfig

    monkeypatch.setenv("MGP_HIST_XCD", xcd)
    if narrow is not None:
        monkeypatch.setenv("MGP_HIST_NARROW", narrow)
    if slice_cells:
        monkeypatch.setenv("MGP_HIST_SLICE_CELLS", str(slice_cells))
    soa = _synth(77, 5 * n_cells, n_cells)
    cfg = EngineConfig(n_cells=n_cells, min_baseq=0, min_mapq=0, dedup_mode="alignment_start", min_reads=0)
    res = run_engine(engine_lib, cfg, soa)
    exp, _ = oracle_lib.oracle_run(cfg, soa)
    assert_same(res, exp, f"{n_cells} cells / {slice_cells}")


@pytest.mark.parametrize("narrow", ["0", "1"])
def test_small_lds_budget(engine_lib, oracle_lib, monkeypatch, narrow):
    """A 4 KiB LDS budget (MGP_HIST_LDS_KB) stands in for a context with more cells
    than grouping pass A's 512-thread form holds (~140k): 5000 cells then take the
    256-thread form, and the histogram many slices of 32- or 8-bit counters."""
    from mgatk2_amd.engine import EngineConfig

    monkeypatch.setenv("MGP_HIST_LDS_KB", "4")
    monkeypatch.setenv("MGP_HIST_NARROW", narrow)
    soa = _synth(78, 60_000, 5_000)
    for mode in ("alignment_and_fragment_length", "none"):
        cfg = EngineConfig(n_cells=5_000, min_baseq=20, min_mapq=30, dedup_mode=mode, min_reads=1)
        res = run_engine(engine_lib, cfg, soa)
        exp, _ = oracle_lib.oracle_run(cfg, soa)
        assert_same(res, exp, f"small LDS budget {mode}")


@pytest.mark.parametrize("bounds", ["0", "1"])
def test_deep_bins_parts_and_direct_buckets(engine_lib, oracle_lib, monkeypatch, bounds):
    """All reads start inside 8 start bins: every bin's parts hold tens of thousands
    of reads (per-part group counts of the histogram feed pass A's slots) and every
    (bin, 64-cell group) bucket exceeds pass B's LDS stage (direct path with the
    bucket walk-back duplicate marking)."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    soa = synth_reads(91, 300_000, 200)
    new = (1000 + soa.start.astype(np.int64) * 64 // 16569).astype(np.int32)  # monotone: order kept
    # ~190 reads per (cell, bin) with 8-bit histogram counters forced: some wrap; the
    # bins' bounds searched per workgroup or up front (k_bin_bounds, MGP_HIST_BOUNDS)
    monkeypatch.setenv("MGP_HIST_NARROW", "1")
    monkeypatch.setenv("MGP_HIST_BOUNDS", bounds)
    soa.start[:] = new
    hdr = soa.payload.view(np.uint8)
    for k in range(4):  # record header: int32 start at +0 (include/mgpileup.h)
        hdr[soa.rec_off.astype(np.int64) + k] = ((new.view(np.uint32) >> (8 * k)) & 0xFF).astype(np.uint8)
    for mode in ("alignment_and_fragment_length", "alignment_start", "none"):
        cfg = EngineConfig(n_cells=200, min_baseq=20, min_mapq=30, dedup_mode=mode, min_reads=1)
        res = run_engine(engine_lib, cfg, soa)
        exp, _ = oracle_lib.oracle_run(cfg, soa)
        assert_same(res, exp, f"deep bins {mode}")


def test_deep_and_shallow_cells_mixed(engine_lib, oracle_lib):
    """Cells above and below 65535 reads in one run: cell-windows of more than
    65535 elements drain their packed 16-bit tile into the output rows between
    segments, the others flush once."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    soa = synth_reads(57, 500_000, 10)
    per_cell = np.bincount(soa.bc[soa.bc >= 0], minlength=10)
    assert per_cell.max() > 65535 > per_cell.min()
    for mode, bias in (("alignment_and_fragment_length", 1.0), ("none", 0.9)):
        cfg = EngineConfig(n_cells=10, min_baseq=20, min_mapq=30, dedup_mode=mode, max_strand_bias=bias,
                           min_reads=1)
        res = run_engine(engine_lib, cfg, soa)
        exp, _ = oracle_lib.oracle_run(cfg, soa)
        assert_same(res, exp, f"deep/shallow {mode}")


def test_long_read_widens_halo_without_changing_other_cells(engine_lib):
    """One read with a 440-base reference span in its own cell widens every
    window's halo (reach R from max_span) for all cells: the other cells' results
    must not change."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import concat_soa, pack_reads, synth_reads

    base = synth_reads(58, 300_000, 40)
    cfg = EngineConfig(n_cells=41, min_baseq=20, min_mapq=30, dedup_mode="alignment_start", min_reads=1)
    a = run_engine(engine_lib, cfg, base)
    assert int(base.start.max()) <= 16560  # the added read keeps coordinate order
    long_read = pack_reads([_read(16560, [(0, 10), (3, 400), (0, 30)], "A" * 40, 40)])
    b = run_engine(engine_lib, cfg, concat_soa([base, long_read]))
    assert b.stats["max_span"] > 64 >= a.stats["max_span"]
    for k in ("counts", "tn5", "depth"):
        np.testing.assert_array_equal(getattr(a, k)[:40], getattr(b, k)[:40], err_msg=k)
    for k in ("n_reads", "covered", "depth_sum", "depth_max", "median_lo", "median_hi"):
        np.testing.assert_array_equal(getattr(a, k)[:40], getattr(b, k)[:40], err_msg=k)


def test_full_size_invariants_and_cell_sample_c3(engine_lib, oracle_lib):
    """BASELINE config C3 at full size (50M reads x 5k cells, `run` parameters):
    size-independent properties over every cell, a bit-exact oracle check of a
    sample of whole cells (cells are independent, so a cell's rows depend only on
    its own reads), and a rerun."""
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.shard import shard_soa
    from mgatk2_amd.synth import cell_cdf, ref_codes

    n, nc, seed = 50_000_000, 5_000, 20251015 + 3
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length",
                       min_reads=1)
    with Engine(cfg) as eng:
        eng.synth(seed, n, cell_cdf(seed, nc), ref_codes(seed))
        eng.run()
        res = eng.fetch()
        eng.run()
        again = eng.fetch()
        sample = eng.download_inputs()
    assert res.stats["total_reads"] == n
    # per position: depth = sum of the 8 (base, strand) counts; no Tn5 where depth is 0 (Q8)
    np.testing.assert_array_equal(res.counts.sum(axis=2, dtype=np.uint64), res.depth.astype(np.uint64))
    assert not np.any(res.tn5[res.depth == 0])
    # per cell statistics
    np.testing.assert_array_equal(res.covered, (res.depth > 0).sum(axis=1))
    np.testing.assert_array_equal(res.depth_sum, res.depth.sum(axis=1, dtype=np.uint64))
    np.testing.assert_array_equal(res.depth_max, res.depth.max(axis=1))
    ok = res.passed.astype(bool)
    assert np.all(res.median_lo[ok] <= res.median_hi[ok]) and np.all(res.median_hi[ok] <= res.depth_max[ok])
    # run statistics and reference-allele tallies over passing cells
    assert res.stats["filtered_reads"] == int(res.n_reads.sum())
    assert res.stats["n_barcodes"] == int((res.n_reads > 0).sum())
    assert res.stats["cells_passed"] == int(ok.sum())
    assert res.stats["duplicate_reads_with_length"] <= res.stats["duplicate_reads_position_only"]
    per_base = res.counts[ok].reshape(int(ok.sum()), -1, 4, 2).sum(axis=(0, 3), dtype=np.uint64)
    np.testing.assert_array_equal(res.ref_tally, per_base)
    # rerun: same arrays
    for k in ("counts", "tn5", "depth", "n_reads", "median_lo", "median_hi", "ref_tally"):
        np.testing.assert_array_equal(getattr(res, k), getattr(again, k), err_msg=f"rerun {k}")
    # a sample of whole cells against the oracle on exactly their reads
    for lo, hi in ((0, 8), (2500, 2508), (nc - 8, nc)):
        sub, _ = shard_soa(sample, lo, hi)
        scfg = EngineConfig(**{**cfg.__dict__, "n_cells": hi - lo})
        exp, _ = oracle_lib.oracle_run(scfg, sub)
        for k in ("counts", "tn5", "depth", "n_reads", "any_paired", "passed", "covered", "depth_sum",
                  "depth_max", "median_lo", "median_hi"):
            np.testing.assert_array_equal(getattr(res, k)[lo:hi], getattr(exp, k), err_msg=f"cells {lo}-{hi} {k}")


def _rows16_invariants(r16, res, lo, hi):
    """Size-independent properties of cells [lo, hi) from their 16-bit rows (exact:
    no wide window) and per-cell statistics."""
    assert not r16.wide.any()
    depth = r16.depth.astype(np.uint64)
    np.testing.assert_array_equal(r16.counts.sum(axis=2, dtype=np.uint64), depth)
    assert not np.any(r16.tn5[r16.depth == 0])
    np.testing.assert_array_equal(res.covered[lo:hi], (r16.depth > 0).sum(axis=1))
    np.testing.assert_array_equal(res.depth_sum[lo:hi], depth.sum(axis=1))
    np.testing.assert_array_equal(res.depth_max[lo:hi], r16.depth.max(axis=1))
    ok = res.passed[lo:hi].astype(bool)
    assert np.all(res.median_lo[lo:hi][ok] <= res.median_hi[lo:hi][ok])
    assert np.all(res.median_hi[lo:hi][ok] <= res.depth_max[lo:hi][ok])
    return r16.counts[ok].reshape(int(ok.sum()), -1, 4, 2).sum(axis=(0, 3), dtype=np.uint64)


def _oracle_cells_from_quality_records(oracle_lib, cfg, seed, n, cdf, ref, lo, hi):
    """The oracle's results for cells [lo, hi) of the global set, from the
    quality-carrying full 128-byte records of exactly those reads (regenerated as
    a cell shard of the same seed): the reference's own per-base filters
    (pileup.py:67-88: end distance, int8 quality >= min_baseq, ACGT) run on the
    raw qualities here, so a 32-byte record built wrong by the producer (the
    device generator's mgp_pack32_record) shows up as a mismatch."""
    from mgatk2_amd.engine import Engine, EngineConfig

    scfg = EngineConfig(**{**cfg.__dict__, "n_cells": hi - lo})
    with Engine(scfg) as e2:
        e2.synth(seed, n, cdf, ref, rec_align=128, pack=False, cells=(lo, hi), shard=(0, 0))
        sub = e2.download_inputs()
    assert sub.n > 1000 * (hi - lo)
    assert not np.any(sub.flag & 0x6000)  # every record full (no packed bit): qualities as in the BAM
    exp, _ = oracle_lib.oracle_run(scfg, sub)
    return exp


def _synth_layout(eng, seed, n, nc, cdf, ref, layout, min_baseq, **shard):
    """The bench's inputs (bench.py): 32-byte records made for min_baseq, four of a
    cell per 128-byte line (quad32), or packed 64-byte records two per line
    (paired64), or packed 64-byte records in BAM order (packed64). shard: a cell
    shard of the global set (cells=(lo, hi), shard=(rank, world)); nc is then the
    shard's cell count."""
    from mgatk2_amd.bam import PLACE_PAIRED, place_records

    p32 = min_baseq if layout == "quad32" else None
    eng.synth(seed, n, cdf, ref, pack32=p32, **shard)
    if layout == "packed64":
        return
    m = eng.resident()[0]
    cols = eng.download_inputs(columns=("bc", "flag", "start", "tlen"))
    roff, pay_b = place_records(cols.bc, cols.flag, np.full(m, 32 if p32 is not None else 64, np.uint32), nc,
                                PLACE_PAIRED, start=cols.start, tlen=cols.tlen)
    del cols
    eng.synth(seed, n, cdf, ref, rec_off=roff, payload_bytes=pay_b, pack32=p32, **shard)
    del roff


FULL_KEYS = ("counts", "tn5", "depth", "n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max",
             "median_lo", "median_hi")


@pytest.mark.parametrize("layout", ["paired64", "quad32"])
def test_full_size_invariants_and_cell_sample_c4(engine_lib, oracle_lib, layout):
    """BASELINE config C4 at full size (200M reads x 10k cells, `run` parameters) in
    the bench's record layouts: the per-cell invariants over every cell (16-bit
    rows: none is wide), the run statistics and tallies, a rerun, and three samples
    of 8 whole cells bit-exact against the oracle on exactly their reads, the
    oracle reading the quality-carrying full records of those reads (for quad32:
    the producer's per-base filter, moved out of the kernel into the 32-byte
    records' codes, is checked at full size)."""
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import cell_cdf, ref_codes

    n, nc, seed = 200_000_000, 10_000, 20251015 + 4
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length",
                       min_reads=1)
    cdf, ref = cell_cdf(seed, nc), ref_codes(seed)
    ranges = ((0, 8), (5000, 5008), (nc - 8, nc))
    with Engine(cfg) as eng:
        _synth_layout(eng, seed, n, nc, cdf, ref, layout, cfg.min_baseq)
        flags = eng.download_inputs(columns=("flag",)).flag
        want = 0x4000 if layout == "quad32" else 0x2000
        assert np.count_nonzero(flags & want) == n  # every record in the layout under test
        del flags
        eng.run()
        res = eng.fetch(dense=False)
        tally = np.zeros_like(res.ref_tally)
        for lo in range(0, nc, 2500):
            tally += _rows16_invariants(eng.fetch_rows16(lo, lo + 2500), res, lo, lo + 2500)
        samples = {r: eng.fetch_cells(*r) for r in ranges}
        first = eng.fetch_rows16(0, 2500).counts
        eng.run()
        again = eng.fetch(dense=False)
        np.testing.assert_array_equal(eng.fetch_rows16(0, 2500).counts, first)
        del first
    assert res.stats["total_reads"] == n and res.stats["error_bits"] == 0
    np.testing.assert_array_equal(res.ref_tally, tally)
    ok = res.passed.astype(bool)
    assert res.stats["filtered_reads"] == int(res.n_reads.sum())
    assert res.stats["n_barcodes"] == int((res.n_reads > 0).sum())
    assert res.stats["cells_passed"] == int(ok.sum())
    assert res.stats["duplicate_reads_with_length"] <= res.stats["duplicate_reads_position_only"]
    for k in ("n_reads", "covered", "depth_sum", "median_lo", "median_hi", "ref_tally"):
        np.testing.assert_array_equal(getattr(res, k), getattr(again, k), err_msg=f"rerun {k}")
    for (lo, hi), got in samples.items():
        exp = _oracle_cells_from_quality_records(oracle_lib, cfg, seed, n, cdf, ref, lo, hi)
        for k in FULL_KEYS:
            np.testing.assert_array_equal(getattr(got, k), getattr(exp, k), err_msg=f"{layout} cells {lo}-{hi} {k}")


@pytest.mark.timeout(600)
def test_c4_eight_cell_shards_equal_the_global_run(engine_lib):
    """BASELINE config C4 in its 8-GPU form, as bench.py splits it: the read-balanced
    contiguous cell ranges of bench.cell_bounds(cdf, 8), rank r's reads generated as
    that cell shard of the global set (its cells' reads plus a share of the reads
    without a whitelisted barcode), quad32 records placed per shard; run here as 8
    sequential shard contexts on one device. Every shard's 16-bit rows (and wide
    flags), per-cell statistics and first reads (by their keys) equal the global
    run's cells bit for bit; the tallies and read counts add up to the global run's
    (the reference's per-cell independence, processors.py:112-144)."""
    import bench
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import cell_cdf, ref_codes

    n, nc, seed, world = 200_000_000, 10_000, 20251015 + 4, 8
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length",
                       min_reads=1)
    cdf, ref = cell_cdf(seed, nc), ref_codes(seed)
    b = bench.cell_bounds(cdf, world)
    assert b[0] == 0 and b[-1] == nc and np.all(np.diff(b) > 0)
    keycols = ("start", "bc", "tlen", "flag", "mapq")
    with Engine(cfg) as eng:
        _synth_layout(eng, seed, n, nc, cdf, ref, "quad32", cfg.min_baseq)
        eng.run()
        whole = eng.fetch(dense=False)
        rows = [eng.fetch_rows16(int(b[r]), int(b[r + 1])) for r in range(world)]
        gk = eng.download_inputs(columns=keycols)
    tally = np.zeros_like(whole.ref_tally)
    sums = dict.fromkeys(("total_reads", "filtered_reads", "duplicate_reads_with_length",
                          "duplicate_reads_position_only", "cells_passed", "n_barcodes"), 0)
    for r in range(world):
        lo, hi = int(b[r]), int(b[r + 1])
        scfg = EngineConfig(**{**cfg.__dict__, "n_cells": hi - lo})
        with Engine(scfg) as e2:
            _synth_layout(e2, seed, n, hi - lo, cdf, ref, "quad32", cfg.min_baseq, cells=(lo, hi), shard=(r, world))
            e2.run()
            part = e2.fetch(dense=False)
            prow = e2.fetch_rows16(0, hi - lo)
            sk = e2.download_inputs(columns=keycols)
        assert part.stats["error_bits"] == 0
        for k in ("counts", "tn5", "depth", "wide"):
            np.testing.assert_array_equal(getattr(prow, k), getattr(rows[r], k), err_msg=f"rank {r} rows {k}")
        for k in FULL_KEYS[3:]:
            np.testing.assert_array_equal(getattr(part, k), getattr(whole, k)[lo:hi], err_msg=f"rank {r} {k}")
        # a cell's first read: the same read of the global set (same keys; bc rebased)
        has = part.n_reads > 0
        fs, fg = part.first_read[has].astype(np.int64), whole.first_read[lo:hi][has].astype(np.int64)
        for k in keycols:
            a, g = getattr(sk, k)[fs], getattr(gk, k)[fg]
            np.testing.assert_array_equal(a, g - lo if k == "bc" else g, err_msg=f"rank {r} first read {k}")
        tally += part.ref_tally
        for k in sums:
            sums[k] += part.stats[k]
        del prow, sk
    np.testing.assert_array_equal(tally, whole.ref_tally)
    for k, v in sums.items():
        assert v == whole.stats[k], k


@pytest.mark.parametrize("layout", ["packed64", "quad32"])
def test_full_size_cell_samples_c5(engine_lib, oracle_lib, layout):
    """BASELINE config C5 on one GPU (1B reads x 100k cells, `run` parameters) in
    the 64-byte and the bench's quad32 layout: sampled cell ranges of the
    full-size run bit-exact against the oracle on the quality-carrying full
    records of exactly their reads (regenerated as a cell shard of the same
    global set), the per-cell invariants over 4 ranges of 2000 cells, and the run
    statistics."""
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import cell_cdf, ref_codes

    n, nc, seed = 1_000_000_000, 100_000, 20251015 + 5
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length",
                       min_reads=1)
    cdf, ref = cell_cdf(seed, nc), ref_codes(seed)
    ranges = ((0, 8), (49_996, 50_012), (nc - 8, nc))
    with Engine(cfg) as eng:
        _synth_layout(eng, seed, n, nc, cdf, ref, layout, cfg.min_baseq)
        eng.run()
        res = eng.fetch(dense=False)
        for lo in (0, 31_000, 64_000, nc - 2000):
            _rows16_invariants(eng.fetch_rows16(lo, lo + 2000), res, lo, lo + 2000)
        samples = {r: eng.fetch_cells(*r) for r in ranges}
    assert res.stats["total_reads"] == n and res.stats["error_bits"] == 0
    assert res.stats["filtered_reads"] == int(res.n_reads.sum())
    assert res.stats["cells_passed"] == int(res.passed.sum())
    for (lo, hi), got in samples.items():
        exp = _oracle_cells_from_quality_records(oracle_lib, cfg, seed, n, cdf, ref, lo, hi)
        for k in FULL_KEYS:
            np.testing.assert_array_equal(getattr(got, k), getattr(exp, k), err_msg=f"{layout} cells {lo}-{hi} {k}")


# ---------------------------------------------------------------------------
# payload placement (mgp_place_records): cell-paired lines; grouping pass A's
# offset sources (dense index / u32 column / u64 column, the input check in k_bin_count)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("cfgname", sorted(CONFIGS))
def test_paired_placement_matches_oracle(engine_lib, oracle_lib, cfgname):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import relocate

    soa = relocate(_synth(1000 + 300_000 + 200, 300_000, 200), paired=True, n_cells=200)
    cfg = EngineConfig(n_cells=200, **CONFIGS[cfgname])
    res = run_engine(engine_lib, cfg, soa)
    exp, _ = oracle_lib.oracle_run(cfg, soa)
    assert_same(res, exp, f"paired {cfgname}")


def _shifted(soa, by=16):
    """The same payload moved by `by` bytes: offsets no longer multiples of 64
    (pass A reads the u64 offset column)."""
    from mgatk2_amd.synth import ReadSoA

    pay = np.zeros(soa.payload.size + by, np.uint8)
    pay[by:] = soa.payload
    return ReadSoA(soa.start, soa.bc, soa.tlen, soa.flag, soa.mapq, soa.span,
                   (soa.rec_off + np.uint64(by)).astype(np.uint64), pay)


def test_offset_sources_give_identical_results(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import relocate

    dense = _synth(5, 250_000, 70)
    paired = relocate(dense, paired=True, n_cells=70)
    cfg = EngineConfig(n_cells=70, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length")
    base = run_engine(engine_lib, cfg, dense)
    for name, soa, batches in [("paired", paired, 1), ("paired x4", paired, 4), ("shifted", _shifted(dense), 1),
                               ("shifted paired x3", _shifted(paired), 3)]:
        assert_same(run_engine(engine_lib, cfg, soa, batches=batches), base, name)


def test_device_generator_with_placement(engine_lib):
    from mgatk2_amd.bam import PLACE_PAIRED, place_records
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import relocate, synth_reads

    n, nc, seed = 90_001, 29, 8
    host = synth_reads(seed, n, nc)
    roff, tot = place_records(host.bc, host.flag, np.full(n, 64, np.uint32), nc, PLACE_PAIRED, start=host.start,
                              tlen=host.tlen)
    exp = relocate(host, paired=True, n_cells=nc)
    np.testing.assert_array_equal(roff, exp.rec_off)
    with engine_lib.Engine(EngineConfig(n_cells=nc)) as eng:
        eng.synth(seed, n, host.extra["cdf"], host.extra["ref"], rec_off=roff, payload_bytes=tot)
        dev = eng.download_inputs()
    for k in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off"):
        np.testing.assert_array_equal(getattr(dev, k), getattr(exp, k), err_msg=k)
    np.testing.assert_array_equal(dev.payload[: exp.payload.size], exp.payload[: dev.payload.size])


# ---------------------------------------------------------------------------
# grouping element forms (mgp_engine.hip): 8-byte compact elements whenever the
# resident reads allow them, the 16-byte form forced with MGP_GROUP_WIDE=1
# ---------------------------------------------------------------------------
def _run_forms(engine_lib, cfg, soa, monkeypatch):
    a = run_engine(engine_lib, cfg, soa)
    monkeypatch.setenv("MGP_GROUP_WIDE", "1")
    try:
        b = run_engine(engine_lib, cfg, soa)
    finally:
        monkeypatch.delenv("MGP_GROUP_WIDE")
    return a, b


@pytest.mark.parametrize("cfgname", sorted(CONFIGS))
def test_compact_and_wide_grouping_agree(engine_lib, oracle_lib, monkeypatch, cfgname):
    """Synthetic reads qualify for the compact element (all packed and paired,
    starts in [0, L), |tlen| < 2^17). Both element forms equal the oracle, on a
    dense set and on a sparse one whose pass-B steps stop at the 32-bin cap."""
    from mgatk2_amd.engine import EngineConfig

    for seed, n, nc in [(5, 300_000, 150), (6, 20_000, 3)]:
        soa = _synth(seed, n, nc)
        cfg = EngineConfig(n_cells=nc, **CONFIGS[cfgname])
        a, b = _run_forms(engine_lib, cfg, soa, monkeypatch)
        exp, _ = oracle_lib.oracle_run(cfg, soa)
        assert_same(a, exp, f"compact {cfgname} {n}x{nc}")
        assert_same(b, exp, f"wide {cfgname} {n}x{nc}")


def test_compact_starts_256_apart_are_not_duplicates(engine_lib, oracle_lib, monkeypatch):
    """Compact elements keep start mod 256: reads of one cell with the same strand
    and |tlen| every 256 positions (equal mod 256, one start bin 32 bins after
    the other) are distinct reads; true duplicates at equal starts still drop."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import pack_reads

    reads = []
    for k in range(40):
        s = 100 + 256 * k
        reads.append(_read(s, [(0, 30)], "ACGT" * 7 + "AC", 0, tlen=150))
        if k % 3 == 0:  # a duplicate under both keys
            reads.append(_read(s, [(0, 30)], "CAGT" * 7 + "CA", 0, tlen=-150))
        if k % 4 == 1:  # same start, other strand
            reads.append(_read(s, [(0, 30)], "GGGT" * 7 + "GG", 0, flag=0x11, tlen=150))
    soa = pack_reads(reads)
    for mode in ("alignment_and_fragment_length", "alignment_start", "none"):
        cfg = EngineConfig(n_cells=1, min_baseq=0, min_mapq=0, min_reads=0, dedup_mode=mode)
        a, b = _run_forms(engine_lib, cfg, soa, monkeypatch)
        exp, _ = oracle_lib.oracle_run(cfg, soa)
        assert_same(a, exp, f"compact {mode}")
        assert_same(b, exp, f"wide {mode}")
        if mode != "none":
            assert exp.stats["duplicate_reads_with_length"] == 14


def test_speculative_compact_falls_back(engine_lib, oracle_lib):
    """Grouping pass A checks key widths and offsets on the reads it loads while it
    writes compact elements; a valid read with |tlen| >= 2^16, or one start past
    mito_len, raises ERR_RESPEC and mgp_sync redoes the run on the standalone check's
    path. Results equal the oracle either way, and a rerun of the same context too."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import ReadSoA

    base = _synth(11, 120_000, 60)
    cfg = EngineConfig(n_cells=60, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length")
    rng = np.random.default_rng(3)
    tl = base.tlen.copy()
    pick = rng.choice(base.n, 40, replace=False)
    tl[pick] = np.where(tl[pick] < 0, -70_000, 70_000) - rng.integers(0, 3, 40)
    for name, soa in [("wide tlen", ReadSoA(base.start, base.bc, tl, base.flag, base.mapq, base.span,
                                            base.rec_off, base.payload)),
                      ("compact", base)]:
        exp, _ = oracle_lib.oracle_run(cfg, soa)
        with engine_lib.Engine(cfg) as eng:
            eng.push(soa)
            for _ in range(2):
                eng.run()
                assert_same(eng.fetch(), exp, name)


@pytest.mark.parametrize("wide", [False, True])
def test_unsorted_detected_at_every_boundary(engine_lib, monkeypatch, wide):
    """The coordinate-order check runs on the speculative path inside grouping pass A
    (a read's predecessor start from the lane below by DPP, from lane 63 of the
    previous slot, or loaded for the first read of a wave's run) and on the fallback
    path in k_check_inputs (MGP_GROUP_WIDE=1). One read moved below its predecessor
    at lane, slot, wave-run, step and start-bin boundaries raises BAMFormatError each
    time; the sorted set runs clean."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import BAMFormatError
    from mgatk2_amd.synth import ReadSoA

    if wide:
        monkeypatch.setenv("MGP_GROUP_WIDE", "1")
    base = _synth(21, 60_000, 40)
    cfg = EngineConfig(n_cells=40, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length")
    st = base.start
    # the first read of some start bins (every part range and wave run starts there)
    bin_first = np.nonzero(np.diff(st // 8) > 0)[0][[3, 40, 700]] + 1
    picks = [1, 63, 64, 65, 511, 512, 513, 2048, 4097, 30_001, base.n - 1, *bin_first.tolist()]
    with engine_lib.Engine(cfg) as eng:
        eng.push(base)
        eng.run()
        eng.sync()
    for i in picks:
        s = st.copy()
        s[i] = s[i - 1] - 1  # below its predecessor only
        soa = ReadSoA(s, base.bc, base.tlen, base.flag, base.mapq, base.span, base.rec_off, base.payload)
        with engine_lib.Engine(cfg) as eng:
            eng.push(soa)
            eng.run()
            with pytest.raises(BAMFormatError):
                eng.sync()


@pytest.mark.parametrize("order", ["reversed", "shuffled"])
def test_scrambled_order_raises_without_faults(engine_lib, order):
    """Reads far from coordinate order give start-bin bounds that are not monotone:
    the histogram flags it and the grouping and pileup kernels stop at entry, so the
    run ends with BAMFormatError and every buffer access stays in bounds. The same
    context then runs the sorted reads bit-exactly."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import BAMFormatError
    from mgatk2_amd.synth import ReadSoA

    base = _synth(23, 80_000, 30)
    cfg = EngineConfig(n_cells=30, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length")
    perm = np.arange(base.n)[::-1] if order == "reversed" else np.random.default_rng(5).permutation(base.n)
    cols = [np.ascontiguousarray(getattr(base, k)[perm]) for k in ("start", "bc", "tlen", "flag", "mapq", "span",
                                                                     "rec_off")]
    bad = ReadSoA(*cols, base.payload)
    exp = run_engine(engine_lib, cfg, base)
    with engine_lib.Engine(cfg) as eng:
        eng.push(bad)
        eng.run()
        with pytest.raises(BAMFormatError):
            eng.sync()
        eng.reset()
        eng.push(base)
        eng.run()
        assert_same(eng.fetch(), exp, f"{order} then sorted")
