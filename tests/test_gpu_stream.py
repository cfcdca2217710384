"""GPU: the ABI v3 paths — cell shards of one synthetic read set (the strong-scaling
bench), cell-range and 16-bit result fetches, streaming runs (MGP_CFG_STREAM: each
push runs the windows it completes while later batches are still being copied),
and the all-reduced speculative-grouping rerun of a communicator run. Every result
is compared bit for bit with a resident run, the oracle or the reference goldens."""

from __future__ import annotations

import numpy as np
import pytest

from golden_io import CASES, Golden, check_result

pytestmark = pytest.mark.gpu

CONFIGS = {
    "tenx": dict(min_baseq=0, min_mapq=0, dedup_mode="alignment_start", min_reads=0),
    "run": dict(min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1),
    "bias": dict(min_baseq=10, min_mapq=1, dedup_mode="none", min_reads=40, max_strand_bias=0.8),
}
KEYS = ("counts", "tn5", "depth", "n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max",
        "median_lo", "median_hi", "ref_tally")
STATS = ("total_reads", "filtered_reads", "n_barcodes", "duplicate_reads_with_length",
         "duplicate_reads_position_only", "cells_passed")


def assert_same(a, b, what="", keys=KEYS, order=True):
    for k in keys:
        x, y = getattr(a, k), getattr(b, k)
        if x is None or y is None:
            continue
        np.testing.assert_array_equal(x, y, err_msg=f"{what}: {k}")
    if order:
        np.testing.assert_array_equal(a.cell_order(), b.cell_order(), err_msg=f"{what}: order")
    for k in STATS:
        assert a.stats[k] == b.stats[k], (what, k, a.stats[k], b.stats[k])


def run_resident(engine_lib, cfg, soa):
    with engine_lib.Engine(cfg) as eng:
        eng.push(soa)
        return eng.finish()


def run_streamed(engine_lib, cfg, soa, batches):
    """Pushes in `batches` coordinate-ordered slices on a streaming context."""
    from dataclasses import replace

    scfg = replace(cfg, stream=True, reserve_reads=soa.n, reserve_payload=int(soa.payload.shape[0]) + 256 * (batches + 1))
    with engine_lib.Engine(scfg) as eng:
        seg0, _ = eng.stream_info()
        cuts = np.linspace(0, soa.n, batches + 1).astype(int)
        for a, b in zip(cuts[:-1], cuts[1:]):
            if b > a:
                eng.push(soa.slice(int(a), int(b)))
        segs, _ = eng.stream_info()
        eng.run()
        res = eng.fetch()
        _, streamed = eng.stream_info()
        return res, segs - seg0, streamed


def _synth(seed, n, nc):
    from mgatk2_amd.synth import synth_reads

    return synth_reads(seed, n, nc)


# ---------------------------------------------------------------------------
# cell shards of one global read set (device generator)
# ---------------------------------------------------------------------------
def test_synth_cell_shards_partition_the_global_set(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.shard import partition_cells
    from mgatk2_amd.synth import cell_cdf, ref_codes

    n, nc, seed, world = 300_000, 60, 4242, 3
    cdf, ref = cell_cdf(seed, nc), ref_codes(seed)
    with engine_lib.Engine(EngineConfig(n_cells=nc)) as eng:
        eng.synth(seed, n, cdf, ref)
        full = eng.download_inputs()
    w = np.diff(np.concatenate([[0], cdf.astype(np.float64)]))
    b = partition_cells(w, world)
    seen = 0
    for r in range(world):
        lo, hi = int(b[r]), int(b[r + 1])
        with engine_lib.Engine(EngineConfig(n_cells=hi - lo)) as eng:
            eng.synth(seed, n, cdf, ref, cells=(lo, hi), shard=(r, world))
            sh = eng.download_inputs()
        i = np.arange(n)
        idx = np.flatnonzero(((full.bc >= lo) & (full.bc < hi)) | ((full.bc < 0) & (i % world == r)))
        assert sh.n == idx.size
        seen += sh.n
        for k in ("start", "tlen", "flag", "mapq", "span"):
            np.testing.assert_array_equal(getattr(sh, k), getattr(full, k)[idx], err_msg=k)
        np.testing.assert_array_equal(sh.bc, np.where(full.bc[idx] >= 0, full.bc[idx] - lo, -1))
        # packed 64-byte records, dense in both sets: record j of the shard is record idx[j]
        rec_sh = sh.payload.reshape(-1, 64)[(sh.rec_off // 64).astype(np.int64)]
        rec_full = full.payload.reshape(-1, 64)[(full.rec_off[idx] // 64).astype(np.int64)]
        np.testing.assert_array_equal(rec_sh, rec_full)
    assert seen == n


def test_shard_runs_equal_the_global_run(engine_lib):
    """Each rank's shard run (cells [lo, hi) of the global set) gives exactly the
    global run's rows of those cells; the tallies sum to the global tallies."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.shard import partition_cells
    from mgatk2_amd.synth import cell_cdf, ref_codes

    n, nc, seed, world = 400_000, 90, 777, 4
    cfg = EngineConfig(n_cells=nc, **CONFIGS["run"])
    cdf, ref = cell_cdf(seed, nc), ref_codes(seed)
    with engine_lib.Engine(cfg) as eng:
        eng.synth(seed, n, cdf, ref)
        whole = eng.finish()
    b = partition_cells(np.diff(np.concatenate([[0], cdf.astype(np.float64)])), world)
    tally = np.zeros_like(whole.ref_tally)
    total = filt = dups = 0
    for r in range(world):
        lo, hi = int(b[r]), int(b[r + 1])
        scfg = EngineConfig(**{**cfg.__dict__, "n_cells": hi - lo})
        with engine_lib.Engine(scfg) as eng:
            eng.synth(seed, n, cdf, ref, cells=(lo, hi), shard=(r, world))
            part = eng.finish()
        for k in KEYS[:-1]:
            np.testing.assert_array_equal(getattr(part, k), getattr(whole, k)[lo:hi], err_msg=f"rank {r} {k}")
        tally += part.ref_tally
        total += part.stats["total_reads"]
        filt += part.stats["filtered_reads"]
        dups += part.stats["duplicate_reads_with_length"]
    np.testing.assert_array_equal(tally, whole.ref_tally)
    assert total == n and filt == whole.stats["filtered_reads"]
    assert dups == whole.stats["duplicate_reads_with_length"]


@pytest.mark.parametrize("streamed", [False, True])
def test_cell_range_of_whole_batches_equals_the_global_run(engine_lib, streamed):
    """mgp_set_cell_range (ABI 5, the streamed multi-device product path): contexts
    that take the same whole batches, each keeping one contiguous cell range, give
    exactly the global run's rows, statistics and first reads of their cells; the
    tallies and read statistics add up (reads of other cells count only toward
    total_reads, like reads without a whitelisted barcode)."""
    from dataclasses import replace

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.shard import partition_cells

    n, nc, world = 400_000, 90, 3
    soa = _synth(4242, n, nc)
    cfg = EngineConfig(n_cells=nc, **CONFIGS["run"])
    whole = run_resident(engine_lib, cfg, soa)
    b = partition_cells(np.bincount(soa.bc[soa.bc >= 0], minlength=nc).astype(np.float64), world)
    tally = np.zeros_like(whole.ref_tally)
    sums = dict.fromkeys(STATS[1:], 0)
    for r in range(world):
        lo, hi = int(b[r]), int(b[r + 1])
        scfg = EngineConfig(**{**cfg.__dict__, "n_cells": hi - lo})
        if streamed:
            scfg = replace(scfg, stream=True, reserve_reads=n, reserve_payload=int(soa.payload.shape[0]) + 4096)
        with engine_lib.Engine(scfg) as eng:
            eng.set_cell_range(lo, hi)
            for a, z in zip(range(0, n, 70_001), list(range(70_001, n, 70_001)) + [n]):
                eng.push(soa.slice(a, z))
            part = eng.finish()
            if streamed:
                assert eng.stream_info()[1]  # (the run was streamed, not rerun resident)
        for k in KEYS[:-1] + ("first_read",):
            np.testing.assert_array_equal(getattr(part, k), getattr(whole, k)[lo:hi], err_msg=f"rank {r} {k}")
        assert part.stats["total_reads"] == n and part.stats["error_bits"] == 0
        tally += part.ref_tally
        for k in sums:
            sums[k] += part.stats[k]
    np.testing.assert_array_equal(tally, whole.ref_tally)
    for k, v in sums.items():
        assert v == whole.stats[k], k


# ---------------------------------------------------------------------------
# cell-range and 16-bit fetches
# ---------------------------------------------------------------------------
def test_fetch_cells_and_rows16_match_fetch(engine_lib):
    from mgatk2_amd.engine import EngineConfig

    soa = _synth(31, 200_000, 40)
    cfg = EngineConfig(n_cells=40, **CONFIGS["tenx"])
    with engine_lib.Engine(cfg) as eng:
        eng.push(soa)
        eng.run()
        full = eng.fetch()
        for lo, hi in ((0, 40), (0, 1), (7, 19), (39, 40), (5, 5)):
            part = eng.fetch_cells(lo, hi)
            for k in KEYS[:-1] + ("first_read",):
                np.testing.assert_array_equal(getattr(part, k), getattr(full, k)[lo:hi], err_msg=f"{lo}-{hi} {k}")
            np.testing.assert_array_equal(part.ref_tally, full.ref_tally)
            r16 = eng.fetch_rows16(lo, hi)
            assert not r16.wide.any()
            np.testing.assert_array_equal(r16.counts.astype(np.uint32), full.counts[lo:hi])
            np.testing.assert_array_equal(r16.tn5.astype(np.uint32), full.tn5[lo:hi])
            np.testing.assert_array_equal(r16.depth.astype(np.uint32), full.depth[lo:hi])
        with pytest.raises(Exception):
            eng.fetch_cells(3, 41)


def test_rows16_wide_windows_saturate_and_fetch_cells_is_exact(engine_lib, oracle_lib):
    """A cell window with more than 65535 reads is flagged wide: its 16-bit rows
    saturate at 65535 (the HDF5 form), the cell-range fetch has the exact values."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    # one cell, 400k reads all starting in positions [0, 60): ~180k deep, so the first
    # window holds more than 65535 reads and is drained into the u32 rows
    deep = synth_reads(91, 400_000, 1)
    assert np.all(deep.rec_off == 64 * np.arange(deep.n, dtype=np.uint64))  # dense packed records
    deep.start[:] = np.sort(deep.start % 60).astype(np.int32)
    deep.payload.reshape(-1, 64)[:, 0:4] = deep.start.view(np.uint8).reshape(-1, 4)
    cfg = EngineConfig(n_cells=1, min_baseq=0, min_mapq=0, dedup_mode="none", min_reads=0)
    with engine_lib.Engine(cfg) as eng:
        eng.push(deep)
        eng.run()
        exact = eng.fetch()
        r16 = eng.fetch_rows16()
    exp, _ = oracle_lib.oracle_run(cfg, deep)
    np.testing.assert_array_equal(exact.counts, exp.counts)
    np.testing.assert_array_equal(exact.depth, exp.depth)
    assert r16.wide[0, 0] == 1
    np.testing.assert_array_equal(r16.depth.astype(np.uint32), np.minimum(exp.depth, 65535))
    np.testing.assert_array_equal(r16.counts.astype(np.uint32), np.minimum(exp.counts, 65535))
    assert exp.depth.max() > 65535


# ---------------------------------------------------------------------------
# streaming runs
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("batches", [1, 3, 17, 64])
@pytest.mark.parametrize("cfgname", sorted(CONFIGS))
def test_streaming_matches_resident(engine_lib, cfgname, batches):
    from mgatk2_amd.engine import EngineConfig

    soa = _synth(5000 + batches, 600_000, 150)
    cfg = EngineConfig(n_cells=150, **CONFIGS[cfgname])
    want = run_resident(engine_lib, cfg, soa)
    got, segs, streamed = run_streamed(engine_lib, cfg, soa, batches)
    assert_same(got, want, f"stream {cfgname} x{batches}")
    np.testing.assert_array_equal(got.first_read, want.first_read)
    assert streamed == (segs > 0)
    if batches >= 3:
        assert segs >= 1  # some window completed before the last push


@pytest.mark.parametrize("cfgname", ["run", "tenx"])
def test_streaming_paired_placement_matches_oracle(engine_lib, oracle_lib, cfgname):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import relocate

    soa = relocate(_synth(77, 400_000, 120), paired=True, n_cells=120)
    cfg = EngineConfig(n_cells=120, **CONFIGS[cfgname])
    got, segs, streamed = run_streamed(engine_lib, cfg, soa, 9)
    exp, _ = oracle_lib.oracle_run(cfg, soa)
    assert segs >= 1 and streamed
    assert_same(got, exp, f"stream paired {cfgname}")


def test_streaming_long_span_halo(engine_lib, oracle_lib):
    """Reads reaching hundreds of positions past their start (declared spans) in
    early batches: the later segments' halos must take them."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import concat_soa, pack_reads

    base = _synth(58, 300_000, 40)
    reads = []
    for s0 in (1200, 2600, 5000, 9000, 12000):
        for k in range(40):
            reads.append(dict(reference_start=s0 + k % 5, cigartuples=[(0, 10), (2, 700), (0, 30)],
                              query_sequence="ACGT" * 10, query_qualities=[37] * 40, bc=40 + k % 2, flag=0x1,
                              mapping_quality=60, template_length=500 + k))
    extra = pack_reads(reads)
    soa = concat_soa([base, extra])
    order = np.argsort(soa.start, kind="stable")
    from mgatk2_amd.shard import shard_soa
    from mgatk2_amd.synth import ReadSoA

    sorted_soa = ReadSoA(soa.start[order], soa.bc[order], soa.tlen[order], soa.flag[order], soa.mapq[order],
                         soa.span[order], soa.rec_off[order], soa.payload)
    sorted_soa, _ = shard_soa(sorted_soa, 0, 42, paired=False, keep_all=True)
    cfg = EngineConfig(n_cells=42, **CONFIGS["tenx"])
    got, segs, streamed = run_streamed(engine_lib, cfg, sorted_soa, 25)
    exp, _ = oracle_lib.oracle_run(cfg, sorted_soa)
    assert segs >= 2 and streamed
    assert got.stats["max_span"] >= 740
    assert_same(got, exp, "stream long spans")


@pytest.mark.parametrize("case", CASES)
def test_streaming_goldens_fall_back_and_match(engine_lib, case):
    """The goldens hold full-layout records, quirk reads and mixed pairedness: a
    streaming run cannot serve them speculatively and reruns resident, with the
    reference's results."""
    g = Golden(case)
    got, segs, streamed = run_streamed(engine_lib, g.config(), g.soa, 7)
    check_result(got, g)


def test_streaming_unsorted_raises(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import BAMFormatError

    soa = _synth(12, 200_000, 20)
    a, b = soa.slice(0, 100_000), soa.slice(100_000, 200_000)
    from dataclasses import replace

    cfg = replace(EngineConfig(n_cells=20, **CONFIGS["run"]), stream=True, reserve_reads=soa.n,
                  reserve_payload=int(soa.payload.shape[0]) + 4096)
    with engine_lib.Engine(cfg) as eng:
        eng.push(b)
        eng.push(a)  # starts go back: not coordinate order
        eng.run()
        with pytest.raises(BAMFormatError):
            eng.sync()
        # the same context then runs sorted input correctly
        eng.reset()
        eng.push(a)
        eng.push(b)
        eng.run()
        got = eng.fetch()
    want = run_resident(engine_lib, EngineConfig(n_cells=20, **CONFIGS["run"]), soa)
    assert_same(got, want, "after unsorted")


def test_streaming_repeated_runs_and_resident_rerun(engine_lib):
    """A second mgp_run on the same resident set (no pushes) runs resident; a new
    streamed set after mgp_reset streams again."""
    from dataclasses import replace

    from mgatk2_amd.engine import EngineConfig

    soa = _synth(99, 300_000, 64)
    cfg = EngineConfig(n_cells=64, **CONFIGS["run"])
    want = run_resident(engine_lib, cfg, soa)
    scfg = replace(cfg, stream=True, reserve_reads=soa.n, reserve_payload=int(soa.payload.shape[0]) + 8192)
    with engine_lib.Engine(scfg) as eng:
        for rep in range(2):
            eng.reset()
            for a in range(0, soa.n, 50_000):
                eng.push(soa.slice(a, min(soa.n, a + 50_000)))
            eng.run()
            assert_same(eng.fetch(), want, f"streamed {rep}")
            assert eng.stream_info()[1]
            eng.run()  # resident rerun of the same set
            assert_same(eng.fetch(), want, f"resident {rep}")
            assert not eng.stream_info()[1]


# ---------------------------------------------------------------------------
# communicator: the speculative grouping's rerun is agreed over the ranks
# ---------------------------------------------------------------------------
def test_single_rank_comm_respec_rerun(engine_lib, oracle_lib):
    """A read with |tlen| >= 2^16 does not fit the compact grouping element: the
    speculative run raises ERR_RESPEC. With a communicator the flag travels in the
    all-reduced buffer and the rerun follows it (one rank here; RCCL refuses two
    ranks on one device)."""
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import concat_soa, pack_reads

    base = _synth(4, 100_000, 9)
    odd = pack_reads([dict(reference_start=int(base.start.max()), cigartuples=[(0, 50)], query_sequence="ACGTA" * 10,
                           query_qualities=[37] * 50, bc=3, flag=0x1, mapping_quality=60, template_length=70_000)])
    soa = concat_soa([base, odd])
    cfg = EngineConfig(n_cells=9, **CONFIGS["run"])
    exp, _ = oracle_lib.oracle_run(cfg, soa)
    with Engine(cfg) as eng:
        eng.comm_init(Engine.comm_unique_id(), 1, 0)
        eng.push(soa)
        got = eng.finish()
    assert_same(got, exp, "comm respec")


def test_repeated_resident_runs_reuse_the_check_bits(engine_lib, oracle_lib):
    """Runs over an unchanged resident set take the previous run's input-check bits
    (no host wait; verified on the device): identical results; a push in between
    drops them (the new set has full-layout records: the general path)."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import concat_soa, synth_reads

    cfg = EngineConfig(n_cells=60, **CONFIGS["run"])
    a = synth_reads(91, 240_000, 60, pack32=cfg.min_baseq)
    a = a.slice(0, int(np.searchsorted(a.start, 8000)))  # the first half of chrM
    with engine_lib.Engine(cfg) as eng:
        eng.push(a)
        eng.run()
        first = eng.fetch()
        for _ in range(3):
            eng.run()
            assert_same(eng.fetch(), first, "cached rerun")
        b = synth_reads(92, 240_000, 60, pack=False)
        b = b.slice(int(np.searchsorted(b.start, 8000)), b.n)  # the second half: coordinate order kept
        assert a.n > 100_000 and b.n > 100_000
        eng.push(b)
        eng.run()
        got = eng.fetch()
    exp_a, _ = oracle_lib.oracle_run(cfg, a)
    assert_same(first, exp_a, "first run")
    exp, _ = oracle_lib.oracle_run(cfg, concat_soa([a, b]))
    assert_same(got, exp, "after push")


# ---------------------------------------------------------------------------
# ABI v3.1: batches without rec_off (dense records in BAM order) and without span
# (the spans from the records' CIGARs on the device)
# ---------------------------------------------------------------------------
def _columnless(soa, a, b, stride, no_start=False):
    from mgatk2_amd.synth import ReadSoA

    return ReadSoA(None if no_start else soa.start[a:b], soa.bc[a:b], soa.tlen[a:b], soa.flag[a:b], soa.mapq[a:b],
                   None, None, np.ascontiguousarray(soa.payload[stride * a:stride * b]))


@pytest.mark.parametrize("no_start", [False, True])
@pytest.mark.parametrize("layout", ["p32", "p64", "full"])
@pytest.mark.parametrize("streamed", [False, True])
def test_push_without_offsets_and_spans(engine_lib, layout, streamed, no_start):
    """The same reads pushed with and without their rec_off / span columns (three
    batches, resident and streaming), and without the start column (ABI 4: the starts
    from the records): identical results, and the device's spans and starts equal the
    producer's (span: max(reference span of the CIGAR, l_seq), the BAM decoder's
    definition) for every read, whatever its CIGAR."""
    from dataclasses import replace

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import relocate, synth_reads

    cfg = EngineConfig(n_cells=30, **CONFIGS["run"])
    kw = dict(pack32=cfg.min_baseq) if layout == "p32" else dict(pack=layout == "p64")
    soa = synth_reads(515, 150_000, 30, **kw)
    stride = {"p32": 32, "p64": 64, "full": 128}[layout]
    soa = relocate(soa, rec_align=stride, n_cells=30)  # dense, BAM order
    assert np.array_equal(soa.rec_off, stride * np.arange(soa.n, dtype=np.uint64)), "dense placement"
    want = run_resident(engine_lib, cfg, soa)
    scfg = replace(cfg, stream=True, reserve_reads=soa.n, reserve_payload=int(soa.payload.shape[0]) + 4096) \
        if streamed else cfg
    cuts = [0, soa.n // 3, (2 * soa.n) // 3 + 7, soa.n]
    with engine_lib.Engine(scfg) as eng:
        for a, b in zip(cuts[:-1], cuts[1:]):
            eng.push(_columnless(soa, a, b, stride, no_start))
        got = eng.finish()
        dev = eng.download_inputs(columns=("span", "start"))
    assert_same(got, want, f"{layout} streamed={streamed} no_start={no_start}")
    np.testing.assert_array_equal(dev.span, soa.span)
    np.testing.assert_array_equal(dev.start, soa.start)


@pytest.mark.parametrize("cfgname", ["run", "tenx"])
@pytest.mark.parametrize("streamed", [False, True])
def test_dense_64_byte_batches_paired_on_the_device(engine_lib, monkeypatch, streamed, cfgname):
    """Dense BAM-order batches of 64-byte records (a streaming producer's, rec_off
    NULL) are paired on the device (k_pair_rank / k_pair_scan / k_pair_place: a
    cell's records two per 128-byte line; batches of 100k, 700k and 700k reads, so
    one and three pairing ranges): the results equal those of the same batches left
    in BAM order (MGP_DEV_PAIR=0), every record lands in a slot of its own, at a
    64-byte multiple, with its bytes unchanged, and the two records sharing a line
    belong to one cell (or are both reads the engine drops)."""
    from dataclasses import replace

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import relocate, synth_reads

    nc = 200
    cfg = EngineConfig(n_cells=nc, **CONFIGS[cfgname])
    soa = relocate(synth_reads(818, 1_500_000, nc, pack=True), rec_align=64, n_cells=nc)
    assert np.array_equal(soa.rec_off, 64 * np.arange(soa.n, dtype=np.uint64))
    if streamed:
        cfg = replace(cfg, stream=True, reserve_reads=soa.n, reserve_payload=int(soa.payload.shape[0]) * 2)
    cuts = [0, 100_000, 800_000, soa.n]
    out = {}
    for pair in ("1", "0"):
        monkeypatch.setenv("MGP_DEV_PAIR", pair)
        with engine_lib.Engine(cfg) as eng:
            for a, b in zip(cuts[:-1], cuts[1:]):
                eng.push(_columnless(soa, a, b, 64, no_start=True))
            res = eng.finish()
            dev = eng.download_inputs(columns=("rec_off", "payload", "bc", "flag"))
        out[pair] = (res, dev)
    assert_same(out["1"][0], out["0"][0], f"paired on the device vs BAM order ({cfgname}, streamed={streamed})")
    dev = out["1"][1]
    off = dev.rec_off.astype(np.int64)
    assert np.all(off % 64 == 0) and np.unique(off).size == soa.n
    recs = dev.payload.reshape(-1, 64)[off // 64]
    np.testing.assert_array_equal(recs, soa.payload.reshape(-1, 64))  # every record's bytes, in read order
    drop = (dev.bc < 0) | ((dev.flag & (0x4 | 0x100 | 0x800)) != 0)
    key = np.where(drop, -1, dev.bc)
    line = off // 128
    order = np.argsort(line, kind="stable")
    ls, ks = line[order], key[order]
    shared = ls[1:] == ls[:-1]
    assert shared.sum() > 0.4 * soa.n  # most records share their line
    assert np.all(ks[1:][shared] == ks[:-1][shared])
    assert np.array_equal(out["0"][1].rec_off.astype(np.int64) % 64, np.zeros(soa.n, np.int64))


@pytest.mark.parametrize("streamed", [False, True])
@pytest.mark.parametrize("layout", ["p64", "p32"])
def test_push16_equals_push(engine_lib, streamed, layout):
    """mgp_push_batch16 (ABI 5: 16-bit barcode index, 0xFFFF = none, and |tlen|; dense
    records): the same results as the 32-bit columns of the same reads, resident and
    streaming (64-byte batches are also paired on the device), with barcode indices
    widened to -1 and |tlen| as the columns; n_cells > 65535 is refused."""
    from dataclasses import replace

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import InvalidInputError
    from mgatk2_amd.synth import ReadSoA, relocate, synth_reads

    nc = 120
    cfg = EngineConfig(n_cells=nc, **CONFIGS["run"])
    stride = 64 if layout == "p64" else 32
    kw = dict(pack=True) if layout == "p64" else dict(pack32=cfg.min_baseq)
    soa = relocate(synth_reads(919, 600_000, nc, **kw), rec_align=stride, n_cells=nc)
    assert int(np.abs(soa.tlen).max()) < 65535
    if streamed:
        cfg = replace(cfg, stream=True, reserve_reads=soa.n, reserve_payload=int(soa.payload.shape[0]) * 2)
    cuts = [0, 150_000, 420_000, soa.n]
    res = {}
    for w16 in (False, True):
        with engine_lib.Engine(cfg) as eng:
            for a, b in zip(cuts[:-1], cuts[1:]):
                if w16:
                    bc = soa.bc[a:b]
                    eng.push(ReadSoA(None, np.where(bc < 0, 0xFFFF, bc).astype(np.uint16),
                                     np.abs(soa.tlen[a:b]).astype(np.uint16), soa.flag[a:b].copy(),
                                     soa.mapq[a:b].copy(), None, None,
                                     np.ascontiguousarray(soa.payload[stride * a:stride * b])))
                else:
                    eng.push(_columnless(soa, a, b, stride, no_start=True))
            res[w16] = eng.finish()
            cols = eng.download_inputs(columns=("bc", "tlen"))
        if w16:
            np.testing.assert_array_equal(cols.bc, soa.bc)
            np.testing.assert_array_equal(cols.tlen, np.abs(soa.tlen))
    assert_same(res[True], res[False], f"push16 {layout} streamed={streamed}")
    with engine_lib.Engine(EngineConfig(n_cells=70_000)) as eng:
        with pytest.raises(InvalidInputError, match="65535"):
            eng.push(ReadSoA(None, np.zeros(4, np.uint16), np.zeros(4, np.uint16), soa.flag[:4].copy(),
                             soa.mapq[:4].copy(), None, None, np.ascontiguousarray(soa.payload[:4 * stride])))


def test_push_without_offsets_rejects_ragged_payloads(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import InvalidInputError
    from mgatk2_amd.synth import relocate, synth_reads

    soa = relocate(synth_reads(516, 1_000, 4, pack32=20), rec_align=32, n_cells=4)
    bad = _columnless(soa, 0, soa.n, 32)
    bad.payload = bad.payload[:-16]  # not n x a stride
    with engine_lib.Engine(EngineConfig(n_cells=4, min_baseq=20)) as eng:
        with pytest.raises(InvalidInputError):
            eng.push(bad)


# ---------------------------------------------------------------------------
# ABI v3.1: a rows target (the 16-bit rows leave the device as the windows complete)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("late", [False, True])
@pytest.mark.parametrize("min_reads", [1, 4500])
@pytest.mark.parametrize("layout", ["p32", "full"])
@pytest.mark.parametrize("streamed", [False, True])
def test_rows16_target_equals_fetch_rows16(engine_lib, streamed, layout, min_reads, late):
    """The rows copied to a pinned target segment by segment equal mgp_fetch_rows16
    of a resident run, for a streamed run of 4 batches and a resident one, also on a
    rerun of the same context; full-layout records make a streamed run rerun resident
    (the target then holds the rerun's rows). With min_reads above some cells' read
    counts the gate (processors.py:22) drops those cells after their rows were sent:
    their target rows are zeroed too (ABI 4). late: the target is set after two of
    the four batches (a streaming run has piled windows by then: they are copied
    when the target is set)."""
    from dataclasses import replace

    from mgatk2_amd.engine import EngineConfig, PinnedBuffer, Rows16
    from mgatk2_amd.synth import synth_reads

    nc = 40
    cfg = EngineConfig(n_cells=nc, **{**CONFIGS["run"], "min_reads": min_reads})
    soa = synth_reads(717, 200_000, nc, **(dict(pack32=cfg.min_baseq) if layout == "p32" else dict(pack=False)))
    with engine_lib.Engine(cfg) as eng:
        eng.push(soa)
        eng.run()
        want = eng.fetch_rows16()
        want_res = eng.fetch()
    if min_reads > 1:  # some cells gated, some passing
        gated = (want_res.n_reads > 0) & (want_res.passed == 0)
        assert gated.any() and want_res.passed.any()
        assert not want.depth[gated].any()
    L = cfg.mito_len
    nw = want.wide.shape[1]
    buf = PinnedBuffer(nc * L * 22 + nc * nw + 64)
    tgt = Rows16(buf.array((nc, L, 8), np.uint16, 0), buf.array((nc, L, 2), np.uint16, nc * L * 16),
                 buf.array((nc, L), np.uint16, nc * L * 20), buf.array((nc, nw), np.uint8, nc * L * 22), want.window_width)
    scfg = replace(cfg, stream=True, reserve_reads=soa.n, reserve_payload=int(soa.payload.shape[0]) + 4096) \
        if streamed else cfg
    with engine_lib.Engine(scfg) as eng:
        if not late:
            eng.set_rows16_target(tgt)
        for rep in range(2):
            for a in (tgt.counts, tgt.tn5, tgt.depth, tgt.wide):
                a.fill(0xAB)
            eng.reset()
            if late:
                eng.set_rows16_target(None)
            cuts = np.linspace(0, soa.n, 5).astype(int)
            for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
                if late and i == 2:
                    if streamed and layout == "p32":
                        assert eng.stream_info()[0] > 0  # windows piled before the target exists
                    eng.set_rows16_target(tgt)
                eng.push(soa.slice(int(a), int(b)))
            eng.run()
            got = eng.fetch()
            for k in ("counts", "tn5", "depth", "wide"):
                np.testing.assert_array_equal(getattr(tgt, k), getattr(want, k), err_msg=f"{k} rep {rep}")
            assert_same(got, want_res, f"rows target streamed={streamed} rep {rep}")
        eng.set_rows16_target(None)


def _rows_targets(nc, L, nw, W):
    """A pinned 16-bit rows target and the 8-bit one beside it (ABI 7)."""
    from mgatk2_amd.engine import PinnedBuffer, Rows8, Rows16

    o8 = nc * L * 22 + nc * nw + 64
    buf = PinnedBuffer(o8 + nc * L * 11 + nc * nw + 64)
    t16 = Rows16(buf.array((nc, L, 8), np.uint16, 0), buf.array((nc, L, 2), np.uint16, nc * L * 16),
                 buf.array((nc, L), np.uint16, nc * L * 20), buf.array((nc, nw), np.uint8, nc * L * 22), W)
    t8 = Rows8(buf.array((nc, L, 8), np.uint8, o8), buf.array((nc, L, 2), np.uint8, o8 + nc * L * 8),
               buf.array((nc, L), np.uint8, o8 + nc * L * 10), buf.array((nc, nw), np.uint8, o8 + nc * L * 11))
    return buf, t16, t8


@pytest.mark.parametrize("late", [False, True])
@pytest.mark.parametrize("gate", [False, True])
@pytest.mark.parametrize("streamed", [False, True])
def test_rows8_target_equals_the_exact_rows(engine_lib, streamed, gate, late):
    """ABI 7 (mgp_set_rows_target): with the 8-bit target beside the 16-bit one, each
    (cell, window) lands in exactly one of them: `narrow` iff every count, tn5 cut and
    depth of the window is at most 255. 8 cells of 40-320 depth (both kinds of window),
    streamed in 4 batches or resident, twice on one context; gate: min_reads between
    the cells' read counts, so the gate (processors.py:22) zeroes some cells after their
    rows were sent; late: the target set after two batches. The merged rows equal the
    exact u32 rows of a resident run."""
    from dataclasses import replace

    from mgatk2_amd.engine import EngineConfig, merge_rows
    from mgatk2_amd.synth import synth_reads

    nc = 8
    soa = synth_reads(717, 800_000, nc, pack=True)
    cfg = EngineConfig(n_cells=nc, **CONFIGS["run"])
    with engine_lib.Engine(cfg) as eng:
        eng.push(soa)
        eng.run()
        ungated = eng.fetch()  # (the narrow flags are the pileup's, before the gate zeroes a cell)
        nw, W = eng.windows()
    nr = ungated.n_reads
    if gate:
        cfg = replace(cfg, min_reads=int(np.sort(nr)[nc // 2]))
    with engine_lib.Engine(cfg) as eng:
        eng.push(soa)
        eng.run()
        want = eng.fetch()
    if gate:
        assert (want.passed == 0).any() and want.passed.any()
    L = cfg.mito_len
    big = np.maximum(ungated.depth, ungated.tn5.max(axis=2))
    fits = np.array([[big[c, k * W:(k + 1) * W].max() <= 255 for k in range(nw)] for c in range(nc)])
    assert fits.any() and not fits.all()
    buf, t16, t8 = _rows_targets(nc, L, nw, W)
    scfg = replace(cfg, stream=True, reserve_reads=soa.n, reserve_payload=int(soa.payload.shape[0]) + 4096) \
        if streamed else cfg
    with engine_lib.Engine(scfg) as eng:
        if not late:
            eng.set_rows_target(t16, t8)
        for rep in range(2):
            for a in (t16.counts, t16.tn5, t16.depth, t16.wide, t8.counts, t8.tn5, t8.depth, t8.narrow):
                a.fill(0xAB)
            eng.reset()
            if late:
                eng.set_rows_target(None)
            cuts = np.linspace(0, soa.n, 5).astype(int)
            for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
                if late and i == 2:
                    eng.set_rows_target(t16, t8)
                eng.push(soa.slice(int(a), int(b)))
            eng.run()
            got = eng.fetch()
            np.testing.assert_array_equal(t8.narrow.astype(bool), fits, err_msg=f"narrow flags rep {rep}")
            assert not t16.wide.any()
            m = merge_rows(t16, t8, 0, nc)
            for k in ("counts", "tn5", "depth"):
                np.testing.assert_array_equal(m[k], getattr(want, k), err_msg=f"{k} rep {rep}")
            assert_same(got, want, f"rows8 target streamed={streamed} rep {rep}")
        eng.set_rows_target(None)


def test_rows8_target_with_a_wide_window(engine_lib):
    """A drained window (more than 65535 reads: wide) is never narrow; its 16-bit rows
    saturate as with the 16-bit target alone, the cell's other windows go 8-bit."""
    from mgatk2_amd.engine import EngineConfig, merge_rows
    from mgatk2_amd.synth import synth_reads

    deep = synth_reads(91, 400_000, 1)  # (as test_rows16_wide_windows_saturate_and_fetch_cells_is_exact)
    deep.start[:] = np.sort(deep.start % 60).astype(np.int32)
    deep.payload.reshape(-1, 64)[:, 0:4] = deep.start.view(np.uint8).reshape(-1, 4)
    cfg = EngineConfig(n_cells=1, min_baseq=0, min_mapq=0, dedup_mode="none", min_reads=0)
    with engine_lib.Engine(cfg) as eng:
        nw, W = eng.windows()
        buf, t16, t8 = _rows_targets(1, cfg.mito_len, nw, W)
        eng.set_rows_target(t16, t8)
        eng.push(deep)
        eng.run()
        exact = eng.fetch()
        eng.set_rows_target(None)
    assert t16.wide[0, 0] == 1 and t8.narrow[0, 0] == 0 and t8.narrow[0, 1:].all()
    m = merge_rows(t16, t8, 0, 1)
    np.testing.assert_array_equal(m["depth"], np.minimum(exact.depth, 65535))
    np.testing.assert_array_equal(m["counts"], np.minimum(exact.counts, 65535))
    np.testing.assert_array_equal(m["tn5"], np.minimum(exact.tn5, 65535))
    assert exact.depth.max() > 65535


@pytest.mark.parametrize("streamed", [False, True])
@pytest.mark.parametrize("fault", ["offset", "misaligned", "cigar", "stride", "lseq", "cigar_off"])
def test_records_outside_the_payload_raise(engine_lib, streamed, fault):
    """A pushed record outside its batch's payload (an offset past the end, a
    misaligned offset, a full record's CIGAR past the end, a dense stride shorter
    than a full record, an l_seq whose qual/seq run past the end, a CIGAR offset
    other than mgp_cigar_offset(l_seq)) makes the run raise InvalidInputError without any kernel
    reading the record; the context then runs a good batch normally (ABI 4)."""
    from dataclasses import replace

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import InvalidInputError
    from mgatk2_amd.synth import ReadSoA, synth_reads

    nc = 8
    cfg = EngineConfig(n_cells=nc, **CONFIGS["run"])
    if streamed:
        cfg = replace(cfg, stream=True, reserve_reads=50_000, reserve_payload=50_000 * 256)
    good = synth_reads(99, 20_000, nc, pack=False)  # full 128-byte records
    with engine_lib.Engine(cfg) as eng:
        eng.push(good)
        want = eng.finish()
    roff = good.rec_off.copy()
    pay = good.payload.copy()
    span = good.span
    if fault == "offset":
        roff[len(roff) // 2] = np.uint64(pay.shape[0] + 4096)
    elif fault == "misaligned":
        roff[7] += np.uint64(8)
    elif fault == "cigar":
        i = len(roff) - 1
        o = int(roff[i])
        pay[o + 8:o + 10] = np.frombuffer(np.uint16(4000).tobytes(), np.uint8)  # n_cigar far past the end
    elif fault == "lseq":  # l_seq far past the end (qual and seq would be read past it), CIGAR left in place
        o = int(roff[len(roff) - 1])
        pay[o + 4:o + 8] = np.frombuffer(np.uint32(100_000).tobytes(), np.uint8)
    elif fault == "cigar_off":  # CIGAR offset inside the record but not at mgp_cigar_offset(l_seq)
        o = int(roff[3])
        pay[o + 12:o + 16] = np.frombuffer(np.uint32(16).tobytes(), np.uint8)
    else:  # dense records at a 64-byte stride: a full record is 128 bytes
        n = 1000
        d = np.zeros(n * 64, np.uint8)
        for i in range(n):
            d[64 * i:64 * i + 64] = good.payload[int(good.rec_off[i]):int(good.rec_off[i]) + 64]
        bad = ReadSoA(good.start[:n].copy(), good.bc[:n].copy(), good.tlen[:n].copy(), good.flag[:n].copy(),
                      good.mapq[:n].copy(), None, None, d)
    if fault != "stride":
        bad = ReadSoA(good.start, good.bc, good.tlen, good.flag, good.mapq, span, roff, pay)
    with engine_lib.Engine(cfg) as eng:
        eng.push(bad)
        with pytest.raises(InvalidInputError, match="outside its batch"):
            eng.finish()
        eng.reset()
        eng.push(good)
        assert_same(eng.finish(), want, "after a rejected batch")
