"""Producer payload placement (mgp_place_records, include/mgpileup_host.h): two
consecutive packed records of one cell per 128-byte line, a cell's reads that
repeat the start, strand and |tlen| of an earlier read of the cell placed with
the dropped reads. The placement moves records, never changes them, so every
consumer (oracle, decoder, shard gather, batch slicing) must give the same
results as with the dense layout. CPU only."""

from __future__ import annotations

import numpy as np
import pytest

from mgatk2_amd.bam import PLACE_DENSE, PLACE_PAIRED, BamFile, place_records, soa_to_bam
from mgatk2_amd.engine import EngineConfig
from mgatk2_amd.synth import FLAG_PACKED, relocate, synth_reads

DROP = 0x4 | 0x100 | 0x800  # unmapped, secondary, supplementary (readers.py:96-97)


def _place_keys(bc, flag, n_cells, start=None, tlen=None, packed=None):
    """The line key of each read (mgp_place.h): its cell, or n_cells for reads the
    engine drops and, given start/tlen, for a packed read repeating an earlier
    packed read's key in the cell at the same start (up to 8 keys kept per start)."""
    key = np.where((bc >= 0) & (bc < n_cells) & ((flag & DROP) == 0), bc, n_cells).astype(np.int64)
    if start is None:
        return key
    seen = {}  # cell -> (start, [keys])
    for i in range(key.size):
        c = int(key[i])
        if c == n_cells or not packed[i]:
            continue
        k = (abs(int(tlen[i])), bool(flag[i] & 0x10))
        st, ks = seen.get(c, (None, []))
        if st != int(start[i]):
            seen[c] = (int(start[i]), [k])
        elif k in ks:
            key[i] = n_cells
        elif len(ks) < 8:
            ks.append(k)
    return key


def _check_paired(bc, flag, rb, n_cells, off, total, start=None, tlen=None):
    off = off.astype(np.int64)
    assert np.all(off % 16 == 0)
    assert np.all(off + rb <= total)
    # no two records overlap
    o = np.argsort(off, kind="stable")
    assert np.all(off[o][1:] >= (off[o] + rb[o])[:-1])
    packed = ((flag & FLAG_PACKED) != 0) & (rb == 64)
    assert np.all(off[~packed] % 128 == 0)
    key = _place_keys(bc, flag, n_cells, start, tlen, packed)
    # per key, the k-th packed record in BAM order sits in line k // 2, half k % 2
    for k in np.unique(key[packed]):
        sel = np.flatnonzero(packed & (key == k))
        lines, half = off[sel] // 128, (off[sel] % 128) // 64
        np.testing.assert_array_equal(half, np.arange(sel.size) % 2)
        np.testing.assert_array_equal(lines[1::2], lines[0::2][: sel.size // 2])
        assert np.all(np.diff(lines[0::2]) > 0)  # lines opened in BAM order


def test_place_records_rules():
    rng = np.random.default_rng(3)
    n, nc = 20_000, 37
    bc = rng.integers(-1, nc, n).astype(np.int32)
    flag = np.full(n, FLAG_PACKED, np.uint16)
    flag[rng.random(n) < 0.05] |= 0x100
    full = rng.random(n) < 0.1
    flag[full] &= ~np.uint16(FLAG_PACKED)
    rb = np.where(full, rng.integers(100, 400, n), 64).astype(np.uint32)
    off, total = place_records(bc, flag, rb, nc, PLACE_PAIRED)
    _check_paired(bc, flag, rb.astype(np.int64), nc, off, total)
    # keyed: repeats of (start, strand, |tlen|) inside a cell go with the dropped reads
    start = np.sort(rng.integers(0, 400, n)).astype(np.int32)
    tlen = (rng.integers(0, 3, n) * rng.choice([-1, 1], n)).astype(np.int32)
    flag[rng.random(n) < 0.5] |= 0x10
    koff, ktotal = place_records(bc, flag, rb, nc, PLACE_PAIRED, start=start, tlen=tlen)
    packed = ((flag & FLAG_PACKED) != 0) & (rb == 64)
    key = _place_keys(bc, flag, nc, start, tlen, packed)
    assert (key == nc).sum() > (_place_keys(bc, flag, nc) == nc).sum() + 1000  # the rule applies
    _check_paired(bc, flag, rb.astype(np.int64), nc, koff, ktotal, start, tlen)
    doff, dtot = place_records(bc, flag, rb, nc, PLACE_DENSE, rec_align=16)
    np.testing.assert_array_equal(doff[1:], np.cumsum((rb.astype(np.int64) + 15) // 16 * 16)[:-1])
    assert dtot == int(((rb.astype(np.int64) + 15) // 16 * 16).sum())


def test_place_records_edges():
    e = np.zeros(0)
    assert place_records(e.astype(np.int32), e.astype(np.uint16), e.astype(np.uint32), 0)[1] == 0
    one = place_records(np.array([0], np.int32), np.array([FLAG_PACKED], np.uint16), np.array([64], np.uint32), 1)
    assert one[0][0] == 0 and one[1] == 128
    with pytest.raises(ValueError):
        place_records(np.array([0], np.int32), np.array([0], np.uint16), np.array([64], np.uint32), 1, mode=7)


@pytest.fixture(scope="module")
def synth():
    return synth_reads(11, 120_000, 40)


def test_relocate_roundtrip(synth):
    p = relocate(synth, paired=True, n_cells=40)
    assert np.any(np.diff(p.rec_off.astype(np.int64)) < 0)  # no longer in BAM order
    rb = np.full(p.n, 64, np.int64)
    _check_paired(p.bc, p.flag, rb, 40, p.rec_off, p.payload.size, p.start, p.tlen)
    d = relocate(p, paired=False, n_cells=40)
    for k in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off"):
        np.testing.assert_array_equal(getattr(d, k), getattr(synth, k), err_msg=k)
    np.testing.assert_array_equal(d.payload[: synth.payload.size], synth.payload)


@pytest.mark.parametrize("cfg", [
    dict(min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1),
    dict(min_baseq=0, min_mapq=0, dedup_mode="alignment_start", min_reads=0),
])
def test_oracle_paired_equals_dense(oracle_lib, synth, cfg):
    c = EngineConfig(n_cells=40, **cfg)
    a, oa = oracle_lib.oracle_run(c, synth)
    b, ob = oracle_lib.oracle_run(c, relocate(synth, paired=True, n_cells=40))
    for k in ("counts", "tn5", "depth", "n_reads", "passed", "ref_tally", "median_lo", "median_hi", "first_read"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    np.testing.assert_array_equal(oa, ob)
    assert a.stats == b.stats


def test_slice_of_paired_payload(synth):
    p = relocate(synth, paired=True, n_cells=40)
    for lo, hi in [(0, 1), (5, 70_001), (100_000, 120_000)]:
        s, d = p.slice(lo, hi), synth.slice(lo, hi)
        r = relocate(s, n_cells=40)
        for k in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off"):
            np.testing.assert_array_equal(getattr(r, k), getattr(d, k), err_msg=f"{k} {lo}:{hi}")
        np.testing.assert_array_equal(r.payload[: d.payload.size], d.payload)


def test_shard_gather_from_paired_source(synth):
    from mgatk2_amd.shard import shard_soa

    p = relocate(synth, paired=True, n_cells=40)
    a, ia = shard_soa(p, 10, 25)
    b, ib = shard_soa(synth, 10, 25)
    np.testing.assert_array_equal(ia, ib)
    ra, rb = relocate(a, n_cells=15), relocate(b, n_cells=15)
    for k in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off"):
        np.testing.assert_array_equal(getattr(ra, k), getattr(rb, k), err_msg=k)
    np.testing.assert_array_equal(ra.payload, rb.payload)


def test_decoder_paired_placement(tmp_path, synth):
    wl = [f"C{i:03d}-1" for i in range(40)]
    sub = synth.slice(0, 30_000)
    soa_to_bam(tmp_path / "x.bam", sub, wl)
    with BamFile(tmp_path / "x.bam") as bam:
        p = bam.read_soa("chrM", wl, pack=True)
        d = bam.read_soa("chrM", wl, pack=True, paired=False)
    assert np.array_equal(d.rec_off, np.arange(d.n, dtype=np.uint64) * 64)
    rb = np.full(p.n, 64, np.int64)
    _check_paired(p.bc, p.flag, rb, 40, p.rec_off, p.payload.size, p.start, p.tlen)
    r = relocate(p, n_cells=40)
    np.testing.assert_array_equal(r.rec_off, d.rec_off)
    np.testing.assert_array_equal(r.payload[: d.payload.size], d.payload[: r.payload.size])


def test_split_by_range_equals_numpy():
    """mgp_split_by_range (the multi-device stream's router): each range's read
    indices in batch order, as one numpy scan per range gives them; empty ranges,
    reads outside every range and negative (unlisted) barcodes included."""
    from mgatk2_amd.shard import split_by_range

    rng = np.random.default_rng(3)
    bc = rng.integers(-3, 1200, 200_001).astype(np.int32)
    for bounds in ([0, 1000], [0, 250, 250, 600, 1000], [100, 101, 900], [0, 1, 2, 3, 4, 5, 6, 7, 1100]):
        got = split_by_range(bc, bounds)
        assert len(got) == len(bounds) - 1
        for d, idx in enumerate(got):
            exp = np.flatnonzero((bc >= bounds[d]) & (bc < bounds[d + 1]))
            np.testing.assert_array_equal(idx, exp)
    assert [x.size for x in split_by_range(np.zeros(0, np.int32), [0, 5, 9])] == [0, 0]
