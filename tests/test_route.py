"""CPU: the host side of a streamed batch on its way to the devices (libmgphost.so,
mgp_route.cpp): the 16-bit batch columns (mgp_batch_columns16) and the multi-device
read router (mgp_route_batch), against numpy restatements of the same selection
(readers.py:96-111: flag and whitelist filters; processors.py:112-144 / SURVEY.md
§8(e): contiguous cell ranges per device)."""

from __future__ import annotations

import numpy as np
import pytest

from mgatk2_amd.bam import RoutePart, batch_columns16, route_batch
from mgatk2_amd.synth import ReadSoA, synth_reads

SKIP = 0x4 | 0x100 | 0x800


def _cols16(soa, n_cells):
    bc16 = np.empty(soa.n, np.uint16)
    tl16 = np.empty(soa.n, np.uint16)
    return batch_columns16(soa, n_cells, bc16, tl16), bc16, tl16


def test_columns16_dense_batch():
    soa = synth_reads(3, 20_000, 40)
    assert np.array_equal(soa.rec_off, 64 * np.arange(soa.n, dtype=np.uint64))
    rc, bc16, tl16 = _cols16(soa, 40)
    assert rc == 3
    np.testing.assert_array_equal(bc16, np.where(soa.bc < 0, 0xFFFF, soa.bc))
    np.testing.assert_array_equal(tl16, np.abs(soa.tlen))


def test_columns16_permuted_records_are_not_dense():
    """reads c1, c2, c1, c2 placed two of a cell per 128-byte line give
    rec_off [0, 128, 64, 192] and a 256-byte payload: the same size and last offset as
    a dense batch, but record i is not at 64 x i."""
    n = 4
    soa = ReadSoA(np.zeros(n, np.int32), np.array([0, 1, 0, 1], np.int32), np.full(n, 200, np.int32),
                  np.full(n, 0x2000, np.uint16), np.full(n, 60, np.uint8), np.zeros(n, np.uint32),
                  np.array([0, 128, 64, 192], np.uint64), np.zeros(256, np.uint8))
    rc, _, _ = _cols16(soa, 2)
    assert rc == 2  # keys fit, records not dense
    soa.rec_off = np.array([0, 64, 128, 192], np.uint64)
    assert _cols16(soa, 2)[0] == 3


@pytest.mark.parametrize("what", ["tlen", "bc", "cells"])
def test_columns16_wide_keys(what):
    soa = synth_reads(4, 5_000, 20)
    nc = 20
    if what == "tlen":
        soa.tlen[77] = -70_000
    elif what == "bc":
        nc = 70_000
        soa.bc[5] = 65_535
    else:
        nc = 70_000
    rc, _, _ = _cols16(soa, nc)
    assert rc == 1  # dense, keys do not fit


def _expected(soa, bounds):
    """Per device: the indices of its reads, in batch order."""
    b = np.asarray(bounds)
    keep = (soa.bc >= b[0]) & (soa.bc < b[-1]) & ((soa.flag & SKIP) == 0)
    dev = np.searchsorted(b, soa.bc, side="right") - 1
    return [np.flatnonzero(keep & (dev == d)) for d in range(len(b) - 1)]


def _record_bytes(payload, off, flag):
    if flag & 0x4000:
        return 32
    if flag & 0x2000:
        return 64
    l_seq = int(payload[off + 4:off + 8].view(np.uint32)[0])
    n_cig = int(payload[off + 8:off + 10].view(np.uint16)[0])
    return 16 + max(64, (l_seq + 3) // 4 * 4) + max(32, (l_seq + 1) // 2 + 15 & ~15) + 4 * n_cig


@pytest.mark.parametrize("layout", ["packed", "full", "pack32", "mixed"])
def test_route_batch_matches_numpy(layout):
    from mgatk2_amd.synth import concat_soa

    nc = 57
    if layout == "mixed":
        soa = concat_soa([synth_reads(7, 3_000, nc, pack=True), synth_reads(8, 3_000, nc, pack=False)])
    else:
        soa = synth_reads(7, 30_000, nc, pack=layout != "full", pack32=20 if layout == "pack32" else None,
                          rec_align=64)
    bounds = np.array([0, 9, 10, 30, 57], np.int32)
    exp = _expected(soa, bounds)
    assert sum(len(e) for e in exp) < soa.n  # some reads go nowhere (no barcode / skipped flags)
    parts = [RoutePart(soa.n, soa.payload.shape[0] + 4096) for _ in range(len(bounds) - 1)]
    first = np.full(nc, 0xFFFFFFFF, np.uint32)
    assert route_batch(soa, bounds, parts, first_index=1000, first_seen=first, n_threads=3)
    for d, (pt, idx) in enumerate(zip(parts, exp)):
        assert pt.n == len(idx)
        sub = pt.soa()
        bc = sub.bc.astype(np.int64)
        np.testing.assert_array_equal(bc, soa.bc[idx] - bounds[d])
        np.testing.assert_array_equal(sub.flag, soa.flag[idx])
        np.testing.assert_array_equal(sub.mapq, soa.mapq[idx])
        if pt.narrow:
            assert layout in ("packed", "pack32")
            np.testing.assert_array_equal(sub.tlen, np.abs(soa.tlen[idx]))
            stride = 32 if layout == "pack32" else 64
            assert sub.payload.shape[0] == stride * len(idx)
            offs = stride * np.arange(len(idx))
        else:
            assert layout in ("full", "mixed")
            np.testing.assert_array_equal(sub.tlen, soa.tlen[idx])
            offs = sub.rec_off.astype(np.int64)
            assert np.all(offs % 64 == 0) and np.all(np.diff(offs) > 0)
        for k, i in enumerate(idx):
            o = int(soa.rec_off[i])
            nb = _record_bytes(soa.payload, o, int(soa.flag[i]))
            np.testing.assert_array_equal(sub.payload[offs[k]:offs[k] + nb], soa.payload[o:o + nb])
        assert not pt.payload[pt.payload_bytes:pt.payload_bytes + 256].any()
    # each cell's first routed read, as a stream index
    for c in range(nc):
        hit = np.flatnonzero((soa.bc == c) & ((soa.flag & SKIP) == 0))
        assert first[c] == (1000 + hit[0] if hit.size else 0xFFFFFFFF)


def test_route_batch_too_small_writes_nothing():
    soa = synth_reads(9, 20_000, 10)
    bounds = np.array([0, 5, 10], np.int32)
    parts = [RoutePart(100, 1 << 20), RoutePart(soa.n, soa.payload.shape[0] + 4096)]
    first = np.full(10, 0xFFFFFFFF, np.uint32)
    assert not route_batch(soa, bounds, parts, first_seen=first)
    assert (first == 0xFFFFFFFF).all()
    # halves until every part fits (what the product's router does)
    got = []
    for a, b in ((0, 50), (50, 100), (100, 150)):
        sub = ReadSoA(None, soa.bc[a:b], soa.tlen[a:b], soa.flag[a:b], soa.mapq[a:b], None, soa.rec_off[a:b],
                      soa.payload)
        assert route_batch(sub, bounds, parts, first_index=a, first_seen=first)
        got.append(parts[0].n)
    assert sum(got) == int(((soa.bc[:150] >= 0) & (soa.bc[:150] < 5) & ((soa.flag[:150] & SKIP) == 0)).sum())
