"""GPU: the txt count files formatted and deflated on the device (mgp_txt_gz_*,
mgatk2_amd/csrc/mgp_txtgz.hip), against the reference's text.

The reference writes, per passing cell, "pos,bc,depth" / "pos,bc,fwd,rev" lines and
gzips each file at compresslevel 9 (src/file_io/writers.py:430-486). The device writes
one gzip member per (file, cell); a file is its members in cell order. Checked here:
* the gunzipped bytes equal the reference's expected text of every golden case (engine
  run, then the device writer on the run's rows);
* edge cases from caller rows (mgp_txt_gz_rows): counts past 16 bits, zero-line cells
  and files, one-line members (fixed / stored blocks), 1- and 4096-byte barcodes, the
  empty barcode, against the host formatter's text (mgp_txt_write_cells, itself pinned
  to the reference by test_writers_golden.py);
* size: on C4-density cells (20k reads per cell through the oracle) each file is no
  larger than zlib level 9's stream of the same text (the reference's gzip.open(...,
  compresslevel=9)); the ratio is printed.
"""

from __future__ import annotations

import gzip
import zlib

import numpy as np
import pytest

from golden_io import CASES, Golden

pytestmark = pytest.mark.gpu

FILES = ("coverage", "A", "C", "G", "T")


def host_text(counts, depth, cells, names, tmp_path) -> dict:
    """The host formatter's text of the same cells (level-1 members, gunzipped)."""
    from mgatk2_amd.bam import txt_write_cells

    prefix = tmp_path / "host"
    txt_write_cells(prefix, counts, depth, cells, names, level=1, append=False)
    return {f: gzip.decompress((tmp_path / f"host.{f}.txt.gz").read_bytes()) for f in FILES}


def device_text(mem) -> dict:
    return {f: gzip.decompress(mem.file_part(i).tobytes()) for i, f in enumerate(FILES)}


def check_members(mem, n):
    """Every nonempty member is a gzip stream of its own, with its text's size."""
    blob = mem.blob.tobytes()
    at = 0
    for f in range(5):
        for k in range(n):
            b = int(mem.member_bytes[f, k])
            if b == 0:
                assert mem.text_bytes[f, k] == 0
                continue
            d = zlib.decompressobj(31)
            txt = d.decompress(blob[at:at + b])
            assert d.eof and not d.unused_data and len(txt) == mem.text_bytes[f, k]
            at += b
    assert at == len(blob)


@pytest.mark.parametrize("case", CASES)
def test_device_txt_equals_reference_goldens(case, engine_lib):
    """Engine run of the golden's reads, then the device writer over the passing cells in
    first-seen order: the gunzipped files equal the reference's txt output."""
    from mgatk2_amd.engine import Engine

    g = Golden(case)
    with Engine(g.config()) as eng:
        eng.push(g.soa)
        eng.run()
        res = eng.fetch(dense=False)
        order = res.cell_order()
        written = order[res.passed[order].astype(bool)]
        mem = eng.txt_gz(written, [g.whitelist[c] for c in written.tolist()])
    check_members(mem, written.size)
    if not g.has("txt_coverage"):
        pytest.skip("(an HDF5 case: no reference txt)")
    got = device_text(mem)
    for f in FILES:
        assert got[f].decode() == str(g.exp(f"txt_{f}")), f"{case}: output.{f}.txt"


def _rows(rng, n, L, scale, zero_frac):
    depth = np.zeros((n, L), np.uint32)
    counts = np.zeros((n, L, 8), np.uint32)
    cov = rng.random((n, L)) > zero_frac
    c = (rng.random((n, L, 8)) < 0.3) * rng.integers(0, scale, (n, L, 8))
    c[..., 0] += rng.integers(1, 3, (n, L)).astype(np.uint32) * cov
    counts[...] = c * cov[..., None]
    depth[...] = counts.sum(axis=2)
    return counts, depth


@pytest.mark.parametrize("scale", [40, 70_000, 5_000_000])
def test_device_txt_rows_edge_cases(scale, engine_lib, tmp_path):
    from mgatk2_amd.engine import txt_gz_rows

    rng = np.random.default_rng(scale)
    L, n = 16569, 9
    counts, depth = _rows(rng, n, L, scale, 0.3)
    counts[2] = 0  # no line in any file
    depth[2] = 0
    counts[3, :, 2:] = 0  # lines only in coverage and A
    depth[3] = counts[3].sum(axis=1)
    counts[4] = 0  # one line
    depth[4] = 0
    counts[4, 777, 5] = 3
    depth[4, 777] = 3
    counts[5, :, :] = 0  # every position a line, counts 1
    counts[5, :, 0] = 1
    depth[5] = 1
    names = ["ACGTACGTACGTACGT-1", "G", "", "AAAC-7", "T" * 4096, "CCCCGGGGTTTTAAAA-1", "x" * 70, "TTTT", "A-1"]
    cells = [0, 1, 2, 3, 4, 5, 6, 7, 8][::-1]
    names = names[::-1]
    mem = txt_gz_rows(counts, depth, cells, names)
    check_members(mem, len(cells))
    assert device_text(mem) == host_text(counts, depth, cells, names, tmp_path)


def test_device_txt_rows_many_small_cells(engine_lib, tmp_path):
    """Thousands of sparse cells (members of a few lines: fixed and stored blocks)."""
    from mgatk2_amd.engine import txt_gz_rows

    rng = np.random.default_rng(7)
    L, n = 16569, 3000
    counts, depth = _rows(rng, n, L, 5, 0.9995)
    names = [f"C{i:05d}-1" for i in range(n)]
    cells = rng.permutation(n)
    mem = txt_gz_rows(counts, depth, cells, [names[c] for c in cells])
    check_members(mem, n)
    assert device_text(mem) == host_text(counts, depth, cells, [names[c] for c in cells], tmp_path)


def test_device_txt_smaller_than_zlib9_on_c4_density(engine_lib, oracle_lib, tmp_path):
    """C4's density (20k reads per cell, `run` parameters) through the oracle: the
    device members of each file are no larger than zlib level 9's single stream of the
    same text (the reference's gzip -9 of the whole file)."""
    from mgatk2_amd.engine import EngineConfig, txt_gz_rows
    from mgatk2_amd.synth import synth_reads

    nc = 12
    soa = synth_reads(20251019, nc * 20_000, nc)
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length",
                       min_reads=1)
    res, _ = oracle_lib.oracle_run(cfg, soa)
    rng = np.random.default_rng(5)
    names = ["".join(rng.choice(list("ACGT"), 16)) + "-1" for _ in range(nc)]
    cells = list(range(nc))
    mem = txt_gz_rows(res.counts, res.depth, cells, names)
    text = host_text(res.counts, res.depth, cells, names, tmp_path)
    assert device_text(mem) == text
    for i, f in enumerate(FILES):
        dev = int(mem.member_bytes[i].sum())
        z9 = len(gzip.compress(text[f], compresslevel=9))
        print(f"{f}: text {len(text[f])} device {dev} zlib9 {z9} ratio {dev / z9:.3f}")
        assert dev <= z9, (f, dev, z9)


def test_device_txt_member_past_32_mb(engine_lib, tmp_path):
    """A member whose text passes 2^25 bytes (every position covered, a 4096-byte
    barcode: ~68 MB of coverage lines): its CRC-32 (per-segment CRCs shifted past the
    bytes after them) and the member still gunzip to the host formatter's text."""
    from mgatk2_amd.engine import txt_gz_rows

    L = 16569
    counts = np.zeros((1, L, 8), np.uint32)
    counts[0, :, 0] = 7
    counts[0, ::3, 3] = 2
    depth = counts.sum(axis=2).astype(np.uint32)
    names = ["ACGT" * 1024]
    mem = txt_gz_rows(counts, depth, [0], names)
    assert mem.text_bytes[0, 0] > 1 << 25
    check_members(mem, 1)
    assert device_text(mem) == host_text(counts, depth, [0], names, tmp_path)


def test_device_txt_with_a_wide_window(engine_lib, tmp_path):
    """A cell with drained windows (more than 65535 reads: its exact u32 rows there, the
    16-bit rows elsewhere) through the engine's writer: the same text as the host
    formatter's from the exact result."""
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import synth_reads

    deep = synth_reads(91, 400_000, 1)
    deep.start[:] = np.sort(deep.start % 3000).astype(np.int32)
    deep.payload.reshape(-1, 64)[:, 0:4] = deep.start.view(np.uint8).reshape(-1, 4)
    cfg = EngineConfig(n_cells=1, min_baseq=0, min_mapq=0, dedup_mode="none", min_reads=0)
    with Engine(cfg) as eng:
        eng.push(deep)
        eng.run()
        exact = eng.fetch()
        r16 = eng.fetch_rows16()
        mem = eng.txt_gz([0], ["ACGTACGTACGTACGT-1"])
    assert r16.wide[0].any() and not r16.wide[0].all()  # (u32 rows in the drained windows, 16-bit elsewhere)
    check_members(mem, 1)
    assert device_text(mem) == host_text(exact.counts, exact.depth, [0], ["ACGTACGTACGTACGT-1"], tmp_path)
