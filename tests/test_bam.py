"""Native BAM ingest (libmgphost.so, include/mgpileup_host.h) — CPU tests.

The golden cases hold the exact reads the reference consumed (through its
pysam stand-in, tests/golden/make_golden.py) and the engine batch they map to.
Writing those reads as a BAM and decoding it with the native reader must give
that batch back bit for bit; the oracle on that batch reproduces the
reference's outputs (test_oracle_golden.py), which pins BAM -> outputs.
The writer itself is checked against an independent decode (gzip + struct,
SAM spec §4.2) so that a symmetric writer/reader bug cannot hide.
"""

from __future__ import annotations

import gzip
import struct

import numpy as np
import pytest

from golden_io import CASES, Golden
from mgatk2_amd.bam import BamFile, BamWriter, soa_to_bam
from mgatk2_amd.exceptions import BAMFormatError, BAMReadError
from mgatk2_amd.synth import FLAG_NOSEQQUAL, pack_reads, unpack_record

KEYS = ["start", "bc", "tlen", "flag", "mapq", "span", "rec_off"]


def _assert_soa_equal(a, b):
    """Same reads and record bytes; the payload placement may differ (the decoder
    pairs packed records per cell): both are compared in the dense layout."""
    from mgatk2_amd.synth import relocate

    nc = max(int(a.bc.max()) if a.n else 0, int(b.bc.max()) if b.n else 0) + 1
    a, b = relocate(a, n_cells=nc), relocate(b, n_cells=nc)
    for k in KEYS:
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    np.testing.assert_array_equal(a.payload[: b.payload.size], b.payload[: a.payload.size])
    assert a.payload.size == b.payload.size


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("index", [True, False])
def test_roundtrip_golden(case, index, tmp_path):
    g = Golden(case)
    soa_to_bam(tmp_path / "x.bam", g.soa, g.whitelist, index=index)
    with BamFile(tmp_path / "x.bam") as bam:
        assert bam.references == ("chr1", "chrM")
        assert bam.lengths == (248956422, 16569)
        assert bam.has_index == index
        got = bam.read_soa("chrM", g.whitelist, rec_align=128, pack=False)
    _assert_soa_equal(got, g.soa)


@pytest.mark.parametrize("case", CASES)
def test_packed_decode_matches_full_decode(case, tmp_path):
    """The decoder's packed records (mgp_pack_record) hold the full records'
    pileup view: same SoA columns (plus MGP_FLAG_PACKED), same start / strand /
    CIGAR, bases with N and quality 0 where the base is not A, C, G or T."""
    from mgatk2_amd.synth import FLAG_PACKED

    g = Golden(case)
    soa_to_bam(tmp_path / "x.bam", g.soa, g.whitelist)
    with BamFile(tmp_path / "x.bam") as bam:
        pk = bam.read_soa("chrM", g.whitelist, pack=True)
        fu = bam.read_soa("chrM", g.whitelist, pack=False)
    for k in ("start", "bc", "tlen", "mapq", "span"):
        np.testing.assert_array_equal(getattr(pk, k), getattr(fu, k), err_msg=k)
    np.testing.assert_array_equal(pk.flag & np.uint16(0xFFFF ^ FLAG_PACKED), fu.flag)
    assert (pk.flag & FLAG_PACKED).any()
    for i in range(pk.n):
        a = unpack_record(pk.payload, int(pk.rec_off[i]), int(pk.flag[i]))
        b = unpack_record(fu.payload, int(fu.rec_off[i]), int(fu.flag[i]))
        assert a["reference_start"] == b["reference_start"] and a["cigartuples"] == b["cigartuples"]
        if pk.flag[i] & FLAG_PACKED:
            acgt = [c in "ACGT" for c in b["query_sequence"]]
            assert a["query_sequence"] == "".join(c if m else "N" for c, m in zip(b["query_sequence"], acgt))
            assert a["query_qualities"] == [q if m else 0 for q, m in zip(b["query_qualities"], acgt)]
            assert bool(a["flag"] & 0x10) == bool(b["flag"] & 0x10)
        else:
            assert a == b


def _independent_decode(path):
    """gzip (BGZF is multi-member gzip) + struct per the SAM spec."""
    raw = gzip.decompress(path.read_bytes())
    assert raw[:4] == b"BAM\1"
    (lt,) = struct.unpack_from("<i", raw, 4)
    p = 8 + lt
    (nref,) = struct.unpack_from("<i", raw, p)
    p += 4
    refs = []
    for _ in range(nref):
        (ln,) = struct.unpack_from("<i", raw, p)
        refs.append(raw[p + 4 : p + 4 + ln - 1].decode())
        p += 4 + ln + 4
    recs = []
    while p < len(raw):
        (bs,) = struct.unpack_from("<i", raw, p)
        r = raw[p + 4 : p + 4 + bs]
        tid, pos, ln, mq, _bin, nc, flag, ls, _nt, _np, tl = struct.unpack_from("<iiBBHHHIiii", r, 0)
        q = 32 + ln
        cig = [(c & 15, c >> 4) for c in struct.unpack_from(f"<{nc}I", r, q)]
        q += 4 * nc
        sb = r[q : q + (ls + 1) // 2]
        seq = "".join("=ACMGRSVTWYHKDBN"[(sb[i // 2] >> (4 * (1 - i % 2))) & 15] for i in range(ls))
        q += (ls + 1) // 2
        qual = list(r[q : q + ls])
        q += ls
        tags = {}
        while q < len(r):
            t, ty = r[q : q + 2].decode(), chr(r[q + 2])
            if ty == "Z":
                z = r.index(b"\0", q + 3)
                tags[t] = r[q + 3 : z].decode()
                q = z + 1
            else:
                raise AssertionError(ty)
        recs.append(dict(tid=tid, pos=pos, mapq=mq, flag=flag, cig=cig, seq=seq, qual=qual, tlen=tl, tags=tags))
        p += 4 + bs
    return refs, recs


def test_writer_independent_decode(tmp_path):
    g = Golden("synth_run")
    soa_to_bam(tmp_path / "x.bam", g.soa, g.whitelist)
    refs, recs = _independent_decode(tmp_path / "x.bam")
    assert refs == ["chr1", "chrM"] and len(recs) == g.soa.n
    for i in range(0, g.soa.n, 7):
        r, d = recs[i], unpack_record(g.soa.payload, int(g.soa.rec_off[i]), int(g.soa.flag[i]))
        assert r["tid"] == 1 and r["pos"] == g.soa.start[i] and r["mapq"] == g.soa.mapq[i]
        assert r["flag"] == int(g.soa.flag[i]) & 0xFFF and r["tlen"] == g.soa.tlen[i]
        assert r["cig"] == d["cigartuples"]
        assert r["seq"] == d["query_sequence"]
        if not (int(g.soa.flag[i]) & FLAG_NOSEQQUAL):
            assert r["qual"] == d["query_qualities"]
        b = int(g.soa.bc[i])
        assert (r["tags"].get("CB") == g.whitelist[b]) if b >= 0 else (r["tags"].get("CB") not in g.whitelist)


def _rd(pos, flag=0, cb="AAAC-1", seq="ACGTACGTAC", cig=None, tid=1, **kw):
    return dict(tid=tid, pos=pos, flag=flag, mapq=60, cigartuples=cig or [(0, len(seq))], query_sequence=seq,
                query_qualities=[30] * len(seq), template_length=kw.get("tlen", 0),
                tags={} if cb is None else {"CB": cb})


def _stream_cols(path, wl, batch, pipe, walk):
    """The columns of a streaming decode of chrM (MGP_BAM_PIPELINE / MGP_BAM_WALK_AHEAD
    as given), batches concatenated."""
    import os

    from mgatk2_amd.bam import StreamSlot

    old = {k: os.environ.get(k) for k in ("MGP_BAM_PIPELINE", "MGP_BAM_WALK_AHEAD")}
    os.environ["MGP_BAM_PIPELINE"], os.environ["MGP_BAM_WALK_AHEAD"] = pipe, walk
    try:
        cols = {k: [] for k in ("start", "bc", "tlen", "flag", "mapq", "span")}
        with BamFile(path, n_threads=4) as b:
            st = b.stream("chrM", wl)
            try:
                slot = StreamSlot(batch, batch * 300 + 2 * 128 * (len(wl) + 1) + (1 << 20))
                while st.next_into(slot):
                    v = slot.soa()
                    for k in cols:
                        cols[k].append(getattr(v, k).copy())
            finally:
                st.close()
        return {k: np.concatenate(v) for k, v in cols.items()}
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_other_contigs_many_blocks_threads(tmp_path):
    """chrM sits between other contigs and spans many BGZF blocks: the index seek,
    the no-index scan and 1 vs 8 inflate threads give the same batch."""
    rng = np.random.default_rng(1)
    w = BamWriter(tmp_path / "x.bam", [("chr1", 10**6), ("chrM", 16569), ("chrX", 10**6)])
    for p in sorted(rng.integers(0, 10**6, 3000)):
        w.write(_rd(int(p), tid=0, cb="CCCC-1"))
    chrm = []
    for p in sorted(rng.integers(0, 16500, 20000)):
        r = _rd(int(p), flag=int(rng.choice([0, 16, 99, 147])), cb=["AAAC-1", "GGGT-1", None, "TTTT-1"][p % 4],
                seq="".join(rng.choice(list("ACGTN"), 40)))
        chrm.append(r)
        w.write(r)
    for p in sorted(rng.integers(0, 10**6, 3000)):
        w.write(_rd(int(p), tid=2))
    w.close(index=True)
    wl = ["AAAC-1", "GGGT-1"]
    with BamFile(tmp_path / "x.bam", n_threads=1) as b1:
        a = b1.read_soa("chrM", wl)
        assert b1.read_soa("chr1", wl).n == 3000
        assert b1.read_soa("chrX", wl).n == 3000
    streamed = {}
    for idx in ("index", "scan"):
        if idx == "scan":
            (tmp_path / "x.bam.bai").unlink()
        for pipe, walk in (("1", "1"), ("1", "0"), ("0", "1"), ("0", "0")):
            for batch in (997, 7000):
                streamed[idx, pipe, walk, batch] = _stream_cols(tmp_path / "x.bam", wl, batch, pipe, walk)
    with BamFile(tmp_path / "x.bam", n_threads=8) as b8:
        assert not b8.has_index
        c = b8.read_soa("chrM", wl)
    _assert_soa_equal(a, c)
    # the streaming decode (index seek or scan; pipelined placement and the prefetch
    # thread's boundary walk on or off) gives the same columns in the same order
    for key, cols in streamed.items():
        for k, v in cols.items():
            np.testing.assert_array_equal(v, getattr(a, k), err_msg=f"{key} {k}")
    exp = pack_reads([dict(reference_start=r["pos"], flag=r["flag"], mapping_quality=60,
                           cigartuples=r["cigartuples"], query_sequence=r["query_sequence"],
                           query_qualities=r["query_qualities"], template_length=0,
                           bc={"AAAC-1": 0, "GGGT-1": 1}.get(r["tags"].get("CB"), -1)) for r in chrm])
    _assert_soa_equal(a, exp)
    assert a.extra["n_with_tag"] == sum(1 for r in chrm if r["tags"])


def test_count_tag_and_bulk(tmp_path):
    w = BamWriter(tmp_path / "x.bam", [("chrM", 16569)])
    reads = [_rd(10, cb="A-1"), _rd(11, cb="B-1"), _rd(12, flag=4, cb="B-1"), _rd(13, flag=1024, cb="C-1"),
             _rd(14, cb=None), _rd(15, cb="A-1"), _rd(16, flag=256, cb="D-1")]
    for r in reads:
        r["tid"] = 0
    for r in reads:
        w.write(r)
    w.close()
    with BamFile(tmp_path / "x.bam") as b:
        # barcode_extraction.py:22-32: unmapped and duplicate reads are not counted
        assert b.count_tag("chrM") == {"A-1": 2, "B-1": 1, "D-1": 1}
        s = b.read_soa("chrM", ["A-1", "Z-1"])
        assert s.bc.tolist() == [0, -1, -1, -1, -1, 0, -1]
        assert s.extra["first_tag_index"] == 0 and s.extra["n_with_tag"] == 6
        s = b.read_soa("chrM", ["bulk"], bulk_cell=0)
        assert s.bc.tolist() == [0] * 7
        s = b.read_soa("chrM", ["A-1", "A-1"])  # duplicates: last index wins (dict semantics)
        assert s.bc.tolist()[0] == 1


def test_long_cigar_cg_tag(tmp_path):
    """> 65535 CIGAR operations are stored in the CG:B,I tag (SAM spec §4.2.2)."""
    import mgatk2_amd.bam as mb

    n_ops = 70000
    cig = [(0, 1) if i % 2 == 0 else (2, 1) for i in range(n_ops - 1)] + [(0, 1)]
    lseq = sum(ln for op, ln in cig if op == 0)
    ref_span = sum(ln for op, ln in cig)
    seq = "A" * lseq
    w = BamWriter(tmp_path / "x.bam", [("chrM", 16569 * 20)])
    # placeholder CIGAR kSmN + CG tag, written by hand
    body_cig = [(4, lseq), (3, ref_span)]
    r = _rd(5, seq=seq, cig=body_cig, tid=0)
    w.write(r)
    w.close(index=False)
    raw = bytearray(gzip.decompress((tmp_path / "x.bam").read_bytes()))
    cg = b"CGBI" + struct.pack("<I", n_ops) + b"".join(struct.pack("<I", (ln << 4) | op) for op, ln in cig)
    # patch the single record: append CG tag and fix block_size
    lt = struct.unpack_from("<i", raw, 4)[0]
    p = 8 + lt + 4
    p += 4 + struct.unpack_from("<i", raw, p)[0] + 4
    bs = struct.unpack_from("<i", raw, p)[0]
    rec = raw[p + 4 : p + 4 + bs] + cg
    out = bytes(raw[:p]) + struct.pack("<i", len(rec)) + bytes(rec)
    data = b"".join(mb._bgzf_block(out[i : i + 0xFF00]) for i in range(0, len(out), 0xFF00)) + mb._BGZF_EOF
    (tmp_path / "y.bam").write_bytes(data)
    assert p + 4 + bs == len(raw)
    with BamFile(tmp_path / "y.bam") as b:
        with pytest.raises(BAMReadError, match="65535"):
            b.read_soa("chrM", ["AAAC-1"])


def test_errors(tmp_path):
    (tmp_path / "bad.bam").write_bytes(b"not a bam file at all")
    with pytest.raises(BAMFormatError):
        BamFile(tmp_path / "bad.bam")
    with pytest.raises(BAMFormatError):
        BamFile(tmp_path / "missing.bam")
    g = Golden("synth_run")
    soa_to_bam(tmp_path / "x.bam", g.soa, g.whitelist, index=False)
    data = (tmp_path / "x.bam").read_bytes()
    (tmp_path / "t.bam").write_bytes(data[: len(data) // 2])  # truncated mid-block
    with BamFile(tmp_path / "t.bam") as b, pytest.raises(BAMReadError):
        b.read_soa("chrM", g.whitelist)
    corrupt = bytearray(data)
    corrupt[2 * len(data) // 3] ^= 0xFF  # CRC / inflate failure past the header block
    (tmp_path / "c.bam").write_bytes(bytes(corrupt))
    with BamFile(tmp_path / "c.bam") as b, pytest.raises(BAMReadError):
        b.read_soa("chrM", g.whitelist)
    # the streaming decode raises on the same files, in every mode (the pipelined one
    # leaves no placement running on the caller's arrays)
    for name in ("t.bam", "c.bam"):
        for pipe in ("1", "0"):
            with pytest.raises(BAMReadError):
                _stream_cols(tmp_path / name, g.whitelist, 997, pipe, pipe)


@pytest.mark.parametrize("case", ["synth_run", "kat_run"])
def test_native_writer_matches_python_writer(case, tmp_path):
    """mgp_bam_write (threaded BGZF, .bai) decodes to the same batch as the Python writer."""
    from mgatk2_amd.bam import write_bam

    g = Golden(case)
    write_bam(tmp_path / "n.bam", g.soa, g.whitelist, n_threads=3)
    soa_to_bam(tmp_path / "p.bam", g.soa, g.whitelist)
    with BamFile(tmp_path / "n.bam") as a, BamFile(tmp_path / "p.bam") as b:
        assert a.has_index
        _assert_soa_equal(a.read_soa("chrM", g.whitelist), b.read_soa("chrM", g.whitelist))
        assert a.count_tag("chrM") == b.count_tag("chrM")
    refs, recs = _independent_decode(tmp_path / "n.bam")
    assert refs == ["chr1", "chrM"] and len(recs) == g.soa.n


def _parse_bai(data: bytes) -> list[dict]:
    """An independent reading of a BAI (SAM spec §5.2): per reference, the smallest
    chunk begin over the real bins and the metadata pseudo-bin 37450's counts."""
    assert data[:4] == b"BAI\1"
    (n_ref,) = struct.unpack_from("<i", data, 4)
    p, out = 8, []
    for _ in range(n_ref):
        (n_bin,) = struct.unpack_from("<i", data, p)
        p += 4
        first, meta = None, None
        for _ in range(n_bin):
            bin_, n_chunk = struct.unpack_from("<Ii", data, p)
            p += 8
            chunks = [struct.unpack_from("<QQ", data, p + 16 * c) for c in range(n_chunk)]
            p += 16 * n_chunk
            if bin_ == 37450:
                meta = chunks
            else:
                b = min(c[0] for c in chunks)
                first = b if first is None else min(first, b)
        (n_intv,) = struct.unpack_from("<i", data, p)
        p += 4 + 8 * n_intv
        out.append(dict(n_bin=n_bin, first=first, meta=meta))
    assert p <= len(data)
    return out


def test_reference_bai_pins_the_index_reader(tmp_path):
    """The reference's only real index (tests/outs/possorted_bam.bam.bai, kept as the
    fixture golden/ref_possorted_bam.bam.bai; its BAM is absent upstream): 194
    references, chrM is reference 22 with 228,149 mapped + 1,619 placed-unmapped
    records. The native reader (mgp_bam.cpp load_index) must give
    those counts, nothing for the references without bins, and refuse the index for
    a header with another reference count."""
    import shutil
    from pathlib import Path

    bai = Path(__file__).parent / "golden" / "ref_possorted_bam.bam.bai"
    data = bai.read_bytes()
    idx = _parse_bai(data)
    assert len(idx) == 194
    assert [i for i, r in enumerate(idx) if r["n_bin"]] == [22]
    assert idx[22]["meta"][1] == (228_149, 1_619)
    assert idx[22]["first"] == idx[22]["meta"][0][0]  # the chrM records start where its extent does
    refs = [(f"chr{i}", 1_000_000) for i in range(194)]
    refs[22] = ("chrM", 16569)
    bam = tmp_path / "hdr.bam"
    BamWriter(bam, refs).close(index=False)
    shutil.copy(bai, str(bam) + ".bai")
    with BamFile(bam) as b:
        assert b.has_index
        assert len(b.references) == 194 and b.references[22] == "chrM"
        assert b.ref_records("chrM") == 228_149 + 1_619
        assert {b.ref_records(f"chr{i}") for i in range(194) if i != 22} == {-1}
    bad = tmp_path / "hdr193.bam"
    BamWriter(bad, refs[:193]).close(index=False)
    shutil.copy(bai, str(bad) + ".bai")
    with pytest.raises(BAMFormatError, match="reference count"):
        BamFile(bad)


@pytest.mark.parametrize("ssse3", [True, False])
def test_decoder_64_byte_records_match_the_definition(ssse3, tmp_path):
    """The decoder's 64-byte records (mgp_pack32_host.h pack64_record_fast: SSSE3
    shuffles and non-temporal stores, or the definition's loop with MGP_NO_SSSE3=1)
    are mgp_pack_record's bytes (include/mgpileup.h, via the Python packer) on random
    reads: every CIGAR operation, 1-50 bases with N and IUPAC codes, qualities up to
    255 (unpackable ones keep the full layout), reads without a barcode tag (records
    ending right after the qualities: the short-tail copy), whole and streamed decode."""
    import os
    import subprocess
    import sys
    from pathlib import Path

    code = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
from test_pack32 import _random_reads
from mgatk2_amd.bam import BamFile, StreamSlot, soa_to_bam
from mgatk2_amd.synth import FLAG_PACKED, pack_reads
rng = np.random.default_rng(77)
reads = _random_reads(rng, 6000)
for i, r in enumerate(reads):
    r["bc"] = -1 if i % 5 == 0 else int(i % 7)
    r["query_qualities"][0] = min(r["query_qualities"][0], 254)  # (0xFF first: BAM's missing QUAL)
want = pack_reads(reads)
soa_to_bam(sys.argv[2], pack_reads(reads, pack=False), [f"BC{i:02d}-1" for i in range(7)])
wl = [f"BC{i:02d}-1" for i in range(7)]
with BamFile(sys.argv[2], n_threads=3) as bf:
    whole = bf.read_soa("chrM", wl, rec_align=64, pack=True, paired=False)
    slot = StreamSlot(1 << 13, 1 << 20)
    parts = []
    with bf.stream("chrM", wl, paired=False) as st:
        while st.next_into(slot):
            s = slot.soa()
            parts.append((s.flag.copy(), s.rec_off.copy(), s.payload.copy()))
def check(flag, off, pay, lo):
    pk = (flag & FLAG_PACKED) != 0
    assert np.array_equal(flag, want.flag[lo:lo + flag.size])
    for i in np.flatnonzero(pk):
        a, b = int(off[i]), int(want.rec_off[lo + i])
        assert np.array_equal(pay[a:a + 64], want.payload[b:b + 64]), (lo + i, reads[lo + i])
    return int(pk.sum())
n = check(whole.flag, whole.rec_off, whole.payload, 0)
lo = m = 0
for f, o, p in parts:
    m += check(f, o, p, lo)
    lo += f.size
assert lo == len(reads) and n == m and 2000 < n < len(reads)
print("ok", n)
'''
    env = dict(os.environ)
    env.pop("MGP_NO_SSSE3", None)
    if not ssse3:
        env["MGP_NO_SSSE3"] = "1"
    root = str(Path(__file__).resolve().parent.parent)
    r = subprocess.run([sys.executable, "-c", code, root, str(tmp_path / "r.bam")], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok")
