"""The C-ABI library loads here (no GPU needed) and exports every symbol the
header declares; host-side packing invariants."""

import re
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent


def header_symbols(name: str = "mgpileup.h"):
    """Functions the header declares for export (static inline helpers excluded)."""
    text = (ROOT / "include" / name).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"static inline[^{]*\{[^}]*\}", "", text)
    return sorted(set(re.findall(r"\b(mgp_[a-z_0-9]+)\s*\(", text)))


def test_host_library_exports_header_symbols():
    from mgatk2_amd.bam import host_library

    lib = host_library()
    syms = header_symbols("mgpileup_host.h")
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(lib, s), f"libmgphost.so does not export {s}"


def test_record_layout_helpers():
    """mgp_seq_offset / mgp_cigar_offset (include/mgpileup.h) == the Python packer's."""
    import subprocess

    from mgatk2_amd.synth import cigar_offset, seq_offset

    src = ROOT / "tests" / "_layout.c"
    src.write_text('#include <stdio.h>\n#include "mgpileup.h"\nint main(void){for(unsigned l=0;l<300;++l)'
                   'printf("%u %u\\n",mgp_seq_offset(l),mgp_cigar_offset(l));return 0;}\n')
    try:
        exe = Path("/tmp") / "mgp_layout_check"
        subprocess.run(["gcc", "-std=c11", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)], check=True)
        out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    finally:
        src.unlink()
    for lseq, line in enumerate(out[:300]):
        so, co = map(int, line.split())
        assert so == int(seq_offset(lseq)) and co == int(cigar_offset(lseq)), lseq
    assert int(seq_offset(50)) == 80 and int(cigar_offset(64)) == 112 and int(cigar_offset(65)) > 112


def test_library_exports_header_symbols():
    from mgatk2_amd.build import build_engine
    from mgatk2_amd import engine

    build_engine()
    lib = engine.load_library()
    syms = header_symbols()
    assert len(syms) >= 19
    for s in syms:
        assert hasattr(lib, s), f"libmgpileup.so does not export {s}"
    assert set(syms) == set(engine.ABI_SYMBOLS)
    assert lib.mgp_abi_version() == engine.ABI_VERSION == 7


def test_no_device_fails_loudly():
    """Without a GPU the engine raises; there is no CPU fallback."""
    import pytest

    from mgatk2_amd import engine

    if engine.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(Exception):
        engine.Engine(engine.EngineConfig(n_cells=1))


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors have the C compiler's sizes and field offsets."""
    import ctypes as C
    import subprocess

    from mgatk2_amd import engine

    structs = {
        "mgp_config": engine.mgp_config, "mgp_batch": engine.mgp_batch, "mgp_batch16": engine.mgp_batch16,
        "mgp_stats": engine.mgp_stats,
        "mgp_result": engine.mgp_result, "mgp_synth_params": engine.mgp_synth_params,
        "mgp_rows16": engine.mgp_rows16, "mgp_rows8": engine.mgp_rows8, "mgp_h5_tiles": engine.mgp_h5_tiles,
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{ROOT}/include/mgpileup.h"', "int main(){"]
    for name, cls in structs.items():
        lines.append(f'printf("%zu\\n", sizeof({name}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("%zu\\n", offsetof({name}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    want = []
    for cls in structs.values():
        want.append(C.sizeof(cls))
        want.extend(getattr(cls, f).offset for f, _ in cls._fields_)
    assert got == want


def test_pack_and_unpack_roundtrip():
    from mgatk2_amd.synth import pack_reads, unpack_record

    reads = [
        dict(reference_start=5, cigartuples=[(4, 2), (0, 7)], query_sequence="ACGTNRY", query_qualities=list(range(7)),
             bc=0, flag=0x11, mapping_quality=7, template_length=-70),
        dict(reference_start=9, cigartuples=[(0, 6)], query_sequence="TTTTGG", query_qualities=[200] * 6, bc=1,
             flag=1, mapping_quality=60, template_length=70),
    ]
    soa = pack_reads(reads, pack=False)
    assert soa.n == 2 and np.all(soa.rec_off % 8 == 0)
    for i, r in enumerate(reads):
        d = unpack_record(soa.payload, int(soa.rec_off[i]), int(soa.flag[i]))
        assert d["reference_start"] == r["reference_start"]
        assert d["cigartuples"] == r["cigartuples"]
        assert d["query_sequence"] == r["query_sequence"]
        assert d["query_qualities"] == r["query_qualities"]
    assert soa.span.tolist() == [7, 6]


def test_packed_layout_roundtrip_and_limits():
    """Packed 64-byte records (include/mgpileup.h): what the pileup reads is
    kept exactly; non-ACGT bases come back as N with quality 0; reads outside
    the layout's limits keep the full layout."""
    from mgatk2_amd.synth import FLAG_PACKED, PACK_BYTES, pack_reads, unpack_record

    ok = [
        dict(reference_start=5, cigartuples=[(4, 2), (0, 7)], query_sequence="ACGTNRY",
             query_qualities=[0, 1, 62, 3, 4, 5, 6], flag=0x11),
        dict(reference_start=16560, cigartuples=[(0, 10), (1, 3), (0, 27), (5, 9)], query_sequence="ACGT" * 10,
             query_qualities=[37] * 40, flag=0x1),
        dict(reference_start=0, cigartuples=[(0, 20), (2, 4000), (0, 30)], query_sequence="T" * 50,
             query_qualities=[2] * 50, flag=0x0),
    ]
    bad = [
        dict(reference_start=1, cigartuples=[(0, 51)], query_sequence="A" * 51, query_qualities=[30] * 51),  # long
        dict(reference_start=1, cigartuples=[(0, 6)], query_sequence="A" * 6, query_qualities=[63] * 6),  # qual 63
        dict(reference_start=1, cigartuples=[(0, 2), (2, 1), (0, 2), (2, 1), (0, 2)], query_sequence="A" * 6,
             query_qualities=[30] * 6),  # 5 operations, 3 aligned blocks
        dict(reference_start=1, cigartuples=[(0, 2), (3, 4096), (0, 4)], query_sequence="A" * 6,
             query_qualities=[30] * 6),  # length >= 4096
        dict(reference_start=1, cigartuples=[(0, 6)], query_sequence="A" * 6, query_qualities=None),
    ]
    soa = pack_reads(ok + bad)
    assert (soa.flag[: len(ok)] & FLAG_PACKED).all() and not (soa.flag[len(ok):] & FLAG_PACKED).any()
    assert np.all(np.diff(soa.rec_off[: len(ok) + 1].astype(np.int64)) == PACK_BYTES)
    for i, r in enumerate(ok):
        d = unpack_record(soa.payload, int(soa.rec_off[i]), int(soa.flag[i]))
        assert d["reference_start"] == r["reference_start"]
        assert d["cigartuples"] == r["cigartuples"]
        want_seq = "".join(c if c in "ACGT" else "N" for c in r["query_sequence"])
        assert d["query_sequence"] == want_seq
        assert d["query_qualities"] == [q if c in "ACGT" else 0 for c, q in zip(r["query_sequence"],
                                                                                  r["query_qualities"])]
        assert bool(d["flag"] & 0x10) == bool(r["flag"] & 0x10)
    full = pack_reads(ok, pack=False)
    assert not (full.flag & FLAG_PACKED).any()


def test_host_synth_is_deterministic_and_sorted():
    from mgatk2_amd.synth import synth_reads

    a = synth_reads(11, 30_000, 9)
    b = synth_reads(11, 30_000, 9, chunk=7_000)
    for k in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off", "payload"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k))
    assert np.all(np.diff(a.start) >= 0)
    assert a.start.min() >= 0 and a.start.max() <= 16569 - 50
    # duplicate structure: ~15% full copies of the previous read's key
    same = (a.start[1:] == a.start[:-1]) & (a.bc[1:] == a.bc[:-1]) & (a.tlen[1:] == a.tlen[:-1])
    assert 0.12 < same.mean() < 0.2


def test_batch_struct_optional_columns():
    """ABI v3.1: a batch without rec_off / span passes NULL pointers (the engine then
    takes dense offsets and the records' spans); every other column is required."""
    import numpy as np

    from mgatk2_amd.engine import batch_struct
    from mgatk2_amd.synth import ReadSoA, synth_reads

    soa = synth_reads(3, 500, 4, pack32=20)
    b = batch_struct(ReadSoA(soa.start, soa.bc, soa.tlen, soa.flag, soa.mapq, None, None, soa.payload))
    assert b.n_reads == soa.n and b.span is None and b.rec_off is None and b.payload_bytes == soa.payload.shape[0]
    full = batch_struct(soa)
    assert full.span == soa.span.ctypes.data and full.rec_off == soa.rec_off.ctypes.data
    assert np.all(soa.span >= 50)
