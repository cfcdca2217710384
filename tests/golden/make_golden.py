"""Generate golden vectors by running the REFERENCE mgatk2 on synthetic inputs.

Runs only in the build container (it reads /root/reference). It imports the
reference's own modules from /root/reference/src with two stubs:

* ``pysam``: an ``AlignmentFile`` whose ``fetch()`` yields pysam-like read
  objects decoded from our engine input (ReadSoA), with pysam's semantics for
  ``query_sequence`` (None when absent), ``query_qualities`` (``array('B')`` or
  None), ``cigartuples`` (None when empty) and the flag properties;
* ``h5py``: a numpy-backed recorder of ``create_dataset`` / slice writes / attrs.

and ``importlib.metadata.version("mgatk2")`` patched (package not installed).
Then it calls the reference ``run_pipeline`` (src/core/pipeline.py:183) exactly
as its CLI does, sequentially, and records:

* reader stats (``BAMReader.collect_reads_by_barcode`` return value),
* every per-cell result of ``process_barcode_worker`` (pileup dicts → arrays),
* the writer outputs: txt files (gunzipped) / captured HDF5 datasets, cell_stats.

Output: tests/golden/<case>.npz (inputs + expected) — data only, no reference
source. Re-run with ``python tests/golden/make_golden.py``.
"""

from __future__ import annotations

import array
import gzip
import importlib
import importlib.metadata
import io
import json
import os
import sys
import tempfile
import types
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
sys.path.insert(0, str(REPO))

from mgatk2_amd.synth import (  # noqa: E402
    FLAG_NOSEQQUAL,
    ReadSoA,
    barcode_names,
    pack_reads,
    synth_reads,
    unpack_record,
)

REF_SRC = Path("/root/reference/src")
L = 16569


# ---------------------------------------------------------------------------
# stubs
# ---------------------------------------------------------------------------
class FakeRead:
    def __init__(self, d, cb):
        self._d = d
        f = d["flag"]
        self.flag = f
        self.is_paired = bool(f & 0x1)
        self.is_proper_pair = bool(f & 0x2)
        self.is_unmapped = bool(f & 0x4)
        self.is_reverse = bool(f & 0x10)
        self.is_secondary = bool(f & 0x100)
        self.is_qcfail = bool(f & 0x200)
        self.is_duplicate = bool(f & 0x400)
        self.is_supplementary = bool(f & 0x800)
        self.reference_start = d["reference_start"]
        self.mapping_quality = d["mapping_quality"]
        self.template_length = d["template_length"]
        self.cigartuples = d["cigartuples"] or None
        seq = d["query_sequence"]
        self.query_sequence = seq if seq else None
        q = d["query_qualities"]
        self.query_qualities = array.array("B", q) if q is not None else None
        self._cb = cb

    def has_tag(self, tag):
        return tag == "CB" and self._cb is not None

    def get_tag(self, tag):
        if not self.has_tag(tag):
            raise KeyError(tag)
        return self._cb


class FakeBam:
    registry: dict = {}

    def __init__(self, path, mode="rb"):
        self.path = str(path)
        self.reads = FakeBam.registry[self.path]
        self.references = ("chr1", "chrM")

    def fetch(self, contig):
        if contig != "chrM":
            return iter(())
        return iter(self.reads)

    def close(self):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


class FakeDataset:
    def __init__(self, shape=None, dtype=None, data=None, fillvalue=0, **kw):
        if data is not None:
            self.data = np.array(data) if dtype is None else np.array(data, dtype=dtype)
        else:
            self.data = np.full(shape, fillvalue, dtype=dtype)
        self.kw = {k: v for k, v in kw.items() if k in ("compression", "compression_opts", "chunks")}
        self.attrs = {}

    def __setitem__(self, key, value):
        self.data[key] = value

    def __getitem__(self, key):
        return self.data[key]

    @property
    def shape(self):
        return self.data.shape


class FakeGroup:
    def __init__(self):
        self.items = {}
        self.attrs = {}

    def create_dataset(self, name, shape=None, dtype=None, data=None, **kw):
        ds = FakeDataset(shape=shape, dtype=dtype, data=data, **kw)
        self.items[name] = ds
        return ds

    def create_group(self, name):
        g = FakeGroup()
        self.items[name] = g
        return g

    def __getitem__(self, k):
        return self.items[k]

    def __contains__(self, k):
        return k in self.items

    def __delitem__(self, k):
        del self.items[k]


class FakeH5File(FakeGroup):
    files: dict = {}

    def __init__(self, path, mode="r", libver=None, **kw):
        super().__init__()
        self.path = str(path)
        FakeH5File.files[Path(path).name] = self

    def flush(self):
        pass

    def close(self):
        pass


def install_stubs():
    pysam = types.ModuleType("pysam")
    pysam.AlignmentFile = FakeBam
    pysam.index = lambda *a, **k: None
    sys.modules["pysam"] = pysam
    h5py = types.ModuleType("h5py")
    h5py.File = FakeH5File
    h5p = types.ModuleType("h5py.h5p")
    h5p.FILE_CREATE = 0

    class _P:
        def set_userblock(self, n):
            pass

    h5p.create = lambda *a: _P()
    h5py.h5p = h5p
    sys.modules["h5py"] = h5py
    sys.modules["h5py.h5p"] = h5p
    real_version = importlib.metadata.version
    importlib.metadata.version = lambda name: "1.0.0" if name == "mgatk2" else real_version(name)
    sys.path.insert(0, str(REF_SRC))


# ---------------------------------------------------------------------------
# inputs
# ---------------------------------------------------------------------------
def soa_to_fake_reads(soa: ReadSoA, whitelist: list[str]) -> list[FakeRead]:
    out = []
    for i in range(soa.n):
        d = unpack_record(soa.payload, int(soa.rec_off[i]))
        f = int(soa.flag[i])
        d["flag"] = f & 0xFFF
        d["mapping_quality"] = int(soa.mapq[i])
        d["template_length"] = int(soa.tlen[i])
        if f & FLAG_NOSEQQUAL:
            # the packer stores qual 0xFF when QUAL is absent; SEQ absent <=> l_seq 0
            if d["query_qualities"] and all(q == 0xFF for q in d["query_qualities"]):
                d["query_qualities"] = None
            if not d["query_sequence"]:
                d["query_sequence"] = None
                d["query_qualities"] = None
        b = int(soa.bc[i])
        if b >= 0:
            cb = whitelist[b]
        else:
            # alternate between an untagged read and a non-whitelisted barcode
            cb = None if (i % 2) else "NNNNNNNNNNNNNNNN-9"
        out.append(FakeRead(d, cb))
    return out


def kat_reads() -> tuple[list[dict], int]:
    """Known-answer reads for the quirks listed in SURVEY.md §8(a) Q1-Q12."""
    R = []
    q30 = lambda n: [30] * n  # noqa: E731

    def add(start, cigar, seq, bc, flag=0x1, mapq=60, qual=None, tlen=200, noqual=False):
        if qual is None and seq is not None and not noqual:
            qual = q30(len(seq))
        R.append(dict(reference_start=start, cigartuples=cigar, query_sequence=seq,
                      query_qualities=None if noqual else qual,
                      bc=bc, flag=flag, mapping_quality=mapq, template_length=tlen))

    acgt = "ACGTACGTACGTACGTACGT"
    # Q1 insertion does not advance the query cursor
    add(100, [(0, 5), (1, 2), (0, 13)], acgt, 0)
    # soft clips (Q3: reverse tn5 includes soft clips), reverse
    add(200, [(4, 5), (0, 45)], "T" * 5 + "ACGT" * 11 + "A", 0, flag=0x11, tlen=-250)
    # deletion / skip / =,X / H,P
    add(300, [(0, 20), (2, 3), (0, 30)], "C" * 50, 1)
    add(400, [(0, 10), (3, 100), (0, 40)], "G" * 50, 1)
    add(600, [(7, 10), (8, 5), (0, 35)], "T" * 50, 1, flag=0x0)
    add(700, [(5, 5), (0, 45), (6, 2)], "A" * 45, 2)
    # N and IUPAC bases skipped; qual >= 128 wraps negative (Q5); low qual
    add(800, [(0, 30)], "ACGTNRYKMACGTNNACGTACGTACGTACG", 2,
        qual=[30] * 10 + [200, 255, 130] + [5] * 5 + [30] * 12)
    # mapq gate (255 passes 30, 0 fails) / tn5 only for passing reads
    add(900, [(0, 40)], "A" * 40, 2, mapq=0)
    add(901, [(0, 40)], "C" * 40, 2, mapq=255)
    # dedup: same (start, strand, |tlen|) -> dup in both modes; other tlen -> dup only
    # in position mode; other strand -> never; QUAL-less dup is never converted
    add(1000, [(0, 30)], "G" * 30, 3, tlen=150)
    add(1000, [(0, 30)], "T" * 30, 3, tlen=-150)
    add(1000, [(0, 30)], "A" * 30, 3, tlen=151)
    add(1000, [(0, 30)], "C" * 30, 3, tlen=150, flag=0x11)
    add(1000, [(0, 30)], "C" * 30, 3, tlen=150, noqual=True)
    # BAM duplicate / QC-fail flags are NOT skipped (Q7)
    add(1100, [(0, 30)], "A" * 30, 3, flag=0x401)
    add(1101, [(0, 30)], "A" * 30, 3, flag=0x201)
    # filtered flags / barcodes
    add(1200, [(0, 30)], "A" * 30, 3, flag=0x4)
    add(1200, [(0, 30)], "A" * 30, 3, flag=0x101)
    add(1200, [(0, 30)], "A" * 30, 3, flag=0x801)
    add(1200, [(0, 30)], "A" * 30, -1)
    # no CIGAR: Tn5 only (dropped by the depth>0 filter, Q8)
    add(1300, [], "ACGTACGTAC", 4)
    add(1310, [], "ACGTACGTAC", 4, flag=0x11)
    # short read: the [5, len-5) window is empty
    add(1400, [(0, 8)], "ACGTACGT", 5)
    # strand bias: 10 fwd / 0 rev A at 2000..; 9 fwd / 1 rev C at 2100..
    for k in range(10):
        add(2000 + k % 3, [(0, 30)], "A" * 30, 5, tlen=100 + k)
    for k in range(10):
        add(2100, [(0, 30)], "C" * 30, 5, tlen=300 + k, flag=0x11 if k == 0 else 0x1)
    # crossing the end of chrM and starting past it (Q4)
    add(16540, [(0, 40)], "ACGT" * 10, 0)
    add(16560, [(0, 40)], "ACGT" * 10, 0, flag=0x11)
    add(16569, [(0, 30)], "A" * 30, 0)
    add(16600, [(0, 30)], "A" * 30, 1)
    R.sort(key=lambda r: r["reference_start"])
    return R, 6


def kat_without_noqual(reads):
    """The KAT set minus its QUAL-less read (with dedup off it would be kept and
    the reference aborts with BAMReadError; tests cover that path separately)."""
    return pack_reads([r for r in reads if r["query_qualities"] is not None or r["query_sequence"] is None])


# ---------------------------------------------------------------------------
# running the reference
# ---------------------------------------------------------------------------
def pileups_to_arrays(results, whitelist, n_cells):
    idx = {b: i for i, b in enumerate(whitelist)}
    counts = np.zeros((n_cells, L, 8), np.uint32)
    tn5 = np.zeros((n_cells, L, 2), np.uint32)
    depth = np.zeros((n_cells, L), np.uint32)
    passed = np.zeros(n_cells, np.uint8)
    qc = {}
    order = []
    for r in results:
        c = idx[r["barcode"]]
        passed[c] = 1
        order.append(c)
        for pos, d in r["pileup"].items():
            for bi, b in enumerate("ACGT"):
                counts[c, pos, 2 * bi] = d[f"{b}_fwd"]
                counts[c, pos, 2 * bi + 1] = d[f"{b}_rev"]
                assert d[b] == d[f"{b}_fwd"] + d[f"{b}_rev"]
            tn5[c, pos, 0] = d["tn5_cuts_fwd"]
            tn5[c, pos, 1] = d["tn5_cuts_rev"]
            depth[c, pos] = d["depth"]
        qc[r["barcode"]] = {k: (float(v) if isinstance(v, (float, np.floating)) else v) for k, v in r["qc"].items()}
    return counts, tn5, depth, passed, qc, np.array(order, np.int32)


def run_reference_case(name, soa, whitelist, params, output_format, workdir):
    import core.pipeline as pipeline
    import processing.processors as processors
    import processing.readers as readers

    bam = Path(workdir) / f"{name}.bam"
    bam.write_bytes(b"")
    Path(str(bam) + ".bai").write_bytes(b"")
    FakeBam.registry[str(bam)] = soa_to_fake_reads(soa, whitelist)
    bcf = Path(workdir) / f"{name}_barcodes.txt"
    bcf.write_text("\n".join(whitelist) + "\n")
    out = Path(workdir) / f"{name}_out"

    captured = {}
    orig_collect = readers.BAMReader.collect_reads_by_barcode

    def collect(self):
        rbb, stats = orig_collect(self)
        captured["stats"] = dict(stats)
        captured["n_reads"] = {b: len(v) for b, v in rbb.items()}
        captured["dict_order"] = list(rbb.keys())
        return rbb, stats

    results = []
    orig_worker = processors.process_barcode_worker

    def worker(args):
        r = orig_worker(args)
        if r:
            results.append(r)
        return r

    readers.BAMReader.collect_reads_by_barcode = collect
    processors.process_barcode_worker = worker
    FakeH5File.files.clear()
    try:
        pipeline.run_pipeline(
            bam_path=str(bam), barcode_file=str(bcf), output_dir=str(out), output_format=output_format,
            sequential=True, n_cores=1, **params,
        )
    finally:
        readers.BAMReader.collect_reads_by_barcode = orig_collect
        processors.process_barcode_worker = orig_worker

    n_cells = len(whitelist)
    counts, tn5, depth, passed, qc, order = pileups_to_arrays(results, whitelist, n_cells)
    n_reads = np.zeros(n_cells, np.uint32)
    for b, k in captured["n_reads"].items():
        n_reads[whitelist.index(b)] = k
    exp = dict(
        counts=counts, tn5=tn5, depth=depth, passed=passed, n_reads=n_reads, order=order,
        dict_order=np.array([whitelist.index(b) for b in captured["dict_order"]], np.int32),
        stats_json=np.array(json.dumps(captured["stats"])),
        qc_json=np.array(json.dumps(qc)),
    )
    od = out / "output"
    if output_format == "txt":
        for fn in ["output.A.txt.gz", "output.C.txt.gz", "output.G.txt.gz", "output.T.txt.gz",
                   "output.coverage.txt.gz"]:
            exp["txt_" + fn.split(".")[1]] = np.array(gzip.decompress((od / fn).read_bytes()).decode())
        exp["txt_depthTable"] = np.array((od / "output.depthTable.txt").read_text())
        exp["txt_refAllele"] = np.array((od / "chrM_refAllele.txt").read_text())
    else:
        cf = FakeH5File.files["counts.h5"]
        mf = FakeH5File.files["metadata.h5"]
        for k, ds in cf.items.items():
            exp["h5c_" + k] = ds.data
        for k, ds in mf.items.items():
            if isinstance(ds, FakeDataset):
                exp["h5m_" + k] = ds.data
        exp["h5c_attrs_json"] = np.array(json.dumps({k: (v if not isinstance(v, np.generic) else v.item())
                                                     for k, v in cf.attrs.items()}))
        exp["h5m_attrs_json"] = np.array(json.dumps({k: (v if not isinstance(v, np.generic) else v.item())
                                                     for k, v in mf.attrs.items()}))
        exp["h5_kw_json"] = np.array(json.dumps({k: ds.kw for k, ds in cf.items.items()}, default=str))
    cs = out / "qc" / "cell_stats.csv"
    exp["cell_stats"] = np.array(cs.read_text() if cs.exists() else "")
    return exp


def save_case(name, soa, whitelist, params, exp):
    cfg = dict(params)
    arrays = dict(
        in_start=soa.start, in_bc=soa.bc, in_tlen=soa.tlen, in_flag=soa.flag, in_mapq=soa.mapq, in_span=soa.span,
        in_rec_off=soa.rec_off, in_payload=soa.payload, whitelist=np.array(whitelist),
        params_json=np.array(json.dumps(cfg)),
    )
    arrays.update({"exp_" + k: v for k, v in exp.items()})
    np.savez_compressed(HERE / f"{name}.npz", **arrays)


TENX = dict(min_baseq=0, min_mapq=0, min_reads_per_cell=0, skip_deduplication=False,
            use_fragment_length_dedup=False, max_strand_bias=1.0, min_distance_from_end=0)
RUN = dict(min_baseq=20, min_mapq=30, min_reads_per_cell=1, skip_deduplication=False,
           use_fragment_length_dedup=True, max_strand_bias=1.0, min_distance_from_end=5)


def main():
    install_stubs()
    cases = []
    kreads, nk = kat_reads()
    kwl = barcode_names(nk, seed=7)
    ksoa = pack_reads(kreads)
    cases.append(("kat_tenx", ksoa, kwl, TENX, "txt"))
    cases.append(("kat_run", ksoa, kwl, RUN, "txt"))
    cases.append(("kat_bias", ksoa, kwl, dict(RUN, max_strand_bias=0.9, min_reads_per_cell=3, min_baseq=0,
                                              min_mapq=0), "txt"))
    cases.append(("kat_nodedup", kat_without_noqual(kreads), kwl, dict(TENX, skip_deduplication=True), "hdf5"))

    ssoa = synth_reads(20251016, 6000, 12)
    swl = barcode_names(12, seed=20251016)
    cases.append(("synth_tenx", ssoa, swl, TENX, "txt"))
    cases.append(("synth_run", ssoa, swl, RUN, "txt"))
    cases.append(("synth_run_h5", ssoa, swl, RUN, "hdf5"))
    cases.append(("synth_bias", ssoa, swl, dict(RUN, max_strand_bias=0.75, min_reads_per_cell=450), "txt"))
    cases.append(("synth_nodedup", ssoa, swl, dict(TENX, skip_deduplication=True), "txt"))

    with tempfile.TemporaryDirectory() as td:
        for name, soa, wl, params, fmt in cases:
            exp = run_reference_case(name, soa, wl, params, fmt, td)
            save_case(name, soa, wl, dict(params, output_format=fmt), exp)
            st = json.loads(str(exp["stats_json"]))
            print(f"{name}: {soa.n} reads, {int(exp['passed'].sum())} cells passed, stats {st}")


if __name__ == "__main__":
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    main()
