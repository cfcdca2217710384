"""End to end: BAM file -> run_pipeline -> output files, against the reference's outputs.

Each golden case holds the reads the reference's ``run_pipeline`` consumed and
the files it wrote (tests/golden/make_golden.py). The reads are written as a
BAM, our ``run_pipeline`` runs on it, and every txt output must match byte for
byte after gunzip.

* CPU tests: host logic only. The engine call is replaced by the oracle, the
  CPU checker. This covers BAM ingest, validation, barcode sources, writers
  and the summary.
* GPU tests (``-m gpu``): the same runs through the HIP engine.
"""

from __future__ import annotations

import gzip
import os

import numpy as np
import pytest

from golden_io import CASES, Golden
from mgatk2_amd.bam import BamWriter, soa_to_bam
from mgatk2_amd.exceptions import InvalidInputError, NoBarcodeTagsError, NoChrMReadsError

TXT_CASES = [c for c in CASES if Golden(c).params["output_format"] == "txt"]


def stream_batches(reader, n_cells, batch_reads=997):
    """The reader's streaming decode (mgp_bam_stream_*) drained into copies of its
    batches (small batches: every golden case takes several, so paired lines and
    placement restart at batch boundaries)."""
    from mgatk2_amd.bam import StreamSlot

    bam, st, _ = reader.open_stream()
    parts = []
    try:
        slot = StreamSlot(batch_reads, batch_reads * 48 + 256 * (n_cells + 1) + (1 << 20))
        while st.next_into(slot):
            v = slot.soa()
            parts.append(type(v)(*[getattr(v, k).copy() for k in ("start", "bc", "tlen", "flag", "mapq", "span",
                                                                  "rec_off", "payload")]))
            parts[-1].extra.update(n_with_tag=st.n_with_tag, first_tag_index=st.first_tag_index)
    finally:
        st.close()
        bam.close()
    return parts


def patch_oracle_engine(monkeypatch, oracle_lib):
    """Stand the oracle in for the engine: the resident path (run_soa) and the
    streamed one (run_stream: the host's streaming decode, then the oracle on the
    concatenated batches)."""
    from mgatk2_amd.processing import processors
    from mgatk2_amd.synth import concat_soa

    def run_soa(self, soa_batches, n_cells):
        soa = soa_batches if not isinstance(soa_batches, list) else concat_soa(soa_batches)
        res, _ = oracle_lib.oracle_run(self.config.engine_config(n_cells), soa)
        self.last_result = res
        return res

    def run_stream(self, reader, n_cells, batch_reads=None, rows_target=True):
        parts = stream_batches(reader, n_cells)
        self.last_timing = {"stream_batches": len(parts)}
        return run_soa(self, parts, n_cells)

    monkeypatch.setattr(processors.CellProcessor, "run_soa", run_soa)
    monkeypatch.setattr(processors.CellProcessor, "run_stream", run_stream)


@pytest.fixture
def oracle_engine(monkeypatch, oracle_lib):
    """Stand the oracle in for the engine (CPU tests of the host logic)."""
    patch_oracle_engine(monkeypatch, oracle_lib)


def _run_case(case, tmp_path, barcode_source="txt"):
    from mgatk2_amd.pipeline import run_pipeline

    g = Golden(case)
    p = g.params
    bam = tmp_path / "possorted_bam.bam"
    soa_to_bam(bam, g.soa, g.whitelist)
    if barcode_source == "txt":
        bfile = tmp_path / "barcodes.tsv"
        bfile.write_text("".join(b + "\n" for b in g.whitelist))
    else:
        bfile = tmp_path / "singlecell.csv"
        rows = ["barcode,is__cell_barcode,passed_filters,excluded_reason"]
        rows += [f"{b},1,{100 + i}," for i, b in enumerate(g.whitelist)]
        rows += ["ZZZZ-1,0,5,lowq"]
        bfile.write_text("\n".join(rows) + "\n")
    out = tmp_path / "out"
    ret = run_pipeline(
        str(bam), str(bfile), str(out), min_baseq=p["min_baseq"], min_mapq=p["min_mapq"],
        min_reads_per_cell=p["min_reads_per_cell"], max_strand_bias=p["max_strand_bias"],
        min_distance_from_end=p["min_distance_from_end"], skip_deduplication=p["skip_deduplication"],
        use_fragment_length_dedup=p["use_fragment_length_dedup"], output_format="txt",
    )
    return g, out, ret


def _check_outputs(g, out, ret):
    od = out / "output"
    for name in ["A", "C", "G", "T", "coverage"]:
        got = gzip.decompress((od / f"output.{name}.txt.gz").read_bytes()).decode()
        assert got == str(g.exp(f"txt_{name}")), f"{g.name}: output.{name}.txt"
    assert (od / "output.depthTable.txt").read_text() == str(g.exp("txt_depthTable"))
    assert (od / "chrM_refAllele.txt").read_text() == str(g.exp("txt_refAllele"))
    assert (out / "qc" / "cell_stats.csv").read_text() == str(g.exp("cell_stats"))
    n_input = int((g.exp("n_reads") > 0).sum())
    n_pass = int(g.exp("passed").sum())
    assert ret["cells_processed"] == n_input and ret["cells_passed_qc"] == n_pass
    assert ret["mean_reads"] == pytest.approx(float(g.exp("n_reads")[g.exp("passed") > 0].sum()) / n_pass)
    summary = (out / "qc" / "summary.txt").read_text().splitlines()
    assert summary[0] == "mgatk2 Run Summary" and summary[1] == "=" * 20
    kv = dict(line.split(": ", 1) for line in summary[2:])
    assert kv["cells_total"] == str(n_input) and kv["cells_passed_qc"] == str(n_pass)
    assert kv["cells_failed_qc"] == str(n_input - n_pass) and kv["reference"] == "chrM"
    assert kv["reference_length"] == "16569"


@pytest.mark.parametrize("case", TXT_CASES)
def test_pipeline_txt_host(case, tmp_path, oracle_engine):
    g, out, ret = _run_case(case, tmp_path)
    _check_outputs(g, out, ret)


def test_pipeline_singlecell_csv(tmp_path, oracle_engine):
    g, out, ret = _run_case("synth_run", tmp_path, barcode_source="csv")
    _check_outputs(g, out, ret)


def test_singlecell_csv_loader(tmp_path):
    from mgatk2_amd.utils import load_singlecell_csv

    f = tmp_path / "singlecell.csv"
    f.write_text("barcode,is__cell_barcode,passed_filters,frac,excluded_reason,tag\n"
                 "AAA-1,1,10,0.5,,x\nCCC-1,0,3,0.1,lowq,y\nGGG-1,1,,,,z\n")
    bcs, meta = load_singlecell_csv(str(f))
    assert bcs == ["AAA-1", "GGG-1"]
    assert meta["passed_filters"] == [10, 0] and meta["frac"] == [0.5, 0]
    assert meta["excluded_reason"] == ["", ""] and meta["tag"] == ["x", "z"]
    assert meta["is__cell_barcode"] == [1, 1]
    f.write_text("barcode,passed_filters\nAAA-1,3\n")
    with pytest.raises(InvalidInputError):
        load_singlecell_csv(str(f))
    f.write_text("barcode,is__cell_barcode\nAAA-1,0\n")
    with pytest.raises(InvalidInputError):
        load_singlecell_csv(str(f))


def test_pipeline_autodetect_barcodes(tmp_path, oracle_engine):
    """barcode_file=None: barcodes come from the BAM's CB counts (barcode_extraction.py)."""
    from mgatk2_amd.file_io.barcode_extraction import extract_barcodes_from_bam
    from mgatk2_amd.pipeline import run_pipeline

    g = Golden("synth_run")
    bam = tmp_path / "x.bam"
    soa_to_bam(bam, g.soa, g.whitelist)
    # expected: str(CB) counts over non-unmapped, non-duplicate records
    counts: dict[str, int] = {}
    for i in range(g.soa.n):
        f = int(g.soa.flag[i]) & 0xFFF
        b = int(g.soa.bc[i])
        tag = g.whitelist[b] if b >= 0 else ("NNNNNNNNNNNNNNNN-9" if i % 2 == 0 else None)
        if tag is None or f & (0x4 | 0x400):
            continue
        counts[tag] = counts.get(tag, 0) + 1
    for mr in (1, 10, 40):
        assert extract_barcodes_from_bam(str(bam), min_reads=mr) == sorted(b for b, n in counts.items() if n >= mr)
    ret = run_pipeline(str(bam), None, str(tmp_path / "o"), min_barcode_reads=10, output_format="txt")
    assert ret["cells_processed"] > 0
    with pytest.raises(InvalidInputError):
        run_pipeline(str(bam), None, str(tmp_path / "o2"), min_barcode_reads=10**9, output_format="txt")


def _tiny_bam(path, refs, tid, n, tag=True):
    w = BamWriter(path, refs)
    for i in range(n):
        w.write(dict(tid=tid, pos=10 + i, flag=0, mapq=60, cigartuples=[(0, 20)], query_sequence="ACGT" * 5,
                     query_qualities=[30] * 20, tags={"CB": "AAAC-1"} if tag else {}))
    w.close()


def test_reader_validation(tmp_path):
    from mgatk2_amd.config import PipelineConfig
    from mgatk2_amd.processing.readers import BAMReader

    _tiny_bam(tmp_path / "a.bam", [("chr1", 1000), ("chr2", 1000)], 0, 5)
    with pytest.raises(NoChrMReadsError):
        BAMReader(str(tmp_path / "a.bam"), PipelineConfig(), {"AAAC-1"})
    # 1001 untagged chrM records -> NoBarcodeTagsError; 1000 are not enough to fail
    _tiny_bam(tmp_path / "b.bam", [("MT", 16569)], 0, 1001, tag=False)
    with pytest.raises(NoBarcodeTagsError) as e:
        BAMReader(str(tmp_path / "b.bam"), PipelineConfig(), {"AAAC-1"})
    assert e.value.total_reads_checked == 1000
    _tiny_bam(tmp_path / "c.bam", [("MT", 16569)], 0, 1000, tag=False)
    cfg = PipelineConfig(mito_chr="chrM")
    BAMReader(str(tmp_path / "c.bam"), cfg, {"AAAC-1"})
    assert cfg.mito_chr == "MT"  # the first present name of chrM/MT/M/chrMT wins (readers.py:43-48)
    # chrM present besides MT: chrM wins even when MT was asked for
    _tiny_bam(tmp_path / "d.bam", [("MT", 16569), ("chrM", 16569)], 1, 3)
    cfg = PipelineConfig(mito_chr="MT")
    BAMReader(str(tmp_path / "d.bam"), cfg, {"AAAC-1"})
    assert cfg.mito_chr == "chrM"


def test_collect_reads_by_barcode_matches_engine_stats(tmp_path, oracle_lib):
    """The dict API (readers.py:63-201) and the engine agree on kept reads and stats."""
    from mgatk2_amd.config import PipelineConfig
    from mgatk2_amd.processing.readers import BAMReader

    for case in ("synth_run", "synth_tenx", "synth_nodedup"):
        g = Golden(case)
        p = g.params
        bam = tmp_path / f"{case}.bam"
        soa_to_bam(bam, g.soa, g.whitelist)
        cfg = PipelineConfig(min_baseq=p["min_baseq"], min_mapq=p["min_mapq"],
                             skip_deduplication=p["skip_deduplication"],
                             use_fragment_length_dedup=p["use_fragment_length_dedup"])
        reads, stats = BAMReader(str(bam), cfg, g.whitelist).collect_reads_by_barcode()
        for k in ("total_reads", "filtered_reads", "n_barcodes"):
            assert stats[k] == g.stats[k], (case, k)
        if not p["skip_deduplication"]:
            assert stats["duplicate_reads_with_length"] == g.stats["duplicate_reads_with_length"]
            assert stats["duplicate_reads_position_only"] == g.stats["duplicate_reads_position_only"]
        assert list(reads) == [g.whitelist[c] for c in g.exp("dict_order")]
        n = np.zeros(len(g.whitelist), np.int64)
        for bc, lst in reads.items():
            n[g.whitelist.index(bc)] = len(lst)
        np.testing.assert_array_equal(n, g.exp("n_reads"))


def test_pipeline_missing_inputs(tmp_path):
    from mgatk2_amd.pipeline import MtDNAPipeline

    with pytest.raises(InvalidInputError):
        MtDNAPipeline(str(tmp_path / "none.bam"), ["A"], tmp_path / "o")
    _tiny_bam(tmp_path / "a.bam", [("chr1", 1000)], 0, 3)
    with pytest.raises(InvalidInputError):
        MtDNAPipeline(str(tmp_path / "a.bam"), ["A"], tmp_path / "o")


@pytest.mark.gpu
@pytest.mark.parametrize("case", TXT_CASES)
def test_pipeline_txt_gpu(case, tmp_path, engine_lib):
    g, out, ret = _run_case(case, tmp_path)
    _check_outputs(g, out, ret)


@pytest.mark.parametrize("case", ["synth_tenx", "kat_tenx"])
def test_cli_tenx_10x_layout(case, tmp_path, oracle_engine, monkeypatch):
    """`tenx -i <project>` with its defaults finds outs/possorted_bam.bam and
    outs/singlecell.csv (cli/utils.py:18-70) and writes the reference's files."""
    from click.testing import CliRunner

    from mgatk2_amd.cli import cli

    g = Golden(case)
    outs = tmp_path / "proj" / "outs"
    outs.mkdir(parents=True)
    soa_to_bam(outs / "possorted_bam.bam", g.soa, g.whitelist)
    rows = ["barcode,is__cell_barcode"] + [f"{b},1" for b in g.whitelist] + ["TTTT-1,0"]
    (outs / "singlecell.csv").write_text("\n".join(rows) + "\n")
    monkeypatch.chdir(tmp_path)
    r = CliRunner().invoke(cli, ["tenx", "-i", str(tmp_path / "proj"), "-o", "res"])
    assert r.exit_code == 0, r.output
    od = tmp_path / "res" / "output"
    for name in ["A", "C", "G", "T", "coverage"]:
        got = gzip.decompress((od / f"output.{name}.txt.gz").read_bytes()).decode()
        assert got == str(g.exp(f"txt_{name}")), name
    assert (od / "output.depthTable.txt").read_text() == str(g.exp("txt_depthTable"))
    assert (tmp_path / "res" / "output.log").exists()
    r = CliRunner().invoke(cli, ["run", "-i", str(outs / "possorted_bam.bam"), "-o", "dry", "--dry-run"])
    assert r.exit_code == 0 and not (tmp_path / "dry" / "output").exists()


H5_CASES = [c for c in CASES if Golden(c).params["output_format"] == "hdf5"]


def _run_case_h5(case, tmp_path):
    from mgatk2_amd.pipeline import run_pipeline

    g = Golden(case)
    p = g.params
    bam = tmp_path / "x.bam"
    soa_to_bam(bam, g.soa, g.whitelist)
    bfile = tmp_path / "barcodes.tsv"
    bfile.write_text("".join(b + "\n" for b in g.whitelist))
    out = tmp_path / "out"
    ret = run_pipeline(
        str(bam), str(bfile), str(out), min_baseq=p["min_baseq"], min_mapq=p["min_mapq"],
        min_reads_per_cell=p["min_reads_per_cell"], max_strand_bias=p["max_strand_bias"],
        skip_deduplication=p["skip_deduplication"], use_fragment_length_dedup=p["use_fragment_length_dedup"],
        output_format="hdf5",
    )
    return g, out, ret


def _check_h5(g, out):
    from mgatk2_amd import h5lite

    with h5lite.File(out / "output" / "counts.h5", "r") as f:
        for k in f.keys():
            np.testing.assert_array_equal(f[k][...], g.exp("h5c_" + k), err_msg=k)
    with h5lite.File(out / "output" / "metadata.h5", "r") as f:
        for k in ["coverage", "mean_depth", "median_depth", "max_depth", "genome_coverage", "total_bases",
                  "reference"]:
            np.testing.assert_array_equal(f[k][...], g.exp("h5m_" + k), err_msg=k)
    assert (out / "qc" / "cell_stats.csv").read_text() == str(g.exp("cell_stats"))


@pytest.mark.parametrize("case", H5_CASES)
def test_pipeline_hdf5_host(case, tmp_path, oracle_engine):
    g, out, _ = _run_case_h5(case, tmp_path)
    _check_h5(g, out)


@pytest.mark.gpu
@pytest.mark.parametrize("case", H5_CASES)
def test_pipeline_hdf5_gpu(case, tmp_path, engine_lib):
    g, out, _ = _run_case_h5(case, tmp_path)
    _check_h5(g, out)


def test_hdf5_report(tmp_path, oracle_engine):
    """hdf5 runs write mgatk2_report.html (analysis/report.py): scRNA layout without
    singlecell.csv, scATAC layout (Tn5 tracks) with it."""
    g, out, _ = _run_case_h5("synth_run_h5", tmp_path)
    page = (out / "mgatk2_report.html").read_text()
    assert "Read start sites" in page and "Number of reads" in page and page.count("data:image/png;base64,") == 4
    from mgatk2_amd.analysis.report import generate_html_report

    import mgatk2_amd.h5lite as h5lite

    with h5lite.File(out / "output" / "metadata.h5", "r") as f:
        n = f["mean_depth"].shape[0]
    # add a barcode_metadata group as the csv path writes it, then the ATAC layout
    meta = out / "output" / "metadata.h5"
    import shutil

    shutil.copy(meta, tmp_path / "m.h5")
    assert generate_html_report(out, "s") is not None  # no barcode_metadata: placeholder for fragments
    page = (out / "mgatk2_report.html").read_text()
    assert "Tn5 transposition frequency" in page and "Tn5 insertion sequence context" in page
    assert n == len(g.whitelist)


def test_insertion_context_matches_loop():
    from mgatk2_amd.analysis.report import insertion_context

    rng = np.random.default_rng(3)
    ref = list(rng.choice(list("ACGTN"), 500, p=[0.24, 0.24, 0.24, 0.24, 0.04]))
    tn5 = rng.integers(0, 5, 500) * (rng.random(500) < 0.5)
    exp = {a + b: 0 for a in "ACGT" for b in "ACGT"}
    for p in range(len(tn5) - 1):
        if tn5[p] > 0 and ref[p] + ref[p + 1] in exp:
            exp[ref[p] + ref[p + 1]] += int(tn5[p])
    assert insertion_context(tn5, ref) == exp


@pytest.mark.gpu
@pytest.mark.parametrize("stream", ["1", "0"])
@pytest.mark.parametrize("case", ["synth_run", "synth_bias", "kat_run"])
def test_pipeline_sharded_gpu(case, stream, tmp_path, engine_lib, monkeypatch):
    """Cells sharded over several engine contexts, run concurrently
    from threads; on a one-GPU box the contexts share device 0. Streamed (each
    decoded batch routed by cell range to the devices' streaming contexts, small
    batches) and resident. Outputs must equal the reference's, like the
    single-context run."""
    from mgatk2_amd.pipeline import run_pipeline

    monkeypatch.setenv("MGP_STREAM", stream)
    monkeypatch.setenv("MGP_STREAM_BATCH", "1500")

    g = Golden(case)
    p = g.params
    bam = tmp_path / "x.bam"
    soa_to_bam(bam, g.soa, g.whitelist)
    bfile = tmp_path / "barcodes.tsv"
    bfile.write_text("".join(b + "\n" for b in g.whitelist))
    out = tmp_path / "out"
    ret = run_pipeline(
        str(bam), str(bfile), str(out), min_baseq=p["min_baseq"], min_mapq=p["min_mapq"],
        min_reads_per_cell=p["min_reads_per_cell"], max_strand_bias=p["max_strand_bias"],
        skip_deduplication=p["skip_deduplication"], use_fragment_length_dedup=p["use_fragment_length_dedup"],
        output_format="txt", devices=[0, 0, 0],
    )
    _check_outputs(g, out, ret)


@pytest.mark.gpu
@pytest.mark.parametrize("stream", ["1", "0"])
def test_pipeline_sharded_hdf5_gpu(stream, tmp_path, engine_lib, monkeypatch):
    """HDF5 output from cells sharded over 3 engine contexts (one GPU): the chunks made
    on the contexts holding their cells (mgp_h5_tiles), the ones across a boundary on the
    host; the files equal the reference's."""
    from mgatk2_amd.pipeline import run_pipeline

    monkeypatch.setenv("MGP_STREAM", stream)
    monkeypatch.setenv("MGP_STREAM_BATCH", "1500")
    g = Golden(H5_CASES[0])
    p = g.params
    bam = tmp_path / "x.bam"
    soa_to_bam(bam, g.soa, g.whitelist)
    bfile = tmp_path / "barcodes.tsv"
    bfile.write_text("".join(b + "\n" for b in g.whitelist))
    out = tmp_path / "out"
    run_pipeline(
        str(bam), str(bfile), str(out), min_baseq=p["min_baseq"], min_mapq=p["min_mapq"],
        min_reads_per_cell=p["min_reads_per_cell"], max_strand_bias=p["max_strand_bias"],
        skip_deduplication=p["skip_deduplication"], use_fragment_length_dedup=p["use_fragment_length_dedup"],
        output_format="hdf5", devices=[0, 0, 0],
    )
    _check_h5(g, out)


@pytest.mark.gpu
def test_pipeline_autodetect_barcodes_gpu(tmp_path, engine_lib, oracle_lib, monkeypatch):
    """barcode_file=None through the HIP engine (pipeline.py:212-223 ->
    barcode_extraction.py:12-46): the native CB count picks the barcodes, the
    engine runs on them; every output equals the oracle's run of the same pipeline."""
    from mgatk2_amd.file_io.barcode_extraction import extract_barcodes_from_bam
    from mgatk2_amd.pipeline import run_pipeline

    g = Golden("synth_run")
    bam = tmp_path / "x.bam"
    soa_to_bam(bam, g.soa, g.whitelist)
    bcs = extract_barcodes_from_bam(str(bam), min_reads=10)
    assert 0 < len(bcs) <= len(g.whitelist) + 1
    ret = run_pipeline(str(bam), None, str(tmp_path / "gpu"), min_barcode_reads=10, output_format="txt")
    assert ret["cells_processed"] > 0

    patch_oracle_engine(monkeypatch, oracle_lib)
    ret2 = run_pipeline(str(bam), None, str(tmp_path / "cpu"), min_barcode_reads=10, output_format="txt")
    assert ret2["cells_processed"] == ret["cells_processed"]
    for name in ("A", "C", "G", "T", "coverage"):
        a = gzip.decompress((tmp_path / "gpu" / "output" / f"output.{name}.txt.gz").read_bytes())
        b = gzip.decompress((tmp_path / "cpu" / "output" / f"output.{name}.txt.gz").read_bytes())
        assert a == b, name
    for rel in ("output/output.depthTable.txt", "output/chrM_refAllele.txt", "qc/cell_stats.csv"):
        assert (tmp_path / "gpu" / rel).read_text() == (tmp_path / "cpu" / rel).read_text(), rel


def test_stream_batches_equal_the_whole_decode(tmp_path, monkeypatch):
    """The streaming decode (mgp_bam_stream_*) gives the whole decode's columns in
    the same order, each record's bytes at its batch's offsets, for every packing /
    placement setting and batch size; the index's record count is the reads'."""
    from mgatk2_amd.bam import BamFile
    from mgatk2_amd.config import PipelineConfig
    from mgatk2_amd.processing.readers import BAMReader
    from mgatk2_amd.synth import concat_soa

    g = Golden("synth_run")
    bam = tmp_path / "x.bam"
    from mgatk2_amd.bam import write_bam

    monkeypatch.setenv("MGP_RECORDS", "64")  # (restored after the test)
    monkeypatch.setenv("MGP_PLACEMENT", "device")
    write_bam(bam, g.soa, g.whitelist)
    with BamFile(bam) as bf:
        assert bf.ref_records("chrM") == g.soa.n
    for q, pack, rec, place in ((20, True, "32", "paired"), (20, True, "64", "paired"), (20, True, "64", "device"),
                                (0, True, "32", "paired"), (20, False, "64", "device")):
        os.environ["MGP_RECORDS"] = rec  # (read at each decode: the producer's record layout and placement)
        os.environ["MGP_PLACEMENT"] = place
        cfg = PipelineConfig(min_baseq=q)
        reader = BAMReader(str(bam), cfg, g.whitelist)
        whole, _ = reader.read_soa(pack=pack)
        for br in (1, 333, 4096, 10**6):
            if not pack:
                break
            parts = stream_batches(reader, len(g.whitelist), br)
            assert sum(p.n for p in parts) == whole.n
            assert all(p.n <= br for p in parts)
            cat = concat_soa(parts)
            for k in ("start", "bc", "tlen", "flag", "mapq", "span"):
                np.testing.assert_array_equal(getattr(cat, k), getattr(whole, k), err_msg=f"q{q} {br} {k}")
            rb = np.where(whole.flag & 0x4000, 32, np.where(whole.flag & 0x2000, 64, 128))
            for i in range(0, whole.n, 7):
                a, b = int(cat.rec_off[i]), int(whole.rec_off[i])
                m = int(rb[i]) if rb[i] < 128 else 112
                assert np.array_equal(cat.payload[a:a + m], whole.payload[b:b + m]), (q, br, i)


@pytest.mark.parametrize("batch", [70_000, 130_000])
def test_stream_pipelined_decode_equals_serial(tmp_path, monkeypatch, batch):
    """The pipelined streaming decode (a chunk's placement on its own thread while the
    pool decodes the next chunk; MGP_BAM_PIPELINE) writes exactly the serial decode's
    batches: columns, offsets and payload bytes, over a BAM of many inflated chunks
    (records carried across chunk ends) and batch cuts inside chunks."""
    from mgatk2_amd.bam import write_bam
    from mgatk2_amd.config import PipelineConfig
    from mgatk2_amd.processing.readers import BAMReader
    from mgatk2_amd.synth import barcode_names, synth_reads

    nc = 300
    soa = synth_reads(17, 300_000, nc)
    names = barcode_names(nc, 17)
    bam = tmp_path / "p.bam"
    write_bam(bam, soa, names)
    out = {}
    for pipe in ("0", "1"):
        monkeypatch.setenv("MGP_BAM_PIPELINE", pipe)
        reader = BAMReader(str(bam), PipelineConfig(min_baseq=20), names)
        out[pipe] = stream_batches(reader, nc, batch)
    assert len(out["0"]) == len(out["1"]) > 1
    for a, b in zip(out["0"], out["1"]):
        for k in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off", "payload"):
            np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
        assert a.extra == b.extra  # the barcode-tag counts of the batch


@pytest.mark.gpu
@pytest.mark.parametrize("rows", ["0", "1"])
@pytest.mark.parametrize("records", ["64", "32"])
@pytest.mark.parametrize("batch", ["997", "50000"])
@pytest.mark.parametrize("case", ["synth_run", "synth_tenx", "synth_bias", "kat_run"])
def test_pipeline_streamed_equals_resident_gpu(case, batch, records, rows, tmp_path, engine_lib, monkeypatch):
    """The production pipeline streamed (batches decoded on a producer thread, each
    pushed as it is ready, windows piled as their reads arrive; the result rows
    fetched after the run, or with MGP_ROWS_TARGET=1 copied back into a pinned target
    as windows complete) writes byte-identical files to the resident run (whole
    decode, one run), and both equal the reference's outputs; with the producer's
    quality-carrying 64-byte records (the default: the kernel filters per base) and
    with its 32-byte records (MGP_RECORDS=32: the producer filters)."""
    if rows == "1" and batch == "50000":
        pytest.skip("(the rows target is covered at the small batches)")
    monkeypatch.setenv("MGP_STREAM_BATCH", batch)
    monkeypatch.setenv("MGP_RECORDS", records)
    monkeypatch.setenv("MGP_ROWS_TARGET", rows)
    from mgatk2_amd import pipeline

    g = Golden(case)
    p = g.params
    bam = tmp_path / "x.bam"
    soa_to_bam(bam, g.soa, g.whitelist)
    bfile = tmp_path / "barcodes.tsv"
    bfile.write_text("".join(b + "\n" for b in g.whitelist))
    from mgatk2_amd.config import PipelineConfig

    outs = {}
    for stream in (True, False):
        cfg = PipelineConfig(min_baseq=p["min_baseq"], min_mapq=p["min_mapq"],
                             min_reads_per_cell=p["min_reads_per_cell"], max_strand_bias=p["max_strand_bias"],
                             skip_deduplication=p["skip_deduplication"],
                             use_fragment_length_dedup=p["use_fragment_length_dedup"])
        out = tmp_path / f"out_{stream}"
        pl = pipeline.MtDNAPipeline(str(bam), g.whitelist, out, config=cfg, output_format="txt", stream=stream)
        ret = pl.run()
        assert pl.timings["streamed"] == stream
        if stream:
            assert pl.timings["stream_batches"] >= (2 if batch == "997" else 1)
        outs[stream] = (out, ret)
    for rel in ("output/output.A.txt.gz", "output/output.C.txt.gz", "output/output.G.txt.gz",
                "output/output.T.txt.gz", "output/output.coverage.txt.gz"):
        a = gzip.decompress((outs[True][0] / rel).read_bytes())
        b = gzip.decompress((outs[False][0] / rel).read_bytes())
        assert a == b, rel
    for rel in ("output/output.depthTable.txt", "output/chrM_refAllele.txt", "qc/cell_stats.csv"):
        assert (outs[True][0] / rel).read_text() == (outs[False][0] / rel).read_text(), rel
    _check_outputs(g, outs[True][0], outs[True][1])


@pytest.mark.parametrize("csv", [False, True])
def test_report_arrays_equal_the_files(tmp_path, oracle_engine, csv):
    """The HTML report reads the writer's in-memory sums (no read-back of the planes):
    they equal what report._load computes from counts.h5 / metadata.h5."""
    from mgatk2_amd.analysis import report
    from mgatk2_amd.config import PipelineConfig
    from mgatk2_amd.file_io import IncrementalHDF5Writer
    from mgatk2_amd.processing.processors import CellProcessor
    from mgatk2_amd.synth import synth_reads

    nc = 30
    soa = synth_reads(5, 60_000, nc)
    cfg = PipelineConfig(min_baseq=20, min_mapq=30)
    names = [f"C{i:03d}-1" for i in range(nc)]
    meta = {"barcode": names[::-1], "total": list(range(100, 100 + nc))} if csv else None
    proc = CellProcessor(cfg, tmp_path)
    res = proc.run_soa(soa, nc)
    w = IncrementalHDF5Writer(tmp_path, cfg, names, barcode_metadata=meta)
    proc.write_results(res, names, w)
    early = w.prepare_report_arrays()  # what the pipeline renders from while finalize runs
    plots = report.render_plots(early, scatac=csv)
    w.finalize(tmp_path / "qc")
    assert w.report_arrays is early
    got = report._from_arrays(w.report_arrays)
    exp = report._load(tmp_path, need_tn5=True, need_meta_group=True)
    np.testing.assert_allclose(got["coverage"], exp["coverage"].mean(axis=1), rtol=1e-12)
    np.testing.assert_array_equal(got["coverage_sum"], exp["coverage"].sum(axis=1, dtype=np.int64))
    for k in ("tn5_fwd", "tn5_rev", "mean_depth", "genome_coverage", "total_bases", "total"):
        np.testing.assert_array_equal(got[k], exp[k], err_msg=k)
    assert got["reference"] == exp["reference"]
    assert report.generate_html_report(tmp_path, "s", arrays=w.report_arrays) is not None
    gen = report.generate_html_report if csv else report.generate_scrna_html_report
    page = gen(tmp_path, "s", arrays=w.report_arrays, plots=plots).read_text()
    assert page.count("data:image/png;base64,") == (5 if csv else 4)


class _OracleEngine:
    """A CPU stand-in for engine.Engine (the oracle behind the same calls) to test
    the host side of the streamed multi-device path: routing, rows-target views,
    first-read mapping and the merge."""

    oracle = None
    pushed: list = []

    def __init__(self, cfg, device=0):
        self.cfg, self.parts, self.rows, self.lo = cfg, [], None, None
        _OracleEngine.pushed.append((cfg, self.parts))

    def set_cell_range(self, lo, hi):  # (mgp_set_cell_range: the barcode indices rebased at push)
        assert hi - lo == self.cfg.n_cells and not self.parts
        self.lo = lo

    def windows(self):
        return -(-self.cfg.mito_len // 1275), 1275

    def set_rows16_target(self, rows):
        self.rows = rows

    def push(self, soa):
        from mgatk2_amd.synth import ReadSoA

        n = soa.n
        bc, tlen = soa.bc, soa.tlen
        if bc.dtype == np.uint16:  # an mgp_batch16: 16-bit barcode index (0xFFFF: none) and |tlen|
            bc = np.where(bc == 0xFFFF, -1, bc.astype(np.int32)).astype(np.int32)
            tlen = tlen.astype(np.int32)
        rec_off = soa.rec_off
        if rec_off is None:  # dense records (the engine places and pairs them)
            stride = soa.payload.shape[0] // max(1, n)
            rec_off = stride * np.arange(n, dtype=np.uint64)
        start = soa.start
        if start is None:  # taken from the records (ABI 4): u16 in 32-byte records, i32 in the others
            at = rec_off.astype(np.int64)
            b = [soa.payload[at + k].astype(np.int64) for k in range(4)]
            s32 = (b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24).astype(np.uint32).view(np.int32)
            start = np.where(soa.flag & 0x4000, b[0] | b[1] << 8, s32).astype(np.int32)
        span = soa.span if soa.span is not None else np.zeros(n, np.uint32)
        part = ReadSoA(*[np.array(a, copy=True) for a in (start, bc, tlen, soa.flag, soa.mapq, span, rec_off,
                                                          soa.payload)])
        if self.lo is not None:
            bc = part.bc
            keep = (bc >= self.lo) & (bc < self.lo + self.cfg.n_cells)
            part.bc[:] = np.where(keep, bc - self.lo, -1)
        self.parts.append(part)

    def copy_wait(self):
        pass

    def run(self):
        from mgatk2_amd.synth import concat_soa

        self.res, _ = self.oracle.oracle_run(self.cfg, concat_soa(self.parts))
        if self.rows is not None:
            self.rows.counts[...] = np.minimum(self.res.counts, 65535)
            self.rows.tn5[...] = np.minimum(self.res.tn5, 65535)
            self.rows.depth[...] = np.minimum(self.res.depth, 65535)
            self.rows.wide[...] = 0

    def sync(self):
        pass

    def fetch(self, dense=True):
        return self.res

    def fetch_rows16(self, lo=0, hi=None, out=None):
        hi = self.cfg.n_cells if hi is None else hi
        out.counts[...] = np.minimum(self.res.counts[lo:hi], 65535)
        out.tn5[...] = np.minimum(self.res.tn5[lo:hi], 65535)
        out.depth[...] = np.minimum(self.res.depth[lo:hi], 65535)
        out.wide[...] = 0
        return out

    def kernel_times(self, last_runs=1):
        return {}

    def txt_gz(self, cells, names, out=None):
        """mgp_txt_gz restated on the host (one gzip member per (file, cell) by the host
        formatter), so the multi-device interleaving of members is tested here."""
        import tempfile

        from mgatk2_amd.bam import txt_write_cells
        from mgatk2_amd.engine import TXT_FILES, TxtMembers

        n = len(names)
        mb, tb = np.zeros((5, n), np.int64), np.zeros((5, n), np.int64)
        per = [[b""] * n for _ in range(5)]
        with tempfile.TemporaryDirectory() as d:
            for k, (c, name) in enumerate(zip(np.asarray(cells).tolist(), names)):
                txt_write_cells(f"{d}/m", self.res.counts, self.res.depth, [c], [name], level=1, append=False)
                for f, fn in enumerate(TXT_FILES):
                    b = open(f"{d}/m.{fn}.txt.gz", "rb").read()
                    per[f][k] = b
                    mb[f, k] = len(b)
                    tb[f, k] = len(gzip.decompress(b)) if b else 0
        blob = np.frombuffer(b"".join(b"".join(x) for x in per) or b"\0", np.uint8)
        return TxtMembers(blob[:int(mb.sum())], mb, tb)

    def h5_tiles(self, cell_of_col, chunks=(1000, 100), sums=None, col_chunks=None):
        """mgp_h5_tiles restated with the host deflate (mgp_h5_plane_tiles); col_chunks:
        only those column chunks (their columns' sums)."""
        from mgatk2_amd.bam import h5_plane_tiles
        from mgatk2_amd.engine import H5_PLANES

        coc = np.asarray(cell_of_col, np.int64)
        if col_chunks is not None:
            coc = coc[col_chunks[0] * chunks[1]:col_chunks[1] * chunks[1]]
        if sums is not None:
            ok = coc[coc >= 0]
            sat = lambda a: np.minimum(a[ok], 65535).astype(np.int64).sum(axis=0)  # noqa: E731
            sums.update(coverage=sat(self.res.depth), tn5_fwd=sat(self.res.tn5[:, :, 0]),
                        tn5_rev=sat(self.res.tn5[:, :, 1]))
        t = (h5_plane_tiles(self.res.counts, coc, list(range(8)), chunks, level=4)
             + h5_plane_tiles(self.res.tn5, coc, [0, 1], chunks, level=4)
             + h5_plane_tiles(self.res.depth, coc, [0], chunks, level=4))
        return dict(zip(H5_PLANES, t))

    def close(self):
        pass


def _stand_in_devices(monkeypatch, oracle_lib):
    from mgatk2_amd.processing import processors

    class HostBuf:
        def __init__(self, nbytes):
            self.buf = np.zeros(int(nbytes) + 64, np.uint8)

        def array(self, shape, dtype, offset=0):
            dt = np.dtype(dtype)
            shape = (int(shape),) if np.ndim(shape) == 0 else tuple(int(x) for x in shape)
            n = int(np.prod(shape)) * dt.itemsize
            return self.buf[offset:offset + n].view(dt).reshape(shape)

    _OracleEngine.oracle = oracle_lib
    _OracleEngine.pushed = []
    monkeypatch.setattr(processors, "Engine", _OracleEngine)
    monkeypatch.setattr(processors, "PinnedBuffer", HostBuf)


@pytest.mark.parametrize("n_dev", [2, 3])
def test_stream_sharded_hdf5_host(n_dev, tmp_path, oracle_lib, monkeypatch):
    """The streamed multi-device path with HDF5 output: each column chunk of the datasets
    deflated by the (stand-in) device holding its cells, the chunks across a device
    boundary on the host (CellProcessor._write_h5); the files equal the reference's."""
    _stand_in_devices(monkeypatch, oracle_lib)
    monkeypatch.setenv("MGP_STREAM_BATCH", "997")
    from mgatk2_amd.pipeline import run_pipeline

    case = H5_CASES[0]
    g = Golden(case)
    p = g.params
    bam = tmp_path / "x.bam"
    soa_to_bam(bam, g.soa, g.whitelist)
    bfile = tmp_path / "barcodes.tsv"
    bfile.write_text("".join(b + "\n" for b in g.whitelist))
    out = tmp_path / "out"
    run_pipeline(
        str(bam), str(bfile), str(out), min_baseq=p["min_baseq"], min_mapq=p["min_mapq"],
        min_reads_per_cell=p["min_reads_per_cell"], max_strand_bias=p["max_strand_bias"],
        skip_deduplication=p["skip_deduplication"], use_fragment_length_dedup=p["use_fragment_length_dedup"],
        output_format="hdf5", devices=list(range(n_dev)),
    )
    _check_h5(g, out)


def test_write_h5_partition(tmp_path, oracle_lib):
    """CellProcessor._write_h5 over 3 stand-in devices holding cell ranges that do not
    fall on 100-column chunk edges, columns shuffled and repeated: every chunk equals
    the host deflate's of the same plane, and the report's column sums are the planes'."""
    import zlib

    from mgatk2_amd.bam import h5_plane_tiles
    from mgatk2_amd.config import PipelineConfig
    from mgatk2_amd.engine import H5_PLANES
    from mgatk2_amd.processing.processors import CellProcessor
    from mgatk2_amd.synth import synth_reads

    nc, L = 260, 16569
    soa = synth_reads(5, 60_000, nc)
    cfg = PipelineConfig()
    res, _ = oracle_lib.oracle_run(cfg.engine_config(nc), soa)
    bounds = [0, 77, 201, nc]
    parts = []
    for lo, hi in zip(bounds[:-1], bounds[1:]):
        e = _OracleEngine.__new__(_OracleEngine)
        e.res = type("R", (), {"counts": res.counts[lo:hi], "tn5": res.tn5[lo:hi], "depth": res.depth[lo:hi]})()
        parts.append((e, lo, hi))
    names = [f"B{i:04d}-1" for i in range(nc)]
    rng = np.random.default_rng(1)
    writer_names = names[:] + [names[int(i)] for i in rng.integers(0, nc, 20)]  # (later duplicates win)
    proc = CellProcessor(cfg, tmp_path)
    proc.enable_device_h5(writer_names)
    proc.config.mito_length = L
    res.passed[:] = 1
    proc._write_h5(res, parts)
    coc, chunks, tiles, sums = res.h5_tiles
    want = (h5_plane_tiles(res.counts, coc, list(range(8)), chunks) + h5_plane_tiles(res.tn5, coc, [0, 1], chunks)
            + h5_plane_tiles(res.depth, coc, [0], chunks))
    for p, w in zip(H5_PLANES, want):
        assert len(tiles[p]) == len(w)
        for i, (a, b) in enumerate(zip(tiles[p], w)):
            assert zlib.decompress(bytes(a)) == zlib.decompress(b), (p, i)
    ok = coc[coc >= 0]
    np.testing.assert_array_equal(sums["coverage"], np.minimum(res.depth[ok], 65535).astype(np.int64).sum(axis=0))
    np.testing.assert_array_equal(sums["tn5_rev"], np.minimum(res.tn5[ok, :, 1], 65535).astype(np.int64).sum(axis=0))


@pytest.mark.parametrize("layout", ["64", "64-paired", "32"])
@pytest.mark.parametrize("rows", ["0", "1"])
@pytest.mark.parametrize("n_dev", [2, 3, 7])
def test_stream_sharded_routing_host(n_dev, rows, layout, tmp_path, oracle_lib, monkeypatch):
    """The streamed multi-device path's host side (CellProcessor._run_stream_sharded:
    every decoded batch routed by the native router (mgp_route_batch) into each
    device's batch of its read-balanced cell range, barcodes rebased, 16-bit columns
    where they fit; the rows fetched per device into its range of one array (or,
    MGP_ROWS_TARGET=1, per-device rows targets as views of one array), first reads
    from the router, tallies and stats merged), with the oracle standing in for each
    device's engine, for the producer's 64-byte records in BAM order, its paired
    placement and its 32-byte records: every output equals the reference's, and no
    device is sent a read of another device's cells."""
    monkeypatch.setenv("MGP_ROWS_TARGET", rows)
    monkeypatch.setenv("MGP_RECORDS", layout[:2])
    monkeypatch.setenv("MGP_PLACEMENT", "paired" if layout.endswith("paired") else "device")
    from mgatk2_amd.engine import PinnedBuffer  # noqa: F401 - (host memory in this stand-in)
    from mgatk2_amd.processing import processors
    from mgatk2_amd.pipeline import run_pipeline

    class HostBuf:
        def __init__(self, nbytes):
            self.buf = np.zeros(int(nbytes) + 64, np.uint8)

        def array(self, shape, dtype, offset=0):
            dt = np.dtype(dtype)
            shape = (int(shape),) if np.ndim(shape) == 0 else tuple(int(x) for x in shape)
            n = int(np.prod(shape)) * dt.itemsize
            return self.buf[offset:offset + n].view(dt).reshape(shape)

    _OracleEngine.oracle = oracle_lib
    _OracleEngine.pushed = []
    monkeypatch.setattr(processors, "Engine", _OracleEngine)
    monkeypatch.setattr(processors, "PinnedBuffer", HostBuf)
    monkeypatch.setenv("MGP_STREAM_BATCH", "997")
    g = Golden("synth_run")
    p = g.params
    bam = tmp_path / "x.bam"
    soa_to_bam(bam, g.soa, g.whitelist)
    bfile = tmp_path / "barcodes.tsv"
    bfile.write_text("".join(b + "\n" for b in g.whitelist))
    out = tmp_path / "out"
    ret = run_pipeline(
        str(bam), str(bfile), str(out), min_baseq=p["min_baseq"], min_mapq=p["min_mapq"],
        min_reads_per_cell=p["min_reads_per_cell"], max_strand_bias=p["max_strand_bias"],
        skip_deduplication=p["skip_deduplication"], use_fragment_length_dedup=p["use_fragment_length_dedup"],
        output_format="txt", devices=list(range(n_dev)),
    )
    _check_outputs(g, out, ret)
    assert len(_OracleEngine.pushed) >= 2
    for cfg, parts in _OracleEngine.pushed:  # every routed read is one of the device's own cells
        for part in parts:
            assert np.all((part.bc >= 0) & (part.bc < cfg.n_cells))
