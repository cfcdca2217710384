"""Writers against the reference's own outputs on the same inputs (tests/golden).

The arrays fed to the writers come from the oracle (the checker), so this
isolates the formatting/layout: txt files must match the reference byte for
byte after gunzip; HDF5 datasets (captured through the same numpy-backed h5py
stand-in the golden generator used) must match exactly.
"""

from __future__ import annotations

import gzip
import json
import sys
from pathlib import Path

import numpy as np
import pytest

from golden_io import CASES, Golden

sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))

TXT_CASES = [c for c in CASES if Golden(c).params["output_format"] == "txt"]
H5_CASES = [c for c in CASES if Golden(c).params["output_format"] == "hdf5"]


def _written(res):
    order = res.cell_order()
    return order[res.passed[order].astype(bool)]


def _config(g):
    from mgatk2_amd.config import PipelineConfig

    p = g.params
    return PipelineConfig(min_baseq=p["min_baseq"], min_mapq=p["min_mapq"], max_strand_bias=p["max_strand_bias"],
                          skip_deduplication=p["skip_deduplication"],
                          use_fragment_length_dedup=p["use_fragment_length_dedup"],
                          min_reads_per_cell=p["min_reads_per_cell"])


@pytest.mark.parametrize("case", TXT_CASES)
def test_txt_writer_matches_reference(case, oracle_lib, tmp_path):
    from mgatk2_amd.file_io import IncrementalTextWriter

    g = Golden(case)
    res, _ = oracle_lib.oracle_run(g.config(), g.soa)
    w = IncrementalTextWriter(tmp_path, _config(g), g.whitelist)
    w.write_cells(res, _written(res), tally=res.ref_tally)
    w.finalize(tmp_path / "qc")
    od = tmp_path / "output"
    for name in ["A", "C", "G", "T", "coverage"]:
        got = gzip.decompress((od / f"output.{name}.txt.gz").read_bytes()).decode()
        assert got == str(g.exp(f"txt_{name}")), f"{case}: output.{name}.txt"
    assert (od / "output.depthTable.txt").read_text() == str(g.exp("txt_depthTable"))
    assert (od / "chrM_refAllele.txt").read_text() == str(g.exp("txt_refAllele"))
    assert (tmp_path / "qc" / "cell_stats.csv").read_text() == str(g.exp("cell_stats"))


@pytest.mark.parametrize("case", TXT_CASES[:2])
def test_txt_writer_dict_api_matches_reference(case, oracle_lib, tmp_path):
    """The reference per-cell API (write_cell(result_dict)) gives the same files."""
    from mgatk2_amd.file_io import IncrementalTextWriter
    from mgatk2_amd.processing.pileup import result_dict

    g = Golden(case)
    res, _ = oracle_lib.oracle_run(g.config(), g.soa)
    w = IncrementalTextWriter(tmp_path, _config(g), g.whitelist)
    for c in _written(res):
        w.write_cell(result_dict(res, int(c), g.whitelist[int(c)], 16569))
    w.finalize(tmp_path / "qc")
    od = tmp_path / "output"
    for name in ["A", "coverage"]:
        got = gzip.decompress((od / f"output.{name}.txt.gz").read_bytes()).decode()
        assert got == str(g.exp(f"txt_{name}"))
    assert (tmp_path / "qc" / "cell_stats.csv").read_text() == str(g.exp("cell_stats"))


@pytest.mark.parametrize("case", H5_CASES)
def test_hdf5_writer_matches_reference(case, oracle_lib, tmp_path):
    import make_golden as mg

    from mgatk2_amd.file_io import IncrementalHDF5Writer

    g = Golden(case)
    res, _ = oracle_lib.oracle_run(g.config(), g.soa)
    h5 = type("h5", (), {"File": mg.FakeH5File})
    mg.FakeH5File.files.clear()
    w = IncrementalHDF5Writer(tmp_path, _config(g), g.whitelist, h5=h5)
    w.write_cells(res, _written(res), tally=res.ref_tally)
    w.finalize(tmp_path / "qc")
    cf, mf = mg.FakeH5File.files["counts.h5"], mg.FakeH5File.files["metadata.h5"]
    for k, ds in cf.items.items():
        exp = g.exp("h5c_" + k)
        np.testing.assert_array_equal(ds.data, exp, err_msg=f"counts.h5/{k}")
        assert ds.data.dtype == exp.dtype, k
    for k, ds in mf.items.items():
        if isinstance(ds, mg.FakeDataset):
            exp = g.exp("h5m_" + k)
            np.testing.assert_array_equal(ds.data, exp, err_msg=f"metadata.h5/{k}")
            assert ds.data.dtype == exp.dtype, k
    exp_keys = {f[len("exp_h5c_"):] for f in g.z.files if f.startswith("exp_h5c_") and not f.endswith("_json")}
    assert set(cf.items) == exp_keys
    assert json.loads(str(g.exp("h5c_attrs_json"))) == {k: (v.item() if hasattr(v, "item") else v)
                                                         for k, v in cf.attrs.items()}
    assert json.loads(str(g.exp("h5m_attrs_json"))) == {k: (v.item() if hasattr(v, "item") else v)
                                                         for k, v in mf.attrs.items()}
    kw = json.loads(str(g.exp("h5_kw_json")))
    for k, ds in cf.items.items():
        assert {a: (list(b) if isinstance(b, tuple) else b) for a, b in ds.kw.items()} == kw[k], k
    assert (tmp_path / "qc" / "cell_stats.csv").read_text() == str(g.exp("cell_stats"))


@pytest.mark.parametrize("case", H5_CASES)
def test_hdf5_files_match_reference(case, oracle_lib, tmp_path):
    """Real counts.h5 / metadata.h5 through libhdf5 (mgatk2_amd.h5lite; chunks
    deflated in parallel and written with H5Dwrite_chunk), read back through
    libhdf5's own filter pipeline, equal the reference's datasets and attrs."""
    from mgatk2_amd import h5lite
    from mgatk2_amd.file_io import IncrementalHDF5Writer

    if not h5lite.available():
        pytest.skip("libhdf5 not present")
    g = Golden(case)
    res, _ = oracle_lib.oracle_run(g.config(), g.soa)
    w = IncrementalHDF5Writer(tmp_path, _config(g), g.whitelist, h5=h5lite.module())
    w.write_cells(res, _written(res), tally=res.ref_tally)
    w.finalize(tmp_path / "qc")
    kw = json.loads(str(g.exp("h5_kw_json")))
    with h5lite.File(tmp_path / "output" / "counts.h5", "r") as f:
        exp_keys = {k[len("exp_h5c_"):] for k in g.z.files if k.startswith("exp_h5c_") and not k.endswith("_json")}
        assert set(f.keys()) == exp_keys
        for k in exp_keys:
            got, exp = f[k][...], g.exp("h5c_" + k)
            assert got.dtype == exp.dtype, k
            np.testing.assert_array_equal(got, exp, err_msg=k)
            if kw[k]:
                assert f[k].chunks == tuple(kw[k]["chunks"]) and f[k].compression == "gzip"
        attrs = {k: (v.item() if hasattr(v, "item") else v) for k, v in f.attrs.items()}
        assert attrs == json.loads(str(g.exp("h5c_attrs_json")))
    with h5lite.File(tmp_path / "output" / "metadata.h5", "r") as f:
        for k in ["coverage", "mean_depth", "median_depth", "max_depth", "genome_coverage", "total_bases",
                  "reference"]:
            got, exp = f[k][...], g.exp("h5m_" + k)
            assert got.dtype == exp.dtype, k
            np.testing.assert_array_equal(got, exp, err_msg=k)
        attrs = {k: (v.item() if hasattr(v, "item") else v) for k, v in f.attrs.items()}
        assert attrs == json.loads(str(g.exp("h5m_attrs_json")))


def test_hdf5_barcode_metadata_group(tmp_path, oracle_lib):
    """singlecell.csv columns land in metadata.h5/barcode_metadata, in whitelist order (writers.py:358-388)."""
    from mgatk2_amd import h5lite
    from mgatk2_amd.file_io import IncrementalHDF5Writer

    if not h5lite.available():
        pytest.skip("libhdf5 not present")
    g = Golden("synth_run_h5")
    res, _ = oracle_lib.oracle_run(g.config(), g.soa)
    wl = g.whitelist
    meta = {"barcode": list(reversed(wl)), "passed_filters": list(range(len(wl))),
            "frac": [0.5] * len(wl), "excluded_reason": [""] * len(wl)}
    w = IncrementalHDF5Writer(tmp_path, _config(g), wl, barcode_metadata=meta, h5=h5lite.module())
    w.write_cells(res, _written(res), tally=res.ref_tally)
    w.finalize(tmp_path / "qc")
    with h5lite.File(tmp_path / "output" / "metadata.h5", "r") as f:
        grp = f["barcode_metadata"]
        assert set(grp.keys()) == set(meta)
        assert [b.decode() for b in grp["barcode"][...]] == wl
        np.testing.assert_array_equal(grp["passed_filters"][...], list(reversed(range(len(wl)))))
        assert grp["frac"][...].dtype == np.float64


def test_hdf5_write_retries_eagain_with_backoff():
    """HDF5 writes and flushes retry EAGAIN (network filesystems) the reference's
    way (writers.py:23-26,266-323): up to 5 attempts, sleeps 0.1, 0.2, 0.4, 0.8 s;
    another errno, or the fifth EAGAIN, raises at once."""
    import ctypes as C
    import errno

    from mgatk2_amd import h5lite

    def failing(fails: int, code: int):
        n = [0]

        def call():
            n[0] += 1
            if n[0] <= fails:
                C.set_errno(code)
                return -1
            return 7

        return call, n

    slept = []
    call, n = failing(3, errno.EAGAIN)
    assert h5lite._ck_retry(call, "w", sleep=slept.append) == 7
    assert n[0] == 4 and slept == [0.1, 0.2, 0.4]
    slept.clear()
    call, n = failing(99, errno.EAGAIN)
    with pytest.raises(OSError) as ei:
        h5lite._ck_retry(call, "w", sleep=slept.append)
    assert ei.value.errno == errno.EAGAIN and n[0] == 5 and slept == [0.1, 0.2, 0.4, 0.8]
    slept.clear()
    call, n = failing(1, errno.ENOSPC)
    with pytest.raises(OSError) as ei:
        h5lite._ck_retry(call, "w", sleep=slept.append)
    assert ei.value.errno == errno.ENOSPC and n[0] == 1 and slept == []
