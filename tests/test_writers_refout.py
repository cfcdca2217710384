"""The txt writers against the reference's own committed outputs on real 10x data
(tests/run_txt_output and tests/tenx_output of the reference: 134 cells, the
`run` and `tenx` parameter sets; fixtures made by tests/golden/make_refout.py).

The input BAM of those runs is absent, so the engine cannot be run on them; but
the per-(position, cell) forward/reverse counts of output.{A,C,G,T}.txt.gz plus
qc/cell_stats.csv are exactly what IncrementalTextWriter consumes
(writers.py:430-510). Writing them back must reproduce every output file: the
coverage lines (coverage = the sum of the 8 counts, SURVEY.md §4 invariant 1),
the count lines, output.depthTable.txt (mean depth over covered positions,
`.2f`, sorted by barcode), chrM_refAllele.txt (first max over A<C<G<T of the
counts summed over cells, N when all zero) and qc/cell_stats.csv
(str(np.mean), covered/16569, n//2 fragments for paired cells). Line order is
compared sorted: the reference writes cells in nondeterministic order."""

from __future__ import annotations

import gzip
import hashlib
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"
L = 16569


def _load(name):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    return {k: z[k] for k in z.files}


def _result(z):
    """An EngineResult holding the reference's per-cell arrays."""
    from mgatk2_amd.engine import EngineResult

    counts = z["counts"].astype(np.uint32)
    n = counts.shape[0]
    res = EngineResult.alloc(n, L, dense=True)
    res.counts[:] = counts
    res.depth[:] = counts.sum(axis=2)
    res.n_reads[:] = z["n_reads"]
    res.any_paired[:] = (z["total_fragments"] != z["n_reads"]).astype(np.uint8)
    res.passed[:] = 1
    res.covered[:] = (res.depth > 0).sum(axis=1)
    res.depth_sum[:] = res.depth.sum(axis=1, dtype=np.uint64)
    res.depth_max[:] = res.depth.max(axis=1)
    return res


def _sorted_sha(path: Path) -> tuple[str, int]:
    with gzip.open(path, "rt") as f:
        lines = f.readlines()
    return hashlib.sha256("".join(sorted(lines)).encode()).hexdigest(), len(lines)


@pytest.mark.parametrize("rows", ["u32", "u16"])
@pytest.mark.parametrize("name", ["refout_run_txt", "refout_tenx"])
def test_txt_writer_reproduces_reference_outputs(name, rows, tmp_path):
    from mgatk2_amd.config import PipelineConfig
    from mgatk2_amd.file_io.writers import IncrementalTextWriter

    z = _load(name)
    res = _result(z)
    if rows == "u16":  # the engine's exact 16-bit rows (Engine.fetch_compact), formatted as they are
        res.counts, res.tn5, res.depth = (a.astype(np.uint16) for a in (res.counts, res.tn5, res.depth))
    barcodes = [str(b) for b in z["barcodes"]]
    cfg = PipelineConfig(bam_file=Path("x.bam"), output_dir=tmp_path, barcode_file=None)
    w = IncrementalTextWriter(tmp_path, cfg, barcodes, gzip_level=1, n_threads=2)
    # write in a shuffled order (the reference's order is nondeterministic) and in two calls
    order = np.random.default_rng(5).permutation(len(barcodes))
    w.write_cells(res, order[:50], barcodes=barcodes)
    w.write_cells(res, order[50:], barcodes=barcodes)
    w.finalize(tmp_path / "qc")
    out = tmp_path / "output"
    want = {str(k): (str(v), int(n)) for k, v, n in zip(z["sha_names"], z["sha_values"], z["sha_lines"])}
    for key in ("A", "C", "G", "T", "coverage"):
        assert _sorted_sha(out / f"output.{key}.txt.gz") == want[key], key
    assert (out / "output.depthTable.txt").read_text() == str(z["depth_table"])
    assert (out / "chrM_refAllele.txt").read_text() == str(z["ref_allele"])
    lines = (tmp_path / "qc" / "cell_stats.csv").read_text().splitlines(keepends=True)
    assert lines[0] == str(z["cell_stats_header"])
    assert "".join(sorted(lines[1:])) == str(z["cell_stats_sorted"])


@pytest.mark.parametrize("name", ["refout_run_txt", "refout_tenx"])
def test_reference_outputs_satisfy_the_invariants(name):
    """SURVEY.md §4's invariants on the reference's real-data outputs, restated
    from the fixture arrays: ref alleles from the summed counts, per-cell means."""
    from mgatk2_amd.file_io.writers import ref_alleles

    z = _load(name)
    counts = z["counts"].astype(np.int64)
    tally = (counts[:, :, 0::2] + counts[:, :, 1::2]).sum(axis=0)
    refs = ref_alleles(tally)
    lines = str(z["ref_allele"]).splitlines()
    assert lines[0] == "pos\tref" and [ln.split("\t")[1] for ln in lines[1:]] == refs
    depth = counts.sum(axis=2)
    table = dict(ln.split("\t") for ln in str(z["depth_table"]).splitlines())
    for c, bc in enumerate(z["barcodes"].tolist()):
        d = depth[c][depth[c] > 0]
        assert table[bc] == f"{d.mean():.2f}"
