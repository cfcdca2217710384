"""Load the committed golden vectors (tests/golden/*.npz, made by make_golden.py)."""

from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from mgatk2_amd.engine import EngineConfig
from mgatk2_amd.synth import ReadSoA

GOLDEN = Path(__file__).resolve().parent / "golden"
# engine cases (make_golden.py); refout_* hold the reference's committed real-data outputs (make_refout.py)
CASES = sorted(p.stem for p in GOLDEN.glob("*.npz") if not p.stem.startswith("refout_"))


class Golden:
    def __init__(self, name: str):
        z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
        self.name = name
        self.z = z
        self.soa = ReadSoA(
            z["in_start"], z["in_bc"], z["in_tlen"], z["in_flag"], z["in_mapq"], z["in_span"], z["in_rec_off"],
            z["in_payload"],
        )
        self.whitelist = [str(x) for x in z["whitelist"]]
        self.params = json.loads(str(z["params_json"]))
        self.stats = json.loads(str(z["exp_stats_json"]))
        self.qc = json.loads(str(z["exp_qc_json"]))

    def exp(self, key):
        return self.z["exp_" + key]

    def has(self, key):
        return ("exp_" + key) in self.z.files

    def config(self) -> EngineConfig:
        p = self.params
        if p["skip_deduplication"]:
            mode = "none"
        elif p["use_fragment_length_dedup"]:
            mode = "alignment_and_fragment_length"
        else:
            mode = "alignment_start"
        # min_distance_from_end is never passed on by the reference (pipeline.py:239-254):
        # the QualityThresholds default of 5 applies (config.py:15)
        return EngineConfig(
            n_cells=len(self.whitelist), min_baseq=p["min_baseq"], min_mapq=p["min_mapq"], min_distance_from_end=5,
            dedup_mode=mode, max_strand_bias=p["max_strand_bias"], min_reads=p["min_reads_per_cell"],
        )


def ref_alleles_from_tally(tally: np.ndarray) -> list[str]:
    out = []
    for row in tally.tolist():
        m = max(range(4), key=lambda b: row[b])  # first max wins: A<C<G<T
        out.append("ACGT"[m] if row[m] > 0 else "N")
    return out


def check_result(res, g: Golden, order=None):
    """Compare an EngineResult (engine or oracle) with a golden case, bit-exact."""
    np.testing.assert_array_equal(res.counts, g.exp("counts"), err_msg=f"{g.name}: counts")
    np.testing.assert_array_equal(res.tn5, g.exp("tn5"), err_msg=f"{g.name}: tn5")
    np.testing.assert_array_equal(res.depth, g.exp("depth"), err_msg=f"{g.name}: depth")
    np.testing.assert_array_equal(res.passed, g.exp("passed"), err_msg=f"{g.name}: passed")
    np.testing.assert_array_equal(res.n_reads, g.exp("n_reads"), err_msg=f"{g.name}: n_reads")
    st = res.stats
    for k in ("total_reads", "filtered_reads", "n_barcodes"):
        assert st[k] == g.stats[k], (g.name, k, st[k], g.stats[k])
    if not g.params["skip_deduplication"]:
        for k in ("duplicate_reads_with_length", "duplicate_reads_position_only"):
            assert st[k] == g.stats[k], (g.name, k, st[k], g.stats[k])
    assert st["cells_passed"] == int(g.exp("passed").sum())
    # dict order of reads_by_barcode == first-seen order
    np.testing.assert_array_equal(res.cell_order(), g.exp("dict_order"), err_msg=f"{g.name}: order")
    # per-cell QC (processors.py:33-51)
    for bc, q in g.qc.items():
        c = g.whitelist.index(bc)
        n = int(res.n_reads[c])
        assert q["total_reads"] == n
        assert q["total_fragments"] == (n // 2 if res.any_paired[c] else n)
        assert q["mean_depth"] == float(res.depth_sum[c]) / float(res.covered[c])
        assert q["coverage_breadth"] == int(res.covered[c]) / 16569
    # reference alleles (writers.py:340-349 / 493-499)
    if g.has("txt_refAllele"):
        lines = str(g.exp("txt_refAllele")).splitlines()
        refs = ref_alleles_from_tally(res.ref_tally)
        assert lines[0] == "pos\tref"
        assert [ln.split("\t")[1] for ln in lines[1:]] == refs, f"{g.name}: refAllele"
    if g.has("h5m_reference"):
        refs = ref_alleles_from_tally(res.ref_tally)
        assert [x.decode() for x in g.exp("h5m_reference").tolist()] == refs
    if g.has("h5m_median_depth"):
        p = res.passed.astype(bool)
        med = np.where(p, (res.median_lo.astype(np.float64) + res.median_hi) / 2.0, 0).astype(np.float32)
        np.testing.assert_array_equal(med, g.exp("h5m_median_depth"))
        mx = np.minimum(res.depth_max, 65535).astype(np.uint16)
        np.testing.assert_array_equal(np.where(p, mx, 0), g.exp("h5m_max_depth"))
