"""The oracle (CPU restatement) against vectors produced by the reference itself."""

import pytest

from golden_io import CASES, Golden, check_result


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(case, oracle_lib):
    g = Golden(case)
    res, order = oracle_lib.oracle_run(g.config(), g.soa)
    check_result(res, g)


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference_on_packed_records(case, oracle_lib, tmp_path):
    """The same reads in the packed 64-byte record layout (written by the native
    BAM decoder, include/mgpileup.h) give the reference's outputs."""
    from mgatk2_amd.bam import BamFile, soa_to_bam
    from mgatk2_amd.synth import FLAG_PACKED

    g = Golden(case)
    soa_to_bam(tmp_path / "x.bam", g.soa, g.whitelist)
    with BamFile(tmp_path / "x.bam") as bam:
        soa = bam.read_soa("chrM", g.whitelist, pack=True)
    assert (soa.flag & FLAG_PACKED).any()
    res, order = oracle_lib.oracle_run(g.config(), soa)
    check_result(res, g)


def test_oracle_badread_raises(oracle_lib):
    """A kept read without QUAL aborts the reference reader (readers.py:158,167-168)."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent / "golden"))
    from make_golden import kat_reads

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import pack_reads

    reads, nc = kat_reads()
    soa = pack_reads(reads)
    cfg = EngineConfig(n_cells=nc, min_baseq=0, min_mapq=0, dedup_mode="none", min_reads=0)
    with pytest.raises(oracle_lib.OracleError) as ei:
        oracle_lib.oracle_run(cfg, soa)
    assert ei.value.code == -5
    # with dedup on, the QUAL-less read is a duplicate and is never converted
    cfg.dedup_mode = "alignment_start"
    oracle_lib.oracle_run(cfg, soa)


def test_oracle_packed_and_full_synth_agree(oracle_lib):
    """The host packer's packed records (synth.pack_bytes) and the full layout of
    the same synthetic reads give the same oracle outputs, at thresholds around
    the packed quality range."""
    import numpy as np

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import FLAG_PACKED, synth_reads

    pk = synth_reads(5, 40_000, 20, pack=True)
    fu = synth_reads(5, 40_000, 20, pack=False)
    assert (pk.flag & FLAG_PACKED).all() and not (fu.flag & FLAG_PACKED).any()
    assert pk.payload.size * 2 == fu.payload.size
    for q in (-5, 0, 30, 62, 63):
        cfg = EngineConfig(n_cells=20, min_baseq=q, min_mapq=30, dedup_mode="alignment_and_fragment_length")
        a, _ = oracle_lib.oracle_run(cfg, pk)
        b, _ = oracle_lib.oracle_run(cfg, fu)
        for k in ("counts", "tn5", "n_reads", "passed", "covered", "depth_sum", "ref_tally"):
            np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=f"{k} q={q}")
