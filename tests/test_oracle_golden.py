"""The oracle (CPU restatement) against vectors produced by the reference itself."""

import pytest

from golden_io import CASES, Golden, check_result


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(case, oracle_lib):
    g = Golden(case)
    res, order = oracle_lib.oracle_run(g.config(), g.soa)
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
