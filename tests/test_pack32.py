"""32-byte records (MGP_FLAG_PACK32, include/mgpileup.h) on CPU: the packers (C
header, Python mirror, native BAM decoder) agree, keep every bit the pileup reads
under the run's min_baseq, and the quad placement puts four of a cell's records
in a 128-byte line. The GPU side is in tests/test_gpu_pack32.py."""

from __future__ import annotations

import numpy as np
import pytest

from golden_io import CASES, Golden, check_result

CONFIGS = {
    "tenx": dict(min_baseq=0, min_mapq=0, dedup_mode="alignment_start", min_reads=0),
    "run": dict(min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1),
    "bias": dict(min_baseq=10, min_mapq=1, dedup_mode="none", min_reads=40, max_strand_bias=0.8),
}


def _same(a, b, what):
    for k in ("counts", "tn5", "depth", "n_reads", "any_paired", "passed", "covered", "depth_sum", "median_lo",
              "median_hi", "ref_tally", "first_read"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=f"{what}: {k}")
    for k in ("total_reads", "filtered_reads", "duplicate_reads_with_length", "duplicate_reads_position_only"):
        assert a.stats[k] == b.stats[k], (what, k)


@pytest.mark.parametrize("cfgname", sorted(CONFIGS))
def test_host_generator_pack32_same_pileup(cfgname, oracle_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import FLAG_PACK32, PACK32_BYTES, synth_reads

    cfg = EngineConfig(n_cells=40, **CONFIGS[cfgname])
    a = synth_reads(321, 60_000, 40)
    b = synth_reads(321, 60_000, 40, pack32=cfg.min_baseq)
    assert (b.flag & FLAG_PACK32).all() and b.payload.size == PACK32_BYTES * b.n
    assert np.all(b.rec_off == PACK32_BYTES * np.arange(b.n, dtype=np.uint64))
    ra, _ = oracle_lib.oracle_run(cfg, a)
    rb, _ = oracle_lib.oracle_run(cfg, b)
    _same(ra, rb, cfgname)


def test_pack32_unpack_roundtrip():
    """A code counts exactly the bases the reference piles: inside an aligned block
    as the reference walks the CIGAR (an insertion does not advance the query
    position, pileup.py Q1: M10 I3 M27 piles query 0..36, never 37..39), at least
    min_dist from either end, int8 quality >= min_baseq, and A/C/G/T."""
    from mgatk2_amd.synth import FLAG_PACK32, pack_reads, unpack_record

    reads = [
        dict(reference_start=5, cigartuples=[(4, 2), (0, 7)], query_sequence="ACGTNRYAC",
             query_qualities=[0, 1, 62, 30, 4, 200, 6, 40, 41], flag=0x11),
        dict(reference_start=16560, cigartuples=[(0, 10), (1, 3), (0, 27), (5, 9)], query_sequence="ACGT" * 10,
             query_qualities=[19, 20, 21, 130] * 10, flag=0x1),
    ]
    blocks = [range(2, 9), range(0, 37)]  # the query positions inside aligned blocks
    for md in (0, 1, 5):
        soa = pack_reads(reads, pack32=20, pack32_dist=md)
        assert (soa.flag & FLAG_PACK32).all()
        for i, r in enumerate(reads):
            d = unpack_record(soa.payload, int(soa.rec_off[i]), int(soa.flag[i]))
            assert d["reference_start"] == r["reference_start"] and d["cigartuples"] == r["cigartuples"]
            assert d["min_baseq"] == 20 and d["min_dist"] == md
            assert bool(d["flag"] & 0x10) == bool(r["flag"] & 0x10)
            n = len(r["query_sequence"])
            q8 = [q - 256 if q >= 128 else q for q in r["query_qualities"]]
            want = "".join(c if c in "ACGT" and q >= 20 and k in blocks[i] and md <= k < n - md else "N"
                           for k, (c, q) in enumerate(zip(r["query_sequence"], q8)))
            assert d["query_sequence"] == want, (i, md)
    assert unpack_record(pack_reads(reads, pack32=20, pack32_dist=0).payload, 0, FLAG_PACK32)["query_sequence"] \
        == "NNGTNNNAC"
    # limits: start >= 65536 or < 0, > 4 CIGAR ops, long reads, min_baseq outside int8 keep other layouts
    bad = [dict(reference_start=70000, cigartuples=[(0, 6)], query_sequence="A" * 6, query_qualities=[30] * 6),
           dict(reference_start=-3, cigartuples=[(0, 6)], query_sequence="A" * 6, query_qualities=[30] * 6),
           dict(reference_start=1, cigartuples=[(0, 51)], query_sequence="A" * 51, query_qualities=[30] * 51)]
    assert not (pack_reads(bad, pack32=20).flag & FLAG_PACK32).any()
    assert not (pack_reads(reads, pack32=128).flag & FLAG_PACK32).any()
    assert not (pack_reads(reads, pack32=20, pack32_dist=16).flag & FLAG_PACK32).any()


def test_quad_placement_four_records_of_a_cell_per_line(oracle_lib):
    from mgatk2_amd.bam import PLACE_PAIRED, place_records
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import FLAG_PACK32, PACK32_BYTES, ReadSoA, relocate, synth_reads

    soa = synth_reads(77, 80_000, 30, pack32=20)
    roff, total = place_records(soa.bc, soa.flag, np.full(soa.n, PACK32_BYTES, np.uint32), 30, PLACE_PAIRED)
    assert np.all(roff % PACK32_BYTES == 0) and np.unique(roff).size == soa.n
    line = roff // 128
    keep = (soa.bc >= 0) & ((soa.flag & 0x904) == 0)
    # a line holds the records of one cell (or of dropped reads), at most 4
    key = np.where(keep, soa.bc, 30)
    order = np.argsort(line, kind="stable")
    l_s, k_s = line[order], key[order]
    same_line = l_s[1:] == l_s[:-1]
    assert np.all(k_s[1:][same_line] == k_s[:-1][same_line])
    assert np.bincount(line.astype(np.int64)).max() <= 4
    assert total < 1.5 * PACK32_BYTES * soa.n  # nearly every line is full
    # the relocated set (shard gather with the producer placement) piles the same
    cfg = EngineConfig(n_cells=30, **CONFIGS["run"])
    quad = relocate(soa, paired=True, n_cells=30)
    assert (quad.flag & FLAG_PACK32).all()
    _same(oracle_lib.oracle_run(cfg, quad)[0], oracle_lib.oracle_run(cfg, soa)[0], "quad")
    assert isinstance(quad, ReadSoA)


@pytest.mark.parametrize("case", CASES)
def test_bam_decoder_pack32_gives_the_reference_results(case, tmp_path, oracle_lib):
    """The golden reads written as a BAM and decoded natively with 32-byte records
    for the case's min_baseq (reads that do not fit keep the 64-byte or full
    layout): the oracle gives the reference's outputs."""
    from mgatk2_amd.bam import BamFile, soa_to_bam
    from mgatk2_amd.synth import FLAG_PACK32

    g = Golden(case)
    cfg = g.config()
    if not -128 <= cfg.min_baseq <= 127:
        pytest.skip("min_baseq outside the 32-byte layout's range")
    soa_to_bam(tmp_path / "x.bam", g.soa, g.whitelist)
    for paired in (False, True):
        with BamFile(tmp_path / "x.bam") as bam:
            soa = bam.read_soa("chrM", g.whitelist, pack=True, paired=paired, pack32=cfg.min_baseq)
        assert (soa.flag & FLAG_PACK32).any()
        res, _ = oracle_lib.oracle_run(cfg, soa)
        check_result(res, g)


def test_oracle_refuses_pack32_made_for_other_thresholds(oracle_lib):
    """Records made for (min_baseq 20, min_dist 5) under a run at min_dist 4 or
    min_baseq 19: the oracle refuses them, as the engine does (ERR_PACKED)."""
    from oracle.oracle import OracleError

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    soa = synth_reads(13, 5_000, 10, pack32=20, pack32_dist=5)
    oracle_lib.oracle_run(EngineConfig(n_cells=10, min_baseq=20, min_distance_from_end=5), soa)
    for kw in (dict(min_baseq=20, min_distance_from_end=4), dict(min_baseq=19, min_distance_from_end=5)):
        with pytest.raises(OracleError):
            oracle_lib.oracle_run(EngineConfig(n_cells=10, **kw), soa)


def _random_reads(rng, n):
    """pysam-like reads over the corners of the 32-byte layout: every CIGAR operation
    (soft clips, insertions, deletions, skips, =/X, hard clips), 1-50 bases with N and
    IUPAC codes, qualities 0-255 (>= 128 wraps negative as int8, pileup.py Q5)."""
    out = []
    for _ in range(n):
        lseq = int(rng.integers(1, 51))
        ops, q = [], 0
        while q < lseq and len(ops) < 4:
            op = int(rng.choice([0, 0, 0, 1, 2, 3, 4, 7, 8, 5]))
            ln = int(rng.integers(1, 20))
            if op in (0, 1, 4, 7, 8):
                ln = min(ln, lseq - q)
                q += ln
            ops.append((op, ln))
        if q < lseq and len(ops) < 4:
            ops.append((0, lseq - q))
        seq = "".join(rng.choice(list("ACGTACGTACGTNRY"), lseq))
        qual = [int(x) for x in rng.integers(0, 256 if rng.random() < 0.3 else 64, lseq)]
        out.append(dict(reference_start=int(rng.integers(0, 16569)), cigartuples=ops, query_sequence=seq,
                        query_qualities=qual, flag=int(rng.choice([0x1, 0x11, 0x0, 0x10])), bc=0))
    out.sort(key=lambda r: r["reference_start"])
    return out


@pytest.mark.parametrize("bmi2", [True, False])
def test_host_pack32_builder_matches_the_definition(bmi2, tmp_path):
    """The host producers' 32-byte builder (mgp_pack32_host.h, used by the BAM decoder
    and mgp_repack32: SSE2 quality compares, BMI2 pdep or the portable deposit) gives
    the bytes of the layout's definition (include/mgpileup.h mgp_pack32_record, via
    its Python mirror) on random reads at every threshold corner; reads that do not
    fit (more than 2 aligned blocks, CIGAR lengths >= 4096) keep their own layout."""
    import subprocess
    import sys
    from pathlib import Path

    code = r'''
import sys, numpy as np
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[1] + "/tests")
from test_pack32 import _random_reads
from mgatk2_amd.synth import FLAG_PACK32, pack_reads
from mgatk2_amd.bam import repack32
rng = np.random.default_rng(2025)
reads = _random_reads(rng, 4000)
reads.append(dict(reference_start=10, cigartuples=[(0, 5000)], query_sequence="A" * 20, query_qualities=[30] * 20,
                  flag=0, bc=0))
reads.sort(key=lambda r: r["reference_start"])
full = pack_reads(reads, pack=False)
n_fit = 0
for q, d in ((20, 5), (0, 0), (-128, 0), (127, 15), (-5, 7), (63, 1), (-127, 2)):
    want = pack_reads(reads, pack=False, pack32=q, pack32_dist=d)
    o, f, k = repack32(full, q, d, n_threads=2)
    assert np.array_equal(f, want.flag), (q, d)
    fit = (want.flag & FLAG_PACK32) != 0
    assert k == int(fit.sum())
    for i in np.flatnonzero(fit):
        r = int(want.rec_off[i])
        assert np.array_equal(o[32 * i:32 * i + 32], want.payload[r:r + 32]), (q, d, i, reads[i])
    assert not o.reshape(-1, 32)[~fit].any()
    n_fit += int(fit.sum())
assert n_fit > 3000 * 7 and not fit.all()
print("ok", n_fit)
'''
    env = dict(__import__("os").environ)
    if not bmi2:
        env["MGP_NO_BMI2"] = "1"
    root = str(Path(__file__).resolve().parent.parent)
    r = subprocess.run([sys.executable, "-c", code, root], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok")
