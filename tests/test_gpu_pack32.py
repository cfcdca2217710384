"""GPU: 32-byte records (MGP_FLAG_PACK32) through the engine — the device
generator against its host mirror, the all-32-byte fast path (dense and
quad-placed), mixed layouts on the any-layout path, streaming, the native BAM
decoder on the reference goldens, and the min_baseq guard. Every result is
compared bit for bit with the oracle on the same reads in the 64-byte layout,
or with the reference goldens."""

from __future__ import annotations

import numpy as np
import pytest

from golden_io import CASES, Golden, check_result

pytestmark = pytest.mark.gpu

CONFIGS = {
    "tenx": dict(min_baseq=0, min_mapq=0, dedup_mode="alignment_start", min_reads=0),
    "run": dict(min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1),
    "bias": dict(min_baseq=10, min_mapq=1, dedup_mode="none", min_reads=40, max_strand_bias=0.8),
}
KEYS = ("counts", "tn5", "depth", "n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max",
        "median_lo", "median_hi", "ref_tally")


def assert_same(a, b, what=""):
    for k in KEYS:
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=f"{what}: {k}")
    np.testing.assert_array_equal(a.cell_order(), b.cell_order(), err_msg=f"{what}: order")
    for k in ("total_reads", "filtered_reads", "n_barcodes", "duplicate_reads_with_length",
              "duplicate_reads_position_only", "cells_passed"):
        assert a.stats[k] == b.stats[k], (what, k, a.stats[k], b.stats[k])


def run(engine_lib, cfg, soa):
    with engine_lib.Engine(cfg) as eng:
        eng.push(soa)
        return eng.finish()


def test_device_generator_pack32_equals_host_mirror(engine_lib):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    for n, nc, seed, q in [(1, 3, 5, 20), (4097, 11, 6, 0), (70_001, 33, 7, 37), (5000, 9, 8, -5)]:
        host = synth_reads(seed, n, nc, pack32=q)
        with engine_lib.Engine(EngineConfig(n_cells=nc)) as eng:
            eng.synth(seed, n, host.extra["cdf"], host.extra["ref"], pack32=q)
            dev = eng.download_inputs()
        for k in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off", "payload"):
            np.testing.assert_array_equal(getattr(dev, k), getattr(host, k), err_msg=f"{k} n={n}")


@pytest.mark.parametrize("placement", ["dense", "quad"])
@pytest.mark.parametrize("cfgname", sorted(CONFIGS))
def test_engine_pack32_matches_oracle_on_64byte_records(engine_lib, oracle_lib, cfgname, placement):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import relocate, synth_reads

    cfg = EngineConfig(n_cells=300, **CONFIGS[cfgname])
    ref = synth_reads(900, 600_000, 300)
    soa = synth_reads(900, 600_000, 300, pack32=cfg.min_baseq)
    if placement == "quad":
        soa = relocate(soa, paired=True, n_cells=300)
    exp, _ = oracle_lib.oracle_run(cfg, ref)
    assert_same(run(engine_lib, cfg, soa), exp, f"pack32 {placement} {cfgname}")


@pytest.mark.parametrize("cfgname", ["run", "tenx"])
def test_engine_mixed_layouts_any_path(engine_lib, oracle_lib, cfgname):
    """32-byte, 64-byte and full records in one run (waves holding all three)."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.shard import shard_soa
    from mgatk2_amd.synth import FLAG_PACK32, FLAG_PACKED, ReadSoA, concat_soa, synth_reads

    cfg = EngineConfig(n_cells=80, **CONFIGS[cfgname])
    n = 200_000
    parts = [synth_reads(31, n, 80, pack32=cfg.min_baseq), synth_reads(31, n, 80), synth_reads(31, n, 80, pack=False)]
    # interleave: read i takes its record from part i % 3 (same reads, three layouts)
    cat = concat_soa(parts)
    idx = np.arange(n) + n * (np.arange(n) % 3)
    mixed = ReadSoA(cat.start[idx], cat.bc[idx], cat.tlen[idx], cat.flag[idx], cat.mapq[idx], cat.span[idx],
                    cat.rec_off[idx], cat.payload)
    mixed, _ = shard_soa(mixed, 0, 80, paired=True, keep_all=True)
    assert (mixed.flag & FLAG_PACK32).any() and (mixed.flag & FLAG_PACKED).any()
    assert ((mixed.flag & (FLAG_PACK32 | FLAG_PACKED)) == 0).any()
    exp, _ = oracle_lib.oracle_run(cfg, parts[1])
    assert_same(run(engine_lib, cfg, mixed), exp, f"mixed {cfgname}")


def test_engine_pack32_streaming(engine_lib, oracle_lib):
    from dataclasses import replace

    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    cfg = EngineConfig(n_cells=150, **CONFIGS["run"])
    ref = synth_reads(44, 500_000, 150)
    soa = synth_reads(44, 500_000, 150, pack32=cfg.min_baseq)
    exp, _ = oracle_lib.oracle_run(cfg, ref)
    scfg = replace(cfg, stream=True, reserve_reads=soa.n, reserve_payload=int(soa.payload.shape[0]) + 65536)
    with engine_lib.Engine(scfg) as eng:
        for a in range(0, soa.n, 37_000):
            eng.push(soa.slice(a, min(soa.n, a + 37_000)))
        segs, _ = eng.stream_info()
        eng.run()
        got = eng.fetch()
        assert segs > 0 and eng.stream_info()[1]
    assert_same(got, exp, "pack32 streamed")


def test_engine_pack32_min_baseq_guard(engine_lib):
    """Records made for (min_baseq 20, min_dist 5) refused by a run at another pair."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.exceptions import InvalidInputError
    from mgatk2_amd.synth import synth_reads

    soa = synth_reads(12, 50_000, 10, pack32=20, pack32_dist=5)
    with pytest.raises(InvalidInputError):
        run(engine_lib, EngineConfig(n_cells=10, **{**CONFIGS["run"], "min_baseq": 21}), soa)
    with pytest.raises(InvalidInputError):  # and for min_dist 5
        run(engine_lib, EngineConfig(n_cells=10, **{**CONFIGS["run"], "min_distance_from_end": 3}), soa)


@pytest.mark.parametrize("case", CASES)
def test_engine_bam_pack32_matches_reference_goldens(case, engine_lib, tmp_path):
    from mgatk2_amd.bam import BamFile, soa_to_bam

    g = Golden(case)
    cfg = g.config()
    soa_to_bam(tmp_path / "x.bam", g.soa, g.whitelist)
    with BamFile(tmp_path / "x.bam") as bam:
        soa = bam.read_soa("chrM", g.whitelist, pack=True, pack32=cfg.min_baseq)
    check_result(run(engine_lib, cfg, soa), g)


@pytest.mark.parametrize("min_dist", [0, 2, 15])
@pytest.mark.parametrize("min_baseq", [0, 30])
def test_engine_pack32_end_distance_and_quality(engine_lib, oracle_lib, min_dist, min_baseq):
    """32-byte records made for other (min_baseq, min_distance_from_end) pairs than the
    default (the codes carry both): the same counts as the oracle on 64-byte records."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import relocate, synth_reads

    cfg = EngineConfig(n_cells=90, min_baseq=min_baseq, min_mapq=20, dedup_mode="alignment_start", min_reads=1,
                       min_distance_from_end=min_dist)
    ref = synth_reads(600 + min_dist, 300_000, 90)
    soa = relocate(synth_reads(600 + min_dist, 300_000, 90, pack32=min_baseq, pack32_dist=min_dist), paired=True,
                   n_cells=90)
    exp, _ = oracle_lib.oracle_run(cfg, ref)
    assert_same(run(engine_lib, cfg, soa), exp, f"pack32 q{min_baseq} d{min_dist}")
