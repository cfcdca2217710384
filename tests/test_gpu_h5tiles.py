"""GPU: the HDF5 count datasets' chunks deflated on the device (mgp_h5_tiles_*,
mgatk2_amd/csrc/mgp_txtgz.hip), against the planes the reference stores.

IncrementalHDF5Writer (src/file_io/writers.py:60-131) keeps 11 u16 datasets of shape
(mito_len, n_barcodes) with gzip-4 chunks of (1000, 100): A/C/G/T fwd/rev, tn5 cuts fwd/rev
and coverage, values min(v, 65535). Checked here:
* every chunk is one complete zlib stream whose bytes are exactly that chunk of the plane
  (edge chunks padded with 0), for columns mapped to cells in any order, empty columns,
  a column count that is not a multiple of 100, and several calls over column ranges;
* a cell with a drained window (values past 16 bits) stores 65535 there;
* size: on C4-density cells the streams total no more than zlib level 4's (the
  reference's compression_opts) of the same chunks; the ratio is printed;
* the pipeline's HDF5 output through it is the reference's (test_pipeline.py -m gpu runs
  every golden case through the device chunks).
"""

from __future__ import annotations

import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _planes(res) -> list[np.ndarray]:
    """The 11 planes [L][cells] of a result (u16, saturated), in mgp_h5_tiles' order."""
    p = [res.counts[:, :, k] for k in range(8)] + [res.tn5[:, :, 0], res.tn5[:, :, 1], res.depth]
    return [np.minimum(a, 65535).astype(np.uint16).T for a in p]


def _expected_chunks(plane: np.ndarray, coc: np.ndarray, chunks) -> list[bytes]:
    L = plane.shape[0]
    full = np.zeros((L, coc.size), np.uint16)
    ok = coc >= 0
    full[:, ok] = plane[:, coc[ok]]
    crow, ccol = chunks
    out = []
    for r0 in range(0, L, crow):
        for c0 in range(0, coc.size, ccol):
            ch = np.zeros((crow, ccol), np.uint16)
            blk = full[r0:r0 + crow, c0:c0 + ccol]
            ch[:blk.shape[0], :blk.shape[1]] = blk
            out.append(ch.tobytes())
    return out


def _check(tiles, res, coc, chunks) -> tuple[int, int]:
    from mgatk2_amd.engine import H5_PLANES

    dev = z4 = 0
    for name, plane in zip(H5_PLANES, _planes(res)):
        exp = _expected_chunks(plane, coc, chunks)
        got = tiles[name]
        assert len(got) == len(exp), name
        for i, (g, e) in enumerate(zip(got, exp)):
            d = zlib.decompressobj()
            assert d.decompress(g) == e, f"{name} chunk {i}"
            assert d.eof and not d.unused_data
            dev += len(g)
            z4 += len(zlib.compress(e, 4))
    return dev, z4


@pytest.mark.parametrize("chunks,cols_per_call", [((1000, 100), 3200), ((1000, 100), 200), ((700, 30), 90)])
def test_device_h5_chunks_equal_the_planes(engine_lib, chunks, cols_per_call):
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    nc = 130
    soa = synth_reads(4242, 400_000, nc)
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1)
    rng = np.random.default_rng(3)
    # 257 columns: the cells in a shuffled order, some twice, and empty columns
    coc = np.concatenate([rng.permutation(nc), rng.integers(0, nc, 60), np.full(67, -1)])
    coc = coc[rng.permutation(coc.size)].astype(np.int64)
    with engine_lib.Engine(cfg) as eng:
        eng.push(soa)
        eng.run()
        res = eng.fetch()
        sums = {}
        tiles = eng.h5_tiles(coc, chunks, cols_per_call=cols_per_call, sums=sums)
    _check(tiles, res, coc, chunks)
    # the report's per-position sums over the stored columns (duplicates count twice)
    ok = coc >= 0
    for k, a in (("coverage", res.depth), ("tn5_fwd", res.tn5[:, :, 0]), ("tn5_rev", res.tn5[:, :, 1])):
        np.testing.assert_array_equal(sums[k], np.minimum(a[coc[ok]], 65535).astype(np.int64).sum(axis=0), err_msg=k)


def test_device_h5_chunks_saturate_a_wide_window(engine_lib):
    """One cell 180k deep at positions [0, 110): its drained window stores 65535."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    deep = synth_reads(91, 400_000, 1)
    deep.start[:] = np.sort(deep.start % 60).astype(np.int32)
    deep.payload.reshape(-1, 64)[:, 0:4] = deep.start.view(np.uint8).reshape(-1, 4)
    cfg = EngineConfig(n_cells=1, min_baseq=0, min_mapq=0, dedup_mode="none", min_reads=0)
    with engine_lib.Engine(cfg) as eng:
        eng.push(deep)
        eng.run()
        res = eng.fetch()
        sums = {}
        tiles = eng.h5_tiles(np.array([0, -1, 0]), (1000, 3), sums=sums)
    assert res.depth.max() > 65535
    np.testing.assert_array_equal(sums["coverage"], 2 * np.minimum(res.depth[0], 65535).astype(np.int64))
    _check(tiles, res, np.array([0, -1, 0]), (1000, 3))


def test_device_h5_chunks_no_larger_than_zlib4_on_c4_density(engine_lib):
    """C4's density (20k reads per cell, `run` parameters), 200 cells: the device streams
    total no more than zlib level 4's of the same chunks (the reference's gzip-4 filter)."""
    from mgatk2_amd.engine import EngineConfig
    from mgatk2_amd.synth import synth_reads

    nc = 200
    soa = synth_reads(20251019, nc * 20_000, nc)
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1)
    coc = np.arange(nc, dtype=np.int64)
    with engine_lib.Engine(cfg) as eng:
        eng.push(soa)
        eng.run()
        res = eng.fetch()
        tiles = eng.h5_tiles(coc)
    dev, z4 = _check(tiles, res, coc, (1000, 100))
    print(f"device {dev} zlib4 {z4} ratio {dev / z4:.4f}")
    assert dev <= z4, (dev, z4)
