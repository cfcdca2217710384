"""Output-stage timing without the engine (SURVEY.md §8(f) writers at scale).

Builds engine-shaped result arrays for BASELINE config C3 (5k cells x chrM; 50M
reads of 50 bp give a depth of ~30 per position per cell) on the host, then times
the txt and HDF5 writers and the HTML report the pipeline runs after the engine,
each broken into its parts. Host-only: runs here and on the GPU box alike.

    python scripts/writers_bench.py [--cells 5000] [--depth 30] [--formats txt,hdf5] [--threads 16]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path
from types import SimpleNamespace

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def fake_result(n_cells: int, L: int, depth: float, seed: int, dtype=np.uint16):
    """Cell-major arrays of the engine's result (Rows16 fields the writers read)."""
    rng = np.random.default_rng(seed)
    scale = rng.gamma(4.0, depth / 4.0, n_cells).astype(np.float32)
    dep = np.empty((n_cells, L), dtype)
    counts = np.zeros((n_cells, L, 8), dtype)
    tn5 = np.zeros((n_cells, L, 2), dtype)
    ref = rng.integers(0, 4, L)
    for c0 in range(0, n_cells, 256):
        c1 = min(n_cells, c0 + 256)
        lam = scale[c0:c1, None]
        d = rng.poisson(np.broadcast_to(lam, (c1 - c0, L))).astype(np.int64)
        dep[c0:c1] = d
        # ~1% of a position's depth on one other base; strands split at random
        alt = np.minimum(d, rng.poisson(np.broadcast_to(lam * 0.01, d.shape)))
        altb = (ref[None, :] + 1 + rng.integers(0, 3, d.shape)) % 4
        split = rng.random(d.shape, np.float32)
        for b in range(4):
            n_b = np.where(ref[None, :] == b, d - alt, 0) + np.where(altb == b, alt, 0)
            f_b = (n_b * split).astype(np.int64)
            counts[c0:c1, :, 2 * b] = f_b
            counts[c0:c1, :, 2 * b + 1] = n_b - f_b
        tn5[c0:c1] = rng.poisson(np.broadcast_to(lam / 25.0, (c1 - c0, L))[..., None].repeat(2, -1))
    covered = (dep > 0).sum(1).astype(np.int64)
    dsum = dep.sum(1, dtype=np.int64)
    srt = np.sort(dep, axis=1)
    return SimpleNamespace(
        counts=counts, depth=dep, tn5=tn5, covered=covered, depth_sum=dsum,
        depth_max=dep.max(1).astype(np.int64), median_lo=srt[:, (L - 1) // 2].astype(np.int64),
        median_hi=srt[:, L // 2].astype(np.int64), n_reads=(dsum // 50).astype(np.int64),
        any_paired=np.ones(n_cells, bool),
    )


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", type=int, default=5000)
    ap.add_argument("--depth", type=float, default=30.0)
    ap.add_argument("--formats", default="txt,hdf5")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default="/tmp/mgp_writers")
    args = ap.parse_args()

    from mgatk2_amd.config import PipelineConfig
    from mgatk2_amd.file_io.writers import IncrementalHDF5Writer, IncrementalTextWriter
    from mgatk2_amd.synth import barcode_names

    L = 16569
    t0 = time.time()
    res = fake_result(args.cells, L, args.depth, 7)
    names = barcode_names(args.cells, 7)
    tally = np.zeros((L, 4), np.int64)
    for c0 in range(0, args.cells, 512):
        cnt = res.counts[c0:c0 + 512].astype(np.int64)
        tally += (cnt[:, :, 0::2] + cnt[:, :, 1::2]).sum(0)
    cfg = PipelineConfig(mito_length=L)
    print(f"[writers] arrays for {args.cells} cells in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    out = {"cells": args.cells, "depth": args.depth}
    cells = np.arange(args.cells, dtype=np.int64)
    for fmt in args.formats.split(","):
        d = Path(args.out) / fmt
        d.mkdir(parents=True, exist_ok=True)
        t = {}
        t0 = time.time()
        if fmt == "txt":
            w = IncrementalTextWriter(d, cfg, names, n_threads=args.threads)
        else:
            w = IncrementalHDF5Writer(d, cfg, names)
        t1 = time.time()
        w.write_cells(res, cells, tally=tally)
        t2 = time.time()
        w.finalize(d / "qc")
        t3 = time.time()
        t.update(init=t1 - t0, write_cells=t2 - t1, finalize=t3 - t2)
        if fmt == "hdf5":
            from mgatk2_amd.analysis.report import generate_scrna_html_report

            t4 = time.time()
            try:
                generate_scrna_html_report(d, "bench", arrays=w.report_arrays)
                t["report"] = time.time() - t4
            except ImportError as e:
                t["report"] = f"skipped: {e}"
        sizes = {p.name: p.stat().st_size for p in (d / "output").iterdir() if p.is_file()}
        t["bytes_out"] = sum(sizes.values())
        t["total"] = sum(v for k, v in t.items() if isinstance(v, float))
        out[fmt] = t
        print(f"[writers] {fmt}: {json.dumps(t)}", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
