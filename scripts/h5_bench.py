"""The device HDF5 chunk deflate (mgp_h5_tiles) alone at C4 size: the engine runs the
synthetic C4 set (device generator), then every chunk of the 11 count planes is made
(columns = the cells); wall times, bytes and the ratio to the raw planes as one JSON
line. Run under `rocprofv3 --kernel-trace --stats` for the kernels' own times.

    python scripts/h5_bench.py [--reads N] [--cells C] [--cols-per-call K] [--repeat R]
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=200_000_000)
    ap.add_argument("--cells", type=int, default=10_000)
    ap.add_argument("--cols-per-call", type=int, default=3200)
    ap.add_argument("--repeat", type=int, default=2)
    args = ap.parse_args()
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import cell_cdf, ref_codes

    seed = 20251015 + 4
    nc = args.cells
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1)
    out = {"reads": args.reads, "cells": nc, "cols_per_call": args.cols_per_call}
    coc = np.arange(nc, dtype=np.int64)
    with Engine(cfg) as eng:
        eng.synth(seed, args.reads, cell_cdf(seed, nc), ref_codes(seed))
        eng.run()
        eng.sync()
        runs = []
        for _ in range(args.repeat):
            t0 = time.perf_counter()
            tiles = eng.h5_tiles(coc, cols_per_call=args.cols_per_call)
            runs.append({"s": round(time.perf_counter() - t0, 3),
                         "bytes": int(sum(len(b) for v in tiles.values() for b in v))})
        out["runs"] = runs
        raw = 11 * (-(-cfg.mito_len // 1000) * 1000) * (-(-nc // 100) * 100) * 2
        out["raw_bytes"] = raw
        out["ratio"] = round(runs[-1]["bytes"] / raw, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
