"""The device txt writer (mgp_txt_gz) alone at C4 size: the engine runs the synthetic
C4 set (device generator), then the passing cells' members are made in chunks of
--chunk cells; per-chunk wall times and totals as one JSON line. Run under
`rocprofv3 --kernel-trace --stats` for the kernels' own times.

    python scripts/txt_bench.py [--reads N] [--cells C] [--chunk K] [--repeat R]
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
    ap.add_argument("--chunk", type=int, default=2048)
    ap.add_argument("--repeat", type=int, default=2)
    args = ap.parse_args()
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.processing.processors import cells_written
    from mgatk2_amd.synth import barcode_names, cell_cdf, ref_codes

    seed = 20251015 + 4
    nc = args.cells
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length", min_reads=1)
    names = barcode_names(nc, seed)
    out = {"reads": args.reads, "cells": nc, "chunk": args.chunk}
    with Engine(cfg) as eng:
        eng.synth(seed, args.reads, cell_cdf(seed, nc), ref_codes(seed))
        eng.run()
        res = eng.fetch(dense=False)
        written = cells_written(res)
        runs = []
        for _ in range(args.repeat):
            t0 = time.perf_counter()
            tot = text = 0
            per = []
            for a in range(0, written.size, args.chunk):
                ch = written[a:a + args.chunk]
                t1 = time.perf_counter()
                mem = eng.txt_gz(ch, [names[c] for c in ch.tolist()])
                per.append(round(time.perf_counter() - t1, 3))
                tot += int(mem.member_bytes.sum())
                text += int(mem.text_bytes.sum())
            runs.append({"s": round(time.perf_counter() - t0, 3), "chunks_s": per, "gz_bytes": tot, "text_bytes": text})
        out["runs"] = runs
        out["GBps_text"] = round(text / min(r["s"] for r in runs) / 1e9, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
