"""PCIe-inclusive rate of the engine at C4: host SoA + payload pushed with
mgp_push_batch (pinned and pageable), then one mgp_run, against the HBM-resident
step of bench.py. Prints one JSON line. Run on the GPU box:
    python scripts/pcie_bench.py [--reads N] [--cells C]
"""

from __future__ import annotations

import argparse
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from mgatk2_amd.engine import Engine, EngineConfig, load_library  # noqa: E402
from mgatk2_amd.synth import ReadSoA, cell_cdf, ref_codes  # noqa: E402


def pinned_like(a: np.ndarray, keep: list) -> np.ndarray:
    """A pinned (mgp_host_alloc) copy of a."""
    lib = load_library()
    p = C.c_void_p()
    if lib.mgp_host_alloc(max(a.nbytes, 1), C.byref(p)) != 0:
        raise RuntimeError("mgp_host_alloc failed")
    keep.append(p)
    buf = (C.c_uint8 * max(a.nbytes, 1)).from_address(p.value)
    out = np.frombuffer(buf, dtype=a.dtype, count=a.size).reshape(a.shape)
    out[...] = a
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=200_000_000)
    ap.add_argument("--cells", type=int, default=10_000)
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    cfg = EngineConfig(n_cells=args.cells, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length")
    seed = 20251015 + 4
    with Engine(cfg) as gen:
        gen.synth(seed, args.reads, cell_cdf(seed, args.cells), ref_codes(seed))
        host = gen.download_inputs()
    keep: list = []
    t0 = time.perf_counter()
    pin = ReadSoA(*[pinned_like(getattr(host, k), keep) for k in
                    ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off", "payload")])
    t_pin = time.perf_counter() - t0
    nbytes = sum(getattr(host, k).nbytes for k in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off",
                                                    "payload"))
    out = {"reads": host.n, "cells": args.cells, "h2d_bytes": nbytes, "pin_copy_s": t_pin}
    with Engine(cfg) as eng:
        for name, soa in (("pinned", pin), ("pageable", host)):
            best = None
            for _ in range(args.reps):
                eng.reset()
                eng.sync() if False else None
                t0 = time.perf_counter()
                eng.push(soa)
                eng.run()
                eng.sync()
                t_all = time.perf_counter() - t0
                kt = eng.kernel_times(1)
                t_run = sum(kt.values()) * 1e-3
                rec = {"total_s": t_all, "engine_s": t_run, "h2d_s": t_all - t_run,
                       "h2d_GBps": nbytes / max(t_all - t_run, 1e-9) / 1e9, "reads_per_s": host.n / t_all}
                if best is None or rec["total_s"] < best["total_s"]:
                    best = rec
            out[name] = best
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
