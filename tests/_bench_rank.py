"""A rank of tests/test_dist.py::test_bench_launcher (CPU): started by bench.launch_workers
with RANK/WORLD_SIZE in its environment, it runs the bench's cell split of one
synthetic set (bench.cell_bounds over the generator's cell weights) through the
oracle on its shard, all-reduces the tallies over gloo and rank 0 checks the merge
against one oracle run over the whole set."""

import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from mgatk2_amd.engine import EngineConfig  # noqa: E402
from mgatk2_amd.shard import merge_results, shard_soa  # noqa: E402
from mgatk2_amd.synth import synth_reads  # noqa: E402
from oracle.oracle import oracle_run  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n, nc = 60_000, 37
    soa = synth_reads(91, n, nc)
    b = bench.cell_bounds(soa.extra["cdf"], world)
    lo, hi = int(b[rank]), int(b[rank + 1])
    cfg = EngineConfig(n_cells=nc, min_baseq=20, min_mapq=30, dedup_mode="alignment_and_fragment_length")
    sub, idx = shard_soa(soa, lo, hi)
    r, _ = oracle_run(EngineConfig(**{**cfg.__dict__, "n_cells": hi - lo}), sub)
    t = torch.from_numpy(r.ref_tally.astype(np.int64))
    dist.all_reduce(t)
    r.ref_tally[:] = t.numpy().astype(np.uint64)
    parts = [None] * world
    dist.all_gather_object(parts, (r, lo, hi, idx))
    if rank == 0:
        merged = merge_results(parts, nc, n, tally_reduced=True)
        whole, _ = oracle_run(cfg, soa)
        for k in ("counts", "tn5", "depth", "n_reads", "passed", "covered", "median_lo", "median_hi", "ref_tally",
                  "first_read"):
            np.testing.assert_array_equal(getattr(merged, k), getattr(whole, k), err_msg=k)
        assert b[0] == 0 and b[-1] == nc and np.all(np.diff(b) > 0)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
