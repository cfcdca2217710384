"""Cell sharding on CPU: partition -> per-shard runs -> merge
equals one run over the whole read set. The per-shard runs use the oracle,
the CPU checker. The multi-process variant runs world_size 2 over gloo: each
rank runs its own shard, the tallies are all-reduced, and rank 0 merges."""

from __future__ import annotations

import os

import numpy as np
import pytest

from golden_io import Golden, check_result

KEYS = ("counts", "tn5", "depth", "n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max",
        "median_lo", "median_hi", "ref_tally")


def _assert_same(a, b):
    for k in KEYS:
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    np.testing.assert_array_equal(a.cell_order(), b.cell_order())
    for k in ("total_reads", "filtered_reads", "n_barcodes", "duplicate_reads_with_length",
              "duplicate_reads_position_only", "cells_passed"):
        assert a.stats[k] == b.stats[k], k


def test_partition_cells():
    from mgatk2_amd.shard import partition_cells

    w = np.array([5, 5, 5, 5, 100, 1, 1, 1])
    for n in (1, 2, 3, 8, 12):
        b = partition_cells(w, n)
        assert b[0] == 0 and b[-1] == w.size and len(b) == n + 1 and np.all(np.diff(b) >= 0)
    assert partition_cells(np.zeros(0), 4).tolist() == [0, 0]
    b = partition_cells(np.ones(1000), 4)
    assert np.diff(b).tolist() == [250, 250, 250, 250]


@pytest.mark.parametrize("n_shards", [1, 2, 3, 5])
@pytest.mark.parametrize("case", ["synth_run", "synth_tenx", "kat_run", "synth_bias"])
def test_shard_merge_equals_whole(case, n_shards, oracle_lib):
    from mgatk2_amd.shard import merge_results, partition_cells, reads_per_cell, shard_soa

    g = Golden(case)
    cfg = g.config()
    whole, _ = oracle_lib.oracle_run(cfg, g.soa)
    nc = len(g.whitelist)
    b = partition_cells(reads_per_cell(g.soa, nc), n_shards)
    parts = []
    for lo, hi in zip(b[:-1].tolist(), b[1:].tolist()):
        sub, idx = shard_soa(g.soa, lo, hi)
        scfg = type(cfg)(**{**cfg.__dict__, "n_cells": hi - lo})
        r, _ = oracle_lib.oracle_run(scfg, sub)
        parts.append((r, lo, hi, idx))
    merged = merge_results(parts, nc, g.soa.n)
    _assert_same(merged, whole)
    check_result(merged, g)


def _rank_main(rank, world, port, case, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch

        from mgatk2_amd.build import build_oracle
        from mgatk2_amd.shard import merge_results, partition_cells, reads_per_cell, shard_soa
        from oracle.oracle import oracle_run

        build_oracle()
        g = Golden(case)
        cfg = g.config()
        nc = len(g.whitelist)
        b = partition_cells(reads_per_cell(g.soa, nc), world)
        lo, hi = int(b[rank]), int(b[rank + 1])
        sub, idx = shard_soa(g.soa, lo, hi)
        r, _ = oracle_run(type(cfg)(**{**cfg.__dict__, "n_cells": hi - lo}), sub)
        t = torch.from_numpy(r.ref_tally.astype(np.int64))
        dist.all_reduce(t)  # the one exchange step (RCCL on the GPU path)
        r.ref_tally[:] = t.numpy().astype(np.uint64)
        objs = [None] * world
        dist.all_gather_object(objs, (r, lo, hi, idx))
        if rank == 0:
            merged = merge_results(objs, nc, g.soa.n, tally_reduced=True)
            whole, _ = oracle_run(cfg, g.soa)
            _assert_same(merged, whole)
            check_result(merged, g)
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported through the queue
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["synth_run", "kat_bias"])
def test_two_rank_gloo(case):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = dict(q.get(timeout=5) for _ in procs)
    assert res == {0: "ok", 1: "ok"}, res
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launcher(world):
    """bench.py's own launcher (`python bench.py --gpus N` without torchrun): N
    worker processes with RANK/WORLD_SIZE set, gloo rendezvous on 127.0.0.1, the
    bench's cell split, per-rank shards through the oracle, tallies all-reduced."""
    import sys
    from pathlib import Path

    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import bench

    script = str(Path(__file__).resolve().parent / "_bench_rank.py")
    assert bench.launch_workers(world, [sys.executable, script]) == 0


def test_bench_kernel_bytes_follow_the_record_layout():
    """The headline roofline counts the pileup's own bytes: a 4-byte element and one
    record of the run's layout per kept read, plus the 16-bit rows per cell."""
    import bench
    from mgatk2_amd.engine import EngineConfig

    cfg = EngineConfig(n_cells=10)
    st = {"filtered_reads": 1000}
    for lay, rec in (("quad32", 32), ("paired", 64), ("full", 128)):
        b = bench.kernel_bytes(2000, 10, st, cfg, lay)
        assert b["pileup"] == (4 + rec) * 1000 + bench.ROW16_BYTES_PER_CELL * 10
        assert b["group_b"] == 12 * 1000
    kr = bench.kernel_rooflines({"pileup": 1.0}, 2000, 10, st, cfg, "quad32")
    assert set(kr) == {"pileup"} and kr["pileup"]["alg_bytes"] == 36 * 1000 + bench.ROW16_BYTES_PER_CELL * 10
