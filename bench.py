"""Benchmark: chrM reads piled up per second (whole node), BASELINE.json's metric.

One step = one pass of the hot path (mgp_run: filter + cell-major grouping +
dedup + CIGAR-walk pileup + strand filter + per-cell stats + reference-allele
tallies, and the RCCL all-reduce of the tallies when N > 1) over the
HBM-resident synthetic workload of BASELINE config C4 (200M chrM reads x 10k
cells, `run` parameters) per GPU. Inputs are generated directly in HBM by the
device generator (bit-identical to mgatk2_amd/synth.py); the timed region starts
with them resident.

Multi-GPU: one process per GPU (torch.distributed.run), cells sharded (each rank
owns its own 10k-cell shard of 200M reads: weak scaling). torch.distributed
(gloo, CPU) is used only for the rendezvous, barriers and the max-over-ranks
time; the data path has no collective except the RCCL tally all-reduce inside
mgp_run. Rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "chrM reads piled-up/sec (whole node) at 200M reads × 10k cells; bit-exact counts"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BYTES_PER_READ = 95  # algorithmic input bytes per L=50 read
BYTES_PER_CELL = 16569 * 10 * 4  # int32 counts (8 planes) + tn5 (2 planes) written once


def workload_name(n_reads: int, n_cells: int) -> str:
    """The BASELINE.json config a run's size matches (C4 is the bench's default)."""
    return {(200_000_000, 10_000): "C4", (50_000_000, 5_000): "C3", (1_000_000, 500): "C2",
            (1_000_000_000, 100_000): "C5 on one GPU"}.get((n_reads, n_cells), "custom")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=200_000_000, help="reads per GPU")
    ap.add_argument("--cells", type=int, default=10_000, help="cells per GPU")
    ap.add_argument("--read-len", type=int, default=50)
    ap.add_argument("--seed", type=int, default=20251015 + 4)
    ap.add_argument("--cpu-sample-reads", type=int, default=20_000_000)
    ap.add_argument("--cpu-sample-cells", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--record-layout", choices=["paired", "packed", "full"], default="paired",
                    help="payload records: packed 64-byte records, two consecutive records of a cell per "
                         "128-byte line (paired, default: the placement of mgp_place_records), packed in BAM "
                         "order, or full 128-byte records")
    ap.add_argument("--check", action="store_true", help="bit-exact check of a sample against the oracle")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as tdist

        tdist.init_process_group("gloo", rank=rank, world_size=world)
        dist = tdist

    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import cell_cdf, ref_codes

    def barrier():
        if dist is not None:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x: float) -> float:
        if dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    n_reads, n_cells = args.reads, args.cells
    seed = args.seed + 1_000_003 * rank
    cfg = EngineConfig(n_cells=n_cells, min_baseq=20, min_mapq=30, min_distance_from_end=5,
                       dedup_mode="alignment_and_fragment_length", max_strand_bias=1.0, min_reads=1)
    eng = Engine(cfg, device=local_rank if os.environ.get("MGP_BENCH_NO_COMM") != "1" else 0)
    t0 = time.time()
    cdf, ref = cell_cdf(seed, n_cells), ref_codes(args.seed)  # one chrM reference for every rank
    packed = args.record_layout in ("packed", "paired")
    eng.synth(seed, n_reads, cdf, ref, read_len=args.read_len, rec_align=64 if packed else 128, pack=packed)
    if args.record_layout == "paired":
        # the producer's placement (mgp_place_records, as the BAM decoder emits it):
        # computed on the host from the generated barcode and flag columns, then the
        # same reads are generated again at those offsets
        from mgatk2_amd.bam import PLACE_PAIRED, place_records

        soa = eng.download_inputs(columns=("bc", "flag", "start", "tlen"))
        roff, pay_b = place_records(soa.bc, soa.flag, np.full(n_reads, 64, np.uint32), n_cells, PLACE_PAIRED,
                                    start=soa.start, tlen=soa.tlen)
        del soa
        eng.synth(seed, n_reads, cdf, ref, read_len=args.read_len, rec_align=64, pack=True, rec_off=roff,
                  payload_bytes=pay_b)
        del roff
    n_res, pay = eng.resident()
    t_gen = time.time() - t0
    if rank == 0:
        print(f"[bench] generated {n_res:,} reads ({pay / 1e9:.2f} GB payload) on device in {t_gen:.1f}s",
              file=sys.stderr, flush=True)

    # MGP_BENCH_NO_COMM=1: rehearse the multi-process path with several ranks on one
    # GPU (RCCL refuses two ranks on one device); the tallies are then not reduced
    if world > 1 and os.environ.get("MGP_BENCH_NO_COMM") != "1":
        uid = Engine.comm_unique_id() if rank == 0 else b"\0" * 128
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(obj[0], world, rank)

    # the timed runs bracket only the pileup with HIP events (its roofline); every
    # other stage boundary would add a marker between two kernels of the stream
    eng.set_stage_timing(os.environ.get("MGP_BENCH_ALL_STAGES") == "1")  # (=1: every stage timed, for A/B)
    for _ in range(args.warmup):
        eng.run()
        eng.sync()

    barrier()
    eng.sync() if args.warmup else None
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run()
    eng.sync()
    barrier()
    dt = time.perf_counter() - t0
    dt = max_over_ranks(dt)

    kt = eng.kernel_times(last_runs=min(args.steps, 64))
    # the per-stage breakdown from a few more (untimed) runs with every stage bracketed
    n_prof = min(3, max(args.steps, 1))
    eng.set_stage_timing(True)
    for _ in range(n_prof):
        eng.run()
    eng.sync()
    kt_all = eng.kernel_times(last_runs=n_prof)
    res = eng.fetch(dense=False)
    total_reads = sum_over_ranks(float(n_res))
    value = total_reads * args.steps / dt
    ms_step = dt / args.steps * 1e3

    # roofline of the dominant stage (HIP events on the compute stream, averaged over the timed steps)
    dom = "pileup"
    alg_bytes = n_res * BYTES_PER_READ + n_cells * BYTES_PER_CELL
    achieved = alg_bytes / (kt[dom] * 1e-3) / 1e9
    step_achieved = alg_bytes / (ms_step * 1e-3) / 1e9
    traffic = None
    pmc = ROOT / "profiles" / "pmc_traffic.json"
    if pmc.exists():
        try:
            d = json.loads(pmc.read_text())
            if (d.get("reads") == n_res and d.get("cells") == n_cells
                    and d.get("record_layout", "full") == args.record_layout):
                traffic = d.get(dom)
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, cfg, local_rank)
    check = None
    if rank == 0 and args.check:
        check = sample_check(args, cfg, local_rank)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "reads/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SURVEY.md §8(d) generator, created in HBM by the device generator)",
            "config": {
                "workload": f"{workload_name(n_reads, n_cells)}: {n_reads / 1e6:g}M chrM reads x {n_cells / 1e3:g}k "
                            f"cells per GPU, run params (q20, mapq30, dedup=alignment_and_fragment_length, "
                            f"min_reads 1), L={args.read_len}",
                "reads_per_gpu": n_res,
                "cells_per_gpu": n_cells,
                "payload_bytes_per_gpu": pay,
                "record_layout": args.record_layout,
                "parallelism": f"cell-sharded x{world} (RCCL all-reduce of ref tallies)",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "alg_bytes_per_launch": alg_bytes,
                "step_achieved": step_achieved,
                "step_frac": step_achieved / HBM_PEAK_GBS,
            },
            "stage_ms": {k: round(v, 4) for k, v in kt_all.items()},
            "cpu_baseline": cpu,
            "stats": res.stats,
            "sample_check": check,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def _sample_inputs(args, cfg, device):
    """A bounded sample of the same workload: same generator, same reads/cell density."""
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import cell_cdf, ref_codes

    n, nc = args.cpu_sample_reads, args.cpu_sample_cells
    seed = args.seed + 77
    scfg = EngineConfig(**{**cfg.__dict__, "n_cells": nc})
    with Engine(scfg, device=device) as e2:
        e2.synth(seed, n, cell_cdf(seed, nc), ref_codes(seed), read_len=args.read_len)
        soa = e2.download_inputs()
    return scfg, soa


def cpu_baseline(args, cfg, device):
    from oracle.oracle import oracle_run

    scfg, soa = _sample_inputs(args, cfg, device)
    t0 = time.perf_counter()
    oracle_run(scfg, soa, dense=False)
    dt = time.perf_counter() - t0
    return {
        "value": soa.n / dt,
        "unit": "reads/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{soa.n:,} reads x {scfg.n_cells} cells of the same generator (20k reads/cell, run params); "
                  f"oracle/mgp_oracle.c single-threaded, {dt:.1f}s",
    }


def sample_check(args, cfg, device):
    from mgatk2_amd.engine import Engine
    from oracle.oracle import oracle_run

    scfg, soa = _sample_inputs(args, cfg, device)
    with Engine(scfg, device=device) as e:
        e.push(soa)
        r = e.finish()
    x, _ = oracle_run(scfg, soa)
    ok = all(np.array_equal(getattr(r, k), getattr(x, k)) for k in
             ("counts", "tn5", "depth", "n_reads", "passed", "ref_tally", "median_lo", "median_hi"))
    return {"reads": soa.n, "cells": scfg.n_cells, "bit_exact": bool(ok)}


if __name__ == "__main__":
    main()
