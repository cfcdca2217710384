"""Benchmark: chrM reads piled up per second (whole node), BASELINE.json's metric.

One step = one pass of the hot path (mgp_run: filter + cell-major grouping +
dedup + CIGAR-walk pileup + strand filter + per-cell stats + reference-allele
tallies, and the RCCL all-reduce of the tallies when N > 1) over BASELINE config
C4: ONE synthetic set of 200M chrM reads x 10k cells, `run` parameters, split by
cell over the N GPUs (strong scaling: rank r owns a read-balanced contiguous cell
range and exactly the reads of those cells, plus an equal share of the reads
without a whitelisted barcode; the reference's per-cell parallelism,
processors.py:112-144). Inputs are generated directly in HBM by the device
generator (bit-identical to mgatk2_amd/synth.py); `value` is timed with them
resident.

Around the timed steps (never inside them), rank 0 also measures:
  * sample_check: 3 samples of 8 whole cells of the timed run, bit for bit
    against the oracle on exactly their reads (cells are independent);
  * pcie: SURVEY.md §8(d)'s engine metric, from the first SoA batch H2D to the
    count matrices in host memory: pinned host batches pushed while earlier
    windows already run (streaming, MGP_CFG_STREAM), then the 16-bit result rows
    and per-cell statistics copied into pinned host memory (every rank, max over
    ranks);
  * cpu_baseline (N = 1 only): the single-threaded C port of the reference's
    path on a bounded sample of the same generator.

Launch: `python bench.py --gpus N` starts N worker processes itself (one per GPU,
RANK/LOCAL_RANK/WORLD_SIZE in their environment, before anything touches a GPU);
under torch.distributed.run the ranks come from the environment. torch.distributed
(gloo, CPU) is used only for the rendezvous, barriers and max-over-ranks; the
data path's only collective is the RCCL tally all-reduce inside mgp_run.
Rank 0 prints one JSON line.
"""

from __future__ import annotations

import argparse
import json
import os
import subprocess
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
ROW16_BYTES_PER_CELL = 16569 * 22  # the pileup's 16-bit rows: 8 + 2 + 1 u16 per position
# payload bytes of one record per layout (include/mgpileup.h)
RECORD_BYTES = {"quad32": 32, "pack32": 32, "paired": 64, "packed": 64, "full": 128}


def workload_name(n_reads: int, n_cells: int) -> str:
    """The BASELINE.json config a run's size matches (C4 is the bench's default)."""
    return {(200_000_000, 10_000): "C4", (50_000_000, 5_000): "C3", (1_000_000, 500): "C2",
            (1_000_000_000, 100_000): "C5"}.get((n_reads, n_cells), "custom")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--reads", type=int, default=200_000_000, help="reads of the whole set (all GPUs)")
    ap.add_argument("--cells", type=int, default=10_000, help="cells of the whole set (all GPUs)")
    ap.add_argument("--read-len", type=int, default=50)
    ap.add_argument("--seed", type=int, default=20251015 + 4)
    ap.add_argument("--weak", action="store_true", help="weak scaling: every rank gets its own full-size set")
    ap.add_argument("--cpu-sample-reads", type=int, default=20_000_000)
    ap.add_argument("--cpu-sample-cells", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the bit-exact sample check")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive (host buffers) leg")
    ap.add_argument("--no-device-paired", action="store_true",
                    help="skip the device leg on quality-carrying 64-byte records (the kernel applies the per-base "
                         "filter)")
    ap.add_argument("--no-host-pack", action="store_true", help="skip timing the host's 32-byte record build")
    ap.add_argument("--pcie-steps", type=int, default=3)
    ap.add_argument("--batch-reads", type=str, default="16000000",
                    help="reads per pushed batch in the PCIe leg; a comma list sweeps (first = reported)")
    ap.add_argument("--record-layout", choices=["quad32", "pack32", "paired", "packed", "full"], default="quad32",
                    help="payload records: 32-byte records made for the run's min_baseq, four consecutive "
                         "records of a cell per 128-byte line (quad32, default: the placement of "
                         "mgp_place_records) or in BAM order (pack32); packed 64-byte records two per line "
                         "(paired) or in BAM order (packed); or full 128-byte records")
    return ap.parse_args()


# ---------------------------------------------------------------------------
# launcher: one worker process per GPU, started before anything touches a GPU
# ---------------------------------------------------------------------------
def launch_workers(n: int, cmd: list[str]) -> int:
    """Start `cmd` n times, as ranks 0..n-1 of one node (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR/PORT in the environment); the first nonzero exit code,
    else 0. The parent never touches a GPU: every HIP call is in the workers."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen(cmd, env=env))
    codes = [p.wait() for p in procs]
    return next((c for c in codes if c != 0), 0)


def cell_bounds(cdf: np.ndarray, world: int) -> np.ndarray:
    """Read-balanced contiguous cell ranges (shard.partition_cells over the
    generator's expected reads per cell)."""
    from mgatk2_amd.shard import partition_cells

    w = np.diff(np.concatenate([[0.0], cdf.astype(np.float64)]))
    return partition_cells(w, world)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_workers(args.gpus, [sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE {world}: running {world} ranks", file=sys.stderr)
    if args.record_layout in ("paired", "quad32", "pack32") and args.read_len > 50:
        raise SystemExit(f"--record-layout {args.record_layout} needs --read-len <= 50 (packed records)")
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

    def reduce(x: float, op: str) -> float:
        if dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
        return float(t.item())

    no_comm = os.environ.get("MGP_BENCH_NO_COMM") == "1"
    device = 0 if no_comm else local_rank
    n_glob, nc_glob = args.reads, args.cells
    seed = args.seed + (1_000_003 * rank if args.weak else 0)
    cdf, ref = cell_cdf(seed, nc_glob), ref_codes(args.seed)  # one chrM reference for every rank
    if world > 1 and not args.weak:
        b = cell_bounds(cdf, world)
        lo, hi = int(b[rank]), int(b[rank + 1])
        shard = dict(cells=(lo, hi), shard=(rank, world))
    else:
        lo, hi = 0, nc_glob
        shard = {}
    n_cells = hi - lo
    cfg = EngineConfig(n_cells=n_cells, min_baseq=20, min_mapq=30, min_distance_from_end=5,
                       dedup_mode="alignment_and_fragment_length", max_strand_bias=1.0, min_reads=1)
    eng = Engine(cfg, device=device)
    t0 = time.time()
    lay = args.record_layout
    packed = lay in ("packed", "paired", "pack32", "quad32")
    p32 = cfg.min_baseq if lay in ("pack32", "quad32") else None  # 32-byte records for the run's min_baseq
    eng.synth(seed, n_glob, cdf, ref, read_len=args.read_len, rec_align=64 if packed else 128, pack=packed,
              pack32=p32, **shard)
    n_res, pay = eng.resident()
    if lay in ("paired", "quad32"):
        # the producer's placement (mgp_place_records, as the BAM decoder emits it):
        # computed on the host from the generated barcode and flag columns, then the
        # same reads are generated again at those offsets
        from mgatk2_amd.bam import PLACE_PAIRED, place_records

        soa = eng.download_inputs(columns=("bc", "flag", "start", "tlen"))
        roff, pay_b = place_records(soa.bc, soa.flag, np.full(n_res, 32 if p32 is not None else 64, np.uint32),
                                    n_cells, PLACE_PAIRED, start=soa.start, tlen=soa.tlen)
        del soa
        eng.synth(seed, n_glob, cdf, ref, read_len=args.read_len, rec_align=64, pack=True, rec_off=roff,
                  payload_bytes=pay_b, pack32=p32, **shard)
        del roff
    n_res, pay = eng.resident()
    t_gen = time.time() - t0
    print(f"[bench] rank {rank}: cells [{lo}, {hi}), {n_res:,} reads ({pay / 1e9:.2f} GB payload) generated "
          f"on device {device} in {t_gen:.1f}s", file=sys.stderr, flush=True)

    # MGP_BENCH_NO_COMM=1: rehearse the multi-process path with several ranks on one
    # GPU (RCCL refuses two ranks on one device); the tallies are then not reduced
    def make_comm(e):
        uid = Engine.comm_unique_id() if rank == 0 else b"\0" * 128
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        e.comm_init(obj[0], world, rank)

    comm_ranks = 1
    if world > 1 and not no_comm:
        make_comm(eng)
        comm_ranks = world

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
    dt_rank = time.perf_counter() - t0
    dt = reduce(dt_rank, "max")

    kt = eng.kernel_times(last_runs=min(args.steps, 64))
    # the per-stage breakdown from a few more (untimed) runs with every stage bracketed
    n_prof = min(3, max(args.steps, 1))
    eng.set_stage_timing(True)
    for _ in range(n_prof):
        eng.run()
    eng.sync()
    kt_all = eng.kernel_times(last_runs=n_prof)
    res = eng.fetch(dense=False)
    total_reads = reduce(float(n_res), "sum")
    value = total_reads * args.steps / dt
    ms_step = dt / args.steps * 1e3

    # roofline of the dominant kernel: its own algorithmic bytes per launch (kernel_rooflines)
    # over its HIP-event time on the compute stream, averaged over the timed steps; the
    # whole step against SURVEY.md §8(d)'s engine-level count (95 B per read + the u32
    # result rows per cell) is step_achieved / step_frac
    dom = "pileup"
    kernels = kernel_rooflines(kt_all, n_res, n_cells, res.stats, cfg, args.record_layout)
    alg_bytes = kernel_bytes(n_res, n_cells, res.stats, cfg, args.record_layout)[dom]
    achieved = alg_bytes / (kt[dom] * 1e-3) / 1e9
    engine_bytes = n_res * BYTES_PER_READ + n_cells * BYTES_PER_CELL
    step_achieved = engine_bytes / (dt_rank / args.steps) / 1e9
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

    check = None
    if rank == 0 and not args.no_check:
        check = sample_check(eng, cfg, res, args, seed, cdf, ref, lo, device)
    eng.close()

    # the same workload on quality-carrying 64-byte records two per line: the kernel
    # applies min_baseq / end distance / ACGT per base (pileup.py:67-86), which the
    # headline's 32-byte records carry resolved (built by the producer, timed below)
    paired = None
    if not args.no_device_paired and args.record_layout == "quad32":
        paired = device_leg(args, cfg, seed, cdf, ref, shard, device, make_comm if comm_ranks > 1 else None,
                            barrier, reduce, "paired")
    host_pack = None
    if rank == 0 and not args.no_host_pack and args.record_layout in ("quad32", "pack32"):
        host_pack = host_pack_leg(args, cfg, device)

    pcie = None
    if not args.no_pcie:
        pcie = pcie_leg(args, cfg, seed, cdf, ref, shard, device, comm_ranks, barrier, reduce, make_comm)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, cfg, local_rank)

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
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SURVEY.md §8(d) generator, created in HBM by the device generator)",
            "bit_exact": None if check is None else check["bit_exact"],
            "config": {
                "workload": f"{workload_name(n_glob, nc_glob)}: {n_glob / 1e6:g}M chrM reads x {nc_glob / 1e3:g}k "
                            f"cells{' per GPU' if args.weak else ' (one set, split by cell over the GPUs)'}, "
                            f"run params (q20, mapq30, dedup=alignment_and_fragment_length, min_reads 1), "
                            f"L={args.read_len}",
                "reads_rank0": n_res,
                "cells_rank0": n_cells,
                "payload_bytes_rank0": pay,
                "record_layout": args.record_layout,
                "parallelism": f"cell-sharded x{world} (RCCL all-reduce of ref tallies over {comm_ranks} ranks)",
                "rank0_step_ms": dt_rank / args.steps * 1e3,
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
                "alg_bytes_what": f"4-byte pileup element + one {RECORD_BYTES[args.record_layout]}-byte record per "
                                  f"kept read, 16-bit result rows ({ROW16_BYTES_PER_CELL} B) per cell",
                "engine_alg_bytes_per_step": engine_bytes,
                "step_achieved": step_achieved,
                "step_frac": step_achieved / HBM_PEAK_GBS,
                "kernels": kernels,
            },
            "stage_ms": {k: round(v, 4) for k, v in kt_all.items()},
            # value is the HBM-resident rate (the task's bench contract: inputs resident
            # when the timed region starts); SURVEY.md §8(d)'s engine metric, from the first
            # H2D to the counts in host memory, is value_pcie
            "value_device": value,
            "value_pcie": None if pcie is None else pcie["value"],
            "device_ms_paired": None if paired is None else paired["ms_per_step"],
            "device_paired": paired,
            "host_pack_ns_per_read": None if host_pack is None else host_pack["ns_per_read_1thread"],
            "host_pack": host_pack,
            "pcie": pcie,
            "cpu_baseline": cpu,
            "stats_rank0": res.stats,
            "sample_check": check,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def device_leg(args, cfg, seed, cdf, ref, shard, device, make_comm, barrier, reduce, layout: str) -> dict:
    """The timed steps again on another record layout of the same reads (untimed
    generation): ms per step (max over ranks) and the stage times."""
    from mgatk2_amd.bam import PLACE_PAIRED, place_records
    from mgatk2_amd.engine import Engine

    eng = Engine(cfg, device=device)
    eng.synth(seed, args.reads, cdf, ref, read_len=args.read_len, rec_align=64, pack=True, **shard)
    n_res, _ = eng.resident()
    if layout == "paired":
        soa = eng.download_inputs(columns=("bc", "flag", "start", "tlen"))
        roff, pay_b = place_records(soa.bc, soa.flag, np.full(n_res, 64, np.uint32), cfg.n_cells, PLACE_PAIRED,
                                    start=soa.start, tlen=soa.tlen)
        del soa
        eng.synth(seed, args.reads, cdf, ref, read_len=args.read_len, rec_align=64, pack=True, rec_off=roff,
                  payload_bytes=pay_b, **shard)
        del roff
    if make_comm is not None:
        make_comm(eng)
    eng.set_stage_timing(False)
    for _ in range(max(1, args.warmup)):
        eng.run()
    eng.sync()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run()
    eng.sync()
    barrier()
    dt = reduce(time.perf_counter() - t0, "max")
    pile = eng.kernel_times(last_runs=min(args.steps, 64)).get("pileup")
    eng.set_stage_timing(True)
    for _ in range(3):
        eng.run()
    eng.sync()
    kt = eng.kernel_times(last_runs=3)
    st = eng.fetch(dense=False).stats
    eng.close()
    return {"record_layout": layout, "what": "packed 64-byte records (qualities and base codes; the kernel applies "
            "min_baseq, min_distance_from_end and ACGT per base), two of a cell per 128-byte line",
            "ms_per_step": dt / args.steps * 1e3, "value": reduce(float(n_res), "sum") * args.steps / dt,
            "pileup_ms": pile, "stage_ms": {k: round(v, 4) for k, v in kt.items()},
            "filtered_reads_rank0": st["filtered_reads"], "error_bits": st["error_bits"]}


def host_pack_leg(args, cfg, device, n: int = 4_000_000) -> dict:
    """The producer's cost of the 32-byte records (what the headline's device step
    does not do): the host builder the BAM decoder calls per record
    (mgp_pack32_host.h via mgp_repack32) over full records of the same generator,
    on one thread and on the host threads."""
    from mgatk2_amd.bam import host_threads, repack32
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.synth import cell_cdf, ref_codes

    seed = args.seed + 91
    nc = 1000
    with Engine(EngineConfig(**{**cfg.__dict__, "n_cells": nc}), device=device) as e2:
        e2.synth(seed, n, cell_cdf(seed, nc), ref_codes(seed), read_len=args.read_len, rec_align=128, pack=False)
        soa = e2.download_inputs()
    out32 = np.empty(n * 32, np.uint8)
    oflag = np.empty(n, np.uint16)
    repack32(soa, cfg.min_baseq, cfg.min_distance_from_end, 1, out32, oflag)  # (pages faulted in)
    t0 = time.perf_counter()
    _, _, k = repack32(soa, cfg.min_baseq, cfg.min_distance_from_end, 1, out32, oflag)
    t1 = time.perf_counter() - t0
    nt = host_threads()
    t0 = time.perf_counter()
    repack32(soa, cfg.min_baseq, cfg.min_distance_from_end, nt, out32, oflag)
    tn = time.perf_counter() - t0
    return {"ns_per_read_1thread": t1 / n * 1e9, "reads_per_s_threads": n / tn, "threads": nt, "packed": k,
            "sample": f"{n:,} full 128-byte records of the generator (run thresholds q{cfg.min_baseq}, "
                      f"min_dist {cfg.min_distance_from_end})"}


def kernel_bytes(n: int, nc: int, stats: dict, cfg, layout: str) -> dict:
    """Each kernel's own algorithmic bytes per launch."""
    L = cfg.mito_len
    nbins = (L + 7) // 8 + 1
    kept = int(stats.get("filtered_reads", 0))
    rec = RECORD_BYTES[layout]
    return {
        # barcode + flag per read, the H rows
        "hist": 6 * n + 4 * nbins * nc,
        # every column of every read (27 B), one 8-byte element per kept-or-duplicate read
        # (the duplicates are a fraction of the valid reads: the kept reads bound it below)
        "group_a": 27 * n + 8 * kept,
        # 8-byte element in, 4-byte pileup element out
        "group_b": 12 * kept,
        # 4-byte element + one record per kept read (an upper bound: kept reads below
        # min_mapq are not gathered), the 16-bit result rows written once
        "pileup": (4 + rec) * kept + ROW16_BYTES_PER_CELL * nc,
        # the 16-bit depth row per cell
        "median": 2 * L * nc,
    }


def kernel_rooflines(kt: dict, n: int, nc: int, stats: dict, cfg, layout: str) -> dict:
    """Each kernel's own algorithmic bytes over its HIP-event time."""
    out = {}
    for k, b in kernel_bytes(n, nc, stats, cfg, layout).items():
        ms = kt.get(k, 0.0)
        if ms > 0:
            gbs = b / (ms * 1e-3) / 1e9
            out[k] = {"alg_bytes": int(b), "ms": round(ms, 4), "GBps": round(gbs, 1),
                      "frac": round(gbs / HBM_PEAK_GBS, 3)}
    return out


def sample_check(eng, cfg, res, args, seed, cdf, ref, cell0: int, device: int) -> dict:
    """3 samples of 8 whole cells of the timed run (first, middle, last cells of the
    rank) bit for bit against the oracle on exactly their reads, plus the run
    statistics' consistency. Cells are independent, so a cell's rows depend only
    on its own reads. The oracle reads the quality-carrying full 128-byte records of
    those reads (regenerated as a cell shard of the same seed): with 32-byte records
    the per-base filter (pileup.py:67-88) was resolved by the producer, and this
    checks that too."""
    from mgatk2_amd.engine import Engine, EngineConfig
    from oracle.oracle import oracle_run

    t0 = time.perf_counter()
    nc = cfg.n_cells
    ranges = sorted({(0, min(8, nc)), (nc // 2, min(nc, nc // 2 + 8)), (max(0, nc - 8), nc)})
    got = {r: eng.fetch_cells(*r) for r in ranges}
    ok = True
    bad = []
    keys = ("counts", "tn5", "depth", "n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max",
            "median_lo", "median_hi")
    for (lo, hi), g in got.items():
        scfg = EngineConfig(**{**cfg.__dict__, "n_cells": hi - lo})
        with Engine(scfg, device=device) as e2:
            e2.synth(seed, args.reads, cdf, ref, read_len=args.read_len, rec_align=128, pack=False,
                     cells=(cell0 + lo, cell0 + hi), shard=(0, 0))
            sub = e2.download_inputs()
        exp, _ = oracle_run(scfg, sub)
        for k in keys:
            if not np.array_equal(getattr(g, k), getattr(exp, k)):
                ok = False
                bad.append(f"{lo}-{hi}:{k}")
    st = res.stats
    consistent = (st["filtered_reads"] == int(res.n_reads.sum()) and st["cells_passed"] == int(res.passed.sum())
                  and st["n_barcodes"] == int((res.n_reads > 0).sum()) and st["error_bits"] == 0)
    return {"bit_exact": bool(ok and consistent), "cells": [list(r) for r in ranges], "mismatches": bad,
            "stats_consistent": bool(consistent), "oracle_input": "full 128-byte records (raw qualities) of the "
            "sampled cells' reads", "seconds": round(time.perf_counter() - t0, 2)}


def pcie_leg(args, cfg, seed, cdf, ref, shard, device, comm_ranks, barrier, reduce, make_comm) -> dict:
    """SURVEY.md §8(d)'s engine metric: host SoA batches in pinned memory -> pushed
    (H2D on the copy stream; with streaming on, each push runs the windows its reads
    complete, overlapping the next batches' copies) -> mgp_run -> the 16-bit result
    rows and per-cell statistics in pinned host memory. The rank's reads are the
    same as the timed run's, in the dense packed layout a streaming producer emits
    (records in BAM order: a batch is a contiguous payload range)."""
    from mgatk2_amd.engine import Engine, EngineConfig, PinnedBuffer, Rows16
    from mgatk2_amd.synth import ReadSoA

    batch_list = [int(x) for x in str(args.batch_reads).split(",") if x.strip()]
    scfg = EngineConfig(**{**cfg.__dict__})
    eng = Engine(scfg, device=device)
    p32 = cfg.min_baseq if args.record_layout in ("pack32", "quad32") else None
    rb = 32 if p32 is not None else 64  # dense records in BAM order
    eng.synth(seed, args.reads, cdf, ref, read_len=args.read_len, rec_align=64, pack=True, pack32=p32, **shard)
    n, pay = eng.resident()
    # the producer's columns: bc, tlen, flag, mapq. No rec_off (dense records in BAM
    # order) and no span (taken from the records' CIGARs on the device): ABI v3.1; no
    # start (taken from the records, which all hold it): ABI 4
    cols = ("bc", "tlen", "flag", "mapq", "payload")
    col_bytes = n * (4 + 4 + 2 + 1)
    hbuf = PinnedBuffer(col_bytes + pay + 4096)
    off = [0]

    def alloc(m, dt):
        a = hbuf.array(m, dt, off[0])
        off[0] = (off[0] + m * np.dtype(dt).itemsize + 63) & ~63
        return a

    host = eng.download_inputs(columns=cols, alloc=alloc)  # the producer's batches: pinned, BAM order
    assert np.all(eng.download_inputs(columns=("rec_off",)).rec_off == rb * np.arange(n, dtype=np.uint64))
    L, nc = cfg.mito_len, cfg.n_cells
    nw, W = eng.windows()
    rbuf = PinnedBuffer(nc * L * 22 + nc * nw + 4096)
    rows = Rows16(rbuf.array((nc, L, 8), np.uint16, 0), rbuf.array((nc, L, 2), np.uint16, nc * L * 16),
                  rbuf.array((nc, L), np.uint16, nc * L * 20), rbuf.array((nc, nw), np.uint8, nc * L * 22), W)
    if comm_ranks > 1:
        make_comm(eng)  # every run all-reduces its tallies, as in the timed steps
    # the rows leave the device as the windows complete, beside the later batches' H2D
    try:
        eng.set_rows16_target(rows)
        rows_target = True
    except Exception as e:  # (pinned memory the device cannot map: copy the rows after the run)
        print(f"[bench] rows target unavailable ({e}); rows fetched after the run", file=sys.stderr)
        rows_target = False

    def batches_for(bs):
        """Batches of bs reads: their columns and their slice of the dense payload."""
        return [ReadSoA(None, host.bc[a:b], host.tlen[a:b], host.flag[a:b], host.mapq[a:b], None, None,
                        host.payload[rb * a:rb * b]) for a, b in ((a, min(n, a + bs)) for a in range(0, n, bs))]

    def one(batches, stream):
        eng.set_streaming(stream)
        eng.reset()
        t0 = time.perf_counter()
        for bt in batches:
            eng.push(bt)
        t_push = time.perf_counter() - t0
        eng.run()
        if not rows_target:
            eng.fetch_rows16(0, nc, out=rows)
        r = eng.fetch(dense=False)  # (waits for the rows' copies too)
        return time.perf_counter() - t0, t_push, r

    legs = []
    for bs in batch_list:
        batches = batches_for(bs)
        one(batches, True)  # warmup (allocations)
        for stream in (True, False):
            ts = []
            seg0 = eng.stream_info()[0]
            for _ in range(args.pcie_steps):
                barrier()
                dt, t_push, r = one(batches, stream)
                ts.append((dt, t_push))
            segs = (eng.stream_info()[0] - seg0) // max(1, args.pcie_steps)
            dt = min(t for t, _ in ts)
            dt_max = reduce(dt, "max")
            legs.append({"batch_reads": bs, "batches": len(batches), "streamed": stream, "segments": int(segs),
                         "s": dt_max, "push_s": round(min(p for _, p in ts), 4),
                         "value": reduce(float(n), "sum") / dt_max})
    stats = r.stats
    h2d = col_bytes + pay
    d2h = nc * L * 22 + nc * nw + nc * 34 + L * 4 * 8  # rows, wide flags, per-cell arrays, tallies
    best = legs[0]
    eng.close()
    return {
        "value": best["value"],
        "unit": "reads/s",
        "what": "pinned host SoA batches (bc, tlen, flag, mapq + dense 32-byte records; no rec_off or span "
                "columns: ABI v3.1, no start column: ABI 4, the engine takes them from the records) -> H2D (streamed: windows run as their reads arrive, and their 16-bit count rows "
                "go back D2H as each window completes) -> run -> every row + per-cell stats in pinned host memory; "
                "max over ranks",
        "h2d_bytes_rank0": h2d,
        "d2h_bytes_rank0": d2h,
        "link_GBps_rank0": round((h2d + d2h) / best["s"] / 1e9, 2),
        "rows_target": rows_target,
        "legs": legs,
        "stats_total_reads_rank0": stats["total_reads"],
    }


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
    import platform

    from oracle.oracle import oracle_run

    scfg, soa = _sample_inputs(args, cfg, device)
    t0 = time.perf_counter()
    oracle_run(scfg, soa, dense=False)
    dt = time.perf_counter() - t0
    cpu = platform.processor() or ""
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": soa.n / dt,
        "unit": "reads/s",
        "cores": 1,
        "kind": "port",
        "cpu": cpu,
        "sample": f"{soa.n:,} reads x {scfg.n_cells} cells of the same generator (20k reads/cell, run params); "
                  f"oracle/mgp_oracle.c single-threaded, {dt:.1f}s",
    }


if __name__ == "__main__":
    main()
