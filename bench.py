"""Benchmark: chrM reads piled up per second (whole node), BASELINE.json's metric.

The step is SURVEY.md §8(d)'s engine metric: one whole pass of the hot path over
BASELINE config C4 (ONE synthetic set of 200M chrM reads x 10k cells, `run`
parameters, split by cell over the N GPUs: rank r owns a read-balanced contiguous
cell range and exactly the reads of those cells, plus an equal share of the reads
without a whitelisted barcode; the reference's per-cell parallelism,
processors.py:112-144), from the first SoA batch's H2D to the count matrices in host
memory. The reads sit in pinned host batches as a streaming producer emits them
(quality-carrying 64-byte records: the kernels apply MAPQ, base quality, end
distance and ACGT per base, pileup.py:33-88); each push copies its batch on the
copy stream and queues the whole hot path (filter + cell-major grouping + dedup +
CIGAR-walk pileup + strand filter) for the windows its reads complete; mgp_run does
the rest, the per-cell stats, the reference-allele tallies and, for N > 1, their
RCCL all-reduce; the 16-bit count rows go to pinned host memory as their windows
complete. `value` = reads of all ranks x K / the slowest rank's time for K steps.

Beside it (never inside the timed steps), the line carries:
  * device: the same hot path with the inputs already resident in HBM (K x
    mgp_run, results left in HBM) on the 32-byte records whose per-base filter the
    producer resolved (value_device, its stage times and per-kernel rooflines),
    and device_paired on the 64-byte records;
  * pcie_pack32: the streamed step on 32-byte records, and a batch-size sweep;
  * sample_check: 3 samples of 8 whole cells of the timed runs, bit for bit
    against the oracle on exactly their reads (cells are independent);
  * host_pack: the producer's cost of the 32-byte records;
  * cpu_baseline (N = 1 only): the single-threaded C port of the reference's
    path on a bounded sample of the same generator;
  * e2e (N = 1 only): the product end to end on a bounded BAM (20M reads x 1000
    cells, BGZF level 6): MtDNAPipeline.run to txt (gzip 9) and to HDF5, wall time
    with BAM ingest and writers separately.

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
from types import SimpleNamespace

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "chrM reads piled-up/sec (whole node) at 200M reads × 10k cells; bit-exact counts"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PCIE_PEAK_GBS = 63.0  # MI355X_MICROARCH.md: host link PCIe Gen5 x16, 63 GB/s (spec) per direction
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
    ap.add_argument("--no-check", action="store_true", help="skip the bit-exact sample checks")
    ap.add_argument("--layout", choices=["packed", "pack32"], default="packed",
                    help="records of the headline (streamed, PCIe-inclusive) step: quality-carrying 64-byte records "
                         "the kernel filters per base (packed, default) or 32-byte records the producer made for "
                         "the run's min_baseq (pack32); dense in BAM order")
    ap.add_argument("--rows", choices=["8", "16"], default="8",
                    help="streamed step's rows target: 8 = the 8-bit target beside the 16-bit one (ABI 7), "
                         "16 = the 16-bit target alone")
    ap.add_argument("--columns", choices=["16", "32"], default="16",
                    help="barcode index and |tlen| columns of the streamed batches: 16-bit (mgp_push_batch16, when "
                         "the cells and every |tlen| fit) or the 32-bit mgp_batch columns")
    ap.add_argument("--device-only", action="store_true",
                    help="no streamed headline: the HBM-resident device leg is the line (kernel A/B runs)")
    ap.add_argument("--no-device", action="store_true", help="skip the HBM-resident device leg (--record-layout)")
    ap.add_argument("--no-pcie", action="store_true",
                    help="skip the extra streamed legs (32-byte records, batch-size sweep)")
    ap.add_argument("--no-device-paired", action="store_true",
                    help="skip the resident device leg on quality-carrying 64-byte records")
    ap.add_argument("--no-host-pack", action="store_true", help="skip timing the host's 32-byte record build")
    ap.add_argument("--no-numa-bind", action="store_true", help="do not move the rank to its GPU's NUMA node")
    ap.add_argument("--pcie-steps", type=int, default=3)
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end leg (BAM -> txt / HDF5 files)")
    ap.add_argument("--e2e-reads", type=int, default=20_000_000,
                    help="reads of the end-to-end leg's synthetic BAM (C4's 20k reads per cell at the default)")
    ap.add_argument("--e2e-cells", type=int, default=1000)
    ap.add_argument("--batch-reads", type=str, default="auto",
                    help="reads per pushed batch of the streamed legs (auto: the rank's reads / 12.5, about one "
                         "position window per batch: 16M at C4 on one GPU, 2M per rank on 8); a comma list also "
                         "sweeps the headline layout (untimed extra; the first is the headline's)")
    ap.add_argument("--record-layout", choices=["quad32", "pack32", "paired", "packed", "full"], default="quad32",
                    help="records of the HBM-resident device leg: 32-byte records made for the run's min_baseq, "
                         "four consecutive records of a cell per 128-byte line (quad32, default: the placement of "
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


def numa_bind(device: int) -> str | None:
    """Run this rank on the CPUs of its GPU's NUMA node (before any pinned host
    memory is allocated, so its pages land on that node): the streamed legs move
    every read across the host link, and on a multi-socket node a batch read from
    the other socket's memory crosses the socket link first. Best effort: the
    node's CPUs intersected with the ones allowed; nothing is changed when the
    PCI topology is unknown."""
    import ctypes as C

    try:
        hip = C.CDLL("libamdhip64.so")
        bus = C.create_string_buffer(64)
        if hip.hipDeviceGetPCIBusId(bus, 64, int(device)) != 0:
            return None
        bdf = bus.value.decode().lower()
        node = int(Path(f"/sys/bus/pci/devices/{bdf}/numa_node").read_text().strip())
        if node < 0:
            return None
        cpus = set()
        for part in Path(f"/sys/devices/system/node/node{node}/cpulist").read_text().strip().split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        if not cpus:
            return None
        os.sched_setaffinity(0, cpus)
        return f"node {node} ({len(cpus)} cpus) for GPU {bdf}"
    except Exception:
        return None


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_workers(args.gpus, [sys.executable, str(Path(__file__).resolve()), *sys.argv[1:]]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE {world}: running {world} ranks", file=sys.stderr)
    if args.read_len > 50:
        raise SystemExit("the packed record layouts need --read-len <= 50")
    dist = None
    if world > 1:
        import torch.distributed as tdist

        tdist.init_process_group("gloo", rank=rank, world_size=world)
        dist = tdist

    from mgatk2_amd.engine import EngineConfig
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
    numa = None if args.no_numa_bind else numa_bind(device)
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

    # MGP_BENCH_NO_COMM=1: rehearse the multi-process path with several ranks on one
    # GPU (RCCL refuses two ranks on one device); the tallies are then not reduced
    def make_comm(e):
        from mgatk2_amd.engine import Engine

        uid = Engine.comm_unique_id() if rank == 0 else b"\0" * 128
        obj = [uid]
        dist.broadcast_object_list(obj, src=0)
        e.comm_init(obj[0], world, rank)

    comm = make_comm if world > 1 and not no_comm else None
    comm_ranks = world if comm is not None else 1
    ctx = Ctx(args, cfg, seed, cdf, ref, shard, device, comm, barrier, reduce, rank, world, lo)

    # the headline: SURVEY.md §8(d)'s engine metric, timed over K whole passes of the
    # hot path from the first SoA batch's H2D to every count row and per-cell
    # statistic in pinned host memory, on the quality-carrying 64-byte records (the
    # kernels apply MAPQ, base quality, end distance and ACGT per base)
    head = None
    if not args.device_only:
        head = stream_leg(ctx, args.layout, batch_sizes(args.batch_reads)[:1], timed=True)
    # the same hot path with the inputs already resident in HBM (the device's own rate),
    # on the 32-byte records whose per-base filter the producer resolved (value_device)
    # and on the 64-byte records the kernel filters (device_paired)
    dev = None
    if not args.no_device:
        dev = device_leg(ctx, args.record_layout)
    paired = None
    if not args.device_only and not args.no_device_paired and args.record_layout != "paired":
        paired = device_leg(ctx, "paired")
    host_pack = None
    if rank == 0 and not args.no_host_pack:
        host_pack = host_pack_leg(args, cfg, device)
    # the streamed leg on the 32-byte records and the batch-size sweep (untimed extras)
    pcie_more = None
    if not args.no_pcie:
        sweep = batch_sizes(args.batch_reads)
        pcie_more = stream_leg(ctx, "pack32", sweep[:1], timed=False)
        if len(sweep) > 1 and not args.device_only:
            pcie_more["sweep_" + args.layout] = stream_leg(ctx, args.layout, sweep, timed=False)["legs"]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, cfg, local_rank)

    e2e = None
    if rank == 0 and world == 1 and not args.no_e2e and not args.device_only:
        e2e = e2e_leg(args)

    if rank == 0:
        main_leg = head if head is not None else dev
        ms_step = main_leg["ms_per_step"]
        workload = (f"{workload_name(n_glob, nc_glob)}: {n_glob / 1e6:g}M chrM reads x {nc_glob / 1e3:g}k "
                    f"cells{' per GPU' if args.weak else ' (one set, split by cell over the GPUs)'}, "
                    f"run params (q20, mapq30, dedup=alignment_and_fragment_length, min_reads 1), "
                    f"L={args.read_len}")
        if head is not None:
            workload += (f"; one step = {head['batches']} pinned host batches of {head['batch_reads'] / 1e6:g}M "
                         f"reads streamed H2D -> streamed hot path -> count rows + per-cell stats in pinned host "
                         f"memory")
        out = {
            "metric": METRIC,
            "value": main_leg["value"],
            "unit": "reads/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak" if args.weak else "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (SURVEY.md §8(d) generator, created in HBM by the device generator; for the streamed "
                    "step copied into pinned host batches before the timed region)",
            "bit_exact": None if main_leg.get("sample_check") is None else main_leg["sample_check"]["bit_exact"],
            "config": {
                "workload": workload,
                "timed_region": main_leg["timed_region"],
                "reads_rank0": main_leg["reads_rank0"],
                "cells_rank0": n_cells,
                "record_layout": main_leg["record_layout"],
                "parallelism": f"cell-sharded x{world} (RCCL all-reduce of ref tallies over {comm_ranks} ranks)",
                "rank0_step_ms": main_leg["rank0_step_ms"],
                "numa": numa,
            },
            "roofline": main_leg["roofline"],
            "stage_ms": main_leg.get("stage_ms"),
            "value_pcie": None if head is None else head["value"],
            "value_device": None if dev is None else dev["value"],
            "device_ms_quad32": None if dev is None else dev["ms_per_step"],
            "device_ms_paired": None if paired is None else paired["ms_per_step"],
            "link": None if head is None else head["link"],
            "stream": None if head is None else {k: head[k] for k in ("batch_reads", "batches", "columns", "segments_per_run",
                                                                     "pileup_launches_per_run", "h2d_bytes_rank0",
                                                                     "d2h_bytes_rank0", "rows_target", "rows",
                                                                     "rows8_windows_frac")},
            "device": dev,
            "device_paired": paired,
            "pcie_pack32": pcie_more,
            "host_pack_ns_per_read": None if host_pack is None else host_pack["ns_per_read_1thread"],
            "host_pack": host_pack,
            "cpu_baseline": cpu,
            "e2e": e2e,
            "stats_rank0": main_leg.get("stats"),
            "sample_check": main_leg.get("sample_check"),
            "stream_kernels": None if head is None else stream_kernels(head["reads_rank0"], n_cells),
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def e2e_leg(args) -> dict:
    """The product end to end on a bounded sample ("also report end-to-end
    wall time including BAM decode and writers separately"): a coordinate-sorted BAM
    (BGZF level 6) of --e2e-reads reads over --e2e-cells cells (the device generator, C4's
    reads per cell at the defaults; written before anything is timed), then
    ``MtDNAPipeline.run`` streamed, once with txt output at the reference's gzip level 9
    and once with HDF5: wall time, BAM ingest, writers. Full-size C4 runs come from
    scripts/e2e_bench.py."""
    import shutil
    import tempfile

    sys.path.insert(0, str(Path(__file__).resolve().parent / "scripts"))
    from e2e_bench import run_e2e

    from mgatk2_amd.bam import host_threads

    out = tempfile.mkdtemp(prefix="mgp_bench_e2e_", dir="/tmp")
    try:
        t = time.time()
        res = run_e2e(args.e2e_reads, args.e2e_cells, host_threads(), out, formats=("txt", "hdf5"),
                      modes=("stream",), gzip_levels=("9",))
        res["leg_seconds"] = round(time.time() - t, 1)
    finally:
        shutil.rmtree(out, ignore_errors=True)
    res["what"] = ("wall = MtDNAPipeline.run (BAM open -> streamed decode + engine -> files closed); bam_ingest = "
                   "the streamed decode, engine work under it; write = writers after the last batch; "
                   "reads_per_s_end_to_end = reads / wall")
    return res


def batch_sizes(spec: str) -> list:
    """--batch-reads: a comma list of read counts or 'auto' (resolved per rank by
    stream_leg from its read count)."""
    return [x.strip() if x.strip() == "auto" else int(x) for x in str(spec).split(",") if x.strip()]


class Ctx:
    """What every leg of one rank needs."""

    def __init__(self, args, cfg, seed, cdf, ref, shard, device, comm, barrier, reduce, rank, world, cell0):
        self.args, self.cfg, self.seed, self.cdf, self.ref, self.shard = args, cfg, seed, cdf, ref, shard
        self.device, self.comm, self.barrier, self.reduce = device, comm, barrier, reduce
        self.rank, self.world, self.cell0 = rank, world, cell0


def pmc_traffic(key: str, n: int, nc: int, layout: str) -> dict | None:
    """The pileup's PMC traffic for this workload (profiles/pmc_traffic*.json, from
    scripts/pmc_traffic.py: 2 x FETCH_SIZE + WRITE_SIZE per launch, gfx950 correction)."""
    f = ROOT / "profiles" / ("pmc_traffic.json" if key == "device" else f"pmc_traffic_{key}.json")
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        if d.get("reads") == n and d.get("cells") == nc and d.get("record_layout") == layout:
            return d
    except Exception:
        pass
    return None


def stream_kernels(n: int, nc: int) -> dict | None:
    """The streamed step's per-kernel GPU time (profiles/stream_kernels.json, from
    scripts/stream_kernels.py over a rocprofv3 --stats run of this step: every kernel's
    calls and ms per step, pairing / check / grouping / pileup / rows), when it is of
    this workload."""
    f = ROOT / "profiles" / "stream_kernels.json"
    try:
        d = json.loads(f.read_text())
        if d.get("reads") == n and d.get("cells") == nc:
            return d
    except (OSError, ValueError):
        pass
    return None


def device_leg(ctx: Ctx, layout: str) -> dict:
    """The hot path with its inputs resident in HBM: K runs of mgp_run (untimed
    generation on the device), ms per step (max over ranks), the stage times, the
    per-kernel rooflines and, on rank 0, the bit-exact sample check."""
    from mgatk2_amd.bam import PLACE_PAIRED, place_records
    from mgatk2_amd.engine import Engine

    args, cfg = ctx.args, ctx.cfg
    eng = Engine(cfg, device=ctx.device)
    packed = layout in ("packed", "paired", "pack32", "quad32")
    p32 = cfg.min_baseq if layout in ("pack32", "quad32") else None  # 32-byte records for the run's min_baseq
    t0 = time.time()
    eng.synth(ctx.seed, args.reads, ctx.cdf, ctx.ref, read_len=args.read_len, rec_align=64 if packed else 128,
              pack=packed, pack32=p32, **ctx.shard)
    n_res, pay = eng.resident()
    if layout in ("paired", "quad32"):
        # the producer's placement (mgp_place_records, as the BAM decoder emits it):
        # computed on the host from the generated barcode and flag columns, then the
        # same reads are generated again at those offsets
        soa = eng.download_inputs(columns=("bc", "flag", "start", "tlen"))
        roff, pay_b = place_records(soa.bc, soa.flag, np.full(n_res, 32 if p32 is not None else 64, np.uint32),
                                    cfg.n_cells, PLACE_PAIRED, start=soa.start, tlen=soa.tlen)
        del soa
        eng.synth(ctx.seed, args.reads, ctx.cdf, ctx.ref, read_len=args.read_len, rec_align=64, pack=True,
                  rec_off=roff, payload_bytes=pay_b, pack32=p32, **ctx.shard)
        del roff
    n_res, pay = eng.resident()
    print(f"[bench] rank {ctx.rank}: device leg {layout}: {n_res:,} reads ({pay / 1e9:.2f} GB payload) generated "
          f"on device {ctx.device} in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    if ctx.comm is not None:
        ctx.comm(eng)
    # the timed runs bracket only the pileup with HIP events (its roofline); every
    # other stage boundary would add a marker between two kernels of the stream
    eng.set_stage_timing(os.environ.get("MGP_BENCH_ALL_STAGES") == "1")  # (=1: every stage timed, for A/B)
    for _ in range(max(1, args.warmup)):
        eng.run()
    eng.sync()
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.run()
    eng.sync()
    ctx.barrier()
    dt_rank = time.perf_counter() - t0
    dt = ctx.reduce(dt_rank, "max")
    kt = eng.kernel_times(last_runs=min(args.steps, 64))
    # the per-stage breakdown from a few more (untimed) runs with every stage bracketed
    eng.set_stage_timing(True)
    for _ in range(3):
        eng.run()
    eng.sync()
    kt_all = eng.kernel_times(last_runs=3)
    res = eng.fetch(dense=False)
    nc = cfg.n_cells
    # roofline of the dominant kernel: its own algorithmic bytes per launch over its
    # HIP-event time on the compute stream, averaged over the timed steps; the whole
    # step against SURVEY.md §8(d)'s engine-level count is step_achieved / step_frac
    dom = "pileup"
    alg = kernel_bytes(n_res, nc, res.stats, cfg, layout)[dom]
    achieved = alg / (kt[dom] * 1e-3) / 1e9
    engine_bytes = n_res * BYTES_PER_READ + nc * BYTES_PER_CELL
    step_achieved = engine_bytes / (dt_rank / args.steps) / 1e9
    pmc = pmc_traffic("device", n_res, nc, layout)
    check = None
    if ctx.rank == 0 and not args.no_check:
        check = sample_check(eng, cfg, res, args, ctx.seed, ctx.cdf, ctx.ref, ctx.cell0, ctx.device)
    eng.close()
    return {
        "record_layout": layout,
        "what": {"quad32": "32-byte records made for the run's min_baseq (per-base filter resolved by the producer), "
                           "four of a cell per 128-byte line",
                 "paired": "packed 64-byte records (qualities and base codes; the kernel applies min_baseq, "
                           "min_distance_from_end and ACGT per base), two of a cell per 128-byte line"}.get(layout, layout),
        "timed_region": "K x mgp_run on inputs resident in HBM (results left in HBM)",
        "value": ctx.reduce(float(n_res), "sum") * args.steps / dt,
        "ms_per_step": dt / args.steps * 1e3,
        "rank0_step_ms": dt_rank / args.steps * 1e3,
        "reads_rank0": n_res,
        "payload_bytes_rank0": pay,
        "stage_ms": {k: round(v, 4) for k, v in kt_all.items()},
        "roofline": {
            "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": None if pmc is None else pmc.get(dom),
            "alg_bytes_per_launch": alg, "launches_per_step": 1, "avg_launch_ms": kt[dom],
            "alg_bytes_what": f"4-byte pileup element + one {RECORD_BYTES[layout]}-byte record per kept read, "
                              f"16-bit result rows ({ROW16_BYTES_PER_CELL} B) per cell",
            "engine_alg_bytes_per_step": engine_bytes, "step_achieved": step_achieved,
            "step_frac": step_achieved / HBM_PEAK_GBS,
            "kernels": kernel_rooflines(kt_all, n_res, nc, res.stats, cfg, layout),
        },
        "stats": res.stats,
        "filtered_reads_rank0": res.stats["filtered_reads"],
        "error_bits": res.stats["error_bits"],
        "sample_check": check,
    }


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
    # the threaded rate: best of 3 (a run of ~40 ms on the box's 16-CPU share of a
    # 256-CPU host is shorter than a scheduler quota period: one throttled period, or a
    # neighbour's burst, once made it read slower than one thread, round 4)
    nt = host_threads()
    tn = float("inf")
    for _ in range(3):
        t0 = time.perf_counter()
        repack32(soa, cfg.min_baseq, cfg.min_distance_from_end, nt, out32, oflag)
        tn = min(tn, time.perf_counter() - t0)
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


def sample_check(eng, cfg, res, args, seed, cdf, ref, cell0: int, device: int, delivered=None) -> dict:
    """3 samples of 8 whole cells of the timed run (first, middle, last cells of the
    rank) bit for bit against the oracle on exactly their reads, plus the run
    statistics' consistency. Cells are independent, so a cell's rows depend only
    on its own reads. The oracle reads the quality-carrying full 128-byte records of
    those reads (regenerated as a cell shard of the same seed): with 32-byte records
    the per-base filter (pileup.py:67-88) was resolved by the producer, and this
    checks that too. delivered (a StreamSet): the rows compared are the ones the
    timed step left in pinned host memory (the bytes that crossed the link) and the
    per-cell statistics are the step's own `res`; otherwise (results left in HBM)
    they are fetched from the device."""
    from mgatk2_amd.engine import Engine, EngineConfig
    from oracle.oracle import oracle_run

    t0 = time.perf_counter()
    nc = cfg.n_cells
    ranges = sorted({(0, min(8, nc)), (nc // 2, min(nc, nc // 2 + 8)), (max(0, nc - 8), nc)})
    if delivered is not None:
        per_cell = ("n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max", "median_lo", "median_hi")
        got = {}
        for lo, hi in ranges:
            d = delivered.cells(lo, hi)
            for k in per_cell:
                d[k] = getattr(res, k)[lo:hi]
            got[(lo, hi)] = SimpleNamespace(**d)
    else:
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
            "sampled cells' reads", "checked": ("the timed step's pinned host rows and per-cell statistics"
                                                if delivered is not None else "rows fetched from the device"),
            "wide_cells": None if delivered is None else len(delivered.exact),
            "windows_from_rows8": (None if delivered is None or delivered.rows8 is None else
                                   sum(int(delivered.rows8.narrow[lo:hi].sum()) for lo, hi in ranges)),
            "windows_checked": None if delivered is None else sum((hi - lo) * delivered.nw for lo, hi in ranges),
            "seconds": round(time.perf_counter() - t0, 2)}


class StreamSet:
    """The producer's side of the streamed step (shared with the full-size GPU test
    of this exact path, tests/test_gpu_stream.py): the engine's resident reads copied
    into pinned host memory as dense records in BAM order (a batch is a contiguous
    payload range), with 16-bit barcode and |tlen| columns (mgp_push_batch16, ABI 5)
    when every read allows, and the pinned 16-bit count rows the engine writes as its
    windows complete (mgp_set_rows16_target), with the 8-bit target beside them
    (mgp_set_rows_target, ABI 7: a (cell, window) whose values all fit a byte leaves as
    half the bytes) unless rows8 is off."""

    def __init__(self, eng, cfg, layout: str, columns16: bool = True, rows8: bool = True):
        from mgatk2_amd.engine import PinnedBuffer, Rows8, Rows16

        self.eng, self.cfg, self.layout = eng, cfg, layout
        self.rb = 32 if layout == "pack32" else 64  # dense records in BAM order
        n, pay = eng.resident()
        self.n, self.pay = n, pay
        # the producer's columns: bc, tlen, flag, mapq. No rec_off (dense records in BAM
        # order) and no span (taken from the records' CIGARs on the device): ABI v3.1; no
        # start (taken from the records, which all hold it): ABI 4
        cols = ("bc", "tlen", "flag", "mapq", "payload")
        # 16-bit barcode and |tlen| columns when every read allows: 7 bytes of columns
        # per read over the link instead of 11
        wide = None
        if columns16 and cfg.n_cells <= 0xFFFF:
            wide = eng.download_inputs(columns=("bc", "tlen"))
            if not np.abs(wide.tlen.astype(np.int64)).max(initial=0) < 0xFFFF:
                wide = None
        self.narrow = wide is not None
        self.col_bytes = n * ((2 + 2) if self.narrow else (4 + 4)) + n * (2 + 1)
        self.hbuf = PinnedBuffer(self.col_bytes + pay + 4096)
        off = [0]

        def alloc(m, dt):
            a = self.hbuf.array(m, dt, off[0])
            off[0] = (off[0] + m * np.dtype(dt).itemsize + 63) & ~63
            return a

        if self.narrow:  # (bc and tlen through host memory, then their 16-bit forms into the pinned batches)
            host = eng.download_inputs(columns=("flag", "mapq", "payload"), alloc=alloc)
            host.bc, host.tlen = alloc(n, np.uint16), alloc(n, np.uint16)
            np.copyto(host.bc, np.where(wide.bc < 0, 0xFFFF, wide.bc).astype(np.uint16))
            np.copyto(host.tlen, np.abs(wide.tlen).astype(np.uint16))
            del wide
        else:
            host = eng.download_inputs(columns=cols, alloc=alloc)  # the producer's batches: pinned, BAM order
        assert np.all(eng.download_inputs(columns=("rec_off",)).rec_off == self.rb * np.arange(n, dtype=np.uint64))
        self.host = host
        L, nc = cfg.mito_len, cfg.n_cells
        nw, W = eng.windows()
        self.nw = nw
        o8 = (nc * L * 22 + nc * nw + 4095) & ~4095  # the 8-bit target after the 16-bit one
        self.rbuf = PinnedBuffer(o8 + (nc * L * 11 + nc * nw if rows8 else 0) + 4096)
        rbuf = self.rbuf
        self.rows = Rows16(rbuf.array((nc, L, 8), np.uint16, 0), rbuf.array((nc, L, 2), np.uint16, nc * L * 16),
                           rbuf.array((nc, L), np.uint16, nc * L * 20), rbuf.array((nc, nw), np.uint8, nc * L * 22), W)
        self.rows8 = Rows8(rbuf.array((nc, L, 8), np.uint8, o8), rbuf.array((nc, L, 2), np.uint8, o8 + nc * L * 8),
                           rbuf.array((nc, L), np.uint8, o8 + nc * L * 10),
                           rbuf.array((nc, nw), np.uint8, o8 + nc * L * 11)) if rows8 else None
        # the rows leave the device as the windows complete, beside the later batches' H2D
        # (MGP_BENCH_ABL_NO_ROWS=1, an A/B only: the rows stay on the device, no D2H)
        self.abl_no_rows = os.environ.get("MGP_BENCH_ABL_NO_ROWS") == "1"
        try:
            if not self.abl_no_rows:
                eng.set_rows_target(self.rows, self.rows8)
            self.rows_target = True
        except Exception as e:  # (pinned memory the device cannot map: copy the rows after the run)
            print(f"[bench] rows target unavailable ({e}); rows fetched after the run", file=sys.stderr)
            self.rows_target = False
        self.h2d = self.col_bytes + pay
        self.d2h = nc * L * 22 + nc * nw + nc * 34 + L * 4 * 8  # rows, wide flags, per-cell arrays, tallies
        # (with the 8-bit target: d2h_bytes() after a step, from the narrow flags)
        self.exact = {}  # cell -> its exact u32 rows (EngineResult of one cell) when a window of it is wide

    def auto_batch(self, b) -> int:
        """'auto': about one position window of reads per batch (the windows a push
        completes run while the next batch is copied)."""
        return max(1_000_000, int(round(self.n / 12.5 / 1e6)) * 1_000_000) if b == "auto" else int(b)

    def batches(self, bs: int) -> list:
        """Batches of bs reads: their columns and their slice of the dense payload."""
        from mgatk2_amd.synth import ReadSoA

        h, rb, n = self.host, self.rb, self.n
        return [ReadSoA(None, h.bc[a:b], h.tlen[a:b], h.flag[a:b], h.mapq[a:b], None, None, h.payload[rb * a:rb * b])
                for a, b in ((a, min(n, a + bs)) for a in range(0, n, bs))]

    def step(self, batches, stream: bool = True):
        """One pass: reset -> push every batch -> mgp_run -> the count rows and per-cell
        statistics in host memory. A cell with a drained window (more than 65535
        elements: its pinned 16-bit rows saturate) gets its exact u32 rows fetched here,
        inside the step (self.exact)."""
        eng = self.eng
        eng.set_streaming(stream)
        eng.reset()
        for bt in batches:
            eng.push(bt)
        eng.run()
        if not self.rows_target:
            eng.fetch_rows16(0, self.cfg.n_cells, out=self.rows)
            if self.rows8 is not None:
                self.rows8.narrow.fill(0)
        res = eng.fetch(dense=False)  # (waits for the rows' copies too)
        self.exact = {}
        if self.rows.wide.any():
            for c in self.rows.wide_cells():
                self.exact[int(c)] = eng.fetch_cells(int(c), int(c) + 1)
        return res

    def cells(self, lo: int, hi: int) -> dict:
        """Cells [lo, hi) as the step delivered them to host memory: the pinned 16-bit
        rows widened to u32 (exact: no wide window), or the exact rows fetched for a
        cell with a wide window."""
        from mgatk2_amd.engine import merge_rows

        out = merge_rows(self.rows, self.rows8, lo, hi)
        for c, e in self.exact.items():
            if lo <= c < hi:
                for k in out:
                    out[k][c - lo] = getattr(e, k)[0]
        return out

    def rows16(self, lo: int, hi: int):
        """Cells [lo, hi) as one 16-bit Rows16 (copies: the 8-bit target's windows
        widened into the 16-bit rows), the form mgp_fetch_rows16 gives."""
        from mgatk2_amd.engine import Rows16, merge_rows

        m = merge_rows(self.rows, self.rows8, lo, hi)
        return Rows16(m["counts"].astype(np.uint16), m["tn5"].astype(np.uint16), m["depth"].astype(np.uint16),
                      self.rows.wide[lo:hi].copy(), self.rows.window_width)

    def d2h_bytes(self) -> int:
        """Bytes of the last step's results to host memory: 22 per position of a 16-bit
        window, 11 of an 8-bit one, the flags, per-cell arrays and tallies."""
        nc, L = self.cfg.n_cells, self.cfg.mito_len
        if self.rows8 is None:
            return self.d2h
        W = self.rows.window_width
        wl = np.minimum(W, L - W * np.arange(self.nw))  # positions per window
        narrow_pos = int((self.rows8.narrow.astype(np.int64) * wl).sum())
        return self.d2h - 11 * narrow_pos + nc * self.nw


def stream_leg(ctx: Ctx, layout: str, batch_list: list, timed: bool) -> dict:
    """SURVEY.md §8(d)'s engine metric: the rank's reads in pinned host SoA batches
    (dense records in BAM order, as a streaming producer emits them: a batch is a
    contiguous payload range) -> pushed (H2D on the copy stream; with streaming on,
    each push runs the whole hot path for the windows its reads complete, overlapping
    the next batches' copies) -> mgp_run -> the 16-bit count rows (written into the
    pinned target as windows complete) and the per-cell statistics in pinned host
    memory. timed: the bench's step (W warmup passes, K timed passes bracketed by
    barrier + device sync, max over ranks), with the pileup's HIP events (every
    segment's launch) for the roofline and the bit-exact sample check of the rows the
    timed step left in host memory; otherwise the best of --pcie-steps passes per
    batch size, streamed and not."""
    from mgatk2_amd.engine import Engine

    args, cfg = ctx.args, ctx.cfg
    eng = Engine(cfg, device=ctx.device)
    p32 = cfg.min_baseq if layout == "pack32" else None
    t0 = time.time()
    eng.synth(ctx.seed, args.reads, ctx.cdf, ctx.ref, read_len=args.read_len, rec_align=64, pack=True, pack32=p32,
              **ctx.shard)
    ss = StreamSet(eng, cfg, layout, columns16=args.columns == "16", rows8=args.rows == "8")
    n, rb, narrow, rows_target = ss.n, ss.rb, ss.narrow, ss.rows_target
    L, nc = cfg.mito_len, cfg.n_cells
    print(f"[bench] rank {ctx.rank}: stream leg {layout}: {n:,} reads ({ss.h2d / 1e9:.2f} GB pinned) "
          f"ready in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    if ctx.comm is not None:
        ctx.comm(eng)  # every run all-reduces its tallies
    eng.set_stage_timing(False)  # HIP events around the pileup launches only
    batch_list = [ss.auto_batch(b) for b in batch_list]
    h2d, d2h = ss.h2d, ss.d2h
    if not timed:
        legs = []
        for bs in batch_list:
            batches = ss.batches(bs)
            ss.step(batches, True)  # warmup (allocations)
            for stream in (True, False):
                ts = []
                seg0 = eng.stream_info()[0]
                for _ in range(args.pcie_steps):
                    ctx.barrier()
                    t1 = time.perf_counter()
                    r = ss.step(batches, stream)
                    ts.append(time.perf_counter() - t1)
                segs = (eng.stream_info()[0] - seg0) // max(1, args.pcie_steps)
                dt_max = ctx.reduce(min(ts), "max")
                legs.append({"batch_reads": bs, "batches": len(batches), "streamed": stream, "segments": int(segs),
                             "s": dt_max, "value": ctx.reduce(float(n), "sum") / dt_max})
        d2h = ss.d2h_bytes()
        eng.close()
        best = max((lg for lg in legs if lg["streamed"]), key=lambda lg: lg["value"])
        return {"record_layout": layout, "value": best["value"], "best_batch_reads": best["batch_reads"],
                "columns_bytes_per_read": 7 if narrow else 11,
                "h2d_bytes_rank0": h2d, "d2h_bytes_rank0": d2h,
                "link_GBps_rank0": round((h2d + d2h) / best["s"] / 1e9, 2), "legs": legs,
                "stats_total_reads_rank0": r.stats["total_reads"]}

    bs = batch_list[0]
    batches = ss.batches(bs)
    for _ in range(max(1, args.warmup)):
        ss.step(batches, True)
    seg0 = eng.stream_info()[0]
    ctx.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = ss.step(batches, True)
    ctx.barrier()
    dt_rank = time.perf_counter() - t0
    dt = ctx.reduce(dt_rank, "max")
    segs = (eng.stream_info()[0] - seg0) / max(1, args.steps)
    streamed = eng.stream_info()[1]
    kt = eng.kernel_times(last_runs=min(args.steps, 64))
    pile_ms = kt.get("pileup", 0.0)  # per run: every segment's launch + the run's last one
    launches = segs + 1
    dom = "pileup"
    alg = kernel_bytes(n, nc, res.stats, cfg, "packed" if rb == 64 else "pack32")[dom]
    achieved = alg / (pile_ms * 1e-3) / 1e9 if pile_ms > 0 else None
    pmc = pmc_traffic("stream", n, nc, layout)
    step_s = dt_rank / args.steps
    check = None
    if ctx.rank == 0 and not args.no_check:
        check = sample_check(eng, cfg, res, args, ctx.seed, ctx.cdf, ctx.ref, ctx.cell0, ctx.device, delivered=ss)
    wide_cells = len(ss.exact)
    d2h = ss.d2h_bytes()
    narrow_frac = None if ss.rows8 is None else float(ss.rows8.narrow.mean())
    eng.close()
    return {
        "record_layout": layout,
        "what": {"packed": "packed 64-byte records (qualities and base codes: the kernel applies min_baseq, "
                           "min_distance_from_end and ACGT per base), dense in BAM order",
                 "pack32": "32-byte records made for the run's min_baseq (per-base filter resolved by the producer), "
                           "dense in BAM order"}[layout],
        "columns": ("u16 bc (0xFFFF: none), u16 |tlen|, u16 flag, u8 mapq: 7 B per read (mgp_push_batch16)" if narrow
                    else "i32 bc, i32 tlen, u16 flag, u8 mapq: 11 B per read (mgp_push_batch)"),
        "timed_region": "K passes of: reset -> push every pinned host batch (H2D on the copy stream; each push "
                        "queues the hot path of the windows its reads complete) -> mgp_run -> every 16-bit count row "
                        "(written into pinned host memory as its windows complete; the exact u32 rows of any cell "
                        "with a drained window fetched) and the per-cell statistics on the host",
        "value": ctx.reduce(float(n), "sum") * args.steps / dt,
        "ms_per_step": dt / args.steps * 1e3,
        "rank0_step_ms": step_s * 1e3,
        "reads_rank0": n,
        "batch_reads": bs,
        "batches": len(batches),
        "streamed": bool(streamed),
        "segments_per_run": segs,
        "pileup_launches_per_run": launches,
        "h2d_bytes_rank0": h2d,
        "d2h_bytes_rank0": d2h,
        "rows_target": rows_target,
        "rows": ("16-bit rows, and 8-bit rows for the (cell, window) pairs whose values all fit a byte "
                 "(mgp_set_rows_target)" if ss.rows8 is not None else "16-bit rows (mgp_set_rows16_target)"),
        "rows8_windows_frac": narrow_frac,
        "wide_cells": wide_cells,
        "link": {"bound": "pcie", "h2d_GBps": round(h2d / step_s / 1e9, 2), "d2h_GBps": round(d2h / step_s / 1e9, 2),
                 "peak_GBps_per_direction": PCIE_PEAK_GBS, "h2d_frac": round(h2d / step_s / 1e9 / PCIE_PEAK_GBS, 3),
                 "what": "H2D bytes of the step (columns + records) over the step time, rank 0; PCIe Gen5 x16 spec "
                         "(MI355X_MICROARCH.md)"},
        "stage_ms": {"pileup_per_run": round(pile_ms, 4)},
        "roofline": {
            "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": None if achieved is None else achieved / HBM_PEAK_GBS,
            "traffic": None if pmc is None else pmc.get(dom),
            "alg_bytes_per_launch": alg / launches, "launches_per_step": launches,
            "avg_launch_ms": pile_ms / launches,
            "alg_bytes_what": f"per step (all launches): 4-byte pileup element + one {rb}-byte record per kept read, "
                              f"16-bit result rows ({ROW16_BYTES_PER_CELL} B) per cell; per launch = / launches",
            "time_what": "HIP events around every pileup launch of the timed steps (the streaming segments' and the "
                         "run's own), summed per step",
        },
        "stats": res.stats,
        "sample_check": check,
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
        "comparison": "the reference's per-read path restated in C on one core (oracle/mgp_oracle.c): at C4's "
                      "density (> 2500 reads per cell) the reference itself runs its cells sequentially on one "
                      "core (processors.py:96-103), and its Python does ~14k reads/s there (SURVEY.md §6 probe), "
                      "so this port is ~130x the reference's own rate; value / this = the GPU's margin over the "
                      "port, not over the reference",
    }


if __name__ == "__main__":
    main()
