"""Cell processing (mirror of src/processing/processors.py).

The reference dispatches one Python call per cell, sequentially or over a
spawn pool (processors.py:63-144). Here every cell goes through the GPU engine
in one run:

* :meth:`CellProcessor.process_soa` — production path: the whole chrM read set
  (engine SoA, BAM order) in, dedup + pileup + filters + statistics on the GPU,
  results streamed to the writer in first-seen cell order.
* :meth:`CellProcessor.process_cells_progressive` / :func:`process_barcode_worker`
  — the reference's dict API (already-deduplicated ``SimpleRead`` lists per
  barcode). The lists are merged into one coordinate-sorted batch and run with
  dedup off, so each cell sees exactly its own reads.
"""

from __future__ import annotations

import gc
import logging
import time

import numpy as np

from ..engine import Engine, EngineResult
from ..synth import ReadSoA, pack_reads
from .pileup import result_dict, simple_reads_to_dicts

logger = logging.getLogger(__name__)

MP_CONTEXT = "spawn"  # kept for API compatibility (processors.py:17); no process pool is used


def _engine_config_for(config, n_cells: int, dedup: bool):
    ec = config.engine_config(n_cells)
    if not dedup:
        ec.dedup_mode = "none"
    return ec


def run_cells_from_reads(config, reads_by_barcode: dict, device: int = 0) -> tuple[EngineResult, list[str]]:
    """Engine run over already-deduplicated per-barcode read lists."""
    barcodes = list(reads_by_barcode)
    dicts = []
    for i, bc in enumerate(barcodes):
        dicts.extend(simple_reads_to_dicts(reads_by_barcode[bc], bc=i))
    dicts.sort(key=lambda d: d["reference_start"])  # stable: per-cell order is kept
    soa = pack_reads(dicts)
    with Engine(_engine_config_for(config, len(barcodes), dedup=False), device=device) as eng:
        eng.push(soa)
        res = eng.finish()
    return res, barcodes


def process_barcode_worker(args):
    """processors.py:20-55: one barcode's reads -> result dict or None."""
    barcode, reads, config = args
    if not reads or len(reads) < config.min_reads_per_cell:
        return None
    res, _ = run_cells_from_reads(config, {barcode: reads})
    if not res.passed[0]:
        return None
    return result_dict(res, 0, barcode, config.mito_length)


class CellProcessor:
    def __init__(self, config, output_dir, device: int = 0, devices: list[int] | None = None):
        self.config = config
        self.output_dir = output_dir
        self.device = device
        self.devices = list(devices) if devices else [device]
        self.last_result: EngineResult | None = None
        self.last_stats: dict = {}
        self.last_timing: dict = {}

    # production path ------------------------------------------------------
    def run_soa(self, soa_batches, n_cells: int) -> EngineResult:
        """Whole read set (one or more BAM-order batches) through the engine:
        filters, dedup, pileup, strand filter, per-cell statistics, tallies."""
        if isinstance(soa_batches, ReadSoA):
            soa_batches = [soa_batches]
        if len(self.devices) > 1:
            return self._run_sharded(soa_batches, n_cells)
        n = sum(b.n for b in soa_batches)
        pay = sum(int(b.payload.shape[0]) for b in soa_batches)
        ec = self.config.engine_config(n_cells, reserve_reads=n, reserve_payload=pay + 256 * len(soa_batches))
        t0 = time.perf_counter()
        with Engine(ec, device=self.device) as eng:
            t1 = time.perf_counter()
            for b in soa_batches:
                eng.push(b)
            eng.run()
            eng.sync()
            t2 = time.perf_counter()
            res = eng.fetch_compact()  # exact 16-bit rows: half the device-to-host bytes
            t3 = time.perf_counter()
            self.last_stats = eng.kernel_times()
        t4 = time.perf_counter()
        # where the engine leg goes (pipeline timings): context + allocation, H2D of
        # the batches + the run, D2H of the results, teardown
        self.last_timing = {"engine_open": t1 - t0, "engine_h2d_run": t2 - t1, "engine_d2h": t3 - t2,
                            "engine_close": t4 - t3}
        self.last_result = res
        return res

    def _run_sharded(self, soa_batches, n_cells: int) -> EngineResult:
        """Cells split into contiguous read-balanced ranges, one engine per device,
        run concurrently (ctypes releases the GIL); results concatenated along
        cells and tallies summed on the host."""
        from concurrent.futures import ThreadPoolExecutor

        from ..shard import merge_results, partition_cells, reads_per_cell, shard_soa
        from ..synth import concat_soa

        soa = soa_batches[0] if len(soa_batches) == 1 else concat_soa(soa_batches)
        b = partition_cells(reads_per_cell(soa, n_cells), len(self.devices))
        shards = [(int(lo), int(hi)) + shard_soa(soa, int(lo), int(hi)) for lo, hi in zip(b[:-1], b[1:])]

        def one(i):
            lo, hi, sub, idx = shards[i]
            ec = self.config.engine_config(hi - lo, reserve_reads=sub.n, reserve_payload=sub.payload.shape[0] + 256)
            with Engine(ec, device=self.devices[i]) as eng:
                if sub.n:
                    eng.push(sub)
                eng.run()
                return eng.fetch_compact(), lo, hi, idx

        with ThreadPoolExecutor(len(self.devices)) as ex:
            parts = list(ex.map(one, range(len(self.devices))))
        res = merge_results(parts, n_cells, soa.n)
        self.last_result = res
        return res

    def write_results(self, res: EngineResult, barcodes: list[str], incremental_writer=None) -> list[dict]:
        """Passing cells in first-seen order to the writer; returns the reference's
        slim result list ({"barcode", "n_reads"} per written cell, processors.py:75)."""
        order = res.cell_order()
        written = order[res.passed[order].astype(bool)]
        failed = int(order.size - written.size)
        if failed:
            logger.warning(f"{failed} cells failed")
        if incremental_writer is not None:
            incremental_writer.write_cells(res, written, barcodes=barcodes, tally=res.ref_tally)
        return [{"barcode": barcodes[int(c)], "n_reads": int(res.n_reads[c])} for c in written]

    def process_soa(self, soa_batches, barcodes: list[str], incremental_writer=None) -> list[dict]:
        res = self.run_soa(soa_batches, len(barcodes))
        return self.write_results(res, barcodes, incremental_writer)

    # reference dict API (processors.py:63-144) ------------------------------
    def process_cells_direct(self, reads_by_barcode, incremental_writer=None):
        res, barcodes = run_cells_from_reads(self.config, reads_by_barcode, self.device)
        self.last_result = res
        reads_by_barcode.clear()
        results, failed = [], 0
        for c, bc in enumerate(barcodes):
            if not res.passed[c]:
                failed += 1
                continue
            r = result_dict(res, c, bc, self.config.mito_length)
            if incremental_writer:
                incremental_writer.write_cell(r)
                results.append({"barcode": bc, "n_reads": r["n_reads"]})
            else:
                results.append(r)
        if failed > 0:
            logger.warning(f"{failed} cells failed")
        gc.collect()
        return results

    def process_cells_progressive(self, reads_by_barcode, incremental_writer=None):
        n_cells = len(reads_by_barcode)
        total = sum(len(r) for r in reads_by_barcode.values())
        avg = total / n_cells if n_cells > 0 else 0
        logger.info(f"Processing {n_cells} cells at an average of {avg:.0f} reads/cell")
        return self.process_cells_direct(reads_by_barcode, incremental_writer)


def cells_written(res: EngineResult) -> np.ndarray:
    order = res.cell_order()
    return order[res.passed[order].astype(bool)]
