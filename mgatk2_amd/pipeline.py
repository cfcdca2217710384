"""Pipeline orchestration (mirror of src/core/pipeline.py:23-269).

Same entry points as the reference (``MtDNAPipeline(...).run()`` and
``run_pipeline(...)``). The flow is the reference's; the work inside is the
build's:

1. native BAM ingest of the chrM records in batches on a producer thread
   (:meth:`BAMReader.open_stream`), each batch pushed to the GPU as soon as it is
   decoded;
2. one streamed engine run: every position window goes through filters, dedup,
   pileup, strand filter and per-cell statistics as soon as its reads have all
   arrived, and its result rows come back while later batches are still decoded
   (:meth:`CellProcessor.run_stream`; ``stream=False`` or ``MGP_STREAM=0``: the whole
   set decoded first, then one run, :meth:`CellProcessor.run_soa`);
3. the writers format the passing cells, in first-seen order, from the
   engine's arrays;
4. ``qc/summary.txt`` and, for HDF5 output, the HTML report.

``self.timings`` records the wall time of each stage (seconds).
"""

from __future__ import annotations

import gc
import logging
import os
import threading
import time
from pathlib import Path
from typing import Any

from .analysis.qc import QCCalculator
from .bam import BamFile
from .config import PipelineConfig
from .exceptions import InvalidInputError
from .file_io import IncrementalHDF5Writer, IncrementalTextWriter, write_run_summary
from .processing.processors import CellProcessor
from .processing.readers import MITO_NAMES, BAMReader

logger = logging.getLogger(__name__)


def _release_in_background(box: list) -> None:
    """Drop the objects in `box` (holding their last references) on a daemon thread:
    their native free releases the GIL, so the unmapping overlaps the caller's next
    stage."""
    import threading

    threading.Thread(target=box.clear, name="mgp-free-inputs", daemon=True).start()


class _Background:
    """fn(*args) on a thread; result() joins and returns its value or raises its error."""

    def __init__(self, fn, *args):
        self._out = self._err = None
        self._t = threading.Thread(target=self._run, args=(fn, args), name="mgp-report-plots", daemon=True)
        self._t.start()

    def _run(self, fn, args):
        try:
            self._out = fn(*args)
        except BaseException as e:  # handed to result()
            self._err = e

    def result(self):
        self._t.join()
        if self._err is not None:
            raise self._err
        return self._out


class MtDNAPipeline:
    """Single-pass mtDNA genotyping pipeline (pipeline.py:23-74)."""

    def __init__(
        self,
        bam_path: str,
        barcodes: list[str],
        output_dir: Path,
        config: PipelineConfig | None = None,
        output_format: str = "standard",
        barcode_metadata=None,
        sample_name: str = "mgatk2",
        report_title: str | None = None,
        report_subtitle: str | None = None,
        working_directory: str | None = None,
        device: int = 0,
        devices: list[int] | None = None,
        stream: bool | None = None,
    ):
        self.bam_path = Path(bam_path)
        # streamed ingest (default; MGP_STREAM=0 decodes the whole chrM set first)
        self.stream = (os.environ.get("MGP_STREAM", "1") != "0") if stream is None else bool(stream)
        self.barcodes = set(barcodes)
        self.barcode_list = list(barcodes)
        self.output_dir = Path(output_dir)
        self.config = config or PipelineConfig()
        self.output_format = output_format.lower()
        self.barcode_metadata = barcode_metadata
        self.sample_name = sample_name
        self.report_title = report_title or sample_name
        self.report_subtitle = report_subtitle or "mgatk2 output analysis"
        self.working_directory = working_directory
        self.device = device
        self.devices = list(devices) if devices else [device]
        self.timings: dict[str, float] = {}
        self.engine_result = None
        self.read_stats: dict = {}

        if not self.bam_path.exists():
            raise InvalidInputError(f"BAM file not found: {bam_path}")
        with BamFile(self.bam_path) as bam:
            refs = list(bam.references)
        if self.config.mito_chr not in refs:
            for alt in MITO_NAMES:
                if alt in refs:
                    logger.warning(f"Using '{alt}' instead of '{self.config.mito_chr}'")
                    self.config.mito_chr = alt
                    break
            else:
                raise InvalidInputError(
                    f"Mitochondrial chromosome '{self.config.mito_chr}' not found. Available: {', '.join(refs[:10])}"
                )
        self.output_dir.mkdir(parents=True, exist_ok=True)

    def _render_plots(self, arrays):
        from .analysis.report import render_plots

        return render_plots(arrays, scatac=self.barcode_metadata is not None)

    def run(self) -> dict[str, Any]:
        t0 = time.time()
        if self.output_format == "hdf5":
            # the report's pyplot import and package listing, under the decode
            try:
                from .analysis.report import prewarm

                prewarm()
            except ImportError:  # pragma: no cover
                pass
        logger.info("Collecting reads from BAM by barcode...")
        reader = BAMReader(str(self.bam_path), self.config, self.barcode_list)
        processor = CellProcessor(self.config, self.output_dir, device=self.device, devices=self.devices)
        txt_writer = None
        if self.output_format != "hdf5":
            # the count files are written from the devices' rows at the end of the run
            # (mgp_txt_gz): the writer's files exist before it
            txt_writer = IncrementalTextWriter(self.output_dir, self.config, self.barcode_list)
            processor.enable_device_txt(txt_writer.prefix, self.barcode_list)
        else:
            # the HDF5 chunks are deflated on the device at the end of the run (mgp_h5_tiles)
            processor.enable_device_h5(self.barcode_list)
        if self.stream:
            # one pass: batches decoded on a producer thread, each pushed to the device as
            # it is ready, the windows piled as their reads arrive (readers.py:84-93)
            res = processor.run_stream(reader, len(self.barcode_list))
            stats = {"total_reads": int(res.stats["total_reads"])}
            t1 = ta = t0 + processor.last_timing.get("stream_decode_end", time.time() - t0)
            tb = t2 = time.time()
        else:
            soa, stats = reader.read_soa()
            t1 = time.time()
            ta = time.time()
            res = processor.run_soa(soa, len(self.barcode_list))
            tb = time.time()
            # the decoded batch (GBs of malloc'd columns and records) is unmapped on a
            # background thread while the writers run: its free took 0.36 s at C3
            box = [soa]
            del soa
            _release_in_background(box)
            t2 = time.time()
        self.engine_result = res
        self.read_stats = {**res.stats, **stats}
        st = self.read_stats
        if not self.config.dedup.skip and st["total_reads"]:
            removed = st["duplicate_reads_with_length"] if self.config.dedup.use_fragment_length \
                else st["duplicate_reads_position_only"]
            logger.info("%d duplicate reads removed (%.1f%%)", removed, removed / st["total_reads"] * 100)
        n_cells_input = int((res.n_reads > 0).sum())  # len(reads_by_barcode)
        if n_cells_input == 0:
            logger.error("No reads found for any barcodes!")
            return {}
        logger.info(f"Kept {st['filtered_reads']:,} reads from {n_cells_input:,} barcodes")

        if self.output_format == "hdf5":
            writer = IncrementalHDF5Writer(self.output_dir, self.config, self.barcode_list,
                                           barcode_metadata=self.barcode_metadata)
        else:
            writer = txt_writer
        cell_results = processor.write_results(res, self.barcode_list, writer)
        if not cell_results:
            logger.error("No cells passed quality filters")
            return {}

        logger.info("Cleaning up...")
        qc_dir = self.output_dir / "qc"
        plots = None
        if self.output_format == "hdf5" and hasattr(writer, "prepare_report_arrays"):
            # the report's figures are rendered from memory while finalize deflates and
            # writes the planes (native code, GIL released)
            plots = _Background(self._render_plots, writer.prepare_report_arrays())
        writer.finalize(qc_dir)
        meta = QCCalculator(self.config).collect_run_metadata(
            str(self.bam_path), str(self.output_dir), n_cells_input, len(cell_results))
        write_run_summary(meta, qc_dir / "summary.txt")
        t3 = time.time()
        gc.collect()

        if self.output_format == "hdf5":
            logger.info("Generating HTML QC report...")
            try:
                from .analysis.report import generate_html_report, generate_scrna_html_report

                gen = generate_html_report if self.barcode_metadata is not None else generate_scrna_html_report
                gen(self.output_dir, self.sample_name, title=self.report_title, subtitle=self.report_subtitle,
                    working_directory=self.working_directory, input_dir=str(self.bam_path.parent),
                    arrays=getattr(writer, "report_arrays", None), plots=plots.result() if plots else None)
            except ImportError:
                logger.warning("matplotlib not installed, skipping HTML report generation")
            except Exception as e:
                logger.warning("Failed to generate HTML report: %s", e)
        t4 = time.time()
        # streamed: bam_ingest ends with the last decoded batch and `engine` is only what the
        # device still did after it (the rest ran under the decode)
        self.timings = {"bam_ingest": t1 - t0, "engine": t2 - t1, "write": t3 - t2, "report": t4 - t3,
                        "total": t4 - t0, "engine_setup": ta - t1, "engine_run_soa": tb - ta,
                        "engine_free_inputs": t2 - tb, "streamed": bool(self.stream),
                        **processor.last_timing}
        logger.info("Pipeline complete")
        logger.info("Elapsed time: %.1fs (ingest %.1fs, engine %.1fs, write %.1fs)", t4 - t0, t1 - t0, t2 - t1,
                    t3 - t2)
        return {
            "cells_processed": n_cells_input,
            "cells_passed_qc": len(cell_results),
            "mean_reads": sum(r["n_reads"] for r in cell_results) / len(cell_results),
        }


def run_pipeline(
    bam_path: str,
    barcode_file: str | None = None,
    output_dir: str = "",
    sample_name: str = "mgatk",
    min_baseq: int = 20,
    min_mapq: int = 30,
    min_reads_per_cell: int = 1,
    max_strand_bias: float = 1.0,
    min_distance_from_end: int = 5,
    skip_deduplication: bool = False,
    use_fragment_length_dedup: bool = True,
    write_cell_bams: bool = False,
    barcode_tag: str = "CB",
    min_barcode_reads: int = 1,
    mito_chr: str = "chrM",
    n_cores: int = 16,
    worker_batch_size: int | None = None,
    io_batch_size: int | None = None,
    max_memory_gb: float = 128.0,
    output_format: str = "standard",
    sequential: bool = False,
    report_title: str | None = None,
    report_subtitle: str | None = None,
    working_directory: str | None = None,
    device: int = 0,
    devices: list[int] | None = None,
) -> dict[str, Any]:
    """pipeline.py:183-269. ``min_distance_from_end`` is accepted and, as in the
    reference, not passed on (the engine uses 5)."""
    barcode_metadata = None
    if barcode_file is None:
        from .file_io.barcode_extraction import extract_barcodes_from_bam

        logger.info("No barcode file provided - extracting barcodes from BAM")
        barcodes = extract_barcodes_from_bam(bam_path, barcode_tag=barcode_tag, mito_chr=mito_chr,
                                             min_reads=min_barcode_reads)
        if not barcodes:
            raise InvalidInputError(
                f"No barcodes found in BAM file with tag '{barcode_tag}' and minimum {min_barcode_reads} reads")
    elif barcode_file.endswith(".csv"):
        from .utils import load_singlecell_csv

        barcodes, barcode_metadata = load_singlecell_csv(barcode_file)
    else:
        from .utils import load_barcode_list

        barcodes = load_barcode_list(barcode_file)

    if worker_batch_size is None:
        worker_batch_size = n_cores
    if io_batch_size is None:
        io_batch_size = max(50, min(int(0.1 * len(barcodes)), 1000))
    config = PipelineConfig(
        min_baseq=min_baseq, min_mapq=min_mapq, max_strand_bias=max_strand_bias,
        skip_deduplication=skip_deduplication, use_fragment_length_dedup=use_fragment_length_dedup,
        n_cores=n_cores, worker_batch_size=worker_batch_size, io_batch_size=io_batch_size,
        max_memory_gb=max_memory_gb, sequential=sequential, min_reads_per_cell=min_reads_per_cell,
        barcode_tag=barcode_tag, mito_chr=mito_chr, write_cell_bams=write_cell_bams,
    )
    pipeline = MtDNAPipeline(
        bam_path=bam_path, barcodes=barcodes, output_dir=Path(output_dir), config=config,
        output_format=output_format, barcode_metadata=barcode_metadata, sample_name=sample_name,
        report_title=report_title, report_subtitle=report_subtitle, working_directory=working_directory,
        device=device, devices=devices,
    )
    return pipeline.run()
