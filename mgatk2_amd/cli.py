"""Command line (mirror of src/cli: base.py, options.py, utils.py, commands/{run,tenx,call}.py).

Same commands, option names, short flags and defaults as the reference, so a
reference command line runs unchanged (``python -m mgatk2_amd run -i ...``).
Added: ``--device`` (HIP device ordinal for the engine).
Not carried over: ``hardmask-fasta`` (FASTA masking utility, outside the hot path).
"""

from __future__ import annotations

import csv
import logging
import multiprocessing
import os
import sys
from datetime import datetime
from pathlib import Path

import click

from . import __version__
from .exceptions import InvalidInputError, ProcessingError

logger = logging.getLogger(__name__)

DEDUP_CHOICES = ["alignment_and_fragment_length", "alignment_start", "none"]


# ---------------------------------------------------------------------------
# options (options.py:6-306)
# ---------------------------------------------------------------------------
def _options(defaults: dict, helps: dict | None = None):
    d = defaults

    def deco(f):
        opts = [
            click.option("--input", "-i", "bam_path", default=".", type=click.Path(exists=True),
                         help="Input BAM file or 10x outs/ directory"),
            click.option("--genome", "-g", "mito_genome", default="chrM", show_default=True,
                         help="Mitochondrial chromosome name (e.g chrM, MT, or M)"),
            click.option("--barcodes", "-b", "barcode_file", default=None, type=click.Path(exists=True),
                         help="Barcode file (singlecell.csv, barcodes.tsv/csv, or auto-detect from BAM)"),
            click.option("--barcode-tag", "-bt", default="CB", show_default=True, help="BAM tag for cell barcode"),
            click.option("--min-barcode-reads", default=10, type=int, show_default=True,
                         help="Minimum reads per barcode when auto-detecting from BAM"),
            click.option("--output", "-o", "output_dir", default=d["output"], type=click.Path(),
                         show_default=True, help="Output directory for analysis results"),
            click.option("--threads", "-t", "ncores", default=None, type=int,
                         help="Number of threads (host side; the pileup runs on the GPU)"),
            click.option("--verbose", "-v", is_flag=True, default=d["verbose"], help="Enable verbose logging"),
            click.option("--batch-size", "batch_size", default=None, type=int,
                         help="Worker batch size (accepted for compatibility)"),
            click.option("--memory", "-m", "max_memory", default=d["memory"], type=float,
                         help="Maximum memory usage in GB"),
            click.option("--quality", "-q", "base_qual", default=d["quality"], type=int, show_default=True,
                         help="Minimum base quality (Phred score)"),
            click.option("--mapq", "min_mapq", default=d["mapq"], type=int, show_default=True,
                         help="Minimum alignment/mapping quality"),
            click.option("--min-reads", "-c", "min_reads", default=d["min_reads"], type=int, show_default=True,
                         help="Minimum deduplicated reads per cell to include in analysis"),
            click.option("--max-strand-bias", "-s", "max_strand_bias", default=1.0, type=float, show_default=True,
                         help="Maximum strand bias (0-1)"),
            click.option("--min-distance-from-end", "-e", "min_distance_from_end", default=d["dist"], type=int,
                         show_default=True, help="Minimum distance from read ends (bp)"),
            click.option("--deduplication", "-d", "dedup_mode",
                         type=click.Choice(DEDUP_CHOICES, case_sensitive=False), default=d["dedup"],
                         show_default=True, help="Deduplication strategy"),
            click.option("--format", "-f", "output_format", type=click.Choice(["txt", "hdf5"], case_sensitive=False),
                         default=d["format"], show_default=True, help="Output format"),
            click.option("--dry-run", is_flag=True, help="Show configuration and exit without processing"),
            click.option("--device", "device", default=0, type=int, show_default=True,
                         help="HIP device ordinal for the pileup engine"),
            click.option("--devices", "devices", default=None,
                         help="Comma-separated HIP devices to shard cells over (e.g. 0,1,2,3)"),
        ]
        for o in reversed(opts):
            f = o(f)
        return f

    return deco


RUN_DEFAULTS = dict(output="mgatk2/", verbose=True, memory=128, quality=20, mapq=30, min_reads=1, dist=5,
                    dedup="alignment_and_fragment_length", format="hdf5")
TENX_DEFAULTS = dict(output="mgatk2", verbose=False, memory=None, quality=0, mapq=0, min_reads=0, dist=0,
                     dedup="alignment_start", format="txt")


# ---------------------------------------------------------------------------
# helpers (cli/utils.py)
# ---------------------------------------------------------------------------
def _find_barcode_file(directory: Path) -> str | None:
    singlecell = directory / "singlecell.csv"
    if singlecell.exists():
        return str(singlecell)
    for pattern in ["filtered_peak_bc_matrix/barcodes.tsv", "filtered_tf_bc_matrix/barcodes.tsv.gz"]:
        if (directory / pattern).exists():
            return str(directory / pattern)
    logger.warning("No barcode file found")
    return None


def auto_detect_10x_structure(bam_path: str, barcode_file: str | None = None) -> tuple[str, str | None]:
    """cli/utils.py:18-52."""
    path = Path(bam_path)
    if path.is_dir():
        bam_file: Path | None = None
        if path.name == "outs" or "outs" in str(path):
            bam_file = path / "possorted_bam.bam"
            if not bam_file.exists():
                bam_file = path.parent / "outs" / "possorted_bam.bam"
        else:
            outs_dir = path / "outs"
            bam_file = outs_dir / "possorted_bam.bam" if outs_dir.exists() else None
        if bam_file and bam_file.exists():
            bam_path = str(bam_file)
            if not barcode_file:
                barcode_file = _find_barcode_file(bam_file.parent)
        else:
            logger.warning(f"No possorted_bam.bam found in {path}")
    elif path.is_file() and not barcode_file and path.parent.name == "outs":
        logger.info("Detected 10x BAM in outs directory")
        barcode_file = _find_barcode_file(path.parent)
    return str(Path(bam_path).resolve()), barcode_file


def normalise_mito_chr(mito_genome: str) -> str:
    """cli/utils.py:76-83."""
    if mito_genome.upper() in ["M", "MT"]:
        return "chrM"
    if mito_genome in ["chrM", "chrMT"]:
        return mito_genome
    logger.warning("Unusual mitochondrial chromosome name: %s", mito_genome)
    return mito_genome


def get_10x_parent_directory_name(bam_path: str) -> str:
    """cli/utils.py:86-108."""
    p = Path(bam_path)
    if p.parent.name == "outs":
        return p.parent.parent.name
    if "outs" in str(p.parent):
        cur = p.parent
        while cur.parent != cur:
            if cur.name == "outs":
                return cur.parent.name
            cur = cur.parent
    return p.parent.name if p.parent.name != "." else "mgatk2"


def setup_file_logging(log_file_path):
    handler = logging.FileHandler(log_file_path, mode="w")
    handler.setLevel(logging.INFO)
    handler.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
    logging.getLogger("mgatk2_amd").addHandler(handler)


def _determine_cores(ncores):
    if ncores is not None:
        return ncores
    for var in ("SLURM_CPUS_PER_TASK", "SLURM_NTASKS"):
        v = os.environ.get(var)
        if v:
            try:
                return int(v)
            except ValueError:
                break
    return max(1, multiprocessing.cpu_count())


def _count_barcodes(barcode_file: str | None) -> str:
    if not barcode_file:
        return "auto-detect from BAM"
    if barcode_file.endswith(".csv"):
        with open(barcode_file) as f:
            reader = csv.DictReader(f)
            headers = reader.fieldnames or []
            col = next((c for c in ("is__cell_barcode", "is_cell_barcode", "is_cell") if c in headers), None)
            return str(sum(1 for row in reader if col and row.get(col, "0") in ("1", "1.0", "True", "true", "TRUE")))
    with open(barcode_file) as f:
        return str(sum(1 for line in f if line.strip()))


def run_pipeline_command(bam_path, output_dir, barcode_file, barcode_tag, min_barcode_reads, mito_genome, ncores,
                         verbose, batch_size, max_memory, base_qual, min_mapq, min_reads, max_strand_bias,
                         min_distance_from_end, dedup_mode, output_format, sequential, dry_run=False,
                         original_bam_path=None, report_title=None, report_subtitle=None, working_directory=None,
                         device=0, devices=None) -> int:
    """cli/utils.py:124-289: returns 0 on success, 1 on a handled error."""
    from .pipeline import run_pipeline
    from .utils import validate_bam_file, validate_barcode_file

    if verbose:
        logging.getLogger("mgatk2_amd").setLevel(logging.DEBUG)
    logger.info("mgatk2 (MI355X engine) version %s", __version__)
    if barcode_file != "bulk":
        bam_path, barcode_file = auto_detect_10x_structure(bam_path, barcode_file)
    skip_dedup = dedup_mode.lower() == "none"
    use_fragment_length_dedup = dedup_mode.lower() in ["alignment_and_fragment_length", "fragment-length", "hybrid"]
    if not dry_run:
        log_file = Path(output_dir) / "output.log"
        log_file.parent.mkdir(parents=True, exist_ok=True)
        setup_file_logging(log_file)
        logger.info("Command executed: %s %s", os.path.realpath(sys.argv[0]) if sys.argv else "mgatk2",
                    " ".join(sys.argv[1:]))
        logger.info("Working directory: %s", os.getcwd())
        logger.info("Execution time: %s", datetime.now().strftime("%Y-%m-%d %H:%M:%S"))
    try:
        validate_bam_file(bam_path)
        if barcode_file:
            validate_barcode_file(barcode_file)
        os.makedirs(output_dir, exist_ok=True)
        mito_chr = normalise_mito_chr(mito_genome)
        cores = _determine_cores(ncores)
        logger.info("  Input BAM:              %s", os.path.realpath(bam_path))
        logger.info("  Input barcodes:         %s",
                    os.path.realpath(barcode_file) if barcode_file else "None (auto-detect from BAM)")
        logger.info("  Output directory:       %s", os.path.realpath(output_dir))
        logger.info("  Mitochondrial chr:      %s", mito_chr)
        logger.info("  Min base quality:       %s", base_qual)
        logger.info("  Min mapping quality:    %s", min_mapq)
        logger.info("  Min reads per cell:     %s", min_reads)
        logger.info("  Max strand bias:        %s", max_strand_bias)
        logger.info("  Deduplication:          %s", dedup_mode)
        logger.info("  Output format:          %s", output_format)
        logger.info("  Barcodes:               %s", _count_barcodes(barcode_file))
        logger.info("  HIP device:             %s", device)
        if dry_run:
            return 0
        if report_title is None:
            report_title = get_10x_parent_directory_name(original_bam_path or bam_path)
        run_args = dict(
            bam_path=bam_path, barcode_file=barcode_file, output_dir=output_dir, sample_name="output_",
            min_baseq=base_qual, min_mapq=min_mapq, min_reads_per_cell=min_reads, output_format=output_format.lower(),
            max_strand_bias=max_strand_bias, min_distance_from_end=min_distance_from_end, barcode_tag=barcode_tag,
            min_barcode_reads=min_barcode_reads, mito_chr=mito_chr, n_cores=cores,
            worker_batch_size=batch_size if batch_size is not None else cores, io_batch_size=None,
            skip_deduplication=skip_dedup, use_fragment_length_dedup=use_fragment_length_dedup,
            sequential=sequential, report_title=report_title, report_subtitle=report_subtitle or
            "mgatk2 output analysis", working_directory=working_directory, device=device,
            devices=[int(x) for x in devices.split(",")] if devices else None,
        )
        if max_memory is not None:
            run_args["max_memory_gb"] = max_memory
        run_pipeline(**run_args)
        return 0
    except InvalidInputError as e:
        logger.error("Input validation failed: %s", e)
        return 1
    except ProcessingError as e:
        logger.error("Processing failed: %s", e)
        return 1
    except Exception as e:
        logger.error("Unexpected error: %s", e)
        if verbose:
            import traceback

            traceback.print_exc()
        return 1


# ---------------------------------------------------------------------------
# commands
# ---------------------------------------------------------------------------
class OrderedGroup(click.Group):
    def list_commands(self, ctx):
        return list(self.commands)


@click.group(cls=OrderedGroup)
@click.version_option(version=__version__)
def cli():
    """mgatk2 (MI355X engine): per-cell mitochondrial pileup on AMD Instinct GPUs."""


@cli.command()
@_options(RUN_DEFAULTS)
def run(bam_path, mito_genome, barcode_file, barcode_tag, min_barcode_reads, output_dir, ncores, verbose, batch_size,
        max_memory, base_qual, min_mapq, min_reads, max_strand_bias, min_distance_from_end, dedup_mode,
        output_format, dry_run, device, devices):
    """Run mgatk2 with optimised defaults"""
    try:
        rc = run_pipeline_command(
            bam_path, output_dir, barcode_file, barcode_tag, min_barcode_reads, mito_genome, ncores, verbose,
            batch_size, max_memory, base_qual, min_mapq, min_reads, max_strand_bias, min_distance_from_end,
            dedup_mode, output_format, ncores == 1, dry_run=dry_run, original_bam_path=bam_path,
            report_title=get_10x_parent_directory_name(bam_path), report_subtitle="mgatk2 output analysis",
            working_directory=os.getcwd(), device=device, devices=devices)
    except KeyboardInterrupt:
        raise SystemExit(130) from None
    if rc:
        raise SystemExit(rc)


@cli.command()
@_options(TENX_DEFAULTS)
def tenx(bam_path, mito_genome, barcode_file, barcode_tag, min_barcode_reads, output_dir, ncores, verbose, batch_size,
         max_memory, base_qual, min_mapq, min_reads, max_strand_bias, min_distance_from_end, dedup_mode,
         output_format, dry_run, device, devices):
    """Run mgatk2 with original mgatk package behaviour"""
    rc = run_pipeline_command(
        bam_path, output_dir, barcode_file, barcode_tag, min_barcode_reads, mito_genome, ncores, verbose,
        batch_size, max_memory, base_qual, min_mapq, min_reads, max_strand_bias, min_distance_from_end, dedup_mode,
        output_format, ncores == 1, dry_run=dry_run, device=device, devices=devices)
    if rc:
        raise SystemExit(rc)


@cli.command()
@click.option("--input", "-i", "bam_path", type=click.Path(exists=True), required=True,
              help="Directory of BAM files (one BAM per cell)")
@click.option("--genome", "-g", "mito_genome", default="chrM", show_default=True)
@click.option("--output", "-o", "output_dir", default="mgatk2/", type=click.Path(), show_default=True)
@click.option("--threads", "-t", "ncores", default=None, type=int)
@click.option("--verbose", "-v", is_flag=True, default=True)
@click.option("--memory", "-m", "max_memory", default=128, type=float, show_default=True)
@click.option("--quality", "-q", "base_qual", default=20, type=int, show_default=True)
@click.option("--mapq", "min_mapq", default=30, type=int, show_default=True)
@click.option("--max-strand-bias", "-s", "max_strand_bias", default=1.0, type=float, show_default=True)
@click.option("--min-distance-from-end", "-e", "min_distance_from_end", default=5, type=int, show_default=True)
@click.option("--deduplication", "-d", "dedup_mode", type=click.Choice(DEDUP_CHOICES, case_sensitive=False),
              default="alignment_and_fragment_length", show_default=True)
@click.option("--format", "-f", "output_format", type=click.Choice(["txt", "hdf5"], case_sensitive=False),
              default="hdf5", show_default=True)
@click.option("--dry-run", is_flag=True)
@click.option("--device", "device", default=0, type=int, show_default=True)
def call(bam_path, mito_genome, output_dir, ncores, verbose, max_memory, base_qual, min_mapq, max_strand_bias,
         min_distance_from_end, dedup_mode, output_format, dry_run, device):
    """Run mgatk2 and treat each bam file as a single cell (commands/call.py)"""
    bam_files = sorted(Path(bam_path).glob("*.bam"))
    if not bam_files:
        logger.error(f"No BAM files (*.bam) found in directory: {bam_path}")
        raise SystemExit(1)
    mito_chr = normalise_mito_chr(mito_genome)
    logger.info("Auto-detected %s BAM files", len(bam_files))
    if dry_run:
        return
    for i, bam_file in enumerate(bam_files, 1):
        out = Path(output_dir) / bam_file.stem
        out.mkdir(parents=True, exist_ok=True)
        logger.info(f"[{i}/{len(bam_files)}] Processing: {bam_file.name} -> {out}")
        run_pipeline_command(str(bam_file), str(out), None, "CB", 10, mito_chr, ncores, verbose, 1, max_memory,
                             base_qual, min_mapq, 0, max_strand_bias, min_distance_from_end, dedup_mode, output_format,
                             ncores == 1, dry_run=False, device=device)
    logger.info("Analysis completed for all %s BAM files", len(bam_files))


def main():
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    cli()


if __name__ == "__main__":
    main()
