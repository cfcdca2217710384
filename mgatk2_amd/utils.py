"""Input helpers (mirror of src/utils/utils.py:14-104)."""

from __future__ import annotations

import csv
import logging
import os

from .exceptions import InvalidInputError

logger = logging.getLogger(__name__)


def load_singlecell_csv(csv_file: str) -> tuple[list[str] | None, dict[str, list] | None]:
    """cellranger-atac singlecell.csv -> (cell barcodes, per-column metadata) (utils.py:14-69).

    Rows with ``is__cell_barcode == "1"`` are kept; values of every column except
    ``barcode``/``excluded_reason`` are converted int -> float -> str, empty -> 0."""
    if csv_file is None:
        return None, None
    try:
        barcodes: list[str] = []
        metadata: dict[str, list] = {}
        with open(csv_file) as f:
            reader = csv.DictReader(f)
            headers = reader.fieldnames
            if headers is None:
                raise InvalidInputError("CSV file has no headers")
            if "is__cell_barcode" not in headers:
                raise InvalidInputError("singlecell.csv missing 'is__cell_barcode' column")
            for header in headers:
                metadata[header] = []
            for row in reader:
                if row.get("is__cell_barcode") != "1":
                    continue
                barcodes.append(row["barcode"])
                for header in headers:
                    value = row[header]
                    if header not in ("barcode", "excluded_reason"):
                        try:
                            value = int(value) if value else 0
                        except ValueError:
                            try:
                                value = float(value) if value else 0.0
                            except ValueError:
                                pass
                    metadata[header].append(value)
        if not barcodes:
            raise InvalidInputError(f"No cells found with is__cell_barcode == 1 in {csv_file}")
        return barcodes, metadata
    except FileNotFoundError as e:
        raise InvalidInputError(f"singlecell.csv file not found: {csv_file}") from e
    except Exception as e:
        logger.error("Error loading singlecell.csv: %s", e)
        raise


def load_barcode_list(barcode_file: str) -> list[str]:
    """Plain barcode file: one barcode per non-empty line (pipeline.py:228-230)."""
    with open(barcode_file) as f:
        return [line.strip() for line in f if line.strip()]


def validate_bam_file(bam_path: str) -> None:
    """utils.py:72-88. The reference builds a missing `.bai` with pysam; the native
    reader does not need one (it scans to the mito contig), so none is written."""
    if not os.path.exists(bam_path):
        raise InvalidInputError(f'BAM file not found: "{bam_path}"')
    if not bam_path.endswith(".bam"):
        raise InvalidInputError(f"Input file must have .bam extension: {bam_path}")
    if not os.path.exists(bam_path + ".bai"):
        logger.info("No BAM index for %s: the mito contig is found by a linear scan", bam_path)


def validate_barcode_file(barcode_file: str) -> None:
    """utils.py:91-104."""
    if not barcode_file:
        return
    if not os.path.exists(barcode_file):
        raise InvalidInputError(f'Barcode file not found: "{barcode_file}"')
    try:
        with open(barcode_file) as f:
            if not f.readline().strip():
                raise InvalidInputError(f"Barcode file is empty: {barcode_file}")
    except Exception as e:
        raise InvalidInputError(f"Cannot read barcode file: {e}") from e
