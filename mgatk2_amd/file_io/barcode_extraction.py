"""Barcode auto-extraction (mirror of src/file_io/barcode_extraction.py:12-46).

One native pass over the mito contig (libmgphost.so `mgp_bam_count_tag`):
counts of ``str(tag value)`` over records that are neither unmapped nor
duplicates; barcodes with ``count >= min_reads`` are returned sorted.
"""

from __future__ import annotations

import logging

from ..bam import BamFile

logger = logging.getLogger(__name__)


def extract_barcodes_from_bam(bam_path: str, barcode_tag: str = "CB", mito_chr: str = "chrM",
                              min_reads: int = 10) -> list[str]:
    logger.info("Extracting barcodes from BAM file...")
    logger.info("  Looking for tag '%s' on chromosome '%s'", barcode_tag, mito_chr)
    try:
        with BamFile(bam_path) as bam:
            counts = bam.count_tag(mito_chr, barcode_tag)
    except Exception as e:
        logger.error("Failed to extract barcodes: %s", e)
        raise
    barcodes = sorted(bc for bc, n in counts.items() if n >= min_reads)
    logger.info("  Found %d total barcodes", len(counts))
    logger.info("  Retained %d barcodes with >= %d reads", len(barcodes), min_reads)
    return barcodes
