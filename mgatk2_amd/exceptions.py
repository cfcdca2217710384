"""Exception taxonomy of the boundary (mirrors src/core/exceptions.py:4-86).

The engine's negative return codes are mapped onto these classes in
mgatk2_amd/engine.py, so callers catch the same exceptions the reference raises.
"""


class MgatkError(Exception):
    """Base exception for mgatk2 errors (exceptions.py:4)."""


class InvalidInputError(MgatkError):
    """Raised when input files are invalid or missing (exceptions.py:8)."""


class ProcessingError(MgatkError):
    """Raised when pipeline processing fails (exceptions.py:12)."""


class BAMReadError(ProcessingError):
    """Raised when BAM file reading fails (exceptions.py:16)."""

    def __init__(self, bam_path: str, message: str):
        self.bam_path = bam_path
        super().__init__(f"BAM read error for {bam_path}: {message}")


class InsufficientDataError(ProcessingError):
    """exceptions.py:24"""

    def __init__(self, n_items: int, min_required: int, item_type: str = "cells"):
        self.n_items = n_items
        self.min_required = min_required
        self.item_type = item_type
        super().__init__(f"Only {n_items} {item_type} found, need >= {min_required}")


class NoChrMReadsError(BAMReadError):
    """exceptions.py:34"""

    def __init__(self, bam_path: str, available_chromosomes: list[str]):
        self.available_chromosomes = available_chromosomes
        chrs = ", ".join(available_chromosomes[:10])
        super().__init__(
            bam_path,
            f"No mitochondrial chromosome (chrM, MT, or M) found.\n"
            f"Available: {chrs}{'...' if len(available_chromosomes) > 10 else ''}",
        )


class NoBarcodeTagsError(BAMReadError):
    """exceptions.py:47"""

    def __init__(self, bam_path: str, barcode_tag: str, total_reads_checked: int):
        self.barcode_tag = barcode_tag
        self.total_reads_checked = total_reads_checked
        super().__init__(
            bam_path,
            (
                f"No reads with barcode tag '{barcode_tag}' found "
                f"(checked {total_reads_checked:,} reads).\n"
                f"This may not be a single-cell BAM file, or wrong tag specified."
            ),
        )


class BAMFormatError(InvalidInputError):
    """exceptions.py:63"""

    def __init__(self, bam_path: str, details: str = ""):
        message = f"BAM file appears corrupted or is not a valid BAM format: {bam_path}"
        if details:
            message += f"\n{details}"
        super().__init__(message)


class HDF5WriteError(ProcessingError):
    """exceptions.py:74"""

    def __init__(self, hdf5_path: str, message: str):
        self.hdf5_path = hdf5_path
        super().__init__(f"HDF5 write error for {hdf5_path}: {message}")
