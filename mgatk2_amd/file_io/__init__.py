"""Output writers (mirror of src/file_io)."""

from .formats import write_cell_stats, write_run_summary
from .writers import IncrementalHDF5Writer, IncrementalTextWriter

__all__ = ["IncrementalHDF5Writer", "IncrementalTextWriter", "write_cell_stats", "write_run_summary"]
