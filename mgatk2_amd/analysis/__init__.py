"""QC metrics and report (mirror of src/analysis)."""

from .qc import QCCalculator

__all__ = ["QCCalculator"]
