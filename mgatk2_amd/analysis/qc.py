"""Quality-control metadata (mirror of src/analysis/qc.py:68-93; the reference's
`calculate_position_stats`, qc.py:21-66, is dead code and is not restated)."""

from __future__ import annotations

import datetime
import logging
from .. import __version__

logger = logging.getLogger(__name__)


class QCCalculator:
    def __init__(self, config):
        self.config = config

    def collect_run_metadata(self, bam_path: str, output_dir: str, n_cells_input: int, n_cells_passed: int) -> dict:
        """qc.py:68-93; the version is this package's."""
        return {
            "mgatk_version": __version__,
            "run_date": datetime.datetime.now().isoformat(),
            "input_bam": str(bam_path),
            "output_dir": str(output_dir),
            "reference": self.config.mito_chr,
            "reference_length": self.config.mito_length,
            "cells_total": n_cells_input,
            "cells_passed_qc": n_cells_passed,
            "cells_failed_qc": n_cells_input - n_cells_passed,
            "parameters": {
                "min_base_quality": self.config.quality.min_baseq,
                "min_mapping_quality": self.config.quality.min_mapq,
                "min_reads_per_cell": self.config.min_reads_per_cell,
                "max_strand_bias": self.config.quality.max_strand_bias,
                "skip_deduplication": self.config.dedup.skip,
                "use_fragment_length_dedup": self.config.dedup.use_fragment_length,
                "barcode_tag": self.config.barcode_tag,
                "mito_chr": self.config.mito_chr,
                "n_cores": self.config.performance.n_cores,
            },
        }
