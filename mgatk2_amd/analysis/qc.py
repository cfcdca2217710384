"""Quality-control metrics (mirror of src/analysis/qc.py:15-93)."""

from __future__ import annotations

import datetime
import logging
from collections import defaultdict

import numpy as np

from .. import __version__

logger = logging.getLogger(__name__)


class QCCalculator:
    def __init__(self, config):
        self.config = config

    def calculate_position_stats(self, cell_results: list[dict]) -> dict[int, dict]:
        """qc.py:21-66 over per-cell result dicts (1-based positions)."""
        position_data: dict[int, dict] = defaultdict(lambda: {"depths": [], "n_cells": 0})
        for result in cell_results:
            for pos, counts in result["pileup"].items():
                if counts["depth"] > 0:
                    position_data[pos + 1]["depths"].append(counts["depth"])
                    position_data[pos + 1]["n_cells"] += 1
        stats = {}
        for pos in range(1, self.config.mito_length + 1):
            if pos in position_data:
                d = position_data[pos]["depths"]
                mean_cov = np.mean(d)
                std_cov = np.std(d)
                stats[pos] = {
                    "n_cells_any": position_data[pos]["n_cells"],
                    "n_cells_10x": sum(1 for x in d if x >= 10),
                    "n_cells_50x": sum(1 for x in d if x >= 50),
                    "mean_cov": mean_cov,
                    "median_cov": np.median(d),
                    "cv": std_cov / mean_cov if mean_cov > 0 else 0,
                }
            else:
                stats[pos] = {"n_cells_any": 0, "n_cells_10x": 0, "n_cells_50x": 0, "mean_cov": 0,
                              "median_cov": 0, "cv": 0}
        return stats

    def position_stats_arrays(self, depth: np.ndarray) -> dict[str, np.ndarray]:
        """Array form of calculate_position_stats over a [cells, L] depth matrix of
        passing cells (n_cells_any/10x/50x, mean/median/cv over covering cells)."""
        d = np.asarray(depth)
        cov = d > 0
        n_any = cov.sum(axis=0)
        with np.errstate(invalid="ignore", divide="ignore"):
            s = np.where(cov, d, 0).astype(np.float64).sum(axis=0)
            mean = np.where(n_any > 0, s / np.maximum(n_any, 1), 0.0)
            sq = np.where(cov, (d - mean[None, :]) ** 2, 0.0).sum(axis=0)
            std = np.sqrt(np.where(n_any > 0, sq / np.maximum(n_any, 1), 0.0))
            cv = np.where(mean > 0, std / np.where(mean > 0, mean, 1), 0.0)
        masked = np.where(cov, d.astype(np.float64), np.nan)
        med = np.zeros(d.shape[1]) if d.shape[0] == 0 else np.nan_to_num(
            np.nanmedian(np.where(n_any[None, :] > 0, masked, 0.0), axis=0))
        return {
            "n_cells_any": n_any,
            "n_cells_10x": (d >= 10).sum(axis=0),
            "n_cells_50x": (d >= 50).sum(axis=0),
            "mean_cov": mean,
            "median_cov": med,
            "cv": cv,
        }

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
