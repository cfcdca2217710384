"""Configuration types (mirror of src/core/config.py:1-114).

Same classes, fields and defaults as the reference, so callers construct them
identically. Behaviour kept on purpose:

* ``PipelineConfig`` does not accept ``min_distance_from_end``: the reference
  never passes it on (src/core/pipeline.py:239-254), so
  ``QualityThresholds.min_distance_from_end`` keeps its default of 5
  (config.py:15) whatever the CLI says.
* ``worker_batch_size`` defaults to ``n_cores`` (config.py:105).

:meth:`PipelineConfig.engine_config` converts to the engine's POD config.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy

from .engine import EngineConfig


@dataclass
class QualityThresholds:
    """Quality filtering parameters (config.py:8-15)."""

    min_baseq: int = 20
    min_mapq: int = 30
    max_strand_bias: float = 1.0
    min_distance_from_end: int = 5


@dataclass
class DeduplicationConfig:
    """Deduplication parameters (config.py:18-23)."""

    skip: bool = False
    use_fragment_length: bool = True


@dataclass
class PerformanceConfig:
    """Resource management (config.py:26-34)."""

    n_cores: int = 8
    worker_batch_size: int = 8
    io_batch_size: int = 100
    max_memory_gb: float = 128.0
    sequential: bool = False


@dataclass
class SimpleRead:
    """Lightweight BAM read (config.py:37-49); used by the per-cell Python API."""

    reference_start: int
    is_reverse: bool
    mapping_quality: int
    query_sequence: bytes
    query_qualities: "numpy.ndarray"
    cigar: list[tuple[int, int]]
    is_proper_pair: bool = False
    is_paired: bool = False
    template_length: int = 0


class PipelineConfig:
    """Pipeline configuration (config.py:77-114)."""

    def __init__(
        self,
        min_baseq: int = 20,
        min_mapq: int = 30,
        max_strand_bias: float = 0.9,
        skip_deduplication: bool = False,
        use_fragment_length_dedup: bool = True,
        n_cores: int = 8,
        worker_batch_size: int | None = None,
        io_batch_size: int | None = None,
        max_memory_gb: float = 128.0,
        sequential: bool = False,
        min_reads_per_cell: int = 1,
        barcode_tag: str = "CB",
        mito_chr: str = "chrM",
        mito_length: int = 16569,
        **kwargs,
    ):
        self.quality = QualityThresholds(min_baseq=min_baseq, min_mapq=min_mapq, max_strand_bias=max_strand_bias)
        self.dedup = DeduplicationConfig(skip=skip_deduplication, use_fragment_length=use_fragment_length_dedup)
        self.performance = PerformanceConfig(
            n_cores=n_cores,
            worker_batch_size=worker_batch_size or n_cores,
            io_batch_size=io_batch_size or 100,
            max_memory_gb=max_memory_gb,
            sequential=sequential,
        )
        self.min_reads_per_cell = min_reads_per_cell
        self.barcode_tag = barcode_tag
        self.mito_chr = mito_chr
        self.mito_length = mito_length

    @property
    def dedup_mode(self) -> str:
        if self.dedup.skip:
            return "none"
        return "alignment_and_fragment_length" if self.dedup.use_fragment_length else "alignment_start"

    def engine_config(self, n_cells: int, reserve_reads: int = 0, reserve_payload: int = 0) -> EngineConfig:
        return EngineConfig(
            n_cells=n_cells,
            min_baseq=self.quality.min_baseq,
            min_mapq=self.quality.min_mapq,
            min_distance_from_end=self.quality.min_distance_from_end,
            dedup_mode=self.dedup_mode,
            max_strand_bias=self.quality.max_strand_bias,
            min_reads=self.min_reads_per_cell,
            mito_len=self.mito_length,
            reserve_reads=reserve_reads,
            reserve_payload=reserve_payload,
        )
