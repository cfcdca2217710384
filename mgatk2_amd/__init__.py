"""mgatk2_amd — MI355X-native per-barcode mitochondrial pileup engine.

Drop-in for the `src/processing` hot path of mgatk2: the host packs chrM reads
into SoA batches, a ctypes C-ABI (include/mgpileup.h) streams them into HBM and
hand-written HIP kernels for gfx950 do dedup, CIGAR-walk pileup, strand filter,
per-cell statistics and reference-allele tallies.
"""

__version__ = "0.1.0"
