"""Per-cell pileup API (mirror of src/processing/pileup.py).

``PileupGenerator.generate_pileup(reads)`` / ``filter_strand_bias(pileup)``
keep the reference's per-cell dict interface (pileup.py:18-154). The counting
runs on the GPU engine (one cell per call): reads are packed into the engine's
SoA batch and the count tile comes back as arrays, which are turned into the
reference's per-position dicts. This path exists for callers of the per-cell
API; the production path (processors.CellProcessor.process_soa) keeps
everything as arrays.
"""

from __future__ import annotations

import numpy as np

from ..engine import Engine, EngineConfig
from ..synth import pack_reads

BASES = ["A", "C", "G", "T"]


def position_dict(counts_row: np.ndarray, tn5_row: np.ndarray) -> dict:
    """One position of the reference pileup dict (pileup.py:109-124)."""
    fw = counts_row[0::2].tolist()
    rv = counts_row[1::2].tolist()
    d = {"depth": int(sum(fw) + sum(rv)), "tn5_cuts_fwd": int(tn5_row[0]), "tn5_cuts_rev": int(tn5_row[1])}
    for bi, b in enumerate(BASES):
        d[b] = int(fw[bi] + rv[bi])
        d[f"{b}_fwd"] = int(fw[bi])
        d[f"{b}_rev"] = int(rv[bi])
    return d


def result_dict(res, c: int, barcode: str, mito_length: int) -> dict:
    """process_barcode_worker's result (processors.py:40-51) for a passing cell of an EngineResult."""
    from ..file_io.writers import cell_qc

    pos = np.flatnonzero(res.depth[c] > 0)
    pileup = {int(p): position_dict(res.counts[c, p], res.tn5[c, p]) for p in pos}
    qc = cell_qc(res, c, barcode, mito_length)
    return {"barcode": barcode, "pileup": pileup, "n_reads": int(res.n_reads[c]), "qc": qc}


def simple_reads_to_dicts(reads, bc: int = 0) -> list[dict]:
    """SimpleRead (config.py:37-49) -> packer dicts."""
    out = []
    for r in reads:
        seq = r.query_sequence
        if isinstance(seq, (bytes, bytearray)):
            seq = seq.decode("ascii")
        q = r.query_qualities
        flag = (0x10 if r.is_reverse else 0) | (0x1 if r.is_paired else 0) | (0x2 if r.is_proper_pair else 0)
        out.append(dict(
            reference_start=int(r.reference_start), cigartuples=list(r.cigar or []), query_sequence=seq,
            query_qualities=None if q is None else (np.asarray(q).astype(np.int64) & 0xFF).tolist(), bc=bc,
            flag=flag, mapping_quality=int(r.mapping_quality), template_length=int(r.template_length),
        ))
    out.sort(key=lambda d: d["reference_start"])  # stable: keeps the caller's order among equal starts
    return out


class PileupGenerator:
    """Generate pileup data from aligned reads with quality filtering (pileup.py:10)."""

    def __init__(self, config, device: int = 0):
        self.config = config
        self.device = device
        self.bases = BASES
        self.base_to_idx = {"A": 0, "C": 1, "G": 2, "T": 3}

    def _engine_config(self, max_strand_bias: float) -> EngineConfig:
        q = self.config.quality
        return EngineConfig(n_cells=1, min_baseq=q.min_baseq, min_mapq=q.min_mapq,
                            min_distance_from_end=q.min_distance_from_end, dedup_mode="none",
                            max_strand_bias=max_strand_bias, min_reads=0, mito_len=self.config.mito_length,
                            keep_tn5=True)

    def generate_pileup(self, reads) -> dict[int, dict[str, int]]:
        """Count bases at each position, stratified by strand (pileup.py:18-126).

        Positions with depth > 0 or a Tn5 cut; no strand filter."""
        if not reads:
            return {}
        soa = pack_reads(simple_reads_to_dicts(reads))
        with Engine(self._engine_config(2.0), device=self.device) as eng:
            eng.push(soa)
            raw = eng.finish_raw()
        counts, tn5 = raw
        L = self.config.mito_length
        keep = np.flatnonzero((counts.reshape(L, 8).sum(1) > 0) | (tn5.reshape(L, 2).sum(1) > 0))
        return {int(p): position_dict(counts[p], tn5[p]) for p in keep}

    def filter_strand_bias(self, pileup: dict[int, dict[str, int]]) -> dict[int, dict[str, int]]:
        """Remove positions where most reads come from a single strand (pileup.py:128-154)."""
        filtered = {}
        max_bias = self.config.quality.max_strand_bias
        for pos, counts in pileup.items():
            fc = counts.copy()
            for base in self.bases:
                fwd, rev = counts[f"{base}_fwd"], counts[f"{base}_rev"]
                total = fwd + rev
                if total > 0 and max(fwd, rev) / total > max_bias:
                    fc[base] = 0
                    fc[f"{base}_fwd"] = 0
                    fc[f"{base}_rev"] = 0
            fc["depth"] = sum(fc[b] for b in self.bases)
            if fc["depth"] > 0:
                filtered[pos] = fc
        return filtered
