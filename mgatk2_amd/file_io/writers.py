"""Output writers (mirror of src/file_io/writers.py).

The reference writers consume one per-position dict per cell
(``write_cell(result)``, writers.py:136,430). Here the engine hands over dense
cell-major arrays (:class:`mgatk2_amd.engine.EngineResult`), and the writers
format directly from them:

* :class:`IncrementalTextWriter` — mgatk txt layout (writers.py:409-510):
  ``output.{A,C,G,T,coverage}.txt.gz``, ``output.depthTable.txt``,
  ``{mito_chr}_refAllele.txt``, ``qc/cell_stats.csv``.
* :class:`IncrementalHDF5Writer` — ``counts.h5`` / ``metadata.h5``
  (writers.py:20-406): uint16 ``[16569, n_barcodes]`` planes saturated at 65535,
  whitelist-indexed columns, per-cell metadata, reference alleles, optional
  ``barcode_metadata`` group. Needs an h5py-compatible module.

Both keep the reference's ``write_cell(result_dict)`` / ``finalize(qc_dir)``
API (for callers of the per-cell path) and add ``write_cells(res, cells)`` for
the array path. Cell order = the order cells are written in (first-seen BAM
order, the reference's sequential order).
"""

from __future__ import annotations

import logging
import os
from pathlib import Path

import numpy as np

from ..bam import txt_write_cells
from .formats import write_cell_stats

logger = logging.getLogger(__name__)

BASES = ["A", "C", "G", "T"]
STRANDS = ["fwd", "rev"]


# ---------------------------------------------------------------------------
# per-cell views of the engine result
# ---------------------------------------------------------------------------
def cell_qc(res, c: int, barcode: str, mito_length: int) -> dict:
    """processors.py:33-51 for a passing cell."""
    n = int(res.n_reads[c])
    covered = int(res.covered[c])
    mean_cov = float(res.depth_sum[c]) / covered  # == np.mean of the kept depths (exact int sum / n)
    return {
        "barcode": barcode,
        "total_reads": n,
        "total_fragments": n // 2 if res.any_paired[c] else n,
        "mean_depth": mean_cov,
        "coverage_breadth": covered / mito_length if mito_length > 0 else 0,
    }


def ref_alleles(tally: np.ndarray) -> list[str]:
    """Reference allele per position: first max over A<C<G<T, N if all zero (writers.py:340-349)."""
    t = np.asarray(tally)
    m = np.argmax(t, axis=1)  # argmax returns the first maximum
    best = t[np.arange(t.shape[0]), m]
    return [("ACGT"[k] if v > 0 else "N") for k, v in zip(m.tolist(), best.tolist())]


def pileup_dict_to_arrays(pileup: dict, mito_length: int):
    """Inverse of the reference per-position dict (pileup.py:100-124) for one cell."""
    counts = np.zeros((mito_length, 8), np.uint32)
    tn5 = np.zeros((mito_length, 2), np.uint32)
    depth = np.zeros(mito_length, np.uint32)
    for pos, d in pileup.items():
        for bi, b in enumerate(BASES):
            counts[pos, 2 * bi] = d.get(f"{b}_fwd", 0)
            counts[pos, 2 * bi + 1] = d.get(f"{b}_rev", 0)
        tn5[pos, 0] = d.get("tn5_cuts_fwd", 0)
        tn5[pos, 1] = d.get("tn5_cuts_rev", 0)
        depth[pos] = d["depth"]
    return counts, tn5, depth


class _OneCell:
    """Adapter: a single reference result dict seen through the EngineResult interface."""

    def __init__(self, result: dict, mito_length: int):
        self.counts, self.tn5, self.depth = pileup_dict_to_arrays(result["pileup"], mito_length)
        self.counts = self.counts[None]
        self.tn5 = self.tn5[None]
        self.depth = self.depth[None]
        qc = result.get("qc", {})
        n = int(result.get("n_reads", qc.get("total_reads", 0)))
        self.n_reads = np.array([n], np.uint32)
        self.any_paired = np.array([qc.get("total_fragments", n) != n], np.uint8)
        d = self.depth[0]
        kept = d[d > 0]
        self.covered = np.array([kept.size], np.uint32)
        self.depth_sum = np.array([int(kept.sum())], np.uint64)
        self.depth_max = np.array([int(kept.max()) if kept.size else 0], np.uint32)
        s = np.sort(kept)
        self.median_lo = np.array([s[(s.size - 1) // 2] if s.size else 0], np.uint32)
        self.median_hi = np.array([s[s.size // 2] if s.size else 0], np.uint32)
        self.qc = qc


# ---------------------------------------------------------------------------
# txt
# ---------------------------------------------------------------------------
class IncrementalTextWriter:
    """mgatk txt format (writers.py:409-510).

    The count files are formatted and deflated natively (libmgphost.so
    `mgp_txt_write_cells`): every call appends gzip members to
    ``output.{A,C,G,T,coverage}.txt.gz``, so no uncompressed copy is kept and
    ``finalize`` has nothing left to compress. The decompressed text equals the
    reference's."""

    def __init__(self, output_dir: Path, config, barcodes: list[str], gzip_level: int | None = None,
                 n_threads: int = 0):
        self.output_dir = Path(output_dir) / "output"
        self.output_dir.mkdir(exist_ok=True, parents=True)
        self.config = config
        self.barcodes = list(barcodes)
        self.cell_stats: list[dict] = []
        self.position_base_counts = np.zeros((config.mito_length, 4), np.int64)
        self.cell_depths: dict[str, float] = {}
        # the reference's compresslevel=9 (writers.py:471-486) by default; MGP_GZIP_LEVEL=1
        # trades ~20 % larger files for a deflate ~15x faster (the decompressed text is the same)
        self.gzip_level = int(os.environ.get("MGP_GZIP_LEVEL", 9)) if gzip_level is None else gzip_level
        self.n_threads = n_threads
        self.prefix = self.output_dir / "output"
        for name in [*BASES, "coverage"]:
            open(self.output_dir / f"output.{name}.txt.gz", "wb").close()

    # array path -----------------------------------------------------------
    def write_cells(self, res, cells, barcodes: list[str] | None = None, tally: np.ndarray | None = None):
        """Write the given cells (indices into `res`) in order."""
        names = barcodes if barcodes is not None else self.barcodes
        L = self.config.mito_length
        cells = np.asarray(cells, dtype=np.int64)
        for c in cells.tolist():
            q = cell_qc(res, c, names[c], L)
            self.cell_stats.append(q)
            self.cell_depths[names[c]] = q["mean_depth"]
        done = getattr(res, "txt_gz_cells", None)
        if done is None or not np.array_equal(np.asarray(done, np.int64), cells):
            txt_write_cells(self.prefix, res.counts, res.depth, cells, [names[c] for c in cells.tolist()],
                            level=self.gzip_level, n_threads=self.n_threads)
        # (else the count files were written on the device: CellProcessor.enable_device_txt)
        if tally is not None:
            self.position_base_counts += tally.astype(np.int64)
        else:
            for c in cells.tolist():
                cnt = res.counts[c].astype(np.int64)
                self.position_base_counts += cnt[:, 0::2] + cnt[:, 1::2]

    # reference per-cell API (writers.py:430-462) ----------------------------
    def write_cell(self, result: dict):
        one = _OneCell(result, self.config.mito_length)
        if "qc" in result:
            self.cell_stats.append(result["qc"])
        kept = one.depth[0][one.depth[0] > 0]
        self.cell_depths[result["barcode"]] = float(kept.sum()) / kept.size if kept.size else 0
        txt_write_cells(self.prefix, one.counts, one.depth, [0], [result["barcode"]], level=self.gzip_level,
                        n_threads=1)
        cnt = one.counts[0].astype(np.int64)
        self.position_base_counts += cnt[:, 0::2] + cnt[:, 1::2]

    def finalize(self, qc_dir: Path):
        with open(self.output_dir / "output.depthTable.txt", "w") as f:
            for cell, depth in sorted(self.cell_depths.items()):
                f.write(f"{cell}\t{depth:.2f}\n")
        refs = ref_alleles(self.position_base_counts)
        with open(self.output_dir / f"{self.config.mito_chr}_refAllele.txt", "w") as f:
            f.write("pos\tref\n")
            f.write("".join(f"{p}\t{r}\n" for p, r in enumerate(refs, start=1)))
        qc_dir = Path(qc_dir)
        qc_dir.mkdir(exist_ok=True, parents=True)
        if self.cell_stats:
            write_cell_stats(self.cell_stats, qc_dir / "cell_stats.csv")


# ---------------------------------------------------------------------------
# HDF5
# ---------------------------------------------------------------------------
def _h5py():
    """h5py when installed, else the ctypes binding of libhdf5 (mgatk2_amd.h5lite)."""
    try:
        import h5py  # noqa: F401

        return h5py
    except ImportError:
        pass
    from .. import h5lite

    if not h5lite.available():  # pragma: no cover - depends on the environment
        raise ImportError("HDF5 output needs h5py or libhdf5 (set MGP_HDF5_LIB); use --format txt")
    return h5lite.module()


def hdf5_columns(writer_barcodes: list[str], names: list[str], cells) -> tuple[np.ndarray, np.ndarray]:
    """The cells of `cells` that IncrementalHDF5Writer.write_cells stores and their
    columns: a cell whose barcode (names[c]) is in the writer's list goes to that
    barcode's column (the last duplicate's, writers.py:146-152)."""
    to_idx = {bc: i for i, bc in enumerate(writer_barcodes)}
    sel, cols = [], []
    for c in np.asarray(cells, dtype=np.int64).tolist():
        j = to_idx.get(names[c])
        if j is not None:
            sel.append(c)
            cols.append(j)
    return np.asarray(sel, np.int64), np.asarray(cols, np.int64)


def hdf5_cell_of_col(n_cols: int, sel: np.ndarray, cols: np.ndarray) -> np.ndarray:
    """Column -> cell of the written cells (-1: an empty column; a later cell of the
    same column wins)."""
    coc = np.full(n_cols, -1, np.int64)
    coc[cols] = sel
    return coc


class IncrementalHDF5Writer:
    """counts.h5 / metadata.h5 (writers.py:20-406)."""

    def __init__(self, output_dir: Path, config, barcodes: list[str], barcode_metadata=None, h5=None):
        self.h5 = h5 if h5 is not None else _h5py()
        self.output_dir = Path(output_dir) / "output"
        self.output_dir.mkdir(exist_ok=True, parents=True)
        self.config = config
        self.barcodes = list(barcodes)
        self.barcode_to_idx = {bc: i for i, bc in enumerate(self.barcodes)}  # last duplicate wins
        self.n_barcodes = len(self.barcodes)
        self.n_positions = config.mito_length
        self.barcode_metadata = barcode_metadata
        self.cell_stats: list[dict] = []
        self.position_base_counts = np.zeros((self.n_positions, 4), np.int64)
        self.cell_depths: dict[str, float] = {}
        L, n = self.n_positions, self.n_barcodes
        # the engine's arrays and their columns (write_cells): the planes are built, chunked
        # and deflated natively at finalize (mgp_h5_plane_tiles); the per-cell API
        # (write_cell) fills dense column buffers instead
        self._sources: list[tuple] = []
        self._planes = self._tn5 = self._coverage = None
        self.report_arrays = None
        self._meta = {
            "mean_depth": np.zeros(n, np.float32),
            "median_depth": np.zeros(n, np.float32),
            "max_depth": np.zeros(n, np.uint16),
            "genome_coverage": np.zeros(n, np.float32),
            "total_bases": np.zeros(n, np.float32),
        }

    def _dense(self):
        """The column buffers of the dense path (flushed once per dataset; the
        reference writes per 250-cell batch), with every recorded source's columns."""
        if self._planes is None:
            L, n = self.n_positions, self.n_barcodes
            self._planes = {f"{b}_{s}": np.zeros((L, n), np.uint16) for b in BASES for s in STRANDS}
            self._tn5 = {s: np.zeros((L, n), np.uint16) for s in STRANDS}
            self._coverage = np.zeros((L, n), np.uint16)
            for res, sel_a, col_a in self._sources:
                for bi, b in enumerate(BASES):
                    for si, s in enumerate(STRANDS):
                        self._planes[f"{b}_{s}"][:, col_a] = np.minimum(res.counts[sel_a, :, 2 * bi + si], 65535).T
                for si, s in enumerate(STRANDS):
                    self._tn5[s][:, col_a] = np.minimum(res.tn5[sel_a, :, si], 65535).T
                self._coverage[:, col_a] = np.minimum(res.depth[sel_a], 65535).T
            self._sources = []

    def _put(self, col: int, counts: np.ndarray, tn5: np.ndarray, depth: np.ndarray, med_lo: int, med_hi: int,
             depth_sum: int, covered: int, depth_max: int):
        self._dense()
        sat = np.minimum(counts, 65535).astype(np.uint16)
        for bi, b in enumerate(BASES):
            self._planes[f"{b}_fwd"][:, col] = sat[:, 2 * bi]
            self._planes[f"{b}_rev"][:, col] = sat[:, 2 * bi + 1]
        t = np.minimum(tn5, 65535).astype(np.uint16)
        self._tn5["fwd"][:, col] = t[:, 0]
        self._tn5["rev"][:, col] = t[:, 1]
        self._coverage[:, col] = np.minimum(depth, 65535).astype(np.uint16)
        mean = float(depth_sum) / covered
        self._meta["mean_depth"][col] = mean
        self._meta["median_depth"][col] = (float(med_lo) + float(med_hi)) / 2.0  # np.median of ints
        self._meta["max_depth"][col] = min(int(depth_max), 65535)
        self._meta["genome_coverage"][col] = covered / self.n_positions * 100
        self._meta["total_bases"][col] = np.float32(np.int64(depth_sum))
        return mean

    def write_cells(self, res, cells, barcodes: list[str] | None = None, tally: np.ndarray | None = None):
        """Columns of the given cells (whitelist index of their barcode), vectorised
        over cells; values as in _put (writers.py:154-264)."""
        names = barcodes if barcodes is not None else self.barcodes
        self.report_arrays = None
        sel_a, col_a = hdf5_columns(self.barcodes, names, cells)
        for c in sel_a.tolist():
            bc = names[c]
            q = cell_qc(res, c, bc, self.n_positions)
            self.cell_stats.append(q)
            self.cell_depths[bc] = q["mean_depth"]
        if sel_a.size:
            self._sources.append((res, sel_a, col_a))
            if self._planes is not None:
                self._dense()
            covered = res.covered[sel_a].astype(np.float64)
            dsum = res.depth_sum[sel_a]
            self._meta["mean_depth"][col_a] = (dsum.astype(np.float64) / covered).astype(np.float32)
            self._meta["median_depth"][col_a] = ((res.median_lo[sel_a].astype(np.float64)
                                                  + res.median_hi[sel_a].astype(np.float64)) / 2.0).astype(np.float32)
            self._meta["max_depth"][col_a] = np.minimum(res.depth_max[sel_a], 65535).astype(np.uint16)
            self._meta["genome_coverage"][col_a] = (res.covered[sel_a] / self.n_positions * 100).astype(np.float32)
            self._meta["total_bases"][col_a] = dsum.astype(np.int64).astype(np.float32)
        if tally is not None:
            self.position_base_counts += tally.astype(np.int64)
        else:
            for c in cells:
                cnt = res.counts[int(c)].astype(np.int64)
                self.position_base_counts += cnt[:, 0::2] + cnt[:, 1::2]

    def _device_tiles(self, coc: np.ndarray, chunks):
        """The device's chunks of the one recorded source (CellProcessor.enable_device_h5:
        (cell_of_col, chunks, tiles, column sums)) when they are of these columns and chunks."""
        if len(self._sources) != 1:
            return None
        dev = getattr(self._sources[0][0], "h5_tiles", None)
        if dev is None or tuple(dev[1]) != tuple(chunks) or not np.array_equal(dev[0], coc):
            return None
        return dev

    def _report_arrays(self, refs: list[str]) -> dict:
        """What the HTML report reads back from the files (report.py _load), from
        memory: per-position sums over the columns of the coverage and Tn5 planes (of
        the saturated u16 values, as stored) and the metadata arrays."""
        L, n = self.n_positions, self.n_barcodes
        sums = {k: np.zeros(L, np.int64) for k in ("coverage", "tn5_fwd", "tn5_rev")}
        dev = None
        if self._planes is None and len(self._sources) == 1 and n:
            res, sel_a, col_a = self._sources[0]
            dev = self._device_tiles(hdf5_cell_of_col(n, sel_a, col_a), (min(1000, L), min(100, n)))
        if dev is not None and len(dev) > 3:  # the device's sums over the stored planes' columns
            sums = {k: np.asarray(dev[3][k], np.int64) for k in ("coverage", "tn5_fwd", "tn5_rev")}
        elif self._planes is not None:
            sums["coverage"] = self._coverage.sum(axis=1, dtype=np.int64)
            sums["tn5_fwd"] = self._tn5["fwd"].sum(axis=1, dtype=np.int64)
            sums["tn5_rev"] = self._tn5["rev"].sum(axis=1, dtype=np.int64)
        else:
            for res, sel_a, _ in self._sources:
                for i in range(0, sel_a.size, 512):
                    part = sel_a[i:i + 512]
                    d = res.depth[part]
                    t = res.tn5[part]
                    if d.dtype != np.uint16:
                        d, t = np.minimum(d, 65535), np.minimum(t, 65535)
                    sums["coverage"] += d.sum(axis=0, dtype=np.int64)
                    sums["tn5_fwd"] += t[:, :, 0].sum(axis=0, dtype=np.int64)
                    sums["tn5_rev"] += t[:, :, 1].sum(axis=0, dtype=np.int64)
        total = None
        if self.barcode_metadata is not None and "total" in self.barcode_metadata:
            bl = self.barcode_metadata.get("barcode", [])
            b2i = {bc: i for i, bc in enumerate(bl)}
            try:
                total = np.asarray([self.barcode_metadata["total"][b2i[bc]] for bc in self.barcodes if bc in b2i],
                                   dtype=np.float64)
            except (TypeError, ValueError, IndexError):
                total = None
        return {"coverage_mean": sums["coverage"] / n if n else np.zeros(L), "coverage_sum": sums["coverage"],
                "tn5_fwd": sums["tn5_fwd"], "tn5_rev": sums["tn5_rev"], "mean_depth": self._meta["mean_depth"],
                "genome_coverage": self._meta["genome_coverage"], "total_bases": self._meta["total_bases"],
                "reference": list(refs), "total": total if total is not None else np.zeros(0)}

    def prepare_report_arrays(self) -> dict:
        """The report's arrays as finalize leaves them, computed now (from memory) so
        the figures can be rendered while finalize writes the files."""
        if self.report_arrays is None:
            self.report_arrays = self._report_arrays(ref_alleles(self.position_base_counts))
        return self.report_arrays

    def write_cell(self, result: dict):
        """Reference per-cell API (writers.py:136-152)."""
        bc = result["barcode"]
        if bc not in self.barcode_to_idx:
            return
        self.report_arrays = None
        one = _OneCell(result, self.n_positions)
        if "qc" in result:
            self.cell_stats.append(result["qc"])
        col = self.barcode_to_idx[bc]
        self.cell_depths[bc] = self._put(
            col, one.counts[0], one.tn5[0], one.depth[0], int(one.median_lo[0]), int(one.median_hi[0]),
            int(one.depth_sum[0]), int(one.covered[0]), int(one.depth_max[0]),
        )
        cnt = one.counts[0].astype(np.int64)
        self.position_base_counts += cnt[:, 0::2] + cnt[:, 1::2]

    def finalize(self, qc_dir: Path):
        h5 = self.h5
        L, n = self.n_positions, self.n_barcodes
        chunks = (min(1000, L), min(100, n)) if n else None
        comp = dict(compression="gzip", compression_opts=4)
        counts_file = h5.File(self.output_dir / "counts.h5", "w", libver="latest")
        counts_file.attrs["n_cells"] = n
        counts_file.attrs["n_positions"] = L
        counts_file.attrs["mito_chr"] = self.config.mito_chr
        counts_file.create_dataset("barcode", data=np.array(self.barcodes, dtype="S"))
        names = [f"{b}_{s}" for b in BASES for s in STRANDS]
        native = (n > 0 and self._planes is None and len(self._sources) == 1
                  and hasattr(counts_file, "create_dataset_from_chunks"))
        if native:
            # the planes straight from the engine's cell-major rows, chunked and deflated in
            # one native pass (the transposes, not the deflate, were the writer's cost)
            from ..bam import h5_plane_tiles

            res, sel_a, col_a = self._sources[0]
            coc = hdf5_cell_of_col(n, sel_a, col_a)
            dev = self._device_tiles(coc, chunks)  # (deflated on the device: CellProcessor.enable_device_h5)
            if dev is not None:
                tiles = dev[2]
            else:
                tiles = {**dict(zip(names, h5_plane_tiles(res.counts, coc, list(range(8)), chunks, level=4))),
                         **dict(zip(("tn5_cuts_fwd", "tn5_cuts_rev"), h5_plane_tiles(res.tn5, coc, [0, 1], chunks,
                                                                                      level=4))),
                         "coverage": h5_plane_tiles(res.depth, coc, [0], chunks, level=4)[0]}
            for k in names + ["tn5_cuts_fwd", "tn5_cuts_rev"]:
                counts_file.create_dataset_from_chunks(k, (L, n), np.uint16, chunks, 4, tiles[k])
        else:
            self._dense()
            for k in names:
                counts_file.create_dataset(k, data=self._planes[k], chunks=chunks, **comp)
            for s in STRANDS:
                counts_file.create_dataset(f"tn5_cuts_{s}", data=self._tn5[s], chunks=chunks, **comp)
        meta = h5.File(self.output_dir / "metadata.h5", "w", libver="latest")
        meta.attrs["mito_chr"] = self.config.mito_chr
        meta.attrs["mito_length"] = L
        if native:
            meta.create_dataset_from_chunks("coverage", (L, n), np.uint16, chunks, 4, tiles["coverage"])
        else:
            meta.create_dataset("coverage", data=self._coverage, chunks=chunks, **comp)
        for k, v in self._meta.items():
            meta.create_dataset(k, data=v)
        refs = ref_alleles(self.position_base_counts)
        meta.create_dataset("reference", data=np.array(refs, dtype="S1"), **comp)
        if self.barcode_metadata is not None:
            grp = meta.create_group("barcode_metadata")
            bl = self.barcode_metadata.get("barcode", [])
            b2i = {bc: i for i, bc in enumerate(bl)}
            reorder = [b2i[bc] for bc in self.barcodes if bc in b2i]
            for col, values_list in self.barcode_metadata.items():
                try:
                    vals = [values_list[i] for i in reorder]
                    arr = np.array(vals)
                    if arr.dtype == object or (len(arr) > 0 and isinstance(arr[0], str)):
                        arr = np.array(vals, dtype="S")
                    grp.create_dataset(col, data=arr, **comp)
                except Exception as e:  # writers.py:387-388
                    logger.warning("Could not store metadata column '%s': %s", col, e)
        counts_file.close()
        meta.close()
        if self.report_arrays is None:
            self.report_arrays = self._report_arrays(refs)
        qc_dir = Path(qc_dir)
        qc_dir.mkdir(exist_ok=True, parents=True)
        if self.cell_stats:
            write_cell_stats(self.cell_stats, qc_dir / "cell_stats.csv")
