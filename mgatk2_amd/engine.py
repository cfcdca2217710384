"""ctypes binding of libmgpileup.so (include/mgpileup.h).

This is the only way the package reaches the GPU: there is no CPU fallback.
If the library is missing or no HIP device is present, :class:`Engine` raises.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from pathlib import Path

import numpy as np

from .exceptions import BAMFormatError, BAMReadError, InvalidInputError, ProcessingError
from .synth import ReadSoA

import os

# MGP_LIB selects an alternative build of the same engine (A/B experiments only)
LIB_PATH = Path(os.environ.get("MGP_LIB") or Path(__file__).resolve().parent / "_lib" / "libmgpileup.so")

MGP_OK = 0
MGP_E_INVALID = -1
MGP_E_HIP = -2
MGP_E_OOM = -3
MGP_E_UNSORTED = -4
MGP_E_BADREAD = -5
MGP_E_SPAN = -6
MGP_E_STATE = -7
MGP_E_COMM = -8

DEDUP_MODES = {"none": 0, "alignment_start": 1, "alignment_and_fragment_length": 2}

# names of every entry point declared in include/mgpileup.h
ABI_SYMBOLS = (
    "mgp_abi_version", "mgp_last_error", "mgp_device_count", "mgp_open", "mgp_close", "mgp_host_alloc",
    "mgp_host_free", "mgp_push_batch", "mgp_reset", "mgp_resident", "mgp_run", "mgp_sync", "mgp_fetch",
    "mgp_finish", "mgp_kernel_times", "mgp_comm_unique_id", "mgp_comm_init", "mgp_synth_generate",
    "mgp_download_inputs", "mgp_set_stage_timing", "mgp_fetch_cells", "mgp_fetch_rows16", "mgp_windows",
    "mgp_stream_info", "mgp_set_streaming", "mgp_set_rows16_target", "mgp_copy_wait", "mgp_set_cell_range",
    "mgp_push_batch16", "mgp_txt_gz_run", "mgp_txt_gz_fetch", "mgp_txt_gz_rows", "mgp_set_rows_target",
    "mgp_h5_tiles_run", "mgp_h5_tiles_fetch",
)
ABI_VERSION = 7
CFG_KEEP_TN5 = 0x1
CFG_STREAM = 0x2


class mgp_config(C.Structure):
    _fields_ = [
        ("min_baseq", C.c_int32),
        ("min_mapq", C.c_int32),
        ("min_dist_from_end", C.c_int32),
        ("dedup_mode", C.c_int32),
        ("max_strand_bias", C.c_double),
        ("min_reads", C.c_int32),
        ("n_cells", C.c_int32),
        ("mito_len", C.c_int32),
        ("flags", C.c_int32),
        ("reserve_reads", C.c_int64),
        ("reserve_payload", C.c_int64),
    ]


class mgp_batch16(C.Structure):
    _fields_ = [
        ("n_reads", C.c_int64),
        ("bc", C.c_void_p),
        ("abs_tlen", C.c_void_p),
        ("flag", C.c_void_p),
        ("mapq", C.c_void_p),
        ("payload", C.c_void_p),
        ("payload_bytes", C.c_int64),
    ]


class mgp_batch(C.Structure):
    _fields_ = [
        ("n_reads", C.c_int64),
        ("start", C.c_void_p),
        ("bc", C.c_void_p),
        ("tlen", C.c_void_p),
        ("flag", C.c_void_p),
        ("mapq", C.c_void_p),
        ("span", C.c_void_p),
        ("rec_off", C.c_void_p),
        ("payload", C.c_void_p),
        ("payload_bytes", C.c_int64),
    ]


class mgp_stats(C.Structure):
    _fields_ = [
        ("total_reads", C.c_int64),
        ("filtered_reads", C.c_int64),
        ("n_barcodes", C.c_int64),
        ("duplicate_reads_with_length", C.c_int64),
        ("duplicate_reads_position_only", C.c_int64),
        ("cells_passed", C.c_int64),
        ("max_span", C.c_int32),
        ("error_bits", C.c_int32),
    ]

    def as_dict(self) -> dict:
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


class mgp_result(C.Structure):
    _fields_ = [
        ("counts", C.c_void_p),
        ("tn5", C.c_void_p),
        ("depth", C.c_void_p),
        ("n_reads", C.c_void_p),
        ("any_paired", C.c_void_p),
        ("passed", C.c_void_p),
        ("covered", C.c_void_p),
        ("depth_sum", C.c_void_p),
        ("depth_max", C.c_void_p),
        ("median_lo", C.c_void_p),
        ("median_hi", C.c_void_p),
        ("first_read", C.c_void_p),
        ("ref_tally", C.c_void_p),
        ("stats", C.POINTER(mgp_stats)),
    ]


class mgp_synth_params(C.Structure):
    _fields_ = [
        ("seed", C.c_uint64),
        ("n_reads", C.c_int64),
        ("read_len", C.c_int32),
        ("n_cells", C.c_int32),
        ("cell_cdf", C.c_void_p),
        ("ref_codes", C.c_void_p),
        ("rec_align", C.c_int32),
        ("pack", C.c_int32),
        ("rec_off", C.c_void_p),
        ("payload_bytes", C.c_int64),
        ("cell_lo", C.c_int32),
        ("cell_hi", C.c_int32),
        ("shard_rank", C.c_int32),
        ("shard_world", C.c_int32),
        ("pack_min_baseq", C.c_int32),
        ("pack_min_dist", C.c_int32),
        ("n_rec_off", C.c_int64),
    ]


class mgp_txt_gz(C.Structure):
    _fields_ = [
        ("n_cells", C.c_int64),
        ("cells", C.c_void_p),
        ("names", C.c_void_p),
        ("name_off", C.c_void_p),
        ("member_bytes", C.c_void_p),
        ("text_bytes", C.c_void_p),
    ]


class mgp_h5_tiles(C.Structure):
    _fields_ = [
        ("n_cols", C.c_int64),
        ("cell_of_col", C.c_void_p),
        ("chunk_rows", C.c_int32),
        ("chunk_cols", C.c_int32),
        ("col_chunk_lo", C.c_int32),
        ("col_chunk_hi", C.c_int32),
        ("chunk_bytes", C.c_void_p),
        ("col_sums", C.c_void_p),
    ]


H5_PLANES = ("A_fwd", "A_rev", "C_fwd", "C_rev", "G_fwd", "G_rev", "T_fwd", "T_rev", "tn5_cuts_fwd", "tn5_cuts_rev",
             "coverage")  # the planes of mgp_h5_tiles, in its order


class mgp_rows16(C.Structure):
    _fields_ = [
        ("counts", C.c_void_p),
        ("tn5", C.c_void_p),
        ("depth", C.c_void_p),
        ("wide", C.c_void_p),
    ]


class mgp_rows8(C.Structure):
    _fields_ = [
        ("counts", C.c_void_p),
        ("tn5", C.c_void_p),
        ("depth", C.c_void_p),
        ("narrow", C.c_void_p),
    ]


_lib = None


def load_library(path: Path | None = None) -> C.CDLL:
    """Load libmgpileup.so; raises if it is absent (no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise ProcessingError(
            f"HIP engine library not found at {p}; build it with `python -m mgatk2_amd.build` "
            "(hipcc --offload-arch=gfx950)"
        )
    lib = C.CDLL(str(p))
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    sig = {
        "mgp_abi_version": ([], C.c_int),
        "mgp_last_error": ([], C.c_char_p),
        "mgp_device_count": ([C.POINTER(C.c_int)], C.c_int),
        "mgp_open": ([C.POINTER(mgp_config), C.c_int, C.POINTER(vp)], C.c_int),
        "mgp_close": ([vp], None),
        "mgp_host_alloc": ([i64, C.POINTER(vp)], C.c_int),
        "mgp_host_free": ([vp], C.c_int),
        "mgp_push_batch": ([vp, C.POINTER(mgp_batch)], C.c_int),
        "mgp_push_batch16": ([vp, C.POINTER(mgp_batch16)], C.c_int),
        "mgp_reset": ([vp], C.c_int),
        "mgp_resident": ([vp, C.POINTER(i64), C.POINTER(i64)], C.c_int),
        "mgp_run": ([vp], C.c_int),
        "mgp_sync": ([vp], C.c_int),
        "mgp_fetch": ([vp, C.POINTER(mgp_result)], C.c_int),
        "mgp_finish": ([vp, C.POINTER(mgp_result)], C.c_int),
        "mgp_kernel_times": (
            [vp, C.c_int, C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int), C.c_char_p, C.c_int], C.c_int
        ),
        "mgp_set_stage_timing": ([vp, C.c_int], C.c_int),
        "mgp_comm_unique_id": ([C.c_char_p], C.c_int),
        "mgp_comm_init": ([vp, C.c_char_p, C.c_int, C.c_int], C.c_int),
        "mgp_synth_generate": ([vp, C.POINTER(mgp_synth_params)], C.c_int),
        "mgp_download_inputs": ([vp] + [vp] * 8, C.c_int),
        "mgp_fetch_cells": ([vp, i32, i32, C.POINTER(mgp_result)], C.c_int),
        "mgp_fetch_rows16": ([vp, i32, i32, C.POINTER(mgp_rows16)], C.c_int),
        "mgp_set_rows16_target": ([vp, C.POINTER(mgp_rows16)], C.c_int),
        "mgp_set_rows_target": ([vp, C.POINTER(mgp_rows16), C.POINTER(mgp_rows8)], C.c_int),
        "mgp_windows": ([vp, C.POINTER(i32), C.POINTER(i32)], C.c_int),
        "mgp_stream_info": ([vp, C.POINTER(i64), C.POINTER(i32)], C.c_int),
        "mgp_set_streaming": ([vp, C.c_int], C.c_int),
        "mgp_set_cell_range": ([vp, C.c_int32, C.c_int32], C.c_int),
        "mgp_copy_wait": ([vp], C.c_int),
        "mgp_txt_gz_run": ([vp, C.POINTER(mgp_txt_gz), C.POINTER(i64)], C.c_int),
        "mgp_h5_tiles_run": ([vp, C.POINTER(mgp_h5_tiles), C.POINTER(i64)], C.c_int),
        "mgp_h5_tiles_fetch": ([vp, vp, i64], C.c_int),
        "mgp_txt_gz_fetch": ([vp, vp, i64], C.c_int),
        "mgp_txt_gz_rows": ([C.c_int, vp, vp, i32, i32, C.POINTER(mgp_txt_gz), vp, i64, C.POINTER(i64)], C.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    if lib.mgp_abi_version() != ABI_VERSION:
        raise ProcessingError("libmgpileup ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def _raise(code: int, what: str):
    lib = load_library()
    msg = (lib.mgp_last_error() or b"").decode(errors="replace")
    text = f"{what}: {msg} (code {code})"
    if code == MGP_E_INVALID or code == MGP_E_SPAN:
        raise InvalidInputError(text)
    if code == MGP_E_UNSORTED:
        raise BAMFormatError("<resident reads>", text)
    if code == MGP_E_BADREAD:
        raise BAMReadError("<resident reads>", text)
    raise ProcessingError(text)


def _ck(code: int, what: str):
    if code != MGP_OK:
        _raise(code, what)


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


@dataclass
class EngineConfig:
    """POD restatement of the hot-path fields of PipelineConfig (config.py:77-114)."""

    n_cells: int
    min_baseq: int = 20
    min_mapq: int = 30
    min_distance_from_end: int = 5
    dedup_mode: str | int = "alignment_and_fragment_length"
    max_strand_bias: float = 1.0
    min_reads: int = 1
    mito_len: int = 16569
    reserve_reads: int = 0
    reserve_payload: int = 0
    keep_tn5: bool = False  # MGP_CFG_KEEP_TN5
    stream: bool = False  # MGP_CFG_STREAM: pushes run the windows they complete (overlapped H2D)

    def to_c(self) -> mgp_config:
        dm = DEDUP_MODES[self.dedup_mode] if isinstance(self.dedup_mode, str) else int(self.dedup_mode)
        flags = (CFG_KEEP_TN5 if self.keep_tn5 else 0) | (CFG_STREAM if self.stream else 0)
        return mgp_config(
            int(self.min_baseq), int(self.min_mapq), int(self.min_distance_from_end), dm,
            float(self.max_strand_bias), int(self.min_reads), int(self.n_cells), int(self.mito_len),
            flags, int(self.reserve_reads), int(self.reserve_payload),
        )


@dataclass
class EngineResult:
    """Host copy of mgp_result (cell-major arrays)."""

    counts: np.ndarray | None  # [n_cells, L, 8] u32
    tn5: np.ndarray | None  # [n_cells, L, 2] u32
    depth: np.ndarray | None  # [n_cells, L] u32
    n_reads: np.ndarray
    any_paired: np.ndarray
    passed: np.ndarray
    covered: np.ndarray
    depth_sum: np.ndarray
    depth_max: np.ndarray
    median_lo: np.ndarray
    median_hi: np.ndarray
    first_read: np.ndarray
    ref_tally: np.ndarray  # [L, 4] u64
    stats: dict

    @staticmethod
    def alloc(n_cells: int, L: int, dense: bool = True) -> EngineResult:
        return EngineResult(
            counts=np.zeros((n_cells, L, 8), np.uint32) if dense else None,
            tn5=np.zeros((n_cells, L, 2), np.uint32) if dense else None,
            depth=np.zeros((n_cells, L), np.uint32) if dense else None,
            n_reads=np.zeros(n_cells, np.uint32),
            any_paired=np.zeros(n_cells, np.uint8),
            passed=np.zeros(n_cells, np.uint8),
            covered=np.zeros(n_cells, np.uint32),
            depth_sum=np.zeros(n_cells, np.uint64),
            depth_max=np.zeros(n_cells, np.uint32),
            median_lo=np.zeros(n_cells, np.uint32),
            median_hi=np.zeros(n_cells, np.uint32),
            first_read=np.zeros(n_cells, np.uint32),
            ref_tally=np.zeros((L, 4), np.uint64),
            stats={},
        )

    def to_c(self, stats: mgp_stats) -> mgp_result:
        return mgp_result(
            _ptr(self.counts), _ptr(self.tn5), _ptr(self.depth), _ptr(self.n_reads), _ptr(self.any_paired),
            _ptr(self.passed), _ptr(self.covered), _ptr(self.depth_sum), _ptr(self.depth_max),
            _ptr(self.median_lo), _ptr(self.median_hi), _ptr(self.first_read), _ptr(self.ref_tally),
            C.pointer(stats),
        )

    def cell_order(self) -> np.ndarray:
        """Cells with >= 1 kept read in first-seen BAM order (dict order of reads_by_barcode)."""
        idx = np.flatnonzero(self.n_reads > 0)
        return idx[np.argsort(self.first_read[idx], kind="stable")]


@dataclass
class Rows16:
    """The pileup's 16-bit result rows of a cell range (mgp_rows16): exact except in
    `wide` (cell, window) pairs, where they saturate at 65535."""

    counts: np.ndarray  # [cells, L, 8] u16
    tn5: np.ndarray  # [cells, L, 2] u16
    depth: np.ndarray  # [cells, L] u16
    wide: np.ndarray  # [cells, n_windows] u8
    window_width: int

    def wide_cells(self) -> np.ndarray:
        """Cells (range-relative) with a window whose 16-bit rows are not exact."""
        return np.flatnonzero(self.wide.any(axis=1))


@dataclass
class Rows8:
    """The 8-bit rows target beside a Rows16 one (mgp_rows8, ABI 7): the rows of the
    (cell, window) pairs whose values all fit a byte (`narrow`); the others are in the
    16-bit target."""

    counts: np.ndarray  # [cells, L, 8] u8
    tn5: np.ndarray  # [cells, L, 2] u8
    depth: np.ndarray  # [cells, L] u8
    narrow: np.ndarray  # [cells, n_windows] u8


def merge_rows(r16: Rows16, r8: Rows8 | None, lo: int, hi: int) -> dict:
    """Cells [lo, hi) of a rows target as u32 arrays (counts, tn5, depth): each window
    from the 8-bit target where it is narrow, else from the 16-bit one (exact unless
    r16.wide)."""
    out = {"counts": r16.counts[lo:hi].astype(np.uint32), "tn5": r16.tn5[lo:hi].astype(np.uint32),
           "depth": r16.depth[lo:hi].astype(np.uint32)}
    if r8 is None:
        return out
    W = r16.window_width
    L = out["depth"].shape[1]
    nar = r8.narrow[lo:hi].astype(bool)
    for k in range(nar.shape[1]):
        m = np.flatnonzero(nar[:, k])
        if m.size == 0:
            continue
        a, b = k * W, min(L, (k + 1) * W)
        for key in ("counts", "tn5", "depth"):
            out[key][m, a:b] = getattr(r8, key)[lo + m, a:b]
    return out


def batch_struct(soa: ReadSoA) -> mgp_batch:
    """The C batch of a ReadSoA. ``span`` and ``rec_off`` may be None (ABI v3.1): the
    spans then come from the records' CIGARs on the device, and the records are dense
    in BAM order (record i at i x payload bytes / n); ``start`` may be None (ABI 4):
    taken from each record on the device."""
    for name in ("start", "bc", "tlen", "flag", "mapq", "span", "rec_off", "payload"):
        a = getattr(soa, name)
        if a is None and name in ("start", "span", "rec_off"):
            continue
        if not a.flags["C_CONTIGUOUS"]:
            raise InvalidInputError(f"batch array {name} must be C-contiguous")
    return mgp_batch(
        soa.n, _ptr(soa.start), _ptr(soa.bc), _ptr(soa.tlen), _ptr(soa.flag), _ptr(soa.mapq), _ptr(soa.span),
        _ptr(soa.rec_off), _ptr(soa.payload), int(soa.payload.shape[0]),
    )


TXT_FILES = ("coverage", "A", "C", "G", "T")  # the member order of mgp_txt_gz (file-major)


@dataclass
class TxtMembers:
    """The gzip members of mgp_txt_gz: `blob` holds them file-major (all coverage
    members in cell order, then A, C, G, T); member_bytes / text_bytes are [5, n]."""

    blob: np.ndarray
    member_bytes: np.ndarray
    text_bytes: np.ndarray

    def file_part(self, f: int) -> np.ndarray:
        """The bytes of file f (0 coverage, 1..4 A..T): its members back to back."""
        per = self.member_bytes.sum(axis=1)
        a = int(per[:f].sum())
        return self.blob[a:a + int(per[f])]


def _txt_job(cells, names: list[str]):
    cells = np.ascontiguousarray(cells, dtype=np.int32)
    enc = [n.encode() for n in names]
    if len(enc) != cells.shape[0]:
        raise InvalidInputError("one barcode per written cell")
    off = np.zeros(len(enc) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in enc])
    blob = np.frombuffer(b"".join(enc) or b"\0", np.uint8)
    n = cells.shape[0]
    mb = np.zeros((5, n), np.int64)
    tb = np.zeros((5, n), np.int64)
    job = mgp_txt_gz(n, _ptr(cells), _ptr(blob), _ptr(off), _ptr(mb), _ptr(tb))
    return job, (cells, blob, off), mb, tb


def txt_gz_rows(counts: np.ndarray, depth: np.ndarray, cells, names: list[str], device: int = 0) -> TxtMembers:
    """mgp_txt_gz_rows: the txt members of `cells` from caller-supplied u32 rows
    (counts [n, L, 8], depth [n, L]), no engine context."""
    lib = load_library()
    counts = np.ascontiguousarray(counts, np.uint32)
    depth = np.ascontiguousarray(depth, np.uint32)
    n_rows, L = depth.shape
    if counts.shape != (n_rows, L, 8):
        raise InvalidInputError("counts must be [n, L, 8]")
    job, keep, mb, tb = _txt_job(cells, names)
    # a bound: every member's text (<= bc + 29 bytes per covered position) plus stored-block overhead
    nnz = np.count_nonzero(depth, axis=1)[np.asarray(keep[0], np.int64)] if len(names) else np.zeros(0, np.int64)
    text = nnz.astype(np.int64) * (np.diff(keep[2]) + 29)
    cap = int((5 * (text + 5 * (text // 65535 + 1) + 96)).sum()) + 64
    out = np.empty(cap, np.uint8)
    tot = C.c_int64()
    _ck(lib.mgp_txt_gz_rows(int(device), _ptr(counts), _ptr(depth), int(n_rows), int(L), C.byref(job), _ptr(out), cap,
                            C.byref(tot)), "mgp_txt_gz_rows")
    return TxtMembers(out[:int(tot.value)], mb, tb)


class Engine:
    """One device context (one GPU). Not thread-safe."""

    def __init__(self, cfg: EngineConfig, device: int = 0):
        self.lib = load_library()
        self.cfg = cfg
        self._c = cfg.to_c()
        h = C.c_void_p()
        _ck(self.lib.mgp_open(C.byref(self._c), int(device), C.byref(h)), "mgp_open")
        self._h = h
        self._keep: list = []  # keep host batches alive until the next sync

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self.lib.mgp_close(self._h)
            self._h = None
        self._keep = []

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- data --------------------------------------------------------------
    def push(self, soa: ReadSoA):
        """mgp_push_batch; a batch whose bc and tlen are uint16 arrays (16-bit barcode
        index, 0xFFFF = none, and |tlen|; dense records, no start / span / rec_off) goes
        through mgp_push_batch16."""
        if soa.bc is not None and soa.bc.dtype == np.uint16:
            for name in ("bc", "tlen", "flag", "mapq", "payload"):
                if not getattr(soa, name).flags["C_CONTIGUOUS"]:
                    raise InvalidInputError(f"batch array {name} must be C-contiguous")
            if soa.tlen.dtype != np.uint16 or soa.start is not None or soa.span is not None or soa.rec_off is not None:
                raise InvalidInputError("a 16-bit batch has uint16 bc and |tlen| and dense records only")
            b = mgp_batch16(soa.n, _ptr(soa.bc), _ptr(soa.tlen), _ptr(soa.flag), _ptr(soa.mapq), _ptr(soa.payload),
                            int(soa.payload.shape[0]))
            _ck(self.lib.mgp_push_batch16(self._h, C.byref(b)), "mgp_push_batch16")
        else:
            b = batch_struct(soa)
            _ck(self.lib.mgp_push_batch(self._h, C.byref(b)), "mgp_push_batch")
        self._keep.append(soa)

    def reset(self):
        _ck(self.lib.mgp_reset(self._h), "mgp_reset")
        self._keep = []

    def resident(self) -> tuple[int, int]:
        n, p = C.c_int64(), C.c_int64()
        _ck(self.lib.mgp_resident(self._h, C.byref(n), C.byref(p)), "mgp_resident")
        return int(n.value), int(p.value)

    def synth(self, seed: int, n_reads: int, cdf: np.ndarray, ref: np.ndarray, read_len: int = 50,
              rec_align: int = 64, pack: bool = True, rec_off: np.ndarray | None = None, payload_bytes: int = 0,
              cells: tuple[int, int] | None = None, shard: tuple[int, int] = (0, 0), pack32: int | None = None,
              pack32_dist: int = 5):
        """Device-side synthetic workload (replaces the resident set). rec_off: an
        explicit placement of the records (e.g. host placement of
        mgp_place_records, `synth.place_records`); None = dense in BAM order.
        cells=(lo, hi): only the reads of those cells of the n_reads-read global set
        (len(cdf) cells; this context's n_cells must be hi - lo), barcodes rebased to
        lo, plus the reads without a whitelisted barcode whose index % world == rank
        for shard=(rank, world) (world 0: none). pack32 (a min_baseq): 32-byte
        records made for that threshold and min_dist_from_end pack32_dist (MGP_FLAG_PACK32)
        instead of packed 64-byte ones."""
        cdf = np.ascontiguousarray(cdf, np.uint32)
        ref = np.ascontiguousarray(ref, np.uint8)
        ro = None if rec_off is None else np.ascontiguousarray(rec_off, np.uint64)
        lo, hi = cells if cells is not None else (0, 0)
        if ro is not None and cells is None and ro.shape[0] != n_reads:
            raise ValueError("rec_off must have n_reads entries")
        p = mgp_synth_params(int(seed), int(n_reads), int(read_len), int(cdf.shape[0]), _ptr(cdf), _ptr(ref),
                             int(rec_align), 2 if pack32 is not None else int(bool(pack)),
                             None if ro is None else _ptr(ro), int(payload_bytes) if ro is not None else 0, int(lo),
                             int(hi), int(shard[0]), int(shard[1]), int(pack32 or 0), int(pack32_dist),
                             0 if ro is None else int(ro.shape[0]))
        _ck(self.lib.mgp_synth_generate(self._h, C.byref(p)), "mgp_synth_generate")

    def download_inputs(self, columns: tuple[str, ...] | None = None, alloc=None) -> ReadSoA:
        """Resident inputs back on the host; `columns` limits the copy to those SoA
        fields (the others are empty arrays). alloc(n, dtype) -> array: where the
        columns go (e.g. views of a PinnedBuffer); np.zeros by default."""
        n, pay = self.resident()

        def col(name, dt, m):
            m = m if columns is None or name in columns else 0
            return alloc(m, dt) if alloc is not None and m else np.zeros(m, dt)

        soa = ReadSoA(
            col("start", np.int32, n), col("bc", np.int32, n), col("tlen", np.int32, n), col("flag", np.uint16, n),
            col("mapq", np.uint8, n), col("span", np.uint32, n), col("rec_off", np.uint64, n),
            col("payload", np.uint8, pay),
        )
        _ck(
            self.lib.mgp_download_inputs(
                self._h, *[_ptr(a) if a.shape[0] else None for a in (soa.start, soa.bc, soa.tlen, soa.flag,
                                                                        soa.mapq, soa.span, soa.rec_off,
                                                                        soa.payload)],
            ),
            "mgp_download_inputs",
        )
        return soa

    # -- compute -----------------------------------------------------------
    def run(self):
        _ck(self.lib.mgp_run(self._h), "mgp_run")

    def sync(self):
        code = self.lib.mgp_sync(self._h)
        self._keep = []
        _ck(code, "mgp_sync")

    def fetch(self, dense: bool = True) -> EngineResult:
        res = EngineResult.alloc(self.cfg.n_cells, self.cfg.mito_len, dense)
        st = mgp_stats()
        cres = res.to_c(st)
        _ck(self.lib.mgp_fetch(self._h, C.byref(cres)), "mgp_fetch")
        res.stats = st.as_dict()
        return res

    def fetch_cells(self, lo: int, hi: int, dense: bool = True) -> EngineResult:
        """mgp_fetch_cells: the results of cells [lo, hi) (cell lo at index 0)."""
        res = EngineResult.alloc(hi - lo, self.cfg.mito_len, dense)
        st = mgp_stats()
        cres = res.to_c(st)
        _ck(self.lib.mgp_fetch_cells(self._h, int(lo), int(hi), C.byref(cres)), "mgp_fetch_cells")
        res.stats = st.as_dict()
        return res

    def fetch_compact(self) -> EngineResult:
        """The run's results with the per-position arrays as the pileup's exact
        16-bit rows (u16 counts/tn5/depth: half the bytes of mgp_fetch's u32 arrays,
        no widening pass on the device). A run with a wide window (a cell window of
        more than 65535 reads) falls back to the exact u32 arrays."""
        res = self.fetch(dense=False)
        r16 = self.fetch_rows16()
        if r16.wide.any():
            return self.fetch(dense=True)
        res.counts, res.tn5, res.depth = r16.counts, r16.tn5, r16.depth
        return res

    def txt_gz(self, cells, names: list[str], out: np.ndarray | None = None) -> TxtMembers:
        """mgp_txt_gz_run + mgp_txt_gz_fetch: the txt count files' gzip members of the run's
        `cells` (context cell indices, in output order) named `names`, formatted and
        deflated on the device (writers.py:430-486). `out`: where the members go (e.g. a
        pinned buffer's view, large enough); a new array otherwise."""
        job, keep, mb, tb = _txt_job(cells, names)
        tot = C.c_int64()
        _ck(self.lib.mgp_txt_gz_run(self._h, C.byref(job), C.byref(tot)), "mgp_txt_gz_run")
        n = int(tot.value)
        if out is None or out.shape[0] < n:
            out = np.empty(max(1, n), np.uint8)
        _ck(self.lib.mgp_txt_gz_fetch(self._h, _ptr(out), int(out.shape[0])), "mgp_txt_gz_fetch")
        return TxtMembers(out[:n], mb, tb)

    def h5_tiles(self, cell_of_col, chunks: tuple[int, int] = (1000, 100), cols_per_call: int = 3200,
                 sums: dict | None = None, col_chunks: tuple[int, int] | None = None) -> dict:
        """mgp_h5_tiles_run / _fetch over every column chunk (cols_per_call columns at a
        time): the zlib streams of the HDF5 count datasets' chunks of the run
        (writers.py:60-131), {plane: [chunk (u8 array), row-major over the chunk grid]} for
        the planes of H5_PLANES; column j holds the run's cell cell_of_col[j] (-1: zeros).
        sums (a dict): filled with the per-position sums over the columns of the stored
        coverage / tn5 planes ("coverage", "tn5_fwd", "tn5_rev", int64 [L]). col_chunks
        (c0, c1): only those column chunks (the lists then row-major over that sub-grid)."""
        coc = np.ascontiguousarray(cell_of_col, np.int32)
        crow, ccol = int(chunks[0]), int(chunks[1])
        nrc = -(-self.cfg.mito_len // crow)
        c0, c1 = (0, -(-coc.size // ccol)) if col_chunks is None else (int(col_chunks[0]), int(col_chunks[1]))
        step = max(1, int(cols_per_call) // ccol)
        grid = {p: [[None] * (c1 - c0) for _ in range(nrc)] for p in H5_PLANES}
        L = self.cfg.mito_len
        acc = np.zeros((3, L), np.int64)
        part = np.zeros((3, L), np.int64)
        for lo in range(c0, c1, step):
            hi = min(c1, lo + step)
            cb = np.zeros(len(H5_PLANES) * nrc * (hi - lo), np.int64)
            job = mgp_h5_tiles(coc.size, _ptr(coc), crow, ccol, lo, hi, _ptr(cb), _ptr(part))
            tot = C.c_int64()
            _ck(self.lib.mgp_h5_tiles_run(self._h, C.byref(job), C.byref(tot)), "mgp_h5_tiles_run")
            buf = np.empty(max(1, int(tot.value)), np.uint8)
            _ck(self.lib.mgp_h5_tiles_fetch(self._h, _ptr(buf), int(buf.shape[0])), "mgp_h5_tiles_fetch")
            offs = np.concatenate([[0], np.cumsum(cb)]).tolist()
            k = 0
            for p in H5_PLANES:
                for rc in range(nrc):
                    row = grid[p][rc]
                    for cc in range(lo, hi):
                        row[cc - c0] = buf[offs[k]:offs[k + 1]]  # (views of the call's buffer)
                        k += 1
            acc += part
        if sums is not None:
            sums.update(coverage=acc[0], tn5_fwd=acc[1], tn5_rev=acc[2])
        return {p: [b for row in grid[p] for b in row] for p in H5_PLANES}

    def windows(self) -> tuple[int, int]:
        nw, w = C.c_int32(), C.c_int32()
        _ck(self.lib.mgp_windows(self._h, C.byref(nw), C.byref(w)), "mgp_windows")
        return int(nw.value), int(w.value)

    def fetch_rows16(self, lo: int = 0, hi: int | None = None, out: Rows16 | None = None) -> Rows16:
        """mgp_fetch_rows16: the 16-bit result rows of cells [lo, hi) (into `out`'s
        arrays when given, e.g. pinned host memory)."""
        hi = self.cfg.n_cells if hi is None else hi
        nw, w = self.windows()
        L, m = self.cfg.mito_len, hi - lo
        if out is None:
            out = Rows16(np.empty((m, L, 8), np.uint16), np.empty((m, L, 2), np.uint16), np.empty((m, L), np.uint16),
                         np.empty((m, nw), np.uint8), w)
        for a, shape in ((out.counts, (m, L, 8)), (out.tn5, (m, L, 2)), (out.depth, (m, L)), (out.wide, (m, nw))):
            if a.shape != shape or not a.flags["C_CONTIGUOUS"]:
                raise InvalidInputError(f"rows16 array of shape {a.shape}, expected {shape}")
        r = mgp_rows16(_ptr(out.counts), _ptr(out.tn5), _ptr(out.depth), _ptr(out.wide))
        _ck(self.lib.mgp_fetch_rows16(self._h, int(lo), int(hi), C.byref(r)), "mgp_fetch_rows16")
        return out

    def set_rows16_target(self, rows: Rows16 | None):
        """mgp_set_rows16_target: every run's 16-bit rows of all cells go to `rows`
        (pinned arrays, e.g. PinnedBuffer views) as its windows complete; sync() waits
        for them. None stops it."""
        if rows is None:
            _ck(self.lib.mgp_set_rows16_target(self._h, None), "mgp_set_rows16_target")
            self._rows_tgt = None
            return
        nw, _ = self.windows()
        L, m = self.cfg.mito_len, self.cfg.n_cells
        for a, shape in ((rows.counts, (m, L, 8)), (rows.tn5, (m, L, 2)), (rows.depth, (m, L)), (rows.wide, (m, nw))):
            if a.shape != shape or not a.flags["C_CONTIGUOUS"]:
                raise InvalidInputError(f"rows16 array of shape {a.shape}, expected {shape}")
        r = mgp_rows16(_ptr(rows.counts), _ptr(rows.tn5), _ptr(rows.depth), _ptr(rows.wide))
        _ck(self.lib.mgp_set_rows16_target(self._h, C.byref(r)), "mgp_set_rows16_target")
        self._rows_tgt = rows  # kept alive while the engine copies into it

    def set_rows_target(self, rows: Rows16 | None, rows8: Rows8 | None = None):
        """mgp_set_rows_target (ABI 7): set_rows16_target with the 8-bit target beside
        it (the windows whose values all fit a byte leave as half the bytes; merge_rows
        reads them back)."""
        if rows is None or rows8 is None:
            self.set_rows16_target(rows)
            return
        nw, _ = self.windows()
        L, m = self.cfg.mito_len, self.cfg.n_cells
        for a, shape in ((rows.counts, (m, L, 8)), (rows.tn5, (m, L, 2)), (rows.depth, (m, L)), (rows.wide, (m, nw)),
                         (rows8.counts, (m, L, 8)), (rows8.tn5, (m, L, 2)), (rows8.depth, (m, L)),
                         (rows8.narrow, (m, nw))):
            if a.shape != shape or not a.flags["C_CONTIGUOUS"]:
                raise InvalidInputError(f"rows array of shape {a.shape}, expected {shape}")
        r = mgp_rows16(_ptr(rows.counts), _ptr(rows.tn5), _ptr(rows.depth), _ptr(rows.wide))
        r8 = mgp_rows8(_ptr(rows8.counts), _ptr(rows8.tn5), _ptr(rows8.depth), _ptr(rows8.narrow))
        _ck(self.lib.mgp_set_rows_target(self._h, C.byref(r), C.byref(r8)), "mgp_set_rows_target")
        self._rows_tgt = (rows, rows8)

    def copy_wait(self):
        """mgp_copy_wait: every pushed batch's H2D copies are done (their host
        buffers may be reused). The batches stay referenced until the next sync."""
        _ck(self.lib.mgp_copy_wait(self._h), "mgp_copy_wait")

    def set_cell_range(self, lo: int, hi: int):
        """mgp_set_cell_range: this context's cells are whitelist indices [lo, hi) of the
        batches pushed from now on (hi - lo = its n_cells); the reads of other cells
        count only toward total_reads."""
        _ck(self.lib.mgp_set_cell_range(self._h, int(lo), int(hi)), "mgp_set_cell_range")

    def set_streaming(self, on: bool):
        """Streaming runs on or off for the next pushes (EngineConfig.stream initially)."""
        _ck(self.lib.mgp_set_streaming(self._h, int(bool(on))), "mgp_set_streaming")

    def stream_info(self) -> tuple[int, bool]:
        """(segments queued by pushes so far, whether the last run was streamed)."""
        n, last = C.c_int64(), C.c_int32()
        _ck(self.lib.mgp_stream_info(self._h, C.byref(n), C.byref(last)), "mgp_stream_info")
        return int(n.value), bool(last.value)

    def finish(self, dense: bool = True) -> EngineResult:
        self.run()
        return self.fetch(dense)

    def finish_raw(self) -> tuple[np.ndarray, np.ndarray]:
        """Unfiltered counts/Tn5 of a single-cell context (PileupGenerator.generate_pileup view)."""
        if self.cfg.n_cells != 1 or self.cfg.max_strand_bias < 1.0 or not self.cfg.keep_tn5:
            raise InvalidInputError("finish_raw needs n_cells=1, max_strand_bias>=1 and keep_tn5")
        self.run()
        r = self.fetch(dense=True)
        return r.counts[0], r.tn5[0]

    def kernel_times(self, last_runs: int = 1) -> dict[str, float]:
        """Per-stage device ms averaged over the last `last_runs` runs (HIP events)."""
        ms = (C.c_float * 32)()
        n = C.c_int()
        names = C.create_string_buffer(512)
        _ck(self.lib.mgp_kernel_times(self._h, int(last_runs), ms, 32, C.byref(n), names, 512), "mgp_kernel_times")
        keys = names.value.decode().split(",")
        return {k: float(ms[i]) for i, k in enumerate(keys[: n.value])}

    def set_stage_timing(self, all_stages: bool = True):
        """HIP events around every stage of the next runs (default), or around the
        pileup only: each event is a marker between two kernels of the stream."""
        _ck(self.lib.mgp_set_stage_timing(self._h, int(bool(all_stages))), "mgp_set_stage_timing")

    # -- multi-GPU ---------------------------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        lib = load_library()
        buf = C.create_string_buffer(128)
        _ck(lib.mgp_comm_unique_id(buf), "mgp_comm_unique_id")
        return buf.raw

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        if len(uid) != 128:
            raise InvalidInputError("RCCL unique id must be 128 bytes")
        _ck(self.lib.mgp_comm_init(self._h, C.c_char_p(uid), int(nranks), int(rank)), "mgp_comm_init")


class _PinnedView:
    """numpy array-interface holder that keeps its PinnedBuffer alive."""

    def __init__(self, owner, addr: int, shape, dtype):
        self._owner = owner
        self.__array_interface__ = {"data": (addr, False), "shape": tuple(shape), "typestr": np.dtype(dtype).str,
                                    "version": 3}


class PinnedBuffer:
    """Page-locked host memory from mgp_host_alloc (hipHostMalloc): H2D/D2H copies
    from it run asynchronously at the link's rate. `array(shape, dtype, offset)`
    gives numpy views, which keep the buffer alive."""

    def __init__(self, nbytes: int):
        self.lib = load_library()
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        _ck(self.lib.mgp_host_alloc(max(self.nbytes, 1), C.byref(p)), "mgp_host_alloc")
        self._p = p

    def array(self, shape, dtype, offset: int = 0) -> np.ndarray:
        dt = np.dtype(dtype)
        shape = (int(shape),) if np.ndim(shape) == 0 else tuple(int(x) for x in shape)
        count = int(np.prod(shape))
        if offset % dt.itemsize or offset + count * dt.itemsize > self.nbytes:
            raise ValueError("pinned view outside the buffer or misaligned")
        return np.asarray(_PinnedView(self, self._p.value + offset, shape, dt))

    def __del__(self):
        try:
            if getattr(self, "_p", None) is not None and self._p.value:
                self.lib.mgp_host_free(self._p)
                self._p = None
        except Exception:
            pass


def device_count() -> int:
    lib = load_library()
    n = C.c_int()
    code = lib.mgp_device_count(C.byref(n))
    return int(n.value) if code == MGP_OK else 0
