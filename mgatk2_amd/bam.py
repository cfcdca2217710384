"""BAM access for the host side.

* :class:`BamFile` — ctypes binding of libmgphost.so (include/mgpileup_host.h):
  the native BGZF/BAM decoder that replaces pysam under the reader
  (src/processing/readers.py:37-92): header, `.bai` seek to chrM, chrM records
  decoded straight into the engine's SoA batch.
* :class:`BamWriter` / :func:`write_bai` — a small BGZF/BAM(/BAI) writer used
  to build test fixtures and synthetic inputs (no pysam needed).
"""

from __future__ import annotations

import ctypes as C
import os
import struct
import zlib
from pathlib import Path

import numpy as np

from .exceptions import BAMFormatError, BAMReadError, ProcessingError
from .synth import SEQ_NT16, ReadSoA

HOST_LIB = Path(os.environ.get("MGP_HOST_LIB") or Path(__file__).resolve().parent / "_lib" / "libmgphost.so")
# (MGP_HOST_LIB: another build of the library, e.g. scripts/sanitize_host.sh's ASan / TSan builds)
_NT16 = {ch: i for i, ch in enumerate(SEQ_NT16)}
CIGAR_OPS = "MIDNSHP=X"


class mgp_bam_batch(C.Structure):
    _fields_ = [
        ("n_reads", C.c_int64),
        ("start", C.POINTER(C.c_int32)),
        ("bc", C.POINTER(C.c_int32)),
        ("tlen", C.POINTER(C.c_int32)),
        ("flag", C.POINTER(C.c_uint16)),
        ("mapq", C.POINTER(C.c_uint8)),
        ("span", C.POINTER(C.c_uint32)),
        ("rec_off", C.POINTER(C.c_uint64)),
        ("payload", C.POINTER(C.c_uint8)),
        ("payload_bytes", C.c_int64),
        ("n_with_tag", C.c_int64),
        ("first_tag_index", C.c_int64),
    ]


class mgp_route_part(C.Structure):
    _fields_ = [
        ("cap_reads", C.c_int64), ("cap_payload", C.c_int64),
        ("bc16", C.c_void_p), ("tlen16", C.c_void_p), ("bc32", C.c_void_p), ("tlen32", C.c_void_p),
        ("flag", C.c_void_p), ("mapq", C.c_void_p), ("rec_off", C.c_void_p), ("payload", C.c_void_p),
        ("n_reads", C.c_int64), ("payload_bytes", C.c_int64), ("narrow", C.c_int32), ("pad", C.c_int32),
    ]


_hlib = None


def cgroup_cpu_quota() -> int | None:
    """CPUs the process's cgroup may use (cgroup v2 cpu.max, else v1
    cpu.cfs_quota_us / cpu.cfs_period_us), rounded up; None when unlimited or unknown."""
    import math

    try:
        rel = "/"
        for line in Path("/proc/self/cgroup").read_text().splitlines():
            parts = line.split(":", 2)
            if len(parts) == 3 and (parts[0] == "0" or "cpu" in parts[1].split(",")):
                rel = parts[2] or "/"
                if parts[0] == "0":
                    break
        for base in (Path("/sys/fs/cgroup") / rel.lstrip("/"), Path("/sys/fs/cgroup")):
            f = base / "cpu.max"
            if f.exists():
                fields = f.read_text().split()  # "<quota|max> <period>"
                if len(fields) >= 2 and fields[0] != "max":
                    return max(1, math.ceil(int(fields[0]) / int(fields[1])))
                return None
        for base in (Path("/sys/fs/cgroup/cpu") / rel.lstrip("/"), Path("/sys/fs/cgroup/cpu"),
                     Path("/sys/fs/cgroup/cpu,cpuacct")):
            fq, fp = base / "cpu.cfs_quota_us", base / "cpu.cfs_period_us"
            if fq.exists() and fp.exists():
                q, p = int(fq.read_text()), int(fp.read_text())
                return max(1, math.ceil(q / p)) if q > 0 and p > 0 else None
    except (OSError, ValueError):
        return None
    return None


def host_threads() -> int:
    """Host worker threads: MGP_HOST_THREADS when set; otherwise the CPUs this process
    may run on (its affinity mask) bounded by its cgroup's CPU quota and by
    OMP_NUM_THREADS when that is set (the machine's standard per-process knob)."""
    v = os.environ.get("MGP_HOST_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    q = cgroup_cpu_quota()
    if q is not None:
        n = min(n, q)
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit() and int(v) > 0:
        n = min(n, int(v))
    return max(1, n)


def host_library() -> C.CDLL:
    global _hlib
    if _hlib is None:
        if not HOST_LIB.exists():
            from .build import build_host

            build_host()
        lib = C.CDLL(str(HOST_LIB))
        vp = C.c_void_p
        lib.mgp_host_last_error.restype = C.c_char_p
        lib.mgp_bam_open.argtypes = [C.c_char_p, C.c_int, C.POINTER(vp)]
        lib.mgp_bam_open.restype = C.c_int
        lib.mgp_bam_close.argtypes = [vp]
        lib.mgp_bam_close.restype = None
        lib.mgp_bam_n_refs.argtypes = [vp]
        lib.mgp_bam_ref_name.argtypes = [vp, C.c_int]
        lib.mgp_bam_ref_name.restype = C.c_char_p
        lib.mgp_bam_ref_len.argtypes = [vp, C.c_int]
        lib.mgp_bam_ref_len.restype = C.c_int64
        lib.mgp_bam_has_index.argtypes = [vp]
        lib.mgp_bam_set_barcodes.argtypes = [vp, C.c_char_p, C.POINTER(C.c_char_p), C.c_int]
        lib.mgp_bam_set_bulk.argtypes = [vp, C.c_int32]
        lib.mgp_bam_set_pack.argtypes = [vp, C.c_int]
        lib.mgp_bam_set_pack32.argtypes = [vp, C.c_int, C.c_int, C.c_int]
        lib.mgp_bam_set_placement.argtypes = [vp, C.c_int]
        lib.mgp_bam_read_ref.argtypes = [vp, C.c_int, C.c_int, C.POINTER(mgp_bam_batch)]
        lib.mgp_bam_free_batch.argtypes = [C.POINTER(mgp_bam_batch)]
        lib.mgp_bam_free_batch.restype = None
        lib.mgp_bam_find_tag.argtypes = [vp, C.c_int, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]
        lib.mgp_bam_find_tag.restype = C.c_int64
        lib.mgp_bam_count_tag.argtypes = [vp, C.c_int, C.c_char_p, C.POINTER(C.POINTER(C.c_uint8)),
                                          C.POINTER(C.c_int64)]
        lib.mgp_bam_count_tag.restype = C.c_int64
        lib.mgp_txt_write_cells.argtypes = [C.c_char_p, vp, vp, C.c_int64, vp, C.c_int64, C.POINTER(C.c_char_p),
                                            C.c_int, C.c_int, C.c_int]
        lib.mgp_txt_write_cells16.argtypes = lib.mgp_txt_write_cells.argtypes
        lib.mgp_deflate_tiles.argtypes = [vp, C.c_int64, C.c_int64, C.c_int32, C.c_int64, C.c_int64, C.c_int, C.c_int,
                                          C.POINTER(C.POINTER(C.c_uint8)), vp]
        lib.mgp_deflate_tiles.restype = C.c_int64
        lib.mgp_place_records.argtypes = [C.c_int64, vp, vp, vp, vp, vp, C.c_int32, C.c_int32, C.c_int32, vp]
        lib.mgp_place_records.restype = C.c_int64
        lib.mgp_gather_offsets.argtypes = [vp, vp, vp, vp, vp, vp, C.c_int64, C.c_int64, vp, C.c_int64, C.c_int32,
                                           C.c_int32, C.c_int32, C.c_int32, vp]
        lib.mgp_gather_offsets.restype = C.c_int64
        lib.mgp_gather_records.argtypes = [vp, vp, vp, C.c_int64, C.c_int64, vp, C.c_int64, vp, C.c_int64, vp,
                                           C.c_int]
        lib.mgp_gather_records.restype = C.c_int
        lib.mgp_split_by_range.argtypes = [vp, C.c_int64, vp, C.c_int32, vp, vp]
        lib.mgp_split_by_range.restype = C.c_int64
        lib.mgp_bam_write.argtypes = [C.c_char_p, C.POINTER(C.c_char_p), C.POINTER(C.c_int64), C.c_int, C.c_int,
                                      C.POINTER(mgp_bam_batch), C.POINTER(C.c_char_p), C.c_int, C.c_char_p,
                                      C.c_char_p, C.c_int, C.c_int, C.c_int]
        lib.mgp_h5_plane_tiles.argtypes = [vp, C.c_int32, C.c_int64, C.c_int64, C.c_int64, vp, C.c_int64, vp,
                                           C.c_int32, C.c_int64, C.c_int64, C.c_int, C.c_int,
                                           C.POINTER(C.POINTER(C.c_uint8)), vp]
        lib.mgp_h5_plane_tiles.restype = C.c_int64
        lib.mgp_repack32.argtypes = [C.c_int64, vp, C.c_int64, vp, vp, C.c_int32, C.c_int32, vp, vp, C.c_int]
        lib.mgp_repack32.restype = C.c_int64
        lib.mgp_bam_ref_records.argtypes = [vp, C.c_int]
        lib.mgp_bam_ref_records.restype = C.c_int64
        lib.mgp_bam_stream_open.argtypes = [vp, C.c_int, C.c_int, C.POINTER(vp)]
        lib.mgp_bam_stream_open.restype = C.c_int
        lib.mgp_bam_stream_next.argtypes = [vp, C.c_int64, C.c_int64, C.POINTER(mgp_bam_batch)]
        lib.mgp_bam_stream_next.restype = C.c_int64
        lib.mgp_bam_stream_close.argtypes = [vp]
        lib.mgp_bam_stream_close.restype = None
        lib.mgp_host_buf_free.argtypes = [vp]
        lib.mgp_host_buf_free.restype = None
        lib.mgp_batch_columns16.argtypes = [C.c_int64, vp, vp, vp, C.c_int64, C.c_int32, vp, vp, C.c_int]
        lib.mgp_batch_columns16.restype = C.c_int
        lib.mgp_route_batch.argtypes = [C.c_int64, vp, vp, vp, vp, vp, vp, C.c_int64, C.c_int32, vp, C.c_int64, vp,
                                        C.POINTER(mgp_route_part), C.c_int]
        lib.mgp_route_batch.restype = C.c_int
        _hlib = lib
    return _hlib


def _err() -> str:
    return (host_library().mgp_host_last_error() or b"").decode(errors="replace")


PLACE_DENSE, PLACE_PAIRED = 0, 1  # include/mgpileup_host.h MGP_PLACE_*


def place_records(bc: np.ndarray, flag: np.ndarray, rec_bytes: np.ndarray, n_cells: int,
                  mode: int = PLACE_PAIRED, rec_align: int = 64, start: np.ndarray | None = None,
                  tlen: np.ndarray | None = None) -> tuple[np.ndarray, int]:
    """Producer placement of payload records (mgp_place_records): returns
    (rec_off, payload_bytes). PLACE_PAIRED puts two consecutive packed records of
    one cell into one 128-byte line; given start and tlen, a read repeating the
    start, strand and |tlen| of an earlier read of its cell goes with the dropped
    reads (a duplicate whenever dedup is on)."""
    lib = host_library()
    n = int(bc.shape[0])
    bc = np.ascontiguousarray(bc, np.int32)
    flag = np.ascontiguousarray(flag, np.uint16)
    rb = np.ascontiguousarray(rec_bytes, np.uint32)
    if flag.shape[0] != n or rb.shape[0] != n:
        raise ValueError("bc, flag and rec_bytes must have the same length")
    keyed = start is not None and tlen is not None
    if keyed:
        start = np.ascontiguousarray(start, np.int32)
        tlen = np.ascontiguousarray(tlen, np.int32)
        if start.shape[0] != n or tlen.shape[0] != n:
            raise ValueError("start and tlen must have the reads' length")
    off = np.empty(n, np.uint64)
    tot = lib.mgp_place_records(n, bc.ctypes.data, flag.ctypes.data, start.ctypes.data if keyed else None,
                                tlen.ctypes.data if keyed else None, rb.ctypes.data, int(n_cells), int(mode),
                                int(rec_align), off.ctypes.data)
    if tot < 0:
        raise ValueError(_err())
    return off, int(tot)


def repack32(soa: ReadSoA, min_baseq: int, min_dist: int = 5, n_threads: int = 0,
             out32: np.ndarray | None = None, out_flag: np.ndarray | None = None) -> tuple[np.ndarray, np.ndarray, int]:
    """libmgphost `mgp_repack32`: the 32-byte records of a batch's full records for one
    run's thresholds, dense in batch order (record i at 32 x i of the returned payload),
    with the new flag words and the number of records packed (the others keep their
    own layout: a zeroed slot and their flag word)."""
    lib = host_library()
    n = soa.n
    out32 = np.empty(n * 32, np.uint8) if out32 is None else out32
    out_flag = np.empty(n, np.uint16) if out_flag is None else out_flag
    if out32.shape[0] < n * 32 or out_flag.shape[0] < n:
        raise ValueError("repack32 output arrays too small")
    pay = np.ascontiguousarray(soa.payload)
    roff = np.ascontiguousarray(soa.rec_off, np.uint64)
    flag = np.ascontiguousarray(soa.flag, np.uint16)
    k = lib.mgp_repack32(n, pay.ctypes.data, int(pay.shape[0]), roff.ctypes.data, flag.ctypes.data, int(min_baseq),
                         int(min_dist), out32.ctypes.data, out_flag.ctypes.data, int(n_threads or host_threads()))
    if k < 0:
        raise ValueError(_err())
    return out32, out_flag, int(k)


class _BatchOwner:
    """Frees an mgp_bam_batch when garbage collected (owner of zero-copy views)."""

    def __init__(self, lib, batch: mgp_bam_batch):
        self.lib = lib
        self.batch = batch

    def __del__(self):
        try:
            self.lib.mgp_bam_free_batch(C.byref(self.batch))
        except Exception:
            pass


class BamFile:
    """Native BAM reader (header, reference list, chrM records -> engine SoA)."""

    def __init__(self, path: str | Path, n_threads: int = 0):
        self.lib = host_library()
        self.path = str(path)
        h = C.c_void_p()
        if self.lib.mgp_bam_open(self.path.encode(), int(n_threads or host_threads()), C.byref(h)) != 0:
            raise BAMFormatError(self.path, f"Cannot open: {_err()}")
        self._h = h
        n = self.lib.mgp_bam_n_refs(h)
        self.references = tuple(self.lib.mgp_bam_ref_name(h, i).decode() for i in range(n))
        self.lengths = tuple(int(self.lib.mgp_bam_ref_len(h, i)) for i in range(n))
        self.has_index = bool(self.lib.mgp_bam_has_index(h))

    def close(self):
        if getattr(self, "_h", None):
            self.lib.mgp_bam_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tid(self, contig: str) -> int:
        return self.references.index(contig)

    def read_soa(self, contig: str, barcodes: list[str], tag: str = "CB", rec_align: int = 64,
                 bulk_cell: int = -1, pack: bool = True, paired: bool | None = None,
                 pack32: int | None = None, pack32_dist: int = 5) -> ReadSoA:
        """Every record of `contig` (fetch order) as an engine batch; bc = whitelist
        index (last duplicate wins, like the reference's dict) or -1. With
        ``bulk_cell >= 0`` every record goes to that cell (bulk calling). pack:
        reads that fit get the packed 64-byte record (include/mgpileup.h), which
        drops the code and quality of non-ACGT bases (off to rebuild SimpleReads).
        paired (default: = pack): two consecutive packed records of a cell share a
        128-byte line (mgp_place_records), so the pileup's gather fetches half the
        lines; the records are then not in BAM order in the payload. pack32 (the
        run's min_baseq): reads that fit get the 32-byte record made for that
        threshold and min_dist_from_end pack32_dist (four to a line when paired)
        before the 64-byte one."""
        self._configure(barcodes, tag, bulk_cell, pack, paired, pack32, pack32_dist)
        b = mgp_bam_batch()
        if self.lib.mgp_bam_read_ref(self._h, self.tid(contig), int(rec_align), C.byref(b)) != 0:
            raise BAMReadError(self.path, f"Read error: {_err()}")
        # zero copy: the arrays view the library's buffers, which are freed when the
        # last array referencing them is gone
        owner = _BatchOwner(self.lib, b)
        n = int(b.n_reads)

        def view(ptr, dtype, count):
            if count == 0:
                return np.zeros(0, dtype)
            nbytes = count * np.dtype(dtype).itemsize
            buf = (C.c_uint8 * nbytes).from_address(C.cast(ptr, C.c_void_p).value)
            buf._owner = owner
            return np.frombuffer(buf, dtype=dtype, count=count)

        soa = ReadSoA(
            view(b.start, np.int32, n), view(b.bc, np.int32, n), view(b.tlen, np.int32, n),
            view(b.flag, np.uint16, n), view(b.mapq, np.uint8, n), view(b.span, np.uint32, n),
            view(b.rec_off, np.uint64, n), view(b.payload, np.uint8, int(b.payload_bytes)),
        )
        soa.extra.update(n_with_tag=int(b.n_with_tag), first_tag_index=int(b.first_tag_index))
        return soa

    def _configure(self, barcodes: list[str], tag: str, bulk_cell: int, pack: bool, paired: bool | None,
                   pack32: int | None, pack32_dist: int) -> None:
        paired = pack if paired is None else paired
        arr = (C.c_char_p * max(1, len(barcodes)))(*[b.encode() for b in barcodes])
        if self.lib.mgp_bam_set_barcodes(self._h, tag.encode(), arr, len(barcodes)) != 0:
            raise ProcessingError(_err())
        if bulk_cell >= 0 and self.lib.mgp_bam_set_bulk(self._h, int(bulk_cell)) != 0:
            raise ProcessingError(_err())
        if self.lib.mgp_bam_set_pack(self._h, int(bool(pack))) != 0:
            raise ProcessingError(_err())
        if self.lib.mgp_bam_set_pack32(self._h, int(pack32 is not None), int(pack32 or 0), int(pack32_dist)) != 0:
            raise ProcessingError(_err())
        if self.lib.mgp_bam_set_placement(self._h, PLACE_PAIRED if paired else PLACE_DENSE) != 0:
            raise ProcessingError(_err())

    def ref_records(self, contig: str) -> int:
        """Records of `contig` per the index's metadata (mapped + placed unmapped), -1 if unknown."""
        return int(self.lib.mgp_bam_ref_records(self._h, self.tid(contig)))

    def stream(self, contig: str, barcodes: list[str], tag: str = "CB", rec_align: int = 64, bulk_cell: int = -1,
               pack: bool = True, paired: bool | None = None, pack32: int | None = None,
               pack32_dist: int = 5) -> BamStream:
        """Streaming decode of `contig` (mgp_bam_stream_*): batches of the records in
        fetch order, decoded into the caller's arrays (:meth:`BamStream.next_into`).
        Same settings as :meth:`read_soa`."""
        self._configure(barcodes, tag, bulk_cell, pack, paired, pack32, pack32_dist)
        h = C.c_void_p()
        if self.lib.mgp_bam_stream_open(self._h, self.tid(contig), int(rec_align), C.byref(h)) != 0:
            raise BAMReadError(self.path, f"Read error: {_err()}")
        return BamStream(self, h)

    def find_tag(self, contig: str, tag: str, max_records: int) -> tuple[int, int]:
        """(index of the first record carrying `tag` among the first `max_records`
        of `contig` or -1, records examined)."""
        n = C.c_int64()
        i = self.lib.mgp_bam_find_tag(self._h, self.tid(contig), tag.encode(), int(max_records), C.byref(n))
        if i < -1:
            raise BAMReadError(self.path, _err())
        return int(i), int(n.value)

    def count_tag(self, contig: str, tag: str = "CB") -> dict[str, int]:
        """Tag value counts over non-unmapped, non-duplicate records (barcode_extraction.py:22-32)."""
        blob = C.POINTER(C.c_uint8)()
        nbytes = C.c_int64()
        n = self.lib.mgp_bam_count_tag(self._h, self.tid(contig), tag.encode(), C.byref(blob), C.byref(nbytes))
        if n < 0:
            raise BAMReadError(self.path, _err())
        try:
            raw = bytes(np.ctypeslib.as_array(blob, shape=(int(nbytes.value),))) if nbytes.value else b""
        finally:
            self.lib.mgp_host_buf_free(C.cast(blob, C.c_void_p))
        out: dict[str, int] = {}
        p = 0
        for _ in range(n):
            z = raw.index(b"\0", p)
            key = raw[p:z].decode()
            (cnt,) = struct.unpack_from("<q", raw, z + 1)
            out[key] = cnt
            p = z + 9
        return out


class StreamSlot:
    """One batch's arrays for :meth:`BamStream.next_into` (any host memory; pinned
    memory, e.g. views of engine.PinnedBuffer, makes the engine's copies async)."""

    COLS = (("start", np.int32), ("bc", np.int32), ("tlen", np.int32), ("flag", np.uint16), ("mapq", np.uint8),
            ("span", np.uint32), ("rec_off", np.uint64))
    # the 16-bit barcode / |tlen| columns of the batch as pushed (mgp_batch_columns16)
    COLS16 = (("bc16", np.uint16), ("tlen16", np.uint16))

    def __init__(self, cap_reads: int, cap_payload: int, alloc=None):
        alloc = alloc or (lambda m, dt: np.empty(m, dt))
        self.cap_reads, self.cap_payload = int(cap_reads), int(cap_payload)
        for name, dt in self.COLS + self.COLS16:
            setattr(self, name, alloc(self.cap_reads, dt))
        self.payload = alloc(self.cap_payload, np.uint8)
        self.n = 0
        self.payload_bytes = 0

    @staticmethod
    def nbytes(cap_reads: int, cap_payload: int) -> int:
        return (sum(int(cap_reads) * np.dtype(dt).itemsize + 64 for _, dt in StreamSlot.COLS + StreamSlot.COLS16)
                + int(cap_payload) + 64)

    def soa(self) -> ReadSoA:
        """The decoded batch as views of the slot's arrays."""
        n, pb = self.n, self.payload_bytes
        return ReadSoA(self.start[:n], self.bc[:n], self.tlen[:n], self.flag[:n], self.mapq[:n], self.span[:n],
                       self.rec_off[:n], self.payload[:pb])


class BamStream:
    """mgp_bam_stream: one pass over a contig in batches (readers.py:84-93)."""

    def __init__(self, bam: BamFile, h: C.c_void_p):
        self.bam = bam  # (outlives the stream)
        self.lib = bam.lib
        self._h = h
        self.n_with_tag = 0
        self.first_tag_index = -1
        self.records = 0

    def next_into(self, slot: StreamSlot) -> int:
        """Decode the next batch into `slot`; returns its records (0 at the end)."""
        b = mgp_bam_batch(0, *[C.cast(getattr(slot, name).ctypes.data, C.POINTER(t)) for (name, _), t in zip(
            StreamSlot.COLS, (C.c_int32, C.c_int32, C.c_int32, C.c_uint16, C.c_uint8, C.c_uint32, C.c_uint64))],
            C.cast(slot.payload.ctypes.data, C.POINTER(C.c_uint8)), 0, 0, -1)
        n = self.lib.mgp_bam_stream_next(self._h, slot.cap_reads, slot.cap_payload, C.byref(b))
        if n < 0:
            raise BAMReadError(self.bam.path, f"Read error: {_err()}")
        slot.n, slot.payload_bytes = int(b.n_reads), int(b.payload_bytes)
        self.n_with_tag, self.first_tag_index = int(b.n_with_tag), int(b.first_tag_index)
        self.records += int(n)
        return int(n)

    def close(self):
        if getattr(self, "_h", None):
            self.lib.mgp_bam_stream_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def batch_columns16(soa: ReadSoA, n_cells: int, bc16: np.ndarray, tlen16: np.ndarray, n_threads: int = 0,
                    dense_only: bool = False) -> int:
    """mgp_batch_columns16: the 16-bit barcode and |tlen| columns of a decoded batch into
    bc16 / tlen16 (room for soa.n). Returns bit 0 = records dense at one stride (every
    offset checked), bit 1 = every key fits 16 bits; 3 = the batch may go as an
    mgp_batch16 (mgp_push_batch16)."""
    n = soa.n
    if bc16.shape[0] < n or tlen16.shape[0] < n or bc16.dtype != np.uint16 or tlen16.dtype != np.uint16:
        raise ValueError("bc16 / tlen16: uint16 arrays of at least n entries")
    ro = soa.rec_off
    if ro is not None and ro.shape[0] != n:
        ro = None if ro.shape[0] == 0 else ro
    rc = host_library().mgp_batch_columns16(
        n, soa.bc.ctypes.data, soa.tlen.ctypes.data, None if ro is None else ro.ctypes.data,
        int(soa.payload.shape[0]), int(n_cells), bc16.ctypes.data, tlen16.ctypes.data, int(n_threads or host_threads()))
    if rc < 0:
        raise ValueError(_err())
    return int(rc)


class RoutePart:
    """One device's batch arrays for :func:`route_batch` (pinned views via alloc(m, dtype)
    make its H2D copies async)."""

    def __init__(self, cap_reads: int, cap_payload: int, alloc=None):
        alloc = alloc or (lambda m, dt: np.empty(m, dt))
        self.cap_reads, self.cap_payload = int(cap_reads), int(cap_payload)
        m = self.cap_reads
        self.bc32, self.tlen32 = alloc(m, np.int32), alloc(m, np.int32)
        self.bc16, self.tlen16 = alloc(m, np.uint16), alloc(m, np.uint16)
        self.flag, self.mapq = alloc(m, np.uint16), alloc(m, np.uint8)
        self.rec_off = alloc(m, np.uint64)
        self.payload = alloc(self.cap_payload, np.uint8)
        self.n, self.payload_bytes, self.narrow = 0, 0, False

    @staticmethod
    def nbytes(cap_reads: int, cap_payload: int) -> int:
        return int(cap_reads) * (4 + 4 + 2 + 2 + 2 + 1 + 8) + int(cap_payload) + 8 * 64

    def c_struct(self) -> mgp_route_part:
        return mgp_route_part(self.cap_reads, self.cap_payload, self.bc16.ctypes.data, self.tlen16.ctypes.data,
                              self.bc32.ctypes.data, self.tlen32.ctypes.data, self.flag.ctypes.data,
                              self.mapq.ctypes.data, self.rec_off.ctypes.data, self.payload.ctypes.data, 0, 0, 0, 0)

    def soa(self) -> ReadSoA:
        """The routed batch as pushed: an mgp_batch16 (uint16 bc / |tlen|, dense records)
        or an mgp_batch with rec_off (no start / span: taken from the records)."""
        n, pb = self.n, self.payload_bytes
        if self.narrow:
            return ReadSoA(None, self.bc16[:n], self.tlen16[:n], self.flag[:n], self.mapq[:n], None, None,
                           self.payload[:pb])
        return ReadSoA(None, self.bc32[:n], self.tlen32[:n], self.flag[:n], self.mapq[:n], None, self.rec_off[:n],
                       self.payload[:pb])


def route_batch(soa: ReadSoA, bounds: np.ndarray, parts: list, first_index: int = 0,
                first_seen: np.ndarray | None = None, n_threads: int = 0) -> bool:
    """mgp_route_batch: every read of `soa` whose cell lies in [bounds[d], bounds[d+1])
    (and whose flag passes readers.py:96) into parts[d] (its RoutePart), in BAM order,
    barcode rebased; first_seen[c - bounds[0]] lowered to each cell's first routed read's
    first_index + i. False (nothing written) when a part's arrays are too small."""
    b = np.ascontiguousarray(bounds, np.int32)
    if b.shape[0] != len(parts) + 1:
        raise ValueError("one part per cell range")
    if first_seen is not None and (first_seen.dtype != np.uint32 or first_seen.shape[0] < int(b[-1] - b[0])):
        raise ValueError("first_seen: uint32, one entry per cell of the ranges")
    cs = (mgp_route_part * len(parts))(*[p.c_struct() for p in parts])
    ro = soa.rec_off if soa.rec_off is not None and soa.rec_off.shape[0] == soa.n else None
    rc = host_library().mgp_route_batch(
        soa.n, soa.bc.ctypes.data, soa.tlen.ctypes.data, soa.flag.ctypes.data, soa.mapq.ctypes.data,
        None if ro is None else ro.ctypes.data, soa.payload.ctypes.data, int(soa.payload.shape[0]), len(parts),
        b.ctypes.data, int(first_index), None if first_seen is None else first_seen.ctypes.data, cs,
        int(n_threads or host_threads()))
    if rc < 0:
        raise BAMFormatError(_err()) if "outside the payload" in _err() else ValueError(_err())
    if rc == 1:
        return False
    for p, c in zip(parts, cs):
        p.n, p.payload_bytes, p.narrow = int(c.n_reads), int(c.payload_bytes), bool(c.narrow)
    return True


def txt_write_cells(prefix: str | Path, counts: np.ndarray, depth: np.ndarray, cells, names: list[str],
                    level: int = 6, n_threads: int = 0, append: bool = True) -> None:
    """Native txt formatter + parallel gzip (libmgphost.so `mgp_txt_write_cells`)."""
    lib = host_library()
    # the engine's exact 16-bit rows are formatted as they are (no widening copy)
    dt = np.uint16 if counts.dtype == np.uint16 and depth.dtype == np.uint16 else np.uint32
    counts = np.ascontiguousarray(counts, dtype=dt)
    depth = np.ascontiguousarray(depth, dtype=dt)
    cells = np.ascontiguousarray(cells, dtype=np.int64)
    L = depth.shape[-1]
    if counts.shape[-2:] != (L, 8) or counts.reshape(-1, L, 8).shape[0] != depth.reshape(-1, L).shape[0]:
        raise ValueError("counts/depth shapes do not match")
    if cells.size and (cells.min() < 0 or cells.max() >= depth.reshape(-1, L).shape[0]):
        raise ValueError("cell index out of range")
    if len(names) != cells.size:
        raise ValueError("one name per written cell")
    arr = (C.c_char_p * max(1, len(names)))(*[n.encode() for n in names])
    fn = lib.mgp_txt_write_cells16 if dt == np.uint16 else lib.mgp_txt_write_cells
    rc = fn(str(prefix).encode(), counts.ctypes.data, depth.ctypes.data, L, cells.ctypes.data,
            cells.size, arr, int(level), int(n_threads or host_threads()), 1 if append else 0)
    if rc != 0:
        raise OSError(_err())


def deflate_tiles(a: np.ndarray, chunks: tuple[int, int], level: int = 4, n_threads: int = 0) -> list[bytes]:
    """Deflate every chunk of a 2-D array as the HDF5 deflate filter stores it
    (libmgphost.so `mgp_deflate_tiles`); chunks in row-major grid order."""
    lib = host_library()
    a = np.ascontiguousarray(a)
    rows, cols = a.shape
    nr, nc = -(-rows // chunks[0]), -(-cols // chunks[1])
    offs = np.zeros(nr * nc + 1, np.int64)
    blob = C.POINTER(C.c_uint8)()
    n = lib.mgp_deflate_tiles(a.ctypes.data, rows, cols, a.dtype.itemsize, chunks[0], chunks[1], int(level),
                              int(n_threads or host_threads()), C.byref(blob), offs.ctypes.data)
    if n < 0:
        raise OSError(_err())
    try:
        raw = C.string_at(blob, int(offs[-1])) if offs[-1] else b""
    finally:
        lib.mgp_host_buf_free(C.cast(blob, C.c_void_p))
    return [raw[offs[i]:offs[i + 1]] for i in range(n)]


def h5_plane_tiles(rows: np.ndarray, cell_of_col: np.ndarray, elems: list[int], chunks: tuple[int, int],
                   level: int = 4, n_threads: int = 0) -> list[list[bytes]]:
    """libmgphost `mgp_h5_plane_tiles`: for each element e of the cell-major rows
    [cells, L, k] (u16 or u32), the deflated chunks of the [L, n_cols] u16 plane
    min(rows[cell_of_col[j], p, e], 65535); chunks row-major over the chunk grid."""
    lib = host_library()
    if rows.ndim == 2:
        rows = rows[:, :, None]
    rows = np.ascontiguousarray(rows)
    if rows.dtype not in (np.uint16, np.uint32):
        raise ValueError("rows must be u16 or u32")
    n_rows, L, k = rows.shape
    coc = np.ascontiguousarray(cell_of_col, np.int64)
    el = np.ascontiguousarray(elems, np.int32)
    if el.size == 0 or el.min() < 0 or el.max() >= k or (coc.size and coc.max() >= n_rows):
        raise ValueError("plane element or cell index out of range")
    nr, nc = -(-L // chunks[0]), -(-coc.size // chunks[1])
    offs = np.zeros(el.size * nr * nc + 1, np.int64)
    blob = C.POINTER(C.c_uint8)()
    n = lib.mgp_h5_plane_tiles(rows.ctypes.data, rows.dtype.itemsize, k, n_rows, L, coc.ctypes.data, coc.size,
                               el.ctypes.data, el.size, int(chunks[0]), int(chunks[1]), int(level),
                               int(n_threads or host_threads()), C.byref(blob), offs.ctypes.data)
    if n < 0:
        raise OSError(_err())
    try:
        raw = C.string_at(blob, int(offs[-1])) if offs[-1] else b""
    finally:
        lib.mgp_host_buf_free(C.cast(blob, C.c_void_p))
    return [[raw[offs[e * n + i]:offs[e * n + i + 1]] for i in range(n)] for e in range(el.size)]


# ---------------------------------------------------------------------------
# writer (fixtures / synthetic inputs)
# ---------------------------------------------------------------------------
_BGZF_EOF = bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")


def _bgzf_block(data: bytes, level: int = 6) -> bytes:
    co = zlib.compressobj(level, zlib.DEFLATED, -15)
    cdata = co.compress(data) + co.flush()
    bsize = len(cdata) + 25
    hdr = struct.pack("<BBBBIBBHBBHH", 31, 139, 8, 4, 0, 0, 255, 6, 66, 67, 2, bsize)
    return hdr + cdata + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data))


def reg2bin(beg: int, end: int) -> int:
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


class BamWriter:
    """Write a coordinate-sorted BAM (+ optional .bai)."""

    BLOCK = 0xFF00

    def __init__(self, path: str | Path, refs: list[tuple[str, int]], text: str | None = None):
        self.path = Path(path)
        self.refs = refs
        self.f = open(self.path, "wb")
        self.coff = 0
        self.buf = bytearray()
        self.records: list[tuple[int, int, int, int, int]] = []  # (tid, beg, end, voff_beg, voff_end)
        if text is None:
            text = "@HD\tVN:1.6\tSO:coordinate\n" + "".join(f"@SQ\tSN:{n}\tLN:{ln}\n" for n, ln in refs)
        tb = text.encode()
        hdr = b"BAM\1" + struct.pack("<i", len(tb)) + tb + struct.pack("<i", len(refs))
        for n, ln in refs:
            nb = n.encode() + b"\0"
            hdr += struct.pack("<i", len(nb)) + nb + struct.pack("<i", ln)
        self._write(hdr)
        self._flush()  # records start in a fresh block

    def _voff(self) -> int:
        return (self.coff << 16) | len(self.buf)

    def _write(self, data: bytes):
        self.buf += data
        while len(self.buf) >= self.BLOCK:
            blk = _bgzf_block(bytes(self.buf[: self.BLOCK]))
            self.f.write(blk)
            self.coff += len(blk)
            del self.buf[: self.BLOCK]

    def _flush(self):
        if self.buf:
            blk = _bgzf_block(bytes(self.buf))
            self.f.write(blk)
            self.coff += len(blk)
            self.buf.clear()

    def write(self, r: dict):
        """r: tid, pos, flag, mapq, cigartuples, query_sequence (or None), query_qualities (or None),
        template_length, tags (dict name -> str/int), query_name, next_tid, next_pos."""
        name = (r.get("query_name", "r") + "\0").encode()
        cig = r.get("cigartuples") or []
        seq = r.get("query_sequence") or ""
        qual = r.get("query_qualities")
        lseq = len(seq)
        cigb = b"".join(struct.pack("<I", (ln << 4) | op) for op, ln in cig)
        codes = [_NT16[c] for c in seq.upper()]
        if lseq & 1:
            codes.append(0)
        seqb = bytes((codes[i] << 4) | codes[i + 1] for i in range(0, len(codes), 2))
        qualb = bytes([0xFF] * lseq) if qual is None else bytes(int(q) & 0xFF for q in qual)
        aux = b""
        for k, v in (r.get("tags") or {}).items():
            if isinstance(v, str):
                aux += k.encode() + b"Z" + v.encode() + b"\0"
            else:
                aux += k.encode() + b"i" + struct.pack("<i", int(v))
        pos = int(r["pos"])
        span = sum(ln for op, ln in cig if op in (0, 2, 3, 7, 8))
        end = pos + max(span, 1)
        bin_ = reg2bin(max(pos, 0), max(end, pos + 1)) if pos >= 0 else 4680
        body = struct.pack(
            "<iiBBHHHIiii", int(r.get("tid", 0)), pos, len(name), int(r.get("mapq", 60)), bin_, len(cig),
            int(r.get("flag", 0)), lseq, int(r.get("next_tid", -1)), int(r.get("next_pos", -1)),
            int(r.get("template_length", 0)),
        ) + name + cigb + seqb + qualb + aux
        vb = self._voff()
        self._write(struct.pack("<I", len(body)) + body)
        self.records.append((int(r.get("tid", 0)), pos, end, vb, self._voff()))

    def close(self, index: bool = True):
        self._flush()
        self.f.write(_BGZF_EOF)
        self.f.close()
        if index:
            write_bai(Path(str(self.path) + ".bai"), len(self.refs), self.records)


def write_bai(path: Path, n_ref: int, records: list[tuple[int, int, int, int, int]]):
    """Minimal BAI: per reference, bins with merged chunks + 16 kbp linear index."""
    per_ref: list[dict] = [dict(bins={}, lin={}) for _ in range(n_ref)]
    for tid, beg, end, vb, ve in records:
        if tid < 0:
            continue
        ref = per_ref[tid]
        b = reg2bin(max(beg, 0), max(end, beg + 1))
        chunks = ref["bins"].setdefault(b, [])
        if chunks and chunks[-1][1] == vb:
            chunks[-1][1] = ve
        else:
            chunks.append([vb, ve])
        for w in range(max(beg, 0) >> 14, (max(end, beg + 1) - 1 >> 14) + 1):
            ref["lin"].setdefault(w, vb)
    out = bytearray(b"BAI\1" + struct.pack("<i", n_ref))
    for ref in per_ref:
        out += struct.pack("<i", len(ref["bins"]))
        for b, chunks in sorted(ref["bins"].items()):
            out += struct.pack("<Ii", b, len(chunks))
            for vb, ve in chunks:
                out += struct.pack("<QQ", vb, ve)
        nl = (max(ref["lin"]) + 1) if ref["lin"] else 0
        out += struct.pack("<i", nl)
        last = 0
        for w in range(nl):
            last = ref["lin"].get(w, last)
            out += struct.pack("<Q", last)
    Path(path).write_bytes(bytes(out))


def write_bam(path: str | Path, soa: ReadSoA, whitelist: list[str], contig: str = "chrM", mito_len: int = 16569,
              index: bool = True, tag: str = "CB", level: int = 1, n_threads: int = 0,
              unlisted: str | None = "NNNNNNNNNNNNNNNN-9") -> None:
    """Native BAM writer (libmgphost.so `mgp_bam_write`): same records as
    :func:`soa_to_bam`, BGZF deflated on a thread pool; for large inputs."""
    lib = host_library()
    refs = [("chr1", 248956422), (contig, mito_len)]
    names = (C.c_char_p * 2)(*[n.encode() for n, _ in refs])
    lens = (C.c_int64 * 2)(*[ln for _, ln in refs])
    arrs = [np.ascontiguousarray(a) for a in (soa.start, soa.bc, soa.tlen, soa.flag, soa.mapq, soa.span,
                                                  soa.rec_off, soa.payload)]
    b = mgp_bam_batch(soa.n, *[C.cast(a.ctypes.data, t) for a, t in zip(arrs, (
        C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_uint16),
        C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_uint8)))],
        int(soa.payload.shape[0]), 0, -1)
    bcs = (C.c_char_p * max(1, len(whitelist)))(*[w.encode() for w in whitelist])
    rc = lib.mgp_bam_write(str(path).encode(), names, lens, 2, 1, C.byref(b), bcs, len(whitelist), tag.encode(),
                           unlisted.encode() if unlisted else None, int(level), int(n_threads or host_threads()),
                           1 if index else 0)
    if rc != 0:
        raise OSError(_err())


def soa_to_bam(path: str | Path, soa: ReadSoA, whitelist: list[str], contig: str = "chrM", mito_len: int = 16569,
               index: bool = True, tag: str = "CB"):
    """Write an engine batch as a BAM (chr1 placeholder + contig). Reads with bc = -1
    alternate between no tag and a non-whitelisted barcode."""
    from .synth import FLAG_NOSEQQUAL, unpack_record

    w = BamWriter(path, [("chr1", 248956422), (contig, mito_len)])
    for i in range(soa.n):
        d = unpack_record(soa.payload, int(soa.rec_off[i]), int(soa.flag[i]))
        f = int(soa.flag[i])
        q = d["query_qualities"]
        seq = d["query_sequence"]
        if f & FLAG_NOSEQQUAL:
            if not seq:
                seq, q = None, None
            elif q and all(x == 0xFF for x in q):
                q = None
        b = int(soa.bc[i])
        tags = {}
        if b >= 0:
            tags[tag] = whitelist[b]
        elif i % 2 == 0:
            tags[tag] = "NNNNNNNNNNNNNNNN-9"
        w.write(dict(tid=1, pos=int(soa.start[i]), flag=f & 0xFFF, mapq=int(soa.mapq[i]),
                     cigartuples=d["cigartuples"], query_sequence=seq, query_qualities=q,
                     template_length=int(soa.tlen[i]), tags=tags, query_name=f"r{i}"))
    w.close(index=index)
