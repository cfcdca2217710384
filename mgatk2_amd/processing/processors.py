"""Cell processing (mirror of src/processing/processors.py).

The reference dispatches one Python call per cell, sequentially or over a
spawn pool (processors.py:63-144). Here every cell goes through the GPU engine
in one run:

* :meth:`CellProcessor.process_soa` — production path: the whole chrM read set
  (engine SoA, BAM order) in, dedup + pileup + filters + statistics on the GPU,
  results streamed to the writer in first-seen cell order.
* :meth:`CellProcessor.process_cells_progressive` / :func:`process_barcode_worker`
  — the reference's dict API (already-deduplicated ``SimpleRead`` lists per
  barcode). The lists are merged into one coordinate-sorted batch and run with
  dedup off, so each cell sees exactly its own reads.
"""

from __future__ import annotations

import gc
import logging
import os
import threading
import time
from queue import Queue

import numpy as np

from ..engine import TXT_FILES, Engine, EngineResult, PinnedBuffer, Rows16
from ..synth import ReadSoA, pack_reads
from .pileup import result_dict, simple_reads_to_dicts

logger = logging.getLogger(__name__)

MP_CONTEXT = "spawn"  # kept for API compatibility (processors.py:17); no process pool is used

# streamed runs: reads per decoded batch and batches in flight (MGP_STREAM_BATCH /
# MGP_STREAM_SLOTS override them, read at each run)
STREAM_BATCH_READS = 4_000_000
STREAM_SLOTS = 3
# cells per mgp_txt_gz call (its device scratch is ~7 GB per 1000 C4 cells)
TXT_CHUNK_CELLS = 2048


def _engine_config_for(config, n_cells: int, dedup: bool):
    ec = config.engine_config(n_cells)
    if not dedup:
        ec.dedup_mode = "none"
    return ec


def run_cells_from_reads(config, reads_by_barcode: dict, device: int = 0) -> tuple[EngineResult, list[str]]:
    """Engine run over already-deduplicated per-barcode read lists."""
    barcodes = list(reads_by_barcode)
    dicts = []
    for i, bc in enumerate(barcodes):
        dicts.extend(simple_reads_to_dicts(reads_by_barcode[bc], bc=i))
    dicts.sort(key=lambda d: d["reference_start"])  # stable: per-cell order is kept
    soa = pack_reads(dicts)
    with Engine(_engine_config_for(config, len(barcodes), dedup=False), device=device) as eng:
        eng.push(soa)
        res = eng.finish()
    return res, barcodes


def process_barcode_worker(args):
    """processors.py:20-55: one barcode's reads -> result dict or None."""
    barcode, reads, config = args
    if not reads or len(reads) < config.min_reads_per_cell:
        return None
    res, _ = run_cells_from_reads(config, {barcode: reads})
    if not res.passed[0]:
        return None
    return result_dict(res, 0, barcode, config.mito_length)


def _pinned_alloc(nbytes: int):
    """alloc(m, dtype) -> consecutive 64-byte aligned views of one pinned buffer."""
    pb = PinnedBuffer(nbytes)
    off = [0]

    def alloc(m, dt):
        a = pb.array(m, dt, off[0])
        off[0] = (off[0] + m * np.dtype(dt).itemsize + 63) & ~63
        return a

    return alloc


def _link_bytes(soa: ReadSoA) -> int:
    """Host-to-device bytes of a pushed batch (its columns and payload)."""
    return sum(int(a.nbytes) for a in (soa.start, soa.bc, soa.tlen, soa.flag, soa.mapq, soa.span, soa.rec_off,
                                       soa.payload) if a is not None)


def _payload_hint(n_reads: int, n_cells: int = 0, batch_reads: int = STREAM_BATCH_READS) -> int:
    """Device payload bytes a streamed run of n_reads needs at once (no regrowth, which
    waits for the queued segments): 64-byte records plus what the on-device pairing
    reserves (mgp_push_batch: one half-empty line per cell and key range of 2^18 reads,
    per batch), or 32-byte records four per line plus their lines."""
    if os.environ.get("MGP_RECORDS", "64") == "32":
        return int(n_reads) * 40 + (64 << 20)
    ranges = -(-int(n_reads) // (1 << 18)) + -(-int(n_reads) // max(1, int(batch_reads))) + 1
    return int(n_reads) * 64 + ranges * (int(n_cells) + 2) * 64 + (64 << 20)


class CellProcessor:
    def __init__(self, config, output_dir, device: int = 0, devices: list[int] | None = None):
        self.config = config
        self.output_dir = output_dir
        self.device = device
        self.devices = list(devices) if devices else [device]
        self.last_result: EngineResult | None = None
        self.last_stats: dict = {}
        self.last_timing: dict = {}
        self.txt_out = None
        self.h5_out = None

    # txt output on the device ----------------------------------------------
    def enable_device_txt(self, prefix, names: list[str]):
        """Write the txt count files (`prefix`.{coverage,A,C,G,T}.txt.gz, appended) from
        the devices' rows before their contexts close: each passing cell's lines
        formatted and deflated on its device (mgp_txt_gz, writers.py:430-486), only the
        gzip members cross the link. The run's result then carries `txt_gz_cells`, the
        cells written, and IncrementalTextWriter.write_cells writes only the rest
        (stats, depth table, reference alleles). MGP_TXT_DEVICE=0, or a gzip level other
        than the reference's 9 (MGP_GZIP_LEVEL), keeps the host formatter."""
        self.txt_out = (str(prefix), list(names))

    def enable_device_h5(self, names: list[str]):
        """Deflate the HDF5 count datasets' chunks (writers.py:60-131) on the devices before
        their contexts close (mgp_h5_tiles): the run's result then carries `h5_tiles`, which
        IncrementalHDF5Writer.finalize writes instead of deflating the planes on the host.
        `names`: the writer's barcodes (its columns). MGP_H5_DEVICE=0 keeps the host deflate."""
        self.h5_out = list(names)

    def _h5_device_on(self) -> bool:
        return self.h5_out is not None and os.environ.get("MGP_H5_DEVICE", "1") != "0"

    def _write_h5(self, res: EngineResult, parts: list) -> float:
        """The written cells' columns (hdf5_columns over the passing cells in first-seen
        order), their chunks deflated on the devices: parts = [(engine, lo, hi)], each
        engine holding the cells [lo, hi) as its 0..hi-lo. A column chunk whose cells lie
        on one device is made there; one that spans two devices' cells (at most one per
        boundary) is deflated on the host from the fetched rows. Returns the seconds spent."""
        from concurrent.futures import ThreadPoolExecutor

        from ..bam import h5_plane_tiles
        from ..engine import H5_PLANES
        from ..file_io.writers import hdf5_cell_of_col, hdf5_columns

        t0 = time.perf_counter()
        names = self.h5_out
        sel, cols = hdf5_columns(names, names, cells_written(res))
        if not (len(names) and sel.size):
            return time.perf_counter() - t0
        n, L = len(names), self.config.mito_length
        coc = hdf5_cell_of_col(n, sel, cols)
        chunks = (min(1000, L), min(100, n))
        crow, ccol = chunks
        nrc, ncc = -(-L // crow), -(-n // ccol)
        los = np.array([lo for _, lo, _ in parts], np.int64)
        his = np.array([hi for _, _, hi in parts], np.int64)
        owner = np.zeros(ncc, np.int64)  # the part making each column chunk, -1: the host
        for cc in range(ncc):
            v = coc[cc * ccol:(cc + 1) * ccol]
            v = v[v >= 0]
            if v.size:
                d = np.searchsorted(his, v, side="right")
                owner[cc] = d[0] if np.all(d == d[0]) else -1
        tiles = {p: [None] * (nrc * ncc) for p in H5_PLANES}
        total = np.zeros((3, L), np.int64)

        def runs(d):  # (c0, c1) runs of consecutive column chunks of part d
            idx = np.flatnonzero(owner == d)
            if not idx.size:
                return []
            cut = np.flatnonzero(np.diff(idx) > 1) + 1
            return [(int(g[0]), int(g[-1]) + 1) for g in np.split(idx, cut)]

        def one(d):
            eng, lo, hi = parts[d]
            local = np.where((coc >= lo) & (coc < hi), coc - lo, -1)
            out = []
            for c0, c1 in runs(d):
                sums = {}
                out.append((c0, c1, eng.h5_tiles(local, chunks, sums=sums, col_chunks=(c0, c1)), sums))
            return out

        if len(parts) > 1:
            with ThreadPoolExecutor(len(parts)) as pool:
                made = list(pool.map(one, range(len(parts))))
        else:
            made = [one(0)]
        for got in made:
            for c0, c1, tl, sums in got:
                w = c1 - c0
                for p in H5_PLANES:
                    src = tl[p]
                    for rc in range(nrc):
                        tiles[p][rc * ncc + c0:rc * ncc + c1] = src[rc * w:(rc + 1) * w]
                total += np.stack([sums["coverage"], sums["tn5_fwd"], sums["tn5_rev"]])
        for cc in np.flatnonzero(owner < 0).tolist():  # chunks across a device boundary
            sub = coc[cc * ccol:(cc + 1) * ccol]
            made_h = (h5_plane_tiles(res.counts, sub, list(range(8)), chunks, level=4)
                      + h5_plane_tiles(res.tn5, sub, [0, 1], chunks, level=4)
                      + h5_plane_tiles(res.depth, sub, [0], chunks, level=4))
            for p, lst in zip(H5_PLANES, made_h):
                for rc in range(nrc):
                    tiles[p][rc * ncc + cc] = lst[rc]
            ok = sub[sub >= 0]
            total[0] += np.minimum(res.depth[ok], 65535).astype(np.int64).sum(axis=0)
            total[1] += np.minimum(res.tn5[ok, :, 0], 65535).astype(np.int64).sum(axis=0)
            total[2] += np.minimum(res.tn5[ok, :, 1], 65535).astype(np.int64).sum(axis=0)
        res.h5_tiles = (coc, chunks, tiles, {"coverage": total[0], "tn5_fwd": total[1], "tn5_rev": total[2]})
        return time.perf_counter() - t0

    def _txt_device_on(self) -> bool:
        if self.txt_out is None or os.environ.get("MGP_TXT_DEVICE", "1") == "0":
            return False
        return os.environ.get("MGP_GZIP_LEVEL", "9") == "9"

    def _write_txt(self, res: EngineResult, parts: list) -> float:
        """The passing cells in first-seen order (processors.py:75's write order) through
        mgp_txt_gz on their devices; parts = [(engine, lo, hi)], each engine holding the
        cells [lo, hi) as its 0..hi-lo. With several devices each writes its own cells (in
        the global order, TXT_CHUNK_CELLS per call, the devices concurrently) and the
        members are interleaved back into the global order. Returns the seconds spent."""
        t0 = time.perf_counter()
        prefix, names = self.txt_out
        written = cells_written(res)
        files = [open(f"{prefix}.{f}.txt.gz", "ab") for f in TXT_FILES]
        try:
            if len(parts) == 1:
                from concurrent.futures import ThreadPoolExecutor

                eng, lo, _ = parts[0]

                def put(mem):
                    for f in range(5):
                        files[f].write(memoryview(mem.file_part(f)))

                # a chunk's members go to the files while the device makes the next chunk's
                with ThreadPoolExecutor(1) as wr:
                    pending = None
                    for a in range(0, written.size, TXT_CHUNK_CELLS):
                        chunk = written[a:a + TXT_CHUNK_CELLS]
                        mem = eng.txt_gz(chunk - lo, [names[c] for c in chunk.tolist()])
                        if pending is not None:
                            pending.result()
                        pending = wr.submit(put, mem)
                    if pending is not None:
                        pending.result()
            else:
                from concurrent.futures import ThreadPoolExecutor

                his = np.array([hi for _, _, hi in parts], np.int64)
                dev = np.searchsorted(his, written, side="right")  # each cell's part

                def one(d):
                    eng, lo, _ = parts[d]
                    sel = written[dev == d]
                    return [eng.txt_gz(ch - lo, [names[c] for c in ch.tolist()])
                            for ch in (sel[a:a + TXT_CHUNK_CELLS] for a in range(0, sel.size, TXT_CHUNK_CELLS))]

                with ThreadPoolExecutor(len(parts)) as pool:
                    mems = list(pool.map(one, range(len(parts))))
                rank = np.zeros(written.size, np.int64)  # a cell's index among its part's cells
                for d in range(len(parts)):
                    rank[dev == d] = np.arange(int((dev == d).sum()))
                call, k_in = np.divmod(rank, TXT_CHUNK_CELLS)
                order = list(zip(dev.tolist(), call.tolist(), k_in.tolist()))
                for f in range(5):
                    views = [[memoryview(m.file_part(f)) for m in ms] for ms in mems]
                    offs = [[np.concatenate([[0], np.cumsum(m.member_bytes[f])]).tolist() for m in ms] for ms in mems]
                    files[f].writelines(views[d][j][offs[d][j][k]:offs[d][j][k + 1]]
                                        for d, j, k in order if offs[d][j][k + 1] > offs[d][j][k])
        finally:
            for fh in files:
                fh.close()
        res.txt_gz_cells = written
        return time.perf_counter() - t0

    # production path ------------------------------------------------------
    def run_soa(self, soa_batches, n_cells: int) -> EngineResult:
        """Whole read set (one or more BAM-order batches) through the engine:
        filters, dedup, pileup, strand filter, per-cell statistics, tallies."""
        if isinstance(soa_batches, ReadSoA):
            soa_batches = [soa_batches]
        if len(self.devices) > 1:
            return self._run_sharded(soa_batches, n_cells)
        n = sum(b.n for b in soa_batches)
        pay = sum(int(b.payload.shape[0]) for b in soa_batches)
        ec = self.config.engine_config(n_cells, reserve_reads=n, reserve_payload=pay + 256 * len(soa_batches))
        t0 = time.perf_counter()
        with Engine(ec, device=self.device) as eng:
            t1 = time.perf_counter()
            for b in soa_batches:
                eng.push(b)
            eng.run()
            eng.sync()
            t2 = time.perf_counter()
            res = eng.fetch_compact()  # exact 16-bit rows: half the device-to-host bytes
            t3 = time.perf_counter()
            self.last_stats = eng.kernel_times()
            t_txt = self._write_txt(res, [(eng, 0, n_cells)]) if self._txt_device_on() else 0.0
            t_h5 = self._write_h5(res, [(eng, 0, n_cells)]) if self._h5_device_on() else 0.0
        t4 = time.perf_counter()
        # where the engine leg goes (pipeline timings): context + allocation, H2D of
        # the batches + the run, D2H of the results, teardown
        self.last_timing = {"engine_open": t1 - t0, "engine_h2d_run": t2 - t1, "engine_d2h": t3 - t2,
                            "engine_close": t4 - t3 - t_txt - t_h5, "txt_device": t_txt, "h5_device": t_h5}
        self.last_result = res
        return res

    def _stream_producer(self, reader, n_cells: int, batch_reads: int | None, pinned: bool = True):
        """The decode side of a streamed run: the native streaming decoder filling a
        ring of batches (pinned: the engine copies from them; pinned=False: the router
        reads them on the host) on a producer thread. Returns (bam, stream, expected
        reads, free queue, full queue, thread, times); the consumer takes filled slots
        from `full` (None at the end, an exception on error) and hands them back
        through `free` (None stops the producer)."""
        from ..bam import StreamSlot

        bam, st, expected = reader.open_stream()
        n_hint = expected if expected > 0 else max(1, os.path.getsize(reader.bam_path) // 30)
        batch_reads = batch_reads or int(os.environ.get("MGP_STREAM_BATCH", STREAM_BATCH_READS))
        n_slots = max(2, int(os.environ.get("MGP_STREAM_SLOTS", STREAM_SLOTS)))
        cap_reads = max(1, min(int(batch_reads), n_hint + 1))
        cap_payload = cap_reads * 48 + 256 * (n_cells + 1) + (1 << 20)
        slot_bytes = StreamSlot.nbytes(cap_reads, cap_payload)
        free: Queue = Queue()
        full: Queue = Queue()
        for _ in range(n_slots):
            free.put(StreamSlot(cap_reads, cap_payload, _pinned_alloc(slot_bytes) if pinned else None))
        times = {"cap_reads": cap_reads, "cap_payload": cap_payload}

        def produce():
            try:
                while True:
                    sl = free.get()
                    if sl is None:
                        return
                    n = st.next_into(sl)
                    full.put(sl if n else None)
                    if not n:
                        times["decode_end"] = time.perf_counter()
                        return
            except BaseException as e:  # noqa: BLE001 - handed to the consumer
                full.put(e)

        producer = threading.Thread(target=produce, name="mgp-bam-decode", daemon=True)
        producer.start()
        return bam, st, n_hint, free, full, producer, times

    @staticmethod
    def _push_view(item, n_cells: int) -> ReadSoA:
        """A decoded batch as pushed. Records dense in BAM order at one stride (every
        offset checked: a paired placement can give the same payload size with its
        records permuted) go without their rec_off / start / span columns (ABI 4: the
        engine places and pairs them on the device and takes start and span from the
        records), and with 16-bit barcode and |tlen| columns when every key fits
        (mgp_push_batch16, ABI 5: 7 bytes of columns per read over the link instead of
        11; MGP_COLUMNS16=0 keeps the 32-bit ones); any other batch with its offsets."""
        from ..bam import batch_columns16

        soa = item.soa()
        n = soa.n
        if not n:
            return soa
        rc = batch_columns16(soa, n_cells, item.bc16, item.tlen16)
        if rc == 3 and os.environ.get("MGP_COLUMNS16", "1") != "0":
            return ReadSoA(None, item.bc16[:n], item.tlen16[:n], soa.flag, soa.mapq, None, None, soa.payload)
        if rc & 1:
            return ReadSoA(None, soa.bc, soa.tlen, soa.flag, soa.mapq, None, None, soa.payload)
        return soa

    def _rows_target(self, n_cells: int, eng=None, windows: tuple[int, int] | None = None) -> Rows16 | None:
        """Pinned 16-bit result rows for all cells (the rows target)."""
        if n_cells <= 0:
            return None
        nw, W = windows if windows is not None else eng.windows()
        L = self.config.mito_length
        rb = PinnedBuffer(n_cells * L * 22 + n_cells * nw + 4096)
        return Rows16(rb.array((n_cells, L, 8), np.uint16, 0), rb.array((n_cells, L, 2), np.uint16, n_cells * L * 16),
                      rb.array((n_cells, L), np.uint16, n_cells * L * 20),
                      rb.array((n_cells, nw), np.uint8, n_cells * L * 22), W)

    def run_stream(self, reader, n_cells: int, batch_reads: int | None = None,
                   rows_target: bool | None = None) -> EngineResult:
        """The production path, streamed (readers.py:84-93's one pass, overlapped with
        the device): the native decoder fills a ring of pinned batches on a producer
        thread while this thread pushes each finished batch to a streaming engine
        context (MGP_CFG_STREAM: its H2D copies, then the hot path of the position
        windows it completes, run behind the next batches' decode); the 16-bit result
        rows are fetched after the run. With a rows target (rows_target=True or
        MGP_ROWS_TARGET=1), each window's rows leave the device as soon as it is piled,
        into pinned host memory the writers read. Results are those of a
        resident run of the same reads (reads a segment cannot serve rerun it).
        Several devices: see :meth:`_run_stream_sharded`."""
        if rows_target is None:
            # the rows fetched after the run by default: pinning a rows target during the
            # decode (GBs at ~0.25 s per GB, on a thread) slowed the decode more than the
            # fetch costs (C4 txt end to end 5.38-5.43 s with the target, 4.72-5.26 s
            # without, fetch 0.16 s; profiles/r05/e2e_rows_*.log); MGP_ROWS_TARGET=1 keeps it
            rows_target = os.environ.get("MGP_ROWS_TARGET", "0") == "1"
        if len(self.devices) > 1:
            return self._run_stream_sharded(reader, n_cells, batch_reads, rows_target)
        t0 = time.perf_counter()
        bam, st, n_hint, free, full, producer, times = self._stream_producer(reader, n_cells, batch_reads)
        try:
            ec = self.config.engine_config(n_cells, reserve_reads=n_hint,
                                           reserve_payload=_payload_hint(n_hint, n_cells, times["cap_reads"]))
            ec.stream = True
            eng = Engine(ec, device=self.device)
            try:
                # the rows target (GBs of pinned memory: ~0.25 s per GB to pin) is allocated
                # on a thread while the first batches go in; the engine copies the rows of
                # the windows piled before it is set when it is set (ABI 4)
                rows, pending = None, None
                if rows_target and n_cells > 0:
                    box: dict = {}
                    wins = eng.windows()

                    def alloc():
                        try:
                            box["rows"] = self._rows_target(n_cells, windows=wins)
                        except BaseException as e:  # noqa: BLE001 - re-raised below
                            box["err"] = e

                    pending = threading.Thread(target=alloc, name="mgp-rows-alloc", daemon=True)
                    pending.start()

                def settle(wait: bool):
                    nonlocal rows, pending
                    if pending is None or (not wait and pending.is_alive()):
                        return
                    pending.join()
                    pending = None
                    if "err" in box:
                        raise box["err"]
                    rows = box.get("rows")
                    if rows is not None:
                        eng.set_rows16_target(rows)

                t1 = time.perf_counter()
                n_batches, h2d = 0, 0
                while True:
                    item = full.get()
                    if item is None:
                        break
                    if isinstance(item, BaseException):
                        raise item
                    if n_batches == 0:
                        times["first_batch"] = time.perf_counter()
                    settle(False)
                    view = self._push_view(item, n_cells)
                    eng.push(view)
                    h2d += _link_bytes(view)
                    eng.copy_wait()  # its pinned arrays may be refilled now
                    free.put(item)
                    n_batches += 1
                settle(True)
                t2 = time.perf_counter()
                eng.run()
                eng.sync()
                t3 = time.perf_counter()
                res = eng.fetch(dense=False)
                if rows is not None and not rows.wide.any():
                    res.counts, res.tn5, res.depth = rows.counts, rows.tn5, rows.depth
                elif rows is not None:
                    res = eng.fetch(dense=True)  # a drained window: the exact u32 arrays
                else:
                    res = eng.fetch_compact()
                t4 = time.perf_counter()
                self.last_stats = eng.kernel_times()
                _, last_streamed = eng.stream_info()
                t_txt = self._write_txt(res, [(eng, 0, n_cells)]) if self._txt_device_on() else 0.0
                t_h5 = self._write_h5(res, [(eng, 0, n_cells)]) if self._h5_device_on() else 0.0
            finally:
                free.put(None)
                eng.close()
            producer.join()
        finally:
            st.close()
            bam.close()
        te = time.perf_counter()
        # where the streamed engine leg goes: setup (pinned ring + rows target, context),
        # the pushes (behind the decode), the run's tail after the last batch, results
        dec_end = times.get("decode_end", t2)
        self.last_timing = {"stream_setup": t1 - t0, "stream_first_batch": times.get("first_batch", t1) - t0,
                            "stream_decode_end": dec_end - t0, "stream_push_end": t2 - t0,
                            "engine_tail": t3 - t2, "engine_fetch": t4 - t3,
                            "engine_close": te - t4 - t_txt - t_h5, "txt_device": t_txt, "h5_device": t_h5,
                            "stream_batches": n_batches, "stream_batch_reads": times["cap_reads"],
                            "streamed_run": bool(last_streamed), "rows_target": rows is not None,
                            "h2d_bytes": int(h2d)}
        self.last_result = res
        return res

    def _run_stream_sharded(self, reader, n_cells: int, batch_reads: int | None, rows_target: bool) -> EngineResult:
        """The streamed path over several devices: one streaming
        context per device, each owning a contiguous whitelist range of cells and fed by
        a thread of its own. The host routes every decoded batch (mgp_route_batch, the
        reference's split of the barcodes over its pool, processors.py:112-144, as a
        split over devices): each kept read's columns and record go to its cell's
        device's pinned batch, in BAM order, the barcode rebased to the device's range;
        reads without a whitelisted barcode, or that readers.py:96 skips, go nowhere
        (they count only toward total_reads, which the decoder counts). So each link
        carries, and each device holds, only its own cells' reads. The ranges are
        read-balanced by the first batch's reads per cell (a cell's reads are spread
        over all of chrM, so the first batch is a fair sample of the whole set). The
        cells' first-seen order (readers.py:104-163) comes from the router: each cell's
        first routed read's index in the stream. Every device's rows go into its cell
        range of one result array, so nothing is concatenated; the tallies are summed
        on the host."""
        from queue import Empty

        from ..bam import RoutePart, host_threads, route_batch
        from ..exceptions import ProcessingError
        from ..shard import partition_cells

        devs = list(self.devices)
        D = len(devs)
        t0 = time.perf_counter()
        bam, st, n_hint, free, full, producer, times = self._stream_producer(reader, n_cells, batch_reads,
                                                                            pinned=False)
        engines, rings, queues, workers, errors = {}, {}, {}, {}, []
        parts: list[tuple[int, int, int]] = []
        rows = None
        first_seen = np.full(max(1, n_cells), 0xFFFFFFFF, np.uint32)
        n_threads = host_threads()
        n_slots = max(2, int(os.environ.get("MGP_STREAM_SLOTS", STREAM_SLOTS)))
        link_bytes = {}
        try:
            first = full.get()
            if isinstance(first, BaseException):
                raise first
            if first is not None:
                times["first_batch"] = time.perf_counter()
                bc = first.soa().bc
                w = np.bincount(bc[(bc >= 0) & (bc < n_cells)], minlength=n_cells).astype(np.float64) + 1e-3
            else:
                w = np.ones(n_cells)
            bounds = partition_cells(w, D)
            parts = [(d, int(bounds[d]), int(bounds[d + 1])) for d in range(D) if bounds[d + 1] > bounds[d]]
            wsum = float(w.sum()) or 1.0
            share = {d: float(w[lo:hi].sum()) / wsum for d, lo, hi in parts}
            for d, lo, hi in parts:
                m = int(n_hint * share[d] * 1.1) + 65536  # the device's share of the reads, with headroom
                ec = self.config.engine_config(hi - lo, reserve_reads=m,
                                               reserve_payload=_payload_hint(m, hi - lo, times["cap_reads"] * share[d]))
                ec.stream = True
                engines[d] = Engine(ec, device=devs[d])
                rings[d], queues[d] = Queue(), Queue()
                link_bytes[d] = 0
            route_bounds = np.array([lo for _, lo, _ in parts] + ([parts[-1][2]] if parts else [0]), np.int32)
            # a device's batch: its share of a decoded batch with headroom (a batch that
            # does not fit is routed in halves)
            cap_r, cap_p = times["cap_reads"], times["cap_payload"]

            def part_caps(d):
                f = min(1.0, share[d] * 1.5 + 0.02)
                return int(cap_r * f) + 65536, int(cap_p * f) + (1 << 20)

            # the rows target (all cells, one pinned array) is pinned on a thread while the
            # first batches go in; each device thread sets its view when it is ready (the
            # engine copies the windows piled before, ABI 4)
            rows_box: dict = {}
            rows_ready = threading.Event()
            if rows_target and parts:
                wins = engines[parts[0][0]].windows()

                def alloc():
                    try:
                        rows_box["rows"] = self._rows_target(n_cells, windows=wins)
                    except BaseException as e:  # noqa: BLE001 - re-raised by the device threads
                        rows_box["err"] = e
                    rows_ready.set()

                threading.Thread(target=alloc, name="mgp-rows-alloc", daemon=True).start()

            def work(d, lo, hi):
                # the device's pinned batches (pinned here, beside the other devices'), then
                # every routed batch pushed, its copy awaited, its arrays back to the ring
                eng = engines[d]
                view_set = not (rows_target and parts)

                def set_view(wait: bool):
                    nonlocal view_set
                    if view_set or (not wait and not rows_ready.is_set()):
                        return
                    rows_ready.wait()
                    view_set = True
                    if "err" in rows_box:
                        raise rows_box["err"]
                    r = rows_box["rows"]
                    if r is not None:
                        eng.set_rows16_target(Rows16(r.counts[lo:hi], r.tn5[lo:hi], r.depth[lo:hi], r.wide[lo:hi],
                                                     r.window_width))

                try:
                    cr, cp = part_caps(d)
                    for _ in range(n_slots):
                        rings[d].put(RoutePart(cr, cp, _pinned_alloc(RoutePart.nbytes(cr, cp))))
                    while True:
                        set_view(False)
                        pt = queues[d].get()
                        if pt is None:
                            break
                        try:
                            sub = pt.soa()
                            eng.push(sub)
                            link_bytes[d] += _link_bytes(sub)
                            eng.copy_wait()
                        finally:
                            rings[d].put(pt)
                    set_view(True)
                    eng.run()
                    eng.sync()
                except BaseException as e:  # noqa: BLE001 - re-raised by the router
                    errors.append(e)
                    while True:  # drain (handing back the batches it was dealt)
                        pt = queues[d].get()
                        if pt is None:
                            break
                        rings[d].put(pt)

            def take(d):
                while True:
                    if errors:
                        raise errors[0]
                    try:
                        return rings[d].get(timeout=0.2)
                    except Empty:
                        continue

            def route(soa, a, b, base):
                """Reads [a, b) of a decoded batch to their devices (halves when a device's
                batch cannot hold its share)."""
                sub = soa if (a, b) == (0, soa.n) else ReadSoA(None, soa.bc[a:b], soa.tlen[a:b], soa.flag[a:b],
                                                               soa.mapq[a:b], None, soa.rec_off[a:b], soa.payload)
                got = [take(d) for d, _, _ in parts]
                if not route_batch(sub, route_bounds, got, base + a, first_seen, n_threads):
                    for (d, _, _), pt in zip(parts, got):
                        rings[d].put(pt)
                    if b - a <= 1:
                        raise ProcessingError("a read's record does not fit a device batch")
                    mid = (a + b) // 2
                    route(soa, a, mid, base)
                    route(soa, mid, b, base)
                    return
                for (d, _, _), pt in zip(parts, got):
                    (queues[d] if pt.n else rings[d]).put(pt)

            for d, lo, hi in parts:
                workers[d] = threading.Thread(target=work, args=(d, lo, hi), name=f"mgp-dev{d}", daemon=True)
                workers[d].start()
            t1 = time.perf_counter()
            n_batches, base, t_route = 0, 0, 0.0
            try:
                item = first
                while item is not None:
                    if isinstance(item, BaseException):
                        raise item
                    if errors:
                        raise errors[0]
                    soa = item.soa()
                    if parts and soa.n:
                        tr = time.perf_counter()
                        route(soa, 0, soa.n, base)
                        t_route += time.perf_counter() - tr
                    base += soa.n
                    free.put(item)
                    n_batches += 1
                    item = full.get()
            finally:
                for d, _, _ in parts:
                    queues[d].put(None)
                for d, _, _ in parts:
                    workers[d].join()
            if errors:
                raise errors[0]
            rows = rows_box.get("rows")
            t2 = time.perf_counter()
            L = self.config.mito_length
            # without a rows target: every device's exact 16-bit rows fetched into its cell
            # range of one host array (the u32 arrays only when a window was drained)
            src = rows
            if rows is None and parts:
                nw, W = engines[parts[0][0]].windows()
                src = Rows16(np.empty((n_cells, L, 8), np.uint16), np.empty((n_cells, L, 2), np.uint16),
                             np.empty((n_cells, L), np.uint16), np.zeros((n_cells, nw), np.uint8), W)
                for d, lo, hi in parts:
                    engines[d].fetch_rows16(lo=0, hi=hi - lo, out=Rows16(src.counts[lo:hi], src.tn5[lo:hi],
                                                                        src.depth[lo:hi], src.wide[lo:hi], W))
            wide = src is None or bool(src.wide.any())
            res = EngineResult.alloc(n_cells, L, dense=wide)
            st_sum = {k: 0 for k in ("filtered_reads", "n_barcodes", "duplicate_reads_with_length",
                                     "duplicate_reads_position_only", "cells_passed")}
            max_span, err = 0, 0
            for d, lo, hi in parts:
                r = engines[d].fetch(dense=wide)
                for k in ("n_reads", "any_paired", "passed", "covered", "depth_sum", "depth_max", "median_lo",
                          "median_hi"):
                    getattr(res, k)[lo:hi] = getattr(r, k)
                if wide:
                    for k in ("counts", "tn5", "depth"):
                        getattr(res, k)[lo:hi] = getattr(r, k)
                res.ref_tally += r.ref_tally
                for k in st_sum:
                    st_sum[k] += int(r.stats[k])
                max_span = max(max_span, int(r.stats["max_span"]))
                err |= int(r.stats["error_bits"])
            # each cell's first read in the BAM (the router's index over the whole stream)
            res.first_read[:] = first_seen[:n_cells]
            if np.any((res.n_reads > 0) != (res.first_read != 0xFFFFFFFF)):
                raise ProcessingError("routed reads and per-cell read counts disagree")
            if not wide:
                res.counts, res.tn5, res.depth = src.counts, src.tn5, src.depth
            res.stats = {"total_reads": int(st.records), **st_sum, "max_span": max_span, "error_bits": err}
            t3 = time.perf_counter()
            self.last_stats = engines[parts[0][0]].kernel_times() if parts else {}
            t_txt = self._write_txt(res, [(engines[d], lo, hi) for d, lo, hi in parts]) \
                if parts and self._txt_device_on() else 0.0
            t_h5 = self._write_h5(res, [(engines[d], lo, hi) for d, lo, hi in parts]) \
                if parts and self._h5_device_on() else 0.0
        finally:
            free.put(None)
            for eng in engines.values():
                eng.close()
            producer.join()
            st.close()
            bam.close()
        te = time.perf_counter()
        self.last_timing = {"stream_setup": t1 - t0, "stream_first_batch": times.get("first_batch", t1) - t0,
                            "stream_decode_end": times.get("decode_end", t2) - t0, "stream_push_end": t2 - t0,
                            "engine_tail": 0.0, "engine_fetch": t3 - t2, "engine_close": te - t3 - t_txt - t_h5,
                            "txt_device": t_txt, "h5_device": t_h5,
                            "stream_batches": n_batches, "stream_batch_reads": times["cap_reads"],
                            "stream_devices": len(parts), "rows_target": rows is not None, "route_s": t_route,
                            "h2d_bytes": int(sum(link_bytes.values())),
                            "cell_bounds": [lo for _, lo, _ in parts] + ([parts[-1][2]] if parts else [])}
        self.last_result = res
        return res

    def _run_sharded(self, soa_batches, n_cells: int) -> EngineResult:
        """Cells split into contiguous read-balanced ranges, one engine per device,
        run concurrently (ctypes releases the GIL); results concatenated along
        cells and tallies summed on the host."""
        from concurrent.futures import ThreadPoolExecutor

        from ..shard import merge_results, partition_cells, reads_per_cell, shard_soa
        from ..synth import concat_soa

        soa = soa_batches[0] if len(soa_batches) == 1 else concat_soa(soa_batches)
        b = partition_cells(reads_per_cell(soa, n_cells), len(self.devices))
        shards = [(int(lo), int(hi)) + shard_soa(soa, int(lo), int(hi)) for lo, hi in zip(b[:-1], b[1:])]

        def one(i):
            lo, hi, sub, idx = shards[i]
            ec = self.config.engine_config(hi - lo, reserve_reads=sub.n, reserve_payload=sub.payload.shape[0] + 256)
            with Engine(ec, device=self.devices[i]) as eng:
                if sub.n:
                    eng.push(sub)
                eng.run()
                return eng.fetch_compact(), lo, hi, idx

        with ThreadPoolExecutor(len(self.devices)) as ex:
            parts = list(ex.map(one, range(len(self.devices))))
        res = merge_results(parts, n_cells, soa.n)
        self.last_result = res
        return res

    def write_results(self, res: EngineResult, barcodes: list[str], incremental_writer=None) -> list[dict]:
        """Passing cells in first-seen order to the writer; returns the reference's
        slim result list ({"barcode", "n_reads"} per written cell, processors.py:75)."""
        order = res.cell_order()
        written = order[res.passed[order].astype(bool)]
        failed = int(order.size - written.size)
        if failed:
            logger.warning(f"{failed} cells failed")
        if incremental_writer is not None:
            incremental_writer.write_cells(res, written, barcodes=barcodes, tally=res.ref_tally)
        return [{"barcode": barcodes[int(c)], "n_reads": int(res.n_reads[c])} for c in written]

    def process_soa(self, soa_batches, barcodes: list[str], incremental_writer=None) -> list[dict]:
        res = self.run_soa(soa_batches, len(barcodes))
        return self.write_results(res, barcodes, incremental_writer)

    # reference dict API (processors.py:63-144) ------------------------------
    def process_cells_direct(self, reads_by_barcode, incremental_writer=None):
        res, barcodes = run_cells_from_reads(self.config, reads_by_barcode, self.device)
        self.last_result = res
        reads_by_barcode.clear()
        results, failed = [], 0
        for c, bc in enumerate(barcodes):
            if not res.passed[c]:
                failed += 1
                continue
            r = result_dict(res, c, bc, self.config.mito_length)
            if incremental_writer:
                incremental_writer.write_cell(r)
                results.append({"barcode": bc, "n_reads": r["n_reads"]})
            else:
                results.append(r)
        if failed > 0:
            logger.warning(f"{failed} cells failed")
        gc.collect()
        return results

    def process_cells_progressive(self, reads_by_barcode, incremental_writer=None):
        n_cells = len(reads_by_barcode)
        total = sum(len(r) for r in reads_by_barcode.values())
        avg = total / n_cells if n_cells > 0 else 0
        logger.info(f"Processing {n_cells} cells at an average of {avg:.0f} reads/cell")
        return self.process_cells_direct(reads_by_barcode, incremental_writer)


def cells_written(res: EngineResult) -> np.ndarray:
    order = res.cell_order()
    return order[res.passed[order].astype(bool)]
