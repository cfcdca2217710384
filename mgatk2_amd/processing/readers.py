"""BAM reading (mirror of src/processing/readers.py).

The reference streams `pysam.AlignmentFile.fetch(mito_chr)` and builds one
Python ``SimpleRead`` per kept record (readers.py:63-201). Here the native
decoder (libmgphost.so, include/mgpileup_host.h) turns every chrM record into
the engine's SoA batch in one pass. The record filters, the whitelist check
and the dedup then run on the GPU (mgatk2_amd/csrc/mgp_engine.hip).

* :meth:`BAMReader.read_soa` is the production path. It returns the whole chrM
  record set as a batch plus the ``total_reads`` statistic. The other counters
  of readers.py:193-199 come from the engine (``EngineResult.stats``).
* :meth:`BAMReader.collect_reads_by_barcode` keeps the reference's dict API.
  It returns ``SimpleRead`` lists per barcode with the same filters, dedup and
  statistics, restated on the host for parity tests and small inputs.
"""

from __future__ import annotations

import os

import logging
from collections import defaultdict
from pathlib import Path

import numpy as np

from ..bam import BamFile
from ..config import PipelineConfig, SimpleRead
from ..exceptions import BAMFormatError, BAMReadError, NoBarcodeTagsError, NoChrMReadsError
from ..synth import FLAG_NOSEQQUAL, ReadSoA, unpack_record

logger = logging.getLogger(__name__)

MITO_NAMES = ["chrM", "MT", "M", "chrMT"]  # readers.py:43
TAG_CHECK_RECORDS = 1001  # readers.py:54-59: records 0..1000 are examined


class BAMReader:
    """Reads and filters BAM files for mtDNA analysis (readers.py:22-33)."""

    def __init__(self, bam_path: str, config: PipelineConfig, barcodes, n_threads: int = 0):
        self.bam_path = Path(bam_path)
        self.config = config
        # the reference takes a set; cell ids need an order, so a list is kept as given
        self.barcode_list = list(barcodes) if not isinstance(barcodes, (set, frozenset)) else sorted(barcodes)
        self.barcodes = set(self.barcode_list)
        self.n_threads = n_threads
        if not self.bam_path.exists():
            raise BAMReadError(str(bam_path), "File does not exist")
        self._validate_bam_file()

    def _open(self) -> BamFile:
        return BamFile(self.bam_path, n_threads=self.n_threads)

    def _validate_bam_file(self):
        """readers.py:35-61: mito contig (first of MITO_NAMES present wins over
        the configured name) and a barcode tag among the first 1001 records."""
        try:
            bam = self._open()
        except BAMFormatError:
            raise
        except Exception as e:  # pragma: no cover - defensive
            raise BAMFormatError(str(self.bam_path), f"Cannot open: {e}") from e
        with bam:
            available = list(bam.references)
            for mito_name in MITO_NAMES:
                if mito_name in available:
                    if self.config.mito_chr != mito_name:
                        logger.info(f"Using mitochondrial chromosome: {mito_name}")
                        self.config.mito_chr = mito_name
                    break
            else:
                raise NoChrMReadsError(str(self.bam_path), available)
            first, checked = bam.find_tag(self.config.mito_chr, self.config.barcode_tag, TAG_CHECK_RECORDS)
            if first < 0 and checked >= TAG_CHECK_RECORDS:
                raise NoBarcodeTagsError(str(self.bam_path), self.config.barcode_tag, TAG_CHECK_RECORDS - 1)

    @property
    def is_bulk_mode(self) -> bool:
        return self.barcodes == {"bulk"}  # readers.py:74

    def read_soa(self, rec_align: int = 64, pack: bool = True) -> tuple[ReadSoA, dict]:
        """Every chrM record as one engine batch (BAM order).

        ``bc`` is the whitelist index (-1 = no tag or not whitelisted). In bulk
        mode every record goes to the ``"bulk"`` cell (readers.py:97-99). With
        packing, reads that fit get the packed 64-byte record, two of a cell to a
        128-byte line (MGP_RECORDS=32: the 32-byte record made for the run's
        min_baseq, four to a line), the others the full one."""
        try:
            with self._open() as bam:
                soa = bam.read_soa(self.config.mito_chr, self.barcode_list, tag=self.config.barcode_tag,
                                   rec_align=rec_align, **self._pack_settings(pack))
        except BAMReadError:
            raise
        except Exception as e:
            raise BAMReadError(str(self.bam_path), f"Read error: {e}") from e
        return soa, {"total_reads": soa.n}

    def _pack_settings(self, pack: bool) -> dict:
        q = int(self.config.quality.min_baseq)
        md = int(self.config.quality.min_distance_from_end)
        bulk = max(i for i, b in enumerate(self.barcode_list) if b == "bulk") if self.is_bulk_mode else -1
        # the producer's records: quality-carrying 64-byte records by default (the kernel
        # applies the per-base filter of pileup.py:67-88); MGP_RECORDS=32: the 32-byte
        # records made for the run's thresholds (the producer resolves it). C4 end to end,
        # one box (profiles/r05/e2e_c4_r5f.json): BAM ingest 5.85-6.01 s with 64-byte
        # records against 6.13-6.71 s with 32-byte ones; the engine is hidden either way
        p32 = os.environ.get("MGP_RECORDS", "64") == "32"
        # where a cell's records are paired two per 128-byte line (the pileup's gathers):
        # "device" (default with 64-byte records): the decoder leaves the records in BAM
        # order (pass 1 and the columns in one pool pass, the records in a second, no
        # placement thread, no duplicate-key stage) and the engine pairs each dense batch
        # on the device (mgp_push_batch); "paired": the decoder's placement thread
        # (mgp_place_records' rule; the 32-byte records always take it, four per line)
        paired = p32 or os.environ.get("MGP_PLACEMENT", "device") == "paired"
        return dict(bulk_cell=bulk, pack=pack, paired=pack and paired,
                    pack32=q if pack and p32 and -128 <= q <= 127 and md <= 15 else None, pack32_dist=md)

    def open_stream(self, rec_align: int = 64, pack: bool = True):
        """The chrM records as a streaming decode (readers.py:84-93's one pass, in
        batches): returns (BamFile, BamStream, expected records or -1). The caller
        pulls batches with ``stream.next_into(slot)`` and closes both."""
        bam = self._open()
        try:
            st = bam.stream(self.config.mito_chr, self.barcode_list, tag=self.config.barcode_tag, rec_align=rec_align,
                            **self._pack_settings(pack))
        except BAMReadError:
            bam.close()
            raise
        except Exception as e:
            bam.close()
            raise BAMReadError(str(self.bam_path), f"Read error: {e}") from e
        return bam, st, bam.ref_records(self.config.mito_chr)

    def collect_reads_by_barcode(self) -> tuple[dict, dict]:
        """readers.py:63-201 on the host: dict[barcode -> list[SimpleRead]] + stats."""
        soa, _ = self.read_soa(rec_align=16, pack=False)  # query_sequence is rebuilt exactly
        index = {b: i for i, b in enumerate(self.barcode_list)}
        names = {i: b for b, i in index.items()}
        reads_by_barcode: dict[str, list] = defaultdict(list)
        seen_len: dict[str, set] = defaultdict(set)
        seen_pos: dict[str, set] = defaultdict(set)
        total = filtered = dup_len = dup_pos = 0
        try:
            for i in range(soa.n):
                total += 1
                f = int(soa.flag[i])
                if f & (0x4 | 0x100 | 0x800):  # unmapped / secondary / supplementary (readers.py:96)
                    continue
                c = int(soa.bc[i])
                if c < 0:
                    continue
                barcode = names[c]
                rev = bool(f & 0x10)
                if not self.config.dedup.skip:
                    start = int(soa.start[i])
                    kl = (start, rev, abs(int(soa.tlen[i])))
                    kp = (start, rev)
                    is_l, is_p = kl in seen_len[barcode], kp in seen_pos[barcode]
                    seen_len[barcode].add(kl)
                    seen_pos[barcode].add(kp)
                    dup_len += is_l
                    dup_pos += is_p
                    if self.config.dedup.use_fragment_length and is_l:
                        continue
                    if not self.config.dedup.use_fragment_length and is_p:
                        continue
                if f & FLAG_NOSEQQUAL:  # .encode() / np.array(None, int8) raise (readers.py:158-159)
                    raise ValueError("read without sequence or base qualities")
                d = unpack_record(soa.payload, int(soa.rec_off[i]), int(soa.flag[i]))
                reads_by_barcode[barcode].append(SimpleRead(
                    reference_start=int(soa.start[i]),
                    is_reverse=rev,
                    mapping_quality=int(soa.mapq[i]),
                    query_sequence=d["query_sequence"].encode("ascii"),
                    query_qualities=np.array(d["query_qualities"], dtype=np.uint8).view(np.int8),
                    cigar=d["cigartuples"],
                    is_proper_pair=bool(f & 0x2),
                    is_paired=bool(f & 0x1),
                    template_length=int(soa.tlen[i]),
                ))
                filtered += 1
        except Exception as e:
            raise BAMReadError(str(self.bam_path), f"Read error: {e}") from e
        stats = {
            "total_reads": total,
            "filtered_reads": filtered,
            "n_barcodes": len(reads_by_barcode),
            "duplicate_reads_with_length": dup_len,
            "duplicate_reads_position_only": dup_pos,
        }
        return dict(reads_by_barcode), stats
