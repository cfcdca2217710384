"""End-to-end timing on one GPU ("Also report end-to-end wall
time including BAM decode and writers separately").

Makes a synthetic coordinate-sorted BAM of BASELINE config C3 (50M chrM reads x
5k cells, `run` parameters) with the device generator and the native BAM writer,
then runs ``run_pipeline`` on it (txt and hdf5 outputs) and prints one JSON line
with the stage times: BAM ingest (native decode into the engine batch), engine
(H2D + run + D2H), writers, QC report.

    python scripts/e2e_bench.py [--reads N] [--cells C] [--threads T] [--out DIR]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def _first_members(path: Path, k: int) -> tuple[bytes, int]:
    """The text of a multi-member gzip file's first k members and their compressed bytes."""
    import zlib

    buf = path.read_bytes()
    pos, parts = 0, []
    for _ in range(k):
        if pos >= len(buf):
            break
        d = zlib.decompressobj(31)
        parts.append(d.decompress(buf[pos:]))
        pos = len(buf) - len(d.unused_data)
    return b"".join(parts), pos


def _zlib9_one(args):
    import gzip

    path, k = args
    text, nbytes = _first_members(Path(path), k)
    return Path(path).name, len(text), nbytes, len(gzip.compress(text, compresslevel=9))


def zlib9_compare(out_dir: Path, k: int) -> dict:
    """The written .txt.gz files against the reference's gzip.open(..., compresslevel=9)
    (writers.py:471-486) on the same text: the first k cells' members of each file (one
    per cell when the device wrote them) recompressed as one zlib-9 stream; a bounded
    sample, zlib 9 runs at ~7 MB/s on this text."""
    from concurrent.futures import ProcessPoolExecutor

    files = [str(out_dir / f"output.{f}.txt.gz") for f in ("coverage", "A", "C", "G", "T")]
    with ProcessPoolExecutor(5) as ex:
        rows = list(ex.map(_zlib9_one, [(f, k) for f in files]))
    return {"sample_cells": k, "files": {n: {"text": t, "written": w, "zlib9": z, "ratio": round(w / z, 4)}
                                         for n, t, w, z in rows},
            "max_ratio": round(max(w / z for _, _, w, z in rows), 4)}


def run_e2e(reads: int, cells: int, threads: int, out: str | Path, formats=("txt", "hdf5"), modes=("stream",),
            records=("64",), gzip_levels=("9",), bam_level: int = 6, reuse_bam: bool = False, devices: str = "0",
            log=sys.stderr, zlib9_sample: int = 100) -> dict:
    """Synthetic BAM (device generator + native writer), then ``run_pipeline`` per
    (record layout, mode, format, gzip level); returns the stage times of each run."""
    from mgatk2_amd.bam import write_bam
    from mgatk2_amd.engine import Engine, EngineConfig
    from mgatk2_amd.pipeline import MtDNAPipeline
    from mgatk2_amd.config import PipelineConfig
    from mgatk2_amd.synth import barcode_names, cell_cdf, ref_codes

    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    seed = 20251015 + 3
    t0 = time.time()
    whitelist = barcode_names(cells, seed)
    bam = out / "possorted_bam.bam"
    tag = out / "possorted_bam.size"
    want = f"{reads} {cells} {bam_level}"
    if reuse_bam and bam.exists() and tag.exists() and tag.read_text() == want:
        t1 = t2 = time.time()
    else:
        with Engine(EngineConfig(n_cells=cells), device=0) as eng:
            eng.synth(seed, reads, cell_cdf(seed, cells), ref_codes(seed), read_len=50)
            soa = eng.download_inputs()
        t1 = time.time()
        write_bam(bam, soa, whitelist, level=bam_level, n_threads=threads)
        del soa
        t2 = time.time()
        tag.write_text(want)
    (out / "barcodes.tsv").write_text("".join(b + "\n" for b in whitelist))
    print(f"[e2e] generated {reads:,} reads in {t1 - t0:.1f}s; BAM {bam.stat().st_size / 1e9:.2f} GB "
          f"written in {t2 - t1:.1f}s", file=log, flush=True)

    name = {(50_000_000, 5_000): "C3", (200_000_000, 10_000): "C4"}.get((reads, cells), "custom")
    res = {"config": f"{name}: {reads:,} reads x {cells} cells, run params (q20 mapq30 "
                     "dedup=alignment_and_fragment_length)", "host_threads": threads, "devices": devices,
           "bam_bytes": bam.stat().st_size, "bam_level": bam_level}
    digests = {}
    runs = [(mode, fmt, rec, lvl) for rec in records for mode in modes
            for fmt in formats for lvl in (gzip_levels if fmt == "txt" else ["-"])]
    for mode, fmt, rec, lvl in runs:
        os.environ["MGP_RECORDS"] = rec
        if lvl != "-":
            os.environ["MGP_GZIP_LEVEL"] = lvl
        cfg = PipelineConfig(min_baseq=20, min_mapq=30, max_strand_bias=1.0, skip_deduplication=False,
                             use_fragment_length_dedup=True, min_reads_per_cell=1, n_cores=threads)
        t = time.time()
        od = out / f"run_{fmt}_{mode}"
        devs = [int(x) for x in devices.split(",")]
        p = MtDNAPipeline(str(bam), whitelist, od, config=cfg, output_format=fmt, stream=mode == "stream",
                          devices=devs if len(devs) > 1 else None)
        ret = p.run()
        wall = time.time() - t
        key = f"{fmt}_{mode}" + (f"_r{rec}" if len(records) > 1 else "") + \
              (f"_z{lvl}" if lvl != "-" and len(gzip_levels) > 1 else "")
        res[key] = {"wall_s": round(wall, 2), "records": rec, "gzip_level": None if lvl == "-" else int(lvl),
                    **{k: (round(v, 3) if isinstance(v, float) else v) for k, v in p.timings.items()},
                    "reads_per_s_end_to_end": round(reads / wall), "cells_passed": ret.get("cells_passed_qc")}
        if fmt == "txt":
            res[key]["txt_gz_bytes"] = sum((od / "output" / f"output.{f}.txt.gz").stat().st_size
                                           for f in ("A", "C", "G", "T", "coverage"))
            if zlib9_sample and lvl == "9":
                res[key]["vs_zlib9"] = zlib9_compare(od / "output", zlib9_sample)
        if fmt == "hdf5":
            html = od / "mgatk2_report.html"
            res[key]["report_html_bytes"] = html.stat().st_size if html.exists() else 0
            res[key]["report_figures"] = html.read_text().count("data:image/png") if html.exists() else 0
        print(f"[e2e] {key}: {res[key]}", file=log, flush=True)
        if fmt == "txt":  # every mode, record layout and level must write the same text
            import gzip
            import hashlib

            h = hashlib.sha256()
            for f in ("A", "C", "G", "T", "coverage"):
                h.update(gzip.decompress((od / "output" / f"output.{f}.txt.gz").read_bytes()))
            digests[key] = h.hexdigest()
        import shutil

        shutil.rmtree(od, ignore_errors=True)
    if len(digests) > 1:
        res["txt_identical_across_runs"] = len(set(digests.values())) == 1
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=50_000_000)
    ap.add_argument("--cells", type=int, default=5_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--out", default="/tmp/mgp_e2e")
    ap.add_argument("--formats", default="txt,hdf5")
    ap.add_argument("--modes", default="stream,resident",
                    help="stream: batches decoded and pushed as they come (the default pipeline); resident: the "
                         "whole chrM set decoded, then one run")
    ap.add_argument("--bam-level", type=int, default=6, help="BGZF level of the synthetic BAM (samtools' default 6)")
    ap.add_argument("--records", default="64",
                    help="producer record layouts to compare (MGP_RECORDS): 32 (32-byte records made for the run's "
                         "thresholds, four per line) and/or 64 (quality-carrying 64-byte records, two per line)")
    ap.add_argument("--gzip-levels", default="9", help="txt gzip levels to time (MGP_GZIP_LEVEL; 9 = the reference's)")
    ap.add_argument("--reuse-bam", action="store_true", help="keep a BAM of the same size already in --out")
    ap.add_argument("--devices", default="0",
                    help="engine devices, comma-separated (cells split over them; '0,0' runs two shards on one GPU)")
    args = ap.parse_args()
    res = run_e2e(args.reads, args.cells, args.threads, args.out, formats=tuple(args.formats.split(",")),
                  modes=tuple(args.modes.split(",")), records=tuple(args.records.split(",")),
                  gzip_levels=tuple(args.gzip_levels.split(",")), bam_level=args.bam_level,
                  reuse_bam=args.reuse_bam, devices=args.devices)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
