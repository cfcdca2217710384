"""Fixtures from the reference's own committed outputs (real 10x data).

The reference repository holds the outputs of `make run` / `make tenx` on its test
BAM (tests/run_txt_output, tests/tenx_output, tests/run_hdf5_output/qc), but not
the BAM itself (.MISSING_LARGE_BLOBS), so they cannot drive the engine. They do
pin the writers: the per-(position, cell) forward/reverse counts in
output.{A,C,G,T}.txt.gz plus qc/cell_stats.csv are everything
IncrementalTextWriter consumes (writers.py:430-510), and the files it produced
are the expected outputs. This script turns them into data:

  counts     [cells, 16569, 8] u16, A_fwd, A_rev, ... T_rev (the txt lines)
  barcodes   cell names (sorted), n_reads / total_fragments from cell_stats.csv
  expected   the reference's coverage / A..T lines (sorted: its parallel order
             is nondeterministic) as sha256 + line counts, and the
             exact bytes of output.depthTable.txt, {chr}_refAllele.txt and the
             sorted cell_stats.csv lines

Run here (the only place /root/reference exists):
    python tests/golden/make_refout.py
"""

from __future__ import annotations

import gzip
import hashlib
from pathlib import Path

import numpy as np

REF = Path("/root/reference/tests")
OUT = Path(__file__).resolve().parent
L = 16569
SETS = {"refout_run_txt": "run_txt_output", "refout_tenx": "tenx_output"}


def sorted_sha(lines: list[str]) -> str:
    return hashlib.sha256("".join(sorted(lines)).encode()).hexdigest()


def read_lines(p: Path) -> list[str]:
    opener = gzip.open if p.suffix == ".gz" else open
    with opener(p, "rt") as f:
        return f.readlines()


def make(name: str, d: str):
    base = REF / d
    stats = read_lines(base / "qc" / "cell_stats.csv")
    header, rows = stats[0], stats[1:]
    assert header.strip() == "barcode,mean_depth,coverage_breadth,total_fragments,total_reads", header
    cells = sorted(r.split(",")[0] for r in rows)
    idx = {c: i for i, c in enumerate(cells)}
    n_reads = np.zeros(len(cells), np.uint32)
    frags = np.zeros(len(cells), np.uint32)
    for r in rows:
        bc, _, _, tf, tr = r.strip().split(",")
        n_reads[idx[bc]] = int(tr)
        frags[idx[bc]] = int(tf)
    counts = np.zeros((len(cells), L, 8), np.uint16)
    shas = {}
    for bi, b in enumerate("ACGT"):
        lines = read_lines(base / "output" / f"output.{b}.txt.gz")
        for ln in lines:
            p, bc, fw, rv = ln.split(",")
            c, pos = idx[bc], int(p) - 1
            assert counts[c, pos, 2 * bi] == 0 and counts[c, pos, 2 * bi + 1] == 0
            counts[c, pos, 2 * bi] = int(fw)
            counts[c, pos, 2 * bi + 1] = int(rv)
        shas[b] = (sorted_sha(lines), len(lines))
    cov = read_lines(base / "output" / "output.coverage.txt.gz")
    shas["coverage"] = (sorted_sha(cov), len(cov))
    depth_table = (base / "output" / "output.depthTable.txt").read_text()
    ref_allele = (base / "output" / "chrM_refAllele.txt").read_text()
    np.savez_compressed(
        OUT / f"{name}.npz",
        source=np.array(d),
        barcodes=np.array(cells),
        n_reads=n_reads,
        total_fragments=frags,
        counts=counts,
        sha_names=np.array(list(shas)),
        sha_values=np.array([v[0] for v in shas.values()]),
        sha_lines=np.array([v[1] for v in shas.values()], np.int64),
        depth_table=np.array(depth_table),
        ref_allele=np.array(ref_allele),
        cell_stats_sorted=np.array("".join(sorted(rows))),
        cell_stats_header=np.array(header),
    )
    print(name, len(cells), "cells", {k: v[1] for k, v in shas.items()})


if __name__ == "__main__":
    for name, d in SETS.items():
        make(name, d)
    # run_hdf5_output's cell_stats.csv is the run_txt one (same run parameters)
    a = sorted(read_lines(REF / "run_hdf5_output" / "qc" / "cell_stats.csv"))
    b = sorted(read_lines(REF / "run_txt_output" / "qc" / "cell_stats.csv"))
    assert a == b, "run_hdf5_output/qc/cell_stats.csv differs from run_txt_output's"
