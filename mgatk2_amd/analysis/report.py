"""HTML QC report (behaviour of src/analysis/report.py).

This module writes ``<output_dir>/mgatk2_report.html``, a self-contained page with
PNG plots embedded as data URIs. The sections follow the reference report:

* scATAC (a singlecell.csv was given, ``generate_html_report``):
  - summary tiles;
  - mean chrM depth per position;
  - mirrored Tn5 cut frequency (fwd above the axis, rev below);
  - dinucleotide context of Tn5 insertions, using the reference allele at pos
    and pos+1;
  - mtDNA depth against total fragments (``barcode_metadata/total``, log-log);
  - coverage breadth against mean depth.
* scRNA (``generate_scrna_html_report``):
  - the read-start-site track replaces the Tn5 tracks;
  - reads (``total_bases / 150``) against depth replaces the fragments plot.

The inputs are ``output/counts.h5`` and ``output/metadata.h5``, read through h5py
when it is installed and otherwise through :mod:`mgatk2_amd.h5lite`.
The ``qc/summary.txt`` key/value lines fill the tiles and the footer. Each
per-position reduction is one numpy call over the position x cell planes.
"""

from __future__ import annotations

import base64
import functools
import html
import io
import logging
import subprocess
import threading
from datetime import datetime
from pathlib import Path

import numpy as np

logger = logging.getLogger(__name__)

DPI = 150
BLUE, MAGENTA, PURPLE = "#2E86AB", "#A23B72", "#9B59B6"
DEPTH_TICKS = [1, 5, 10, 20, 30, 40, 50, 100, 200, 300, 400, 500, 1000, 5000, 10000]


def _h5():
    try:
        import h5py

        return h5py
    except ImportError:
        from .. import h5lite

        return h5lite.module()


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    return plt


def _png(fig) -> str:
    plt = _plt()
    buf = io.BytesIO()
    fig.savefig(buf, format="png", dpi=DPI, bbox_inches="tight")
    plt.close(fig)
    return "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode("ascii")


def _style(ax):
    for side in ("top", "right"):
        ax.spines[side].set_visible(False)
    ax.tick_params(colors="black")


def _placeholder(text: str, size=(6, 5)) -> str:
    plt = _plt()
    fig, ax = plt.subplots(figsize=size)
    ax.text(0.5, 0.5, text, ha="center", va="center", fontsize=14, color="gray")
    ax.axis("off")
    return _png(fig)


# ---------------------------------------------------------------------------
# plots
# ---------------------------------------------------------------------------
def coverage_track(coverage: np.ndarray) -> str:
    """Mean depth per chrM position over the cells (columns) of the coverage plane."""
    plt = _plt()
    cov = np.asarray(coverage)
    mean = cov.mean(axis=1) if cov.ndim == 2 and cov.shape[1] else (cov if cov.ndim == 1 else np.zeros(cov.shape[0]))
    pos = np.arange(1, mean.size + 1)
    fig, ax = plt.subplots(figsize=(10, 3.5))
    ax.plot(pos, mean, linewidth=0.8, color=BLUE)
    ax.set_xlabel("chrM (bp)", fontsize=10)
    ax.set_ylabel("Mean depth", fontsize=10)
    ax.set_xlim(0, max(1, pos[-1] if pos.size else 1))
    _style(ax)
    return _png(fig)


def tn5_track(tn5_fwd: np.ndarray, tn5_rev: np.ndarray) -> str:
    """Tn5 cuts per position summed over cells: forward up, reverse mirrored down."""
    plt = _plt()
    pos = np.arange(1, tn5_fwd.size + 1)
    fig, ax = plt.subplots(figsize=(10, 3.5))
    ax.fill_between(pos, 0, tn5_fwd, linewidth=0.5, color=MAGENTA, alpha=0.6, label="Forward")
    ax.fill_between(pos, 0, -tn5_rev.astype(np.int64), linewidth=0.5, color=BLUE, alpha=0.8, label="Reverse")
    ax.axhline(0, color="black", linewidth=0.8)
    ax.set_xlabel("chrM (bp)", fontsize=10)
    ax.set_ylabel("Tn5 cut sites (n)", fontsize=10)
    ax.set_xlim(0, max(1, pos[-1] if pos.size else 1))
    ax.legend(loc="upper right", frameon=False, fontsize=8)
    _style(ax)
    return _png(fig)


def read_start_track(starts: np.ndarray) -> str:
    plt = _plt()
    pos = np.arange(1, starts.size + 1)
    fig, ax = plt.subplots(figsize=(10, 3.5))
    ax.fill_between(pos, 0, starts, linewidth=0.5, color=BLUE, alpha=0.8)
    ax.set_xlabel("chrM (bp)", fontsize=10)
    ax.set_ylabel("Read start sites (n)", fontsize=10)
    ax.set_xlim(0, max(1, pos[-1] if pos.size else 1))
    _style(ax)
    return _png(fig)


def insertion_context(tn5_total: np.ndarray, reference: list[str]) -> dict[str, int]:
    """Tn5 cuts at position p credited to the reference dinucleotide (p, p+1); the last
    position has no successor, and dinucleotides with N are not counted."""
    ref = np.array([r if r in "ACGT" and len(r) == 1 else "N" for r in reference])
    idx = np.full(ref.size, -1, np.int64)
    for k, b in enumerate("ACGT"):
        idx[ref == b] = k
    t = np.asarray(tn5_total, np.int64)[:-1]
    a, b = idx[:-1], idx[1:]
    ok = (t > 0) & (a >= 0) & (b >= 0)
    sums = np.bincount(a[ok] * 4 + b[ok], weights=t[ok], minlength=16).astype(np.int64)
    return {x + y: int(sums[4 * i + j]) for i, x in enumerate("ACGT") for j, y in enumerate("ACGT")}


def insertion_context_plot(ctx: dict[str, int]) -> str:
    plt = _plt()
    total = sum(ctx.values())
    if total == 0:
        return _placeholder("No Tn5 cut data available", (8, 4))
    names = sorted(ctx)
    pct = [ctx[d] / total * 100 for d in names]
    gc = [(d.count("G") + d.count("C")) / 2 for d in names]
    colors = [MAGENTA if g == 0 else BLUE if g == 1 else PURPLE for g in gc]
    fig, ax = plt.subplots(figsize=(8, 4))
    bars = ax.bar(names, pct, color=colors, alpha=0.8, edgecolor="black", linewidth=0.5)
    for bar, p in zip(bars, pct):
        if p > 0.5:
            ax.text(bar.get_x() + bar.get_width() / 2, p, f"{p:.1f}%", ha="center", va="bottom", fontsize=7)
    ax.set_xlabel("Dinucleotide context", fontsize=10)
    ax.set_ylabel("Tn5 insertion frequency (%)", fontsize=10)
    ax.set_ylim(0, max(pct) * 1.1)
    plt.setp(ax.get_xticklabels(), rotation=45, ha="right")
    _style(ax)
    fig.tight_layout()
    return _png(fig)


def _loglog_depth(x: np.ndarray, depth: np.ndarray, xlabel: str) -> str:
    plt = _plt()
    from matplotlib.ticker import FixedLocator, FuncFormatter

    m = (x > 0) & (depth > 0)
    if not m.any():
        return _placeholder("No data available\n(all values are zero)")
    fig, ax = plt.subplots(figsize=(6, 5))
    ax.scatter(x[m], depth[m], s=10, color="black", edgecolors="none")
    ax.set_xscale("log")
    ax.set_yscale("log")
    ax.set_xlabel(xlabel, fontsize=10)
    ax.set_ylabel("mtDNA depth (log10)", fontsize=10)
    ax.yaxis.set_major_locator(FixedLocator(DEPTH_TICKS))
    ax.xaxis.set_major_formatter(FuncFormatter(lambda v, _: f"{int(v):,}"))
    ax.yaxis.set_major_formatter(FuncFormatter(lambda v, _: f"{int(v):,}"))
    _style(ax)
    return _png(fig)


def depth_vs_coverage_plot(mean_depth: np.ndarray, breadth: np.ndarray) -> str:
    plt = _plt()
    m = (mean_depth > 0) & (breadth > 0)
    if not m.any():
        return _placeholder("No data available")
    fig, ax = plt.subplots(figsize=(6, 5))
    ax.scatter(mean_depth[m], breadth[m], s=20, color="black", edgecolors="none")
    ax.set_xlabel("Mean mtDNA depth", fontsize=10)
    ax.set_ylabel("Coverage breadth (%)", fontsize=10)
    ax.set_xlim(0, 105)
    _style(ax)
    return _png(fig)


# ---------------------------------------------------------------------------
# page
# ---------------------------------------------------------------------------
def _title(title, sample_name, working_directory, input_dir) -> str:
    """10x-aware title: the run folder holding outs/ (report.py:433-461)."""
    if title is not None:
        return title
    for cand, parent_ok in ((input_dir, False), (working_directory, True)):
        if cand is None:
            continue
        p = Path(cand)
        if p.name == "outs":
            return p.parent.name
        if (p / "outs").exists():
            return p.name
        if parent_ok and p.parent.name == "outs":
            return p.parent.parent.name
        return p.name
    return sample_name


def _summary(output_dir: Path) -> dict[str, str]:
    f = output_dir / "qc" / "summary.txt"
    out: dict[str, str] = {}
    if f.exists():
        for line in f.read_text().splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                out[k.strip()] = v.strip()
    return out


@functools.lru_cache(maxsize=1)
def _env() -> str:
    try:
        r = subprocess.run(["pip", "list"], capture_output=True, text=True, timeout=30)
        return r.stdout if r.returncode == 0 else "pip not available"
    except Exception:
        return "pip not available"


def prewarm() -> threading.Thread:
    """Start a daemon thread that pays the report's fixed costs early (the pyplot
    import and the ``pip list`` of the environment section, ~1.5 s together), so a
    pipeline can overlap them with the BAM decode and the engine."""

    def work():
        try:
            _plt()
        except ImportError:
            pass
        _env()

    t = threading.Thread(target=work, name="mgp-report-prewarm", daemon=True)
    t.start()
    return t


CSS = """
body{font-family:-apple-system,'Segoe UI',Arial,sans-serif;margin:0;padding:20px;background:#f5f5f5;color:#000}
.container{max-width:1200px;margin:0 auto;background:#fff;padding:30px;border-radius:8px;box-shadow:0 2px 4px #0002}
h1{border-bottom:3px solid #000;padding-bottom:10px;margin-bottom:5px}
.subtitle{color:#666;font-size:1.1em;font-style:italic;margin-bottom:20px}
h2{margin-top:30px;border-left:4px solid #000;padding-left:10px}
.tiles{display:grid;grid-template-columns:repeat(auto-fit,minmax(200px,1fr));gap:15px;margin:20px 0}
.tile{background:#f8f9fa;padding:15px;border-radius:5px;border-left:3px solid #2E86AB}
.tile .k{font-size:.85em;text-transform:uppercase}.tile .v{font-size:1.5em;font-weight:bold;margin-top:5px}
.plot{margin:20px 0;text-align:center}.plot img{max-width:100%;height:auto}
.pair{display:grid;grid-template-columns:repeat(2,1fr);gap:20px}
.footer{margin-top:40px;padding-top:20px;border-top:1px solid #ddd;font-size:.9em;text-align:center}
.env{margin-top:30px;padding:15px;background:#f8f9fa;border-radius:5px;font-size:.8em}
.env pre{background:#fff;padding:10px;max-height:300px;overflow:auto;white-space:pre-wrap}
"""


def _page(title, subtitle, working_directory, tiles, sections, pair, summary, output_dir) -> str:
    esc = html.escape
    tile_html = "".join(f'<div class="tile"><div class="k">{esc(k)}</div><div class="v">{esc(v)}</div></div>'
                        for k, v in tiles)
    sec_html = "".join(f'<h2>{esc(h)}</h2><div class="plot"><img src="{img}" alt="{esc(h)}">{note}</div>'
                       for h, img, note in sections)
    pair_html = "".join(f'<div><h2>{esc(h)}</h2><div class="plot"><img src="{img}" alt="{esc(h)}"></div></div>'
                        for h, img in pair)
    wd = f"<p><strong>Working directory:</strong> {esc(working_directory)}</p>" if working_directory else ""
    return f"""<!DOCTYPE html>
<html><head><meta charset="UTF-8"><meta name="viewport" content="width=device-width, initial-scale=1.0">
<title>{esc(title)} - mgatk2 Report</title><style>{CSS}</style></head>
<body><div class="container">
<h1>{esc(title)}</h1><div class="subtitle">{esc(subtitle)}</div>
<p><strong>Date:</strong> {datetime.now().strftime("%d/%m/%Y, %H:%M")}</p>{wd}
<h2>Summary statistics</h2><div class="tiles">{tile_html}</div>
{sec_html}
<div class="pair">{pair_html}</div>
<div class="footer">Generated by mgatk2 (MI355X engine) v{esc(summary.get("mgatk_version", "?"))} |
Reference: {esc(summary.get("reference", "chrM"))} | Output: {esc(Path(output_dir).name)}</div>
<div class="env"><details><summary>Python packages</summary><pre>{esc(_env())}</pre></details></div>
</div></body></html>
"""


def _load(output_dir: Path, need_tn5: bool, need_meta_group: bool):
    h5 = _h5()
    counts_file = output_dir / "output" / "counts.h5"
    meta_file = output_dir / "output" / "metadata.h5"
    if not counts_file.exists() or not meta_file.exists():
        logger.error("Output files not found in %s", output_dir)
        return None
    d = {}
    with h5.File(meta_file, "r") as f:
        d["coverage"] = np.asarray(f["coverage"][...])
        d["mean_depth"] = np.asarray(f["mean_depth"][...])
        d["genome_coverage"] = np.asarray(f["genome_coverage"][...])
        d["total_bases"] = np.asarray(f["total_bases"][...])
        ref = f["reference"][...]
        d["reference"] = [x.decode() if isinstance(x, bytes) else str(x) for x in ref]
        if need_meta_group:
            try:
                d["total"] = np.asarray(f["barcode_metadata"]["total"][...], dtype=np.float64)
            except KeyError:
                d["total"] = np.zeros(0)
    if need_tn5:
        with h5.File(counts_file, "r") as f:
            d["tn5_fwd"] = np.asarray(f["tn5_cuts_fwd"][...]).sum(axis=1, dtype=np.int64)
            d["tn5_rev"] = np.asarray(f["tn5_cuts_rev"][...]).sum(axis=1, dtype=np.int64)
    return d


def _tiles(d, summary):
    md = d["mean_depth"]
    return [("Total cells", f"{md.size:,}"), ("Cells passing QC", summary.get("cells_passed_qc", "N/A")),
            ("Mean depth", f"{(md.mean() if md.size else 0.0):.1f}×")]


def _from_arrays(a: dict) -> dict:
    """The writer's in-memory report arrays (IncrementalHDF5Writer.report_arrays) in
    _load's form: the coverage plane as its per-position column mean."""
    return {"coverage": np.asarray(a["coverage_mean"], np.float64), "coverage_sum": a["coverage_sum"],
            "mean_depth": a["mean_depth"], "genome_coverage": a["genome_coverage"], "total_bases": a["total_bases"],
            "reference": a["reference"], "total": a["total"], "tn5_fwd": a["tn5_fwd"], "tn5_rev": a["tn5_rev"]}


def _atac_plots(d: dict):
    ctx = insertion_context(d["tn5_fwd"] + d["tn5_rev"], d["reference"])
    total = d["total"]
    depth_frag = _loglog_depth(total, d["mean_depth"][: total.size] if total.size else total,
                               "Total fragments (log10)") if total.size == d["mean_depth"].size else \
        _placeholder("No data available\n(no fragment totals)")
    sections = [("chrM coverage", coverage_track(d["coverage"]), ""),
                ("Tn5 transposition frequency", tn5_track(d["tn5_fwd"], d["tn5_rev"]), ""),
                ("Tn5 insertion sequence context", insertion_context_plot(ctx),
                 '<p style="color:#666;font-size:.9em">magenta = AT-rich, blue = GC-rich, purple = mixed</p>')]
    pair = [("Depth per cell", depth_frag),
            ("chrM coverage", depth_vs_coverage_plot(d["mean_depth"], d["genome_coverage"]))]
    return sections, pair


def _scrna_plots(d: dict):
    starts = d["coverage"].sum(axis=1, dtype=np.int64) if d["coverage"].ndim == 2 else \
        d.get("coverage_sum", d["coverage"])
    sections = [("chrM coverage", coverage_track(d["coverage"]), ""),
                ("Read start sites", read_start_track(starts), "")]
    pair = [("Number of reads", _loglog_depth(d["total_bases"] / 150.0, d["mean_depth"], "Number of reads (log10)")),
            ("chrM coverage", depth_vs_coverage_plot(d["mean_depth"], d["genome_coverage"]))]
    return sections, pair


def render_plots(arrays: dict, scatac: bool):
    """The report's figures from the writer's in-memory arrays, before the page is
    put together: a pipeline renders them while the HDF5 files are still being
    written (the deflate runs in native code without the GIL)."""
    d = _from_arrays(arrays)
    return _atac_plots(d) if scatac else _scrna_plots(d)


def generate_html_report(output_dir: Path, sample_name: str = "mgatk2", title: str | None = None,
                         subtitle: str | None = None, working_directory: str | None = None,
                         input_dir: str | None = None, arrays: dict | None = None, plots=None):
    """scATAC report (singlecell.csv metadata present). ``arrays``: the writer's
    in-memory sums (the files are then not read back); ``plots``: the figures
    already rendered from them (render_plots)."""
    output_dir = Path(output_dir)
    d = _from_arrays(arrays) if arrays is not None else _load(output_dir, need_tn5=True, need_meta_group=True)
    if d is None:
        return None
    summary = _summary(output_dir)
    sections, pair = plots if plots is not None else _atac_plots(d)
    page = _page(
        _title(title, sample_name, working_directory, input_dir), subtitle or "mgatk2 output analysis",
        working_directory, _tiles(d, summary), sections, pair, summary, output_dir)
    out = output_dir / "mgatk2_report.html"
    out.write_text(page)
    return out


def generate_scrna_html_report(output_dir: Path, sample_name: str = "mgatk2", title: str | None = None,
                               subtitle: str | None = None, working_directory: str | None = None,
                               input_dir: str | None = None, arrays: dict | None = None, plots=None):
    """scRNA report (no singlecell.csv): read-start track and reads-vs-depth plot."""
    output_dir = Path(output_dir)
    d = _from_arrays(arrays) if arrays is not None else _load(output_dir, need_tn5=False, need_meta_group=False)
    if d is None:
        return None
    summary = _summary(output_dir)
    sections, pair = plots if plots is not None else _scrna_plots(d)
    page = _page(
        _title(title, sample_name, working_directory, input_dir), subtitle or "mgatk2 output analysis",
        working_directory, _tiles(d, summary), sections, pair, summary, output_dir)
    out = output_dir / "mgatk2_report.html"
    out.write_text(page)
    return out
