"""Small text formatters (mirror of src/file_io/formats.py:9-57)."""

from __future__ import annotations

from pathlib import Path

CELL_STATS_COLUMNS = ["barcode", "mean_depth", "coverage_breadth", "total_fragments", "total_reads"]


def write_cell_stats(cell_stats: list[dict], output_path: Path):
    """qc/cell_stats.csv (formats.py:9-24): values printed with str()."""
    if not cell_stats:
        return
    with open(output_path, "w") as f:
        f.write(",".join(CELL_STATS_COLUMNS) + "\n")
        for stats in cell_stats:
            f.write(",".join(str(stats.get(k, "NA")) for k in CELL_STATS_COLUMNS) + "\n")


def write_run_summary(run_metadata: dict, output_path: Path):
    """qc/summary.txt (formats.py:49-57)."""
    with open(output_path, "w") as f:
        f.write("mgatk2 Run Summary\n")
        f.write("=" * 20 + "\n")
        for key, value in run_metadata.items():
            if key != "parameters":
                f.write(f"{key}: {value}\n")
