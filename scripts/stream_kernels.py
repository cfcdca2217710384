"""The streamed headline step's per-kernel table from a rocprofv3 --stats summary of
`bench.py` (head-only: W warmup + K timed passes, nothing else launched per pass):
every kernel's calls and GPU milliseconds per step, into a JSON that bench.py attaches
to its line when the workload matches (profiles/stream_kernels.json).

    python scripts/stream_kernels.py KERNEL_STATS.csv PASSES OUT.json --reads N --cells C
"""

from __future__ import annotations

import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("passes", type=int)
    ap.add_argument("out")
    ap.add_argument("--reads", type=int, default=200_000_000)
    ap.add_argument("--cells", type=int, default=10_000)
    ap.add_argument("--source", default="")
    a = ap.parse_args()
    rows = {}
    for r in csv.DictReader(open(a.stats)):
        name = r["Name"].split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]
        calls, tot = int(r["Calls"]), float(r["TotalDurationNs"])
        if calls < a.passes:  # (set-up kernels: the generator, one-time fills)
            continue
        e = rows.setdefault(name, [0, 0.0])
        e[0] += calls
        e[1] += tot
    table = {k: {"calls_per_step": round(c / a.passes, 2), "ms_per_step": round(t / a.passes / 1e6, 4)}
             for k, (c, t) in sorted(rows.items(), key=lambda kv: -kv[1][1])}
    out = {"reads": a.reads, "cells": a.cells, "record_layout": "packed", "passes": a.passes, "source": a.source,
           "gpu_ms_per_step": round(sum(v["ms_per_step"] for v in table.values()), 3), "kernels": table}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
