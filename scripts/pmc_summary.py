"""Summarise rocprofv3 --pmc CSVs: per kernel, mean counter value per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/pmc_*/**/*counter_collection.csv", recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "?").split("(")[0]
            acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in sorted(acc.items()):
    print(k)
    for c, v in sorted(cs.items()):
        # values are per dispatch (already summed over dimensions by rocprofv3)
        print(f"   {c:28s} n={len(v):3d} mean={sum(v) / len(v):.6g}")
