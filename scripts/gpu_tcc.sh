#!/bin/bash
# Fabric request counts (reads, writes by size) and L2 hit/miss for the C4 step's
# kernels: one rocprofv3 PMC pass per counter group (at most 4 TCC counters each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-base}
K="k_pileup|k_group_a|k_group_b|k_bin_count|k_median"
i=0
for grp in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$K" --output-format csv \
        -d gpurun_out/tcc_${TAG}_$i -o pmc -- python bench.py --steps 2 --warmup 0 --no-cpu-baseline \
        > gpurun_out/tcc_${TAG}_$i.log 2>&1 || exit $?
done
python - "$TAG" <<'PY'
import csv, glob, sys, re
from collections import defaultdict
tag = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"gpurun_out/tcc_{tag}_*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = re.match(r"(?:void )?(\w+)", row["Kernel_Name"]).group(1)
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in sorted(acc.items()):
    print(k, {c: f"{sum(v) / len(v):.4g}" for c, v in sorted(d.items())})
PY
