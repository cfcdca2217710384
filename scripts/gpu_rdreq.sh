#!/bin/bash
# HBM read requests of k_pileup by size (TCC_EA0_RDREQ_{32B,64B,128B}) for the
# packed and full record layouts: one PMC pass per layout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lay in packed full; do
    timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
        TCC_EA0_RDREQ_128B_sum --kernel-include-regex "k_pileup" --output-format csv -d gpurun_out/rdreq_$lay -o pmc \
        -- python bench.py --steps 2 --warmup 0 --no-cpu-baseline --record-layout $lay \
        > gpurun_out/rdreq_$lay.log 2>&1 || exit $?
done
python - <<'PY'
import csv, glob
from collections import defaultdict
for lay in ("packed", "full"):
    acc = defaultdict(list)
    for f in glob.glob(f"gpurun_out/rdreq_{lay}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(lay, {k: f"{sum(v) / len(v):.4g}" for k, v in sorted(acc.items())})
PY
