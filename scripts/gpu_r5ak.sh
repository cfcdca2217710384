#!/bin/bash
# Round 5: SQ counters of the streamed step's k_pileup (one PMC pass, 8 SQ counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
HEAD="--steps 2 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired --no-host-pack --no-e2e"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-include-regex "k_pileup" --output-format csv -d gpurun_out/sq_head -o pmc \
    -- python bench.py $HEAD > gpurun_out/sq_head.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/sq_head.log; exit 1; }
f=$(find gpurun_out/sq_head -name "*counter_collection.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:24s} n={len(v):3d} mean per launch {sum(v) / len(v):.4g}")
PY
