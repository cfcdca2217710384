#!/bin/bash
# Per-kernel times of one short bench (rocprofv3 kernel trace + stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof -o run -- \
    python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/kprof.log 2>&1 || exit $?
f=$(find gpurun_out/kprof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats.csv
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/kernel_stats.csv")):
    print(f'{r["Name"].split("(")[0][:48]:48s} calls={r["Calls"]:>4s} avg_ms={float(r["AverageNs"])/1e6:9.4f}')
PY
