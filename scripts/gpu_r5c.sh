#!/bin/bash
# Round 5: streamed-step A/B (payload copy over 1/2/4 streams, segment width) and the
# rocprof kernel stats of the streamed step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ab_stream.sh MGP_H2D_SPLIT=2 MGP_H2D_SPLIT=4 MGP_SEG_MIN_WIN=2 MGP_SEG_MIN_WIN=3 \
    MGP_H2D_SPLIT=2,MGP_SEG_MIN_WIN=2 > gpurun_out/abs_r5c.txt 2>&1; rc=$?
cat gpurun_out/abs_r5c.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof_s -o run -- \
    python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired \
    --no-host-pack > gpurun_out/kprof_s.log 2>&1 || { tail -5 gpurun_out/kprof_s.log; exit 1; }
f=$(find gpurun_out/kprof_s -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_stream_r5c.csv
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/kernel_stats_stream_r5c.csv")):
    print(f'{r["Name"].split("(")[0][:48]:48s} calls={r["Calls"]:>5s} avg_ms={float(r["AverageNs"])/1e6:9.4f} tot_ms={float(r["TotalDurationNs"])/1e6:9.2f}')
PY
grep '^{' gpurun_out/kprof_s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline'], d['ms_per_step'])"
