#!/bin/bash
# Round 5: per-dispatch durations of the streamed step's kernels (kernel trace), to see
# where the pileup's 13 launches spend their time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
HEAD="--steps 3 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired --no-host-pack --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ktr_head -o run -- python bench.py $HEAD \
    > gpurun_out/ktr_head.log 2>&1 || { tail -5 gpurun_out/ktr_head.log; exit 1; }
f=$(find gpurun_out/ktr_head -name "*kernel_trace.csv" | head -1)
cp "$f" gpurun_out/kernel_trace_head_r5aa.csv
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/kernel_trace_head_r5aa.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pile = [r for r in rows if "k_pileup" in r["Kernel_Name"]]
print("pileup dispatches", len(pile))
last = pile[-13:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  start {(s - t0) / 1e6:9.3f} ms  dur {(e - s) / 1e3:8.1f} us  grid {r.get('Grid_Size_X', r.get('Grid_Size', '?'))} x {r.get('Grid_Size_Y', '?')}")
# kernels of the last step between the first and last pileup, with gaps
seg = [r for r in rows if int(r["Start_Timestamp"]) >= int(last[0]["Start_Timestamp"]) - 3_000_000 and int(r["End_Timestamp"]) <= int(last[-1]["End_Timestamp"]) + 3_000_000]
tot = {}
for r in seg:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    tot[n] = tot.get(n, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for n, v in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"  {n:40s} {v:8.3f} ms")
PY
