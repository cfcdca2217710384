#!/bin/bash
# A/B of the stage events on one box: the timed steps with every stage bracketed
# by HIP events (MGP_BENCH_ALL_STAGES=1) against the pileup's only (the default).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $A > gpurun_out/ev_0warm.log 2>&1 || exit $?
timeout -k 10 300 $A > gpurun_out/ev_1pile.log 2>&1 || exit $?
MGP_BENCH_ALL_STAGES=1 timeout -k 10 300 $A > gpurun_out/ev_2all.log 2>&1 || exit $?
timeout -k 10 300 $A > gpurun_out/ev_3pile.log 2>&1 || exit $?
MGP_BENCH_ALL_STAGES=1 timeout -k 10 300 $A > gpurun_out/ev_4all.log 2>&1 || exit $?
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/ev_*.log")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"],3), round(d["roofline"]["frac"],3), {k:v for k,v in d["stage_ms"].items() if v})
PY
