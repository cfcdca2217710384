#!/bin/bash
# A/B of payload layouts on one box (bench.py --record-layout), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for r in 1 2; do
  for lay in ${LAYOUTS:-paired packed}; do
    timeout -k 10 300 $A --record-layout $lay > gpurun_out/lay_${lay}_$r.log 2>&1 || exit $?
  done
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/lay_*.log")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"],3), round(d["roofline"]["frac"],3), {k:v for k,v in d["stage_ms"].items() if v})
PY
