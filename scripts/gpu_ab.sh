#!/bin/bash
# A/B: bench the default library and a variant (MGP_LIB), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=${1:?variant .so}
A="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
for r in 1 2; do
  timeout -k 10 300 $A > gpurun_out/ab_base_$r.log 2>&1 || exit $?
  MGP_LIB=$V timeout -k 10 300 $A > gpurun_out/ab_var_$r.log 2>&1 || exit $?
done
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/ab_*.log")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"],3), {k:v for k,v in d["stage_ms"].items() if v})
PY
