#!/bin/bash
# A/B of library variants on one box: a discarded warm-up run, then base, each
# variant, and base again (order effects show up as base/base2 differences).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A="python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $A > gpurun_out/abl_0warm.log 2>&1 || exit $?
timeout -k 10 300 $A > gpurun_out/abl_1base.log 2>&1 || exit $?
for v in "$@"; do
  MGP_LIB=mgatk2_amd/_lib/$v timeout -k 10 300 $A > gpurun_out/abl_2_$(basename $v .so).log 2>&1 || exit $?
done
timeout -k 10 300 $A > gpurun_out/abl_3base2.log 2>&1 || exit $?
python - <<'PY'
import json,glob
for f in sorted(glob.glob("gpurun_out/abl_*.log")):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"],3), {k:v for k,v in d["stage_ms"].items() if v})
PY
