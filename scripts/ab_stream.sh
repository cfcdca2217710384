#!/bin/bash
# A/B of the streamed headline step (bench.py's default line): each variant is an
# environment setting list (NAME=V,NAME2=V2) or "base"; the line's step, link rate and
# the streamed pileup's HIP-event time per run.
#   scripts/ab_stream.sh [MGP_H2D_SPLIT=2 ...]   (extra bench args in BARGS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BARGS=${BARGS:-"--steps 5 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired --no-host-pack"}
for v in base "$@"; do
    envset=()
    if [ "$v" != base ]; then IFS=',' read -ra envset <<< "$v"; fi
    tag=${v//[^A-Za-z0-9_=]/_}
    timeout -k 10 300 env "${envset[@]}" python bench.py $BARGS > "gpurun_out/abs_$tag.log" 2>&1 || { echo "$v failed"; tail -5 "gpurun_out/abs_$tag.log"; exit 1; }
    python - "$tag" "$v" <<'PY'
import json, sys
line = [l for l in open(f"gpurun_out/abs_{sys.argv[1]}.log") if l.startswith("{")][-1]
d = json.loads(line)
r = d["roofline"]
print(f"{sys.argv[2]:36s} ms/step {d['ms_per_step']:.2f} value {d['value'] / 1e9:.4f} G/s h2d {d['link']['h2d_GBps']:.1f} GB/s "
      f"pileup/run {d['stage_ms']['pileup_per_run']:.3f} ms launches {r['launches_per_step']:.0f} frac {r['frac']:.3f}")
PY
done
