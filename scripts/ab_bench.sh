#!/bin/bash
# Default bench with the default library and A/B variants (MGP_LIB), stage times per run.
#   scripts/ab_bench.sh [variant.so ...]   (extra bench args in BARGS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BARGS=${BARGS:-"--device-only --steps 10 --warmup 2 --no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack"}
for lib in base "$@"; do
    # a variant is a library (libmgpileup_x.so) or an environment setting (ENV:NAME=VALUE)
    unset MGP_LIB
    envset=()
    if [[ $lib == ENV:* ]]; then envset=("${lib#ENV:}"); elif [ "$lib" != base ]; then export MGP_LIB=mgatk2_amd/_lib/$lib; fi
    timeout -k 10 240 env "${envset[@]}" python bench.py $BARGS > "gpurun_out/ab_$lib.log" 2>&1 || { echo "$lib failed"; tail -5 "gpurun_out/ab_$lib.log"; exit 1; }
    python - "$lib" <<'PY'
import json, sys
line = [l for l in open(f"gpurun_out/ab_{sys.argv[1]}.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[1]:32s} ms/step {d['ms_per_step']:.3f}", " ".join(f"{k} {v:.3f}" for k, v in d["stage_ms"].items()))
PY
done
