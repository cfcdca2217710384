#!/bin/bash
# Round 3 (session 2) end pass: A/B of VARIANTS against the current library (C4 and the
# 8-GPU share), then gpu_final.sh (GPU suite, default bench line, rocprofv3 kernel
# stats, FETCH/WRITE PMC passes).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "${VARIANTS:-}" ]; then SKIP_TESTS=1 bash scripts/gpu_r3e.sh || exit 1; fi
bash scripts/gpu_final.sh
