#!/bin/bash
# Round 3 (session 2): GPU suite, the default bench line (PCIe leg included), then
# the A/B of VARIANTS (scripts/gpu_r3e.sh without its tests).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-x}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$V.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$V.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$V.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/bench_$V.log 2>&1 || { tail -20 gpurun_out/bench_$V.log; exit 1; }
tail -c 1500 gpurun_out/bench_$V.log
[ -n "${VARIANTS:-}" ] && SKIP_TESTS=1 bash scripts/gpu_r3e.sh
exit 0
