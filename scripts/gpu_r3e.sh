#!/bin/bash
# Round 3 (session 2): A/B of VARIANTS against the current library (C4 and the 8-GPU
# share), then the GPU suite on the current library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-x}
IFS=';' read -ra SIZES <<< "${ABSIZES:-;--reads 25000000 --cells 1250}"
for args in "${SIZES[@]}"; do
    echo "== A/B $args"
    BARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-check --no-pcie $args" \
        bash scripts/ab_bench.sh ${VARIANTS:-} || exit 1
done
if [ "${SKIP_TESTS:-0}" = 0 ]; then
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/pytest_gpu_$V.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$V.log; exit 1; }
    tail -2 gpurun_out/pytest_gpu_$V.log
fi
