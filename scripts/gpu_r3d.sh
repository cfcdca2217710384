#!/bin/bash
# Round 3 (session 2): the GPU suite on the current library, A/B against VARIANTS at C4
# and at the 8-GPU share of C4 (timed steps as the bench times them: only the pileup
# bracketed), then the C3 end-to-end pipeline (scripts/e2e_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-x}
if [ "${SKIP_TESTS:-0}" = 0 ]; then
    timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/pytest_gpu_$V.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$V.log; exit 1; }
    tail -2 gpurun_out/pytest_gpu_$V.log
fi
for args in "" "--reads 25000000 --cells 1250"; do
    echo "== A/B $args"
    BARGS="--steps 20 --warmup 3 --no-cpu-baseline --no-check --no-pcie $args" \
        bash scripts/ab_bench.sh ${VARIANTS:-} || exit 1
done
if [ "${E2E:-1}" = 1 ]; then
    timeout -k 10 400 python -u scripts/e2e_bench.py --out /tmp/mgp_e2e > gpurun_out/e2e_c3_$V.log 2>&1 \
        || { tail -20 gpurun_out/e2e_c3_$V.log; exit 1; }
    tail -3 gpurun_out/e2e_c3_$V.log | cut -c1-1500
fi
