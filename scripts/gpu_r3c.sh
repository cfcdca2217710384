#!/bin/bash
# Round 3 (session 2): the end-of-round pass on the committed library (gpu_final.sh),
# then A/B of the variant libraries given in VARIANTS at C4 and at the 8-GPU share of C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${SKIP_FINAL:-0}" = 0 ]; then
    bash scripts/gpu_final.sh || exit 1
fi
for args in "" "--reads 25000000 --cells 1250"; do
    echo "== A/B $args"
    MGP_BENCH_ALL_STAGES=1 BARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-check --no-pcie $args" \
        bash scripts/ab_bench.sh ${VARIANTS:-} || exit 1
done
