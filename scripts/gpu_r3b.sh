#!/bin/bash
# Round 3 second pass: pass-A variants A/B, the C3 end-to-end pipeline (txt) and the C5
# PCIe-inclusive batch-size sweep. Each step has its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-ab,e2e,c5}
if [[ $STEPS == *ab* ]]; then
    timeout -k 10 400 bash scripts/ab_bench.sh ${AB_LIBS:-} > gpurun_out/ab_r3b.txt 2>&1 || { cat gpurun_out/ab_r3b.txt; exit 1; }
    cat gpurun_out/ab_r3b.txt
fi
if [[ $STEPS == *e2e* ]]; then
    timeout -k 10 400 python -u scripts/e2e_bench.py --formats txt --out /tmp/mgp_e2e > gpurun_out/e2e_c3.log 2>&1 \
        || { tail -20 gpurun_out/e2e_c3.log; exit 1; }
    tail -2 gpurun_out/e2e_c3.log | cut -c1-2000
fi
if [[ $STEPS == *c5* ]]; then
    timeout -k 10 600 python -u bench.py --reads 1000000000 --cells 100000 --steps 3 --warmup 1 --no-cpu-baseline \
        --batch-reads 16000000,1000000,4000000,64000000 > gpurun_out/bench_c5_sweep.log 2>&1 \
        || { tail -20 gpurun_out/bench_c5_sweep.log; exit 1; }
    tail -c 3000 gpurun_out/bench_c5_sweep.log
fi
