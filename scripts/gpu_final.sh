#!/bin/bash
# End-of-round pass: the whole GPU suite, the default bench line, the rocprofv3 kernel
# stats and the FETCH/WRITE PMC passes of the default bench (gpu_round3.sh steps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-final}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$V.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_$V.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$V.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$V.log 2>&1 || { tail -20 gpurun_out/bench_$V.log; exit 1; }
tail -c 600 gpurun_out/bench_$V.log
STEPS=rocprof,pmc bash scripts/gpu_round3.sh > gpurun_out/prof_$V.log 2>&1 || { tail -20 gpurun_out/prof_$V.log; exit 1; }
grep "rc=" gpurun_out/prof_$V.log
