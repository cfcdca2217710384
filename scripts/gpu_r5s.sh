#!/bin/bash
# Round 5: the default bench line (now with the end-to-end leg), then C4 end to end with
# the SIMD 64-byte record build and the pooled record list, and the same BAM with the
# definition's record loop (MGP_NO_SSSE3=1) for A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r5s}
if [[ ${STEPS:-bench,e2e} == *bench* ]]; then
    timeout -k 10 600 python -u bench.py > gpurun_out/bench_$V.log 2>&1 || { tail -20 gpurun_out/bench_$V.log; exit 1; }
    grep '^{' gpurun_out/bench_$V.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['bit_exact']); print(json.dumps(d['e2e']))"
fi
if [[ ${STEPS:-bench,e2e} == *e2e* ]]; then
    MGP_HOST_PROFILE=1 timeout -k 10 400 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --formats txt,hdf5 \
        --modes stream --gzip-levels 1 --out /tmp/mgp_e2e_c4 > gpurun_out/e2e_c4_$V.log 2>&1 \
        || { tail -20 gpurun_out/e2e_c4_$V.log; exit 1; }
    grep "^\[mgp_bam_stream\]\|wall_s" gpurun_out/e2e_c4_$V.log | cut -c1-400
    MGP_NO_SSSE3=1 MGP_HOST_PROFILE=1 timeout -k 10 200 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 \
        --formats txt --modes stream --gzip-levels 1 --out /tmp/mgp_e2e_c4 --reuse-bam > gpurun_out/e2e_c4_nossse3_$V.log 2>&1 \
        || { tail -20 gpurun_out/e2e_c4_nossse3_$V.log; exit 1; }
    grep "^\[mgp_bam_stream\]\|wall_s" gpurun_out/e2e_c4_nossse3_$V.log | cut -c1-400
    MGP_HOST_PROFILE=1 timeout -k 10 200 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 \
        --formats txt --modes stream --gzip-levels 1 --out /tmp/mgp_e2e_c4 --reuse-bam > gpurun_out/e2e_c4b_$V.log 2>&1 \
        || { tail -20 gpurun_out/e2e_c4b_$V.log; exit 1; }
    grep "^\[mgp_bam_stream\]\|wall_s" gpurun_out/e2e_c4b_$V.log | cut -c1-400
fi
