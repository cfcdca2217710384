#!/bin/bash
# Round 5: record-copy workgroups per pairing range (MGP_PAIR_SPLIT 1 / 4 / 16 builds):
# the streamed C4 step and one rank's 8-GPU share, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
    for v in split1 split4 base; do
        unset MGP_LIB
        [ $v != base ] && export MGP_LIB=mgatk2_amd/_lib/libmgpileup_$v.so
        bash scripts/ab_stream.sh | sed "s/^base/$v/" >> gpurun_out/abs_r5ac.txt 2>&1
        BARGS="--reads 25000000 --cells 1250 --steps 10 --warmup 2 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired --no-host-pack --no-e2e" \
            bash scripts/ab_stream.sh | sed "s/^base/$v share8/" >> gpurun_out/abs_r5ac.txt 2>&1
    done
done
unset MGP_LIB
cat gpurun_out/abs_r5ac.txt
