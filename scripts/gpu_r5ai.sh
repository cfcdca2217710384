#!/bin/bash
# Round 5: the record copy with non-temporal loads/stores (MGP_PAIR_NT=1) against the
# default and one copy workgroup per range: the streamed C4 step and the 8-GPU share.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    -k "dense_64 or push16 or cell_range" > gpurun_out/pytest_pairnt.log 2>&1 || { tail -20 gpurun_out/pytest_pairnt.log; exit 1; }
for i in 1 2; do
    for v in pairnt base split1; do
        unset MGP_LIB
        [ $v != base ] && export MGP_LIB=mgatk2_amd/_lib/libmgpileup_$v.so
        bash scripts/ab_stream.sh | sed "s/^base/$v/" >> gpurun_out/abs_r5ai.txt 2>&1
    done
done
unset MGP_LIB
cat gpurun_out/abs_r5ai.txt
