#!/bin/bash
# Round 5: k_pair_place over 16 workgroups per range: the pairing/stream tests, then the
# streamed step's kernel trace and the A/B of the step (MGP_PAIR_SPLIT=1 build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_stream_r5ab.log 2>&1 || { tail -30 gpurun_out/pytest_stream_r5ab.log; exit 1; }
tail -1 gpurun_out/pytest_stream_r5ab.log
bash scripts/gpu_r5aa.sh || exit 1
for i in 1 2; do
    MGP_LIB=mgatk2_amd/_lib/libmgpileup_split1.so bash scripts/ab_stream.sh | sed 's/^base/split1/' >> gpurun_out/abs_r5ab.txt 2>&1
    bash scripts/ab_stream.sh >> gpurun_out/abs_r5ab.txt 2>&1
done
cat gpurun_out/abs_r5ab.txt
