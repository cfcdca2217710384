#!/bin/bash
# Round 5: on-device pairing of dense 64-byte batches: the stream tests, then the
# streamed step with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_stream_r5m.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_stream_r5m.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_stream_r5m.log | head -20; exit $rc; }
bash scripts/ab_stream.sh MGP_DEV_PAIR=0 > gpurun_out/abs_r5m.txt 2>&1; rc=$?
cat gpurun_out/abs_r5m.txt
exit $rc
