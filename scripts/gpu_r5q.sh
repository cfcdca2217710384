#!/bin/bash
# Round 5: 16-bit columns (mgp_push_batch16): the stream tests, then the streamed step
# with 16-bit and 32-bit columns, and the small bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_stream_r5q.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_stream_r5q.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_stream_r5q.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --reads 2000000 --cells 500 --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_small_r5q.log 2>&1 || { tail -20 gpurun_out/bench_small_r5q.log; exit 1; }
grep '^{' gpurun_out/bench_small_r5q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['bit_exact'], d['stream'])"
BARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired --no-host-pack --columns 32" \
    bash scripts/ab_stream.sh > gpurun_out/abs_r5q32.txt 2>&1; cat gpurun_out/abs_r5q32.txt
bash scripts/ab_stream.sh > gpurun_out/abs_r5q16.txt 2>&1; rc=$?
cat gpurun_out/abs_r5q16.txt
exit $rc
