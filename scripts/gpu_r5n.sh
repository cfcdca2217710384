#!/bin/bash
# Round 5: the product's placement A/B at C4 end to end (decoder pairs records on its
# placement thread vs BAM-order records paired on the device), after the pipeline GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_pipe_r5n.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_pipe_r5n.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_pipe_r5n.log | head -20; exit $rc; }
export MGP_HOST_PROFILE=1
E="python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --threads 16 --modes stream --formats txt --gzip-levels 1 --out /tmp/mgp_e2e --reuse-bam"
rm -f gpurun_out/e2e_place_r5n.log
for pl in device paired device paired; do
    echo "== MGP_PLACEMENT=$pl" >> gpurun_out/e2e_place_r5n.log
    MGP_PLACEMENT=$pl timeout -k 10 400 $E >> gpurun_out/e2e_place_r5n.log 2>&1 || { tail -20 gpurun_out/e2e_place_r5n.log; exit 1; }
done
MGP_PLACEMENT=device timeout -k 10 400 $E --formats hdf5 >> gpurun_out/e2e_place_r5n.log 2>&1 || exit 1
grep -E "^==|^\[e2e\] (txt|hdf5)|mgp_bam_stream" gpurun_out/e2e_place_r5n.log | cut -c1-300
