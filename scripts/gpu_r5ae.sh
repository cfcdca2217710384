#!/bin/bash
# Round 5: the stream tests at one-cell pileup chunks, then C4 end to end with the
# pooled txt writer (gzip 9 and 1) and HDF5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r5ae}
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_pipeline.py -m gpu -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_stream_$V.log 2>&1 || { tail -30 gpurun_out/pytest_stream_$V.log; exit 1; }
tail -1 gpurun_out/pytest_stream_$V.log
MGP_TXT_PROFILE=1 MGP_HOST_PROFILE=1 timeout -k 10 500 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 \
    --modes stream --formats txt,hdf5 --gzip-levels 9,1 --out /tmp/mgp_e2e_c4 > gpurun_out/e2e_c4_$V.log 2>&1 \
    || { tail -20 gpurun_out/e2e_c4_$V.log; exit 1; }
grep "^{" gpurun_out/e2e_c4_$V.log > gpurun_out/e2e_c4_$V.json
grep "\[mgp_txt\]" gpurun_out/e2e_c4_$V.log
python -c "
import json; d=json.load(open('gpurun_out/e2e_c4_$V.json'))
print(d.get('txt_identical_across_runs'), {k: (v['wall_s'], v['bam_ingest'], v['write']) for k, v in d.items() if isinstance(v, dict)})"
