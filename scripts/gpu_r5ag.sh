#!/bin/bash
# Round 5: pipeline GPU tests with and without the rows target, then C4 end to end at the
# new default (rows fetched after the run): txt gzip 9 and 1, HDF5.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r5ag}
timeout -k 10 700 python -u -m pytest tests/test_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_pipe_$V.log 2>&1 || { tail -30 gpurun_out/pytest_pipe_$V.log; exit 1; }
tail -1 gpurun_out/pytest_pipe_$V.log
MGP_HOST_PROFILE=1 timeout -k 10 500 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 \
    --modes stream --formats txt,hdf5 --gzip-levels 9,1 --out /tmp/mgp_e2e_c4 > gpurun_out/e2e_c4_$V.log 2>&1 \
    || { tail -20 gpurun_out/e2e_c4_$V.log; exit 1; }
grep "^{" gpurun_out/e2e_c4_$V.log > gpurun_out/e2e_c4_$V.json
python -c "
import json; d=json.load(open('gpurun_out/e2e_c4_$V.json'))
print(d.get('txt_identical_across_runs'), {k: (v['wall_s'], v['bam_ingest'], v['write'], v['engine_fetch']) for k, v in d.items() if isinstance(v, dict)})"
timeout -k 10 200 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --modes stream --formats txt,hdf5 \
    --gzip-levels 1 --out /tmp/mgp_e2e_c4 --reuse-bam > gpurun_out/e2e_c4b_$V.log 2>&1 || { tail -20 gpurun_out/e2e_c4b_$V.log; exit 1; }
grep "^{" gpurun_out/e2e_c4b_$V.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print({k: (v['wall_s'], v['bam_ingest'], v['write']) for k, v in d.items() if isinstance(v, dict)})"
