#!/bin/bash
# Round 5: C4 end to end with the one-pass BAM-order decode (records written in the
# columns' pass), txt gzip 1 twice, hdf5 once, txt gzip 9 once; then the 8-context run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export MGP_HOST_PROFILE=1
E="python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --threads 16 --modes stream --out /tmp/mgp_e2e --reuse-bam"
timeout -k 10 600 $E --formats txt,hdf5,txt --gzip-levels 1 > gpurun_out/e2e_c4_r5o.log 2>&1 || { tail -20 gpurun_out/e2e_c4_r5o.log; exit 1; }
timeout -k 10 400 $E --formats txt --gzip-levels 9 > gpurun_out/e2e_c4z9_r5o.log 2>&1 || { tail -20 gpurun_out/e2e_c4z9_r5o.log; exit 1; }
timeout -k 10 400 $E --formats txt --gzip-levels 1 --devices 0,0,0,0,0,0,0,0 > gpurun_out/e2e_c4x8_r5o.log 2>&1 || { tail -20 gpurun_out/e2e_c4x8_r5o.log; exit 1; }
for f in e2e_c4_r5o e2e_c4z9_r5o e2e_c4x8_r5o; do grep '^{' gpurun_out/$f.log > gpurun_out/$f.json; grep -E "^\[e2e\] (txt|hdf5)|mgp_bam_stream" gpurun_out/$f.log | cut -c1-300; done
