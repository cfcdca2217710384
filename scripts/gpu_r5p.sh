#!/bin/bash
# Round 5: C4 through 8 engine contexts of one GPU (64-byte records, paired on each
# device) against one context, txt gzip 1, on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export MGP_HOST_PROFILE=1
E="python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --threads 16 --modes stream --formats txt --gzip-levels 1 --out /tmp/mgp_e2e --reuse-bam"
timeout -k 10 600 $E > gpurun_out/e2e_c4_r5p.log 2>&1 || { tail -20 gpurun_out/e2e_c4_r5p.log; exit 1; }
timeout -k 10 400 $E --devices 0,0,0,0,0,0,0,0 > gpurun_out/e2e_c4x8_r5p.log 2>&1 || { tail -20 gpurun_out/e2e_c4x8_r5p.log; exit 1; }
timeout -k 10 400 $E > gpurun_out/e2e_c4b_r5p.log 2>&1 || { tail -20 gpurun_out/e2e_c4b_r5p.log; exit 1; }
for f in e2e_c4_r5p e2e_c4x8_r5p e2e_c4b_r5p; do grep '^{' gpurun_out/$f.log > gpurun_out/$f.json; grep -E "^\[e2e\] (txt|hdf5)|mgp_bam_stream" gpurun_out/$f.log | cut -c1-300; done
