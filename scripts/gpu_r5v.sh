#!/bin/bash
# Round 5 final C4 end to end: txt at gzip 9 (default) and 1, HDF5, and C4 through 8
# engine contexts of one GPU (txt gzip 1), with the decoder's stage profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r5v}
E="python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --modes stream --out /tmp/mgp_e2e_c4"
MGP_HOST_PROFILE=1 timeout -k 10 500 $E --formats txt,hdf5 --gzip-levels 9,1 > gpurun_out/e2e_c4_final_$V.log 2>&1 \
    || { tail -20 gpurun_out/e2e_c4_final_$V.log; exit 1; }
grep "^{" gpurun_out/e2e_c4_final_$V.log > gpurun_out/e2e_c4_final_$V.json
grep -o "'wall_s': [0-9.]*\|'bam_ingest': [0-9.]*\|'write': [0-9.]*" gpurun_out/e2e_c4_final_$V.log | tr '\n' ' '; echo
MGP_HOST_PROFILE=1 timeout -k 10 200 $E --formats txt --gzip-levels 1 --reuse-bam --devices 0,0,0,0,0,0,0,0 \
    > gpurun_out/e2e_c4x8_final_$V.log 2>&1 || { tail -20 gpurun_out/e2e_c4x8_final_$V.log; exit 1; }
grep "^{" gpurun_out/e2e_c4x8_final_$V.log > gpurun_out/e2e_c4x8_final_$V.json
grep -o "'wall_s': [0-9.]*\|'bam_ingest': [0-9.]*\|'write': [0-9.]*" gpurun_out/e2e_c4x8_final_$V.log | tr '\n' ' '; echo
MGP_HOST_PROFILE=1 timeout -k 10 200 $E --formats txt --gzip-levels 1 --reuse-bam > gpurun_out/e2e_c4b_final_$V.log 2>&1 \
    || { tail -20 gpurun_out/e2e_c4b_final_$V.log; exit 1; }
grep -o "'wall_s': [0-9.]*\|'bam_ingest': [0-9.]*\|'write': [0-9.]*" gpurun_out/e2e_c4b_final_$V.log | tr '\n' ' '; echo
