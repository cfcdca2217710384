#!/bin/bash
# Round 5: C4 end to end (BAM -> files) on one GPU: producer record layout A/B (32-byte
# records the host filters vs 64-byte records the kernel filters), txt at gzip 9 and 1,
# hdf5; then the cells over 8 engine contexts of this GPU (the 8-device product path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export MGP_HOST_PROFILE=1
timeout -k 10 700 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --threads 16 --modes stream \
    --formats txt,hdf5 --records 32,64 --gzip-levels 9,1 --out /tmp/mgp_e2e > gpurun_out/e2e_c4_r5f.log 2>&1; rc=$?
grep '^{' gpurun_out/e2e_c4_r5f.log > gpurun_out/e2e_c4_r5f.json
grep -E "^\[e2e\]|mgp_bam_stream" gpurun_out/e2e_c4_r5f.log | cut -c1-400
[ $rc -eq 0 ] || { tail -20 gpurun_out/e2e_c4_r5f.log; exit $rc; }
timeout -k 10 400 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --threads 16 --modes stream \
    --formats txt --records 32 --gzip-levels 1 --devices 0,0,0,0,0,0,0,0 --reuse-bam --out /tmp/mgp_e2e \
    > gpurun_out/e2e_c4x8_r5f.log 2>&1; rc=$?
grep '^{' gpurun_out/e2e_c4x8_r5f.log > gpurun_out/e2e_c4x8_r5f.json
grep -E "^\[e2e\]|mgp_bam_stream" gpurun_out/e2e_c4x8_r5f.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
# bench.py's multi-rank path: 2 ranks on this one GPU (no RCCL: it refuses two ranks on a device)
MGP_BENCH_NO_COMM=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/rehearse2_r5f.log 2>&1; rc=$?
grep '^{' gpurun_out/rehearse2_r5f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','n_gpus','bit_exact','value_device')}, d['stream'])"
exit $rc
