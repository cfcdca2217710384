#!/bin/bash
# Round 5 final pass B: one rank's 8-GPU share of C4 on one GPU (25M reads x 1250 cells),
# a 2-rank rehearsal of the multi-process line (both ranks on this GPU, no RCCL), then the
# kernel stats and FETCH/WRITE PMC passes of the streamed and resident legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r5fb}
timeout -k 10 300 python -u bench.py --reads 25000000 --cells 1250 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
    --no-pcie --no-device-paired --no-host-pack > gpurun_out/bench_share8_$V.log 2>&1 || { tail -20 gpurun_out/bench_share8_$V.log; exit 1; }
grep '^{' gpurun_out/bench_share8_$V.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('share8: value', d['value'], 'ms', d['ms_per_step'], 'link', d['link']['h2d_GBps'], 'device ms', d['device_ms_quad32'], 'bit_exact', d['bit_exact'])"
MGP_BENCH_NO_COMM=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline \
    > gpurun_out/rehearse2_$V.log 2>&1 || { tail -20 gpurun_out/rehearse2_$V.log; exit 1; }
grep '^{' gpurun_out/rehearse2_$V.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('2 ranks: value', d['value'], 'ms', d['ms_per_step'], 'n_gpus', d['n_gpus'], 'bit_exact', d['bit_exact'], 'e2e', d['e2e'])"
STEPS=prof,pmc V=$V bash scripts/gpu_r5g.sh
