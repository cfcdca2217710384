#!/bin/bash
# Round 3 (session 2): the multi-process bench path rehearsed with 2 ranks on this one
# GPU (no RCCL: it refuses two ranks on one device), then C5 (1B reads x 100k cells) on
# one GPU without the CPU leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-x}
MGP_BENCH_NO_COMM=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/rehearse2_$V.log 2>&1 || { tail -20 gpurun_out/rehearse2_$V.log; exit 1; }
tail -c 800 gpurun_out/rehearse2_$V.log
timeout -k 10 500 python -u bench.py --reads 1000000000 --cells 100000 --steps 5 --warmup 1 --no-cpu-baseline \
    --no-check --no-pcie > gpurun_out/bench_c5_$V.log 2>&1 || { tail -20 gpurun_out/bench_c5_$V.log; exit 1; }
tail -c 800 gpurun_out/bench_c5_$V.log
