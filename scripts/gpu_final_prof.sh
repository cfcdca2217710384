#!/bin/bash
# The headline step's kernel table and the pileup's HBM traffic for the round's profiles:
# one rocprofv3 --kernel-trace --stats run of the head-only bench (2 warmup + 5 timed passes)
# -> gpurun_out/final_ks (kernel_stats.csv + the bench line), then the PMC passes of
# scripts/pmc_stream.sh -> gpurun_out/pmc_traffic_stream.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
HEAD="--steps 5 --warmup 2 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired --no-host-pack --no-e2e"
rm -rf gpurun_out/final_ks
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_ks -o run -- python3 bench.py $HEAD \
    > gpurun_out/final_ks.log 2>&1 || { echo "kernel trace failed"; tail -5 gpurun_out/final_ks.log; exit 1; }
f=$(find gpurun_out/final_ks -name "*kernel_stats.csv" | head -1)
python3 scripts/stream_kernels.py "$f" 7 gpurun_out/stream_kernels.json --source "$f (scripts/gpu_final_prof.sh, 2 warmup + 5 timed passes)" > /dev/null
scripts/pmc_stream.sh
