#!/bin/bash
# Round 5: the streamed step's pileup granularity: workgroups per one-window launch
# (MGP_PILE_WG_STREAM; cells per chunk = ceil(cells / it), at least 2) and windows per
# segment (MGP_SEG_MIN_WIN), alternating, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
    bash scripts/ab_stream.sh MGP_PILE_WG_STREAM=1024 MGP_PILE_WG_STREAM=3334 MGP_PILE_WG_STREAM=5000 \
        MGP_SEG_MIN_WIN=2 MGP_SEG_MIN_WIN=2,MGP_PILE_WG_STREAM=1024 >> gpurun_out/abs_r5y.txt 2>&1 \
        || { cat gpurun_out/abs_r5y.txt; exit 1; }
done
cat gpurun_out/abs_r5y.txt
