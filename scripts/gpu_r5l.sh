#!/bin/bash
# Round 5: why a streamed one-window pileup launch costs 1.5x a resident window:
# resident pileup on dense BAM-order 64-byte records vs cell-paired ones, and the
# streamed step at smaller chunks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for lay in packed paired; do
    BARGS="--device-only --record-layout $lay --steps 10 --warmup 2 --no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack" \
        bash scripts/ab_bench.sh > gpurun_out/ab_lay_$lay.txt 2>&1 || { cat gpurun_out/ab_lay_$lay.txt; exit 1; }
    echo "$lay: $(cat gpurun_out/ab_lay_$lay.txt)"
done
bash scripts/ab_stream.sh MGP_PILE_WG_STREAM=8192 MGP_PILE_WG_STREAM=8192,MGP_SEG_MIN_WIN=2 MGP_PILE_WG_STREAM=4096,MGP_SEG_MIN_WIN=3 \
    > gpurun_out/abs_r5l.txt 2>&1; rc=$?
cat gpurun_out/abs_r5l.txt
exit $rc
