#!/bin/bash
# Round 5: one rank's 8-GPU share (25M reads x 1250 cells): pileup chunks of at least 1
# cell (1250 workgroups per one-window launch) against 2 (625), alternating; plus the
# 4-GPU share (2500 cells) with 1 against 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
S8="--reads 25000000 --cells 1250 --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-device --no-device-paired --no-host-pack --no-e2e"
S4="--reads 50000000 --cells 2500 --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --no-device --no-device-paired --no-host-pack --no-e2e"
for i in 1 2; do
    BARGS="$S8" bash scripts/ab_stream.sh MGP_PILE_MIN_CPB_STREAM=1 MGP_PILE_MIN_CPB_STREAM=1,MGP_PILE_WG_STREAM=4096 | sed 's/^/share8 /' >> gpurun_out/abs_r5ad.txt 2>&1
    BARGS="$S4" bash scripts/ab_stream.sh MGP_PILE_MIN_CPB_STREAM=1,MGP_PILE_WG_STREAM=4096 | sed 's/^/share4 /' >> gpurun_out/abs_r5ad.txt 2>&1
done
cat gpurun_out/abs_r5ad.txt
grep -h '"bit_exact"' gpurun_out/abs_MGP_PILE_MIN_CPB_STREAM=1*.log | python -c "import sys,json; [print('bit_exact', json.loads(l)['bit_exact']) for l in sys.stdin if l.startswith('{')]"
