#!/bin/bash
# Round 5: C4 end to end, the decoder's placement A/B (cell-paired records vs BAM
# order: one decoder pass, no placement thread), 64-byte records, txt gzip 1, twice each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export MGP_HOST_PROFILE=1
E="python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --threads 16 --modes stream --formats txt --gzip-levels 1 --out /tmp/mgp_e2e --reuse-bam"
rm -f gpurun_out/e2e_place_r5k.log
for pl in paired dense paired dense; do
    echo "== MGP_PLACEMENT=$pl" >> gpurun_out/e2e_place_r5k.log
    MGP_PLACEMENT=$pl timeout -k 10 400 $E >> gpurun_out/e2e_place_r5k.log 2>&1 || { tail -20 gpurun_out/e2e_place_r5k.log; exit 1; }
done
MGP_PLACEMENT=dense timeout -k 10 400 $E --formats hdf5 >> gpurun_out/e2e_place_r5k.log 2>&1 || exit 1
grep -E "^==|^\[e2e\] (txt|hdf5)|mgp_bam_stream" gpurun_out/e2e_place_r5k.log | cut -c1-330
